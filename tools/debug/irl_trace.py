"""Per-wave step timeline of irl_kernel (VERDICT r5 ask 4: where does the step lose its cycles?).
Loads the trace build (tools/debug/irl_trace.sh -> tools/debug/trace_lib/libzaru_hip.so, kernels/irl.hip
with ZR_IRL_TRACE), runs hand_landmark_lite at 341 ROIs twice (the second run is read), and prints
for each irl launch the median over the first 16 workgroups and the steady-state steps of:
  M = the MFMA waves' work per step: expand of chunk t (m_expand) + projection of chunk t - 2,
  D = the depthwise waves' work per step: staging (last step's loads stored, the next issued:
      d_staging) + the row tasks (d_depthwise),
  period = step start to next step start, and the barrier wait of each role (period - work),
in shader clocks (s_memtime).

    python tools/debug/irl_trace.py [batch] > gpurun_out/irl_trace.txt
"""
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import zaru_amd._lib as L  # noqa: E402

L.LIB_PATH = os.path.join(REPO, "tools", "debug", "trace_lib", "libzaru_hip.so")
from zaru_amd._lib import DeviceBuffer, synchronize  # noqa: E402
from zaru_amd.nn import NeuralNetwork, model_bytes  # noqa: E402

WG, LAUNCHES, SLOTS = 16, 32, 256
# the hand network's irl launches in plan order: (K, plane, stride, expanded channels)
LAYERS = [(3, 14, 1, 288), (3, 14, 1, 288), (5, 14, 1, 288), (5, 14, 1, 384), (5, 14, 1, 384),
          (5, 14, 2, 384), (5, 7, 1, 672), (5, 7, 1, 672), (5, 7, 1, 672)]


def main():
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 341
    lib = L.lib()
    lib.zr_debug_irl_trace.argtypes = [C.POINTER(C.c_uint64), C.c_size_t, C.c_int]
    nn = NeuralNetwork.from_onnx(model_bytes("hand_landmark_lite")).load()
    shape = nn.inputs()[0][1]
    x = np.random.default_rng(0).uniform(-1, 1, size=(batch,) + tuple(shape[1:])).astype(np.float32)
    din = DeviceBuffer.from_array(x)
    outs = [DeviceBuffer(int(np.prod(s)) * 4) for s in nn.output_shapes(batch)]
    buf = np.zeros(LAUNCHES * WG * 8 * SLOTS, dtype=np.uint64)
    for _ in range(2):
        nn.estimate_device(batch, din.ptr, [o.ptr for o in outs])
        synchronize()
    n = lib.zr_debug_irl_trace(buf.ctypes.data_as(C.POINTER(C.c_uint64)), buf.size, 0)
    assert n == buf.size, n
    tr = buf.reshape(LAUNCHES, WG, 8, SLOTS).astype(np.int64)
    rows = []
    for li, (k, hw, s, cexp) in enumerate(LAYERS):
        launch = len(LAYERS) + li  # the second run
        t = tr[launch]
        nch = cexp // 16
        steps = range(2, nch)  # steady state: both roles busy
        m_work, d_work, period, total, m_first, d_first, d_stores = [], [], [], [], [], [], []
        for w in range(WG):
            if t[w, 0, 0] == 0:
                continue
            total.append(t[w, 0, 255] - t[w, 0, 0])
            for st in steps:
                s0, sm, s1, s2 = 4 * st + 2, 4 * st + 3, 4 * st + 4, 4 * st + 6
                period.append(np.median(t[w, :, s2] - t[w, :, s0]))
                m_work.append(np.median(t[w, 0:4, s1] - t[w, 0:4, s0]))
                d_work.append(np.median(t[w, 4:8, s1] - t[w, 4:8, s0]))
                m_first.append(np.median(t[w, 0:4, sm] - t[w, 0:4, s0]))
                d_first.append(np.median(t[w, 4:8, sm] - t[w, 4:8, s0]))
                d_stores.append(np.median(t[w, 4:8, 4 * st + 5] - t[w, 4:8, s0]))
        if not period:
            continue
        r = dict(layer=f"irl K{k} {hw}^2 s{s} x{cexp}", steps=nch + 2, kernel_clocks=float(np.median(total)),
                 period=float(np.median(period)), m_work=float(np.median(m_work)), d_work=float(np.median(d_work)))
        r["m_expand"] = float(np.median(m_first))
        r["m_project"] = r["m_work"] - r["m_expand"]
        r["d_staging"] = float(np.median(d_first))
        r["d_depthwise"] = r["d_work"] - r["d_staging"]
        r["d_stores"] = float(np.median(d_stores))  # (of d_staging: storing last step's loads)
        r["m_wait"] = r["period"] - r["m_work"]
        r["d_wait"] = r["period"] - r["d_work"]
        r["steps_share"] = r["period"] * (nch + 2) / r["kernel_clocks"]
        rows.append(r)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
