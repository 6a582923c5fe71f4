"""Where does a stale HIP error come from after the communicator test's sequence (VERDICT r5
weak 1: `hipErrorCapturedEvent` reported by a pipeline launched after a one-rank RCCL gather
on the NULL stream, synchronize, ncclCommDestroy)?  Replays the sequence in one process and
peeks at the thread's HIP last-error slot (hipPeekAtLastError: no reset) after every step,
then runs a device-post Remove pipeline.  `--stream null|real` picks the gather's stream.

    python tools/debug/comm_pending_probe.py --stream null
"""
import argparse
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# ZARU_PROBE_ROOT: import zaru_amd from another tree (alt/r05: the round-5 build, package + .so)
sys.path.insert(0, os.path.join(REPO, os.environ["ZARU_PROBE_ROOT"]) if os.environ.get("ZARU_PROBE_ROOT") else REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stream", choices=["null", "real"], default="null")
    ap.add_argument("--gathers", type=int, default=2)
    ap.add_argument("--skip-destroy", action="store_true")
    ap.add_argument("--repeat", type=int, default=1, help="replay the whole sequence this many times")
    ap.add_argument("--force-pending", action="store_true",
                    help="leave a HIP error pending before the gathers (hipSetDevice(9999) through ctypes), as the "
                         "round-5 library's unconsumed memcpy2d failure did")
    a = ap.parse_args()
    for it in range(a.repeat):
        print(f"=== iteration {it}", flush=True)
        if not one(a, it):
            print("STALE ERROR REPRODUCED", flush=True)
            break


def one(a, it):
    import numpy as np
    from zaru_amd._lib import Comm, DeviceBuffer, lib, synchronize
    hip = C.CDLL(os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib", "libamdhip64.so"))
    hip.hipGetErrorName.restype = C.c_char_p
    log = []

    def peek(what):
        e = hip.hipPeekAtLastError()
        log.append({"after": what, "code": e, "name": hip.hipGetErrorName(e).decode()})
        print(f"{what:48s} -> {e} {log[-1]['name']}", flush=True)

    peek("start")
    comm = Comm(Comm.unique_id(), 1, 0, 0)
    peek("zr_comm_create")
    src, dst = DeviceBuffer(256), DeviceBuffer(256)
    peek("DeviceBuffer x2")
    st = None
    if a.stream == "real":
        sp = C.c_void_p()
        lib().zr_stream_create(C.byref(sp))
        st = sp.value
        peek("zr_stream_create")
    rc = lib().zr_memcpy2d_async(dst.ptr, 4, src.ptr, 256, 256, 1, 2, None)
    peek(f"zr_memcpy2d_async(pitch < width) rc={rc}")
    if a.force_pending:
        peek(f"hipSetDevice(9999) rc={hip.hipSetDevice(9999)}")
    for k in range(a.gathers):
        try:
            comm.all_gather_async(src.ptr, dst.ptr, 256, st)
            peek(f"all_gather #{k} ok")
        except Exception as e:  # noqa: BLE001
            peek(f"all_gather #{k} raised {e}")
    synchronize(st)
    peek("zr_stream_synchronize(stream)")
    if not a.skip_destroy:
        comm.close()
        peek("zr_comm_destroy")
    e = hip.hipDeviceSynchronize()
    peek(f"hipDeviceSynchronize rc={e}")
    import zaru_amd.host as H
    H.set_models_dir(os.path.join(REPO, "zaru_amd", "models"))
    if it == 0:
        print("zaru_amd from", os.path.dirname(H.__file__), flush=True)
    W, Hh, NF = 1920, 1080, 2
    f = np.random.default_rng(1).integers(0, 256, size=(NF, Hh, W, 4), dtype=np.uint8)
    buf = DeviceBuffer.from_array(f)
    flist = [(buf.ptr + i * Hh * W * 4, W, Hh, W * 4) for i in range(NF)]
    peek("frames uploaded")
    p = H.DetectTrackPipeline("hand", 0, 4, 4, 3, True, nms_mode="remove", det_threshold=0.05, device_post=True)
    peek("pipeline created")
    p.set_frames(flist, [[] for _ in range(NF)])
    peek("set_frames")
    ok = True
    try:
        p.run_frames()
        peek("run_frames ok")
    except Exception as ex:  # noqa: BLE001
        peek(f"run_frames raised {ex}")
        ok = False
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", f"comm_probe_{a.stream}_{it}.json"), "w") as fh:
        json.dump(log, fh, indent=1)
    return ok


if __name__ == "__main__":
    main()
