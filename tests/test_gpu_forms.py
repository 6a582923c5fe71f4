"""The kernel forms the launchers choose between compute the same arithmetic in the same order,
so switching a form (ZARU_HIP_FORMS, read once per process) must not change one bit of any model
output.  Each configuration runs in a child process (the switches are process-wide); the
batch is large enough that every form the default build picks is exercised (LDS-DMA staged
VALU and MFMA forms, the windowed V4 taps, the image-row head GEMM); the warp-specialized MFMA
form has a test of its own at 1024 hand ROIs.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
from zaru_amd.nn import NeuralNetwork, model_bytes
out = {}
for model, s in (("face_detection_short_range", 128), ("face_landmark", 192),
                 ("palm_detection_lite", 192), ("hand_landmark_lite", 224)):
    rng = np.random.default_rng(5)
    x = rng.uniform(-1.0, 1.0, size=(36, 3, s, s)).astype(np.float32)
    net = NeuralNetwork.from_onnx(model_bytes(model)).load()
    for i, o in enumerate(net.estimate(x)):
        out[f"{model}/{i}"] = o
np.savez(sys.argv[2], **out)
"""

# each setting turns one form off ("-form"); "all_off" every form
SWITCHES = {
    "default": "",
    "no_valu_db": "-valu_db",
    "no_valu": "-valu",
    "no_dma": "-dma",
    "no_v4": "-v4,-dma",
    "no_rows": "-rows",
    "no_vres": "-vres",
    "no_vstore": "-vstore",
    "no_ws": "-ws",
    "no_groups": "-groups",
    "no_dwgap": "-dwgap",
    "no_rt": "-rt",
    "no_ir": "-ir",
    "no_irl": "-irl",
    "no_bneck": "-bneck",
    "no_pin": "-pin",
    "irl_lds0": "",  # + ZARU_HIP_IRL_LDS (EXTRA_ENV): irl's plain LDS layout / padded, single-buffered rows
    "irl_lds2": "",
    "dma_pad": "",  # + ZARU_HIP_DMA_PAD=1: the bank-padded LDS channel stride of the pin layouts
    "all_off": "-dma,-v4,-valu,-valu_db,-rows,-vres,-vstore,-ws,-groups,-dwgap,-rt,-ir,-irl,-pin",
}
EXTRA_ENV = {"irl_lds0": {"ZARU_HIP_IRL_LDS": "0"}, "irl_lds2": {"ZARU_HIP_IRL_LDS": "2"},
             "dma_pad": {"ZARU_HIP_DMA_PAD": "1"}}  # name -> extra env


@pytest.fixture(scope="module")
def outputs(tmp_path_factory):
    d = tmp_path_factory.mktemp("forms")
    res = {}
    for name, env in SWITCHES.items():
        path = str(d / f"{name}.npz")
        e = dict(os.environ)
        e["ZARU_HIP_FORMS"] = env
        e.update(EXTRA_ENV.get(name, {}))
        subprocess.run([sys.executable, "-c", CHILD, REPO, path], env=e, check=True, timeout=110)
        with np.load(path) as z:
            res[name] = {k: z[k] for k in z.files}
    return res


@pytest.mark.parametrize("name", [n for n in SWITCHES if n != "default"])
def test_form_switch_is_bitwise_neutral(outputs, name):
    base, other = outputs["default"], outputs[name]
    assert base.keys() == other.keys()
    for k in base:
        assert np.array_equal(base[k], other[k]), (name, k, float(np.abs(base[k] - other[k]).max()))


# A full-plane conv with a non-square kernel (x[N,4,3,5] -> Conv 6x4x3x5 -> y[N,6,1,1]) through
# gemm_kernel<., true> (the image-row form switched off, as for a step with a residual): its
# im2col walk must wrap ky at the kernel height, not the width.
NONSQUARE_CHILD = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[1] + "/tests")
from test_lib_cpu import _fld, _vfld, _tensor, _value_info
from zaru_amd.nn import NeuralNetwork
rng = np.random.default_rng(3)
w = rng.uniform(-1, 1, (6, 4, 3, 5)).astype(np.float32)
node = _fld(1, b"x") + _fld(1, b"w") + _fld(2, b"y") + _fld(4, b"Conv")
graph = (_fld(1, node) + _fld(5, _tensor(b"w", w.shape, 1, w.tobytes())) +
         _fld(11, _value_info(b"x", [1, 4, 3, 5])) + _fld(12, _value_info(b"y", [1, 6, 1, 1])))
net = NeuralNetwork.from_onnx(_fld(7, graph)).load()
x = rng.uniform(-1, 1, (8, 4, 3, 5)).astype(np.float32)
got = net.estimate(x)[0].reshape(8, 6)
want = np.einsum("nchw,mchw->nm", x.astype(np.float64), w.astype(np.float64))
err = float(np.abs(got - want).max())
assert err < 1e-5, err
print("nonsquare ok", err)
"""


@pytest.mark.parametrize("forms", ["", "-rows"])
def test_nonsquare_full_plane_conv(forms):
    e = dict(os.environ, ZARU_HIP_FORMS=forms)
    r = subprocess.run([sys.executable, "-c", NONSQUARE_CHILD, REPO], env=e, capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]


# The warp-specialized form runs only on launches with about a tile per CU or more (the hand
# network's 14^2 / 7^2 blocks from ~940 ROIs): a batch of its own, with the launched kernels read
# back from the session profile so the test knows the form ran.  The fused low-resolution
# inverted residual (irl) takes those blocks by default, so both sides run without it.
WS_CHILD = r"""
import sys, ctypes as C, numpy as np
sys.path.insert(0, sys.argv[1])
from zaru_amd.nn import NeuralNetwork, model_bytes
from zaru_amd._lib import lib, check
net = NeuralNetwork.from_onnx(model_bytes("hand_landmark_lite")).load()
check(lib().zr_profile_enable(net._h, 1))
x = np.random.default_rng(9).uniform(-1.0, 1.0, size=(1024, 3, 224, 224)).astype(np.float32)
outs = net.estimate(x)
need = C.c_size_t()
buf = C.create_string_buffer(1 << 20)  # (a read returns and clears the aggregate: one call)
check(lib().zr_profile_read(net._h, buf, len(buf), C.byref(need)))
kernels = np.array([l.split()[0] for l in buf.value.decode().splitlines() if l.strip()])
np.savez(sys.argv[2], kernels=kernels, **{f"o{i}": o for i, o in enumerate(outs)})
"""


def test_ws_form_is_bitwise_neutral(tmp_path):
    res = {}
    for name, env in (("default", "-irl"), ("no_ws", "-irl,-ws")):
        path = str(tmp_path / f"{name}.npz")
        subprocess.run([sys.executable, "-c", WS_CHILD, REPO, path], env=dict(os.environ, ZARU_HIP_FORMS=env),
                       check=True, timeout=110)
        with np.load(path) as z:
            res[name] = {k: z[k] for k in z.files}
    ws = [k for k in res["default"]["kernels"] if k.startswith("dwpw_ws_kernel")]
    assert len(ws) == 4, res["default"]["kernels"]  # 3x3 14^2, 5x5 14^2, 5x5/2 14->7, 5x5 7^2
    assert not any(k.startswith("dwpw_ws_kernel") for k in res["no_ws"]["kernels"])
    for k in res["default"]:
        if k != "kernels":
            assert np.array_equal(res["default"][k], res["no_ws"][k]), (k, float(np.abs(res["default"][k] - res["no_ws"][k]).max()))


# The row-task depthwise (form "rt", dwpw_dma_body RT > 0) picks its task width from the layer's
# column tile, which depends on the batch: the bench's batches (palm 256 / 85 frames, hand 341
# ROIs, FaceMesh and BlazeFace 341 images) exercise the 2-, 4- and 8-wide tasks.
RT_CHILD = r"""
import sys, ctypes as C, numpy as np
sys.path.insert(0, sys.argv[1])
from zaru_amd.nn import NeuralNetwork, model_bytes
from zaru_amd._lib import lib, check
out, kernels = {}, []
for model, s, b in (("palm_detection_lite", 192, 256), ("palm_detection_lite", 192, 85),
                    ("hand_landmark_lite", 224, 341), ("face_landmark", 192, 341),
                    ("face_detection_short_range", 128, 341)):
    net = NeuralNetwork.from_onnx(model_bytes(model)).load()
    check(lib().zr_profile_enable(net._h, 1))
    x = np.random.default_rng(b).uniform(-1.0, 1.0, size=(b, 3, s, s)).astype(np.float32)
    for i, o in enumerate(net.estimate(x)):
        out[f"{model}/{b}/{i}"] = o
    need = C.c_size_t()
    buf = C.create_string_buffer(1 << 20)
    check(lib().zr_profile_read(net._h, buf, len(buf), C.byref(need)))
    kernels += [l.split()[0] for l in buf.value.decode().splitlines() if l.strip()]
np.savez(sys.argv[2], kernels=np.array(kernels), **out)
"""


def test_rt_form_is_bitwise_neutral_at_bench_batches(tmp_path):
    res = {}
    for name, env in (("default", ""), ("no_rt", "-rt")):
        path = str(tmp_path / f"{name}.npz")
        subprocess.run([sys.executable, "-c", RT_CHILD, REPO, path], env=dict(os.environ, ZARU_HIP_FORMS=env),
                       check=True, timeout=110)
        with np.load(path) as z:
            res[name] = {k: z[k] for k in z.files}
    def rt(k):  # dwpw_dma_kernel / dwpw_dma_group_kernel<K,S,WM,MTW,DFKC,RT>
        return k.split("<", 1)[1].rstrip(">").split(",")[5]
    widths = {rt(k) for k in res["default"]["kernels"] if k.startswith("dwpw_dma")}
    # row tasks of 2 (12^2 / 6^2 / 14^2 / 28^2) and 4 (palm 48^2, FaceMesh 24^2: the MTW-2 layouts
    # are capped at 4 since round 6, rt_hi)
    assert {"2", "4"} <= widths, widths
    assert {rt(k) for k in res["no_rt"]["kernels"] if k.startswith("dwpw_dma")} == {"0"}
    for k in res["default"]:
        if k != "kernels":
            assert np.array_equal(res["default"][k], res["no_rt"][k]), (k, float(np.abs(res["default"][k] - res["no_rt"][k]).max()))


# Two images per workgroup at 7^2 (form "irl2", irl_kernel NI = 2) applies once the ROIs
# outnumber the CUs: 341 (odd: the last workgroup's second image is past the end) and 1024.
IRL2_CHILD = r"""
import sys, ctypes as C, numpy as np
sys.path.insert(0, sys.argv[1])
from zaru_amd.nn import NeuralNetwork, model_bytes
from zaru_amd._lib import lib, check
out, kernels = {}, []
net = NeuralNetwork.from_onnx(model_bytes("hand_landmark_lite")).load()
check(lib().zr_profile_enable(net._h, 1))
for b in (341, 1024):
    x = np.random.default_rng(b).uniform(-1.0, 1.0, size=(b, 3, 224, 224)).astype(np.float32)
    for i, o in enumerate(net.estimate(x)):
        out[f"{b}/{i}"] = o
need = C.c_size_t()
buf = C.create_string_buffer(1 << 20)
check(lib().zr_profile_read(net._h, buf, len(buf), C.byref(need)))
kernels += [l.split()[0] for l in buf.value.decode().splitlines() if l.strip()]
np.savez(sys.argv[2], kernels=np.array(kernels), **out)
"""


def test_irl2_form_is_bitwise_neutral(tmp_path):
    res = {}
    for name, env in (("default", ""), ("no_irl2", "-irl2")):
        path = str(tmp_path / f"{name}.npz")
        subprocess.run([sys.executable, "-c", IRL2_CHILD, REPO, path], env=dict(os.environ, ZARU_HIP_FORMS=env),
                       check=True, timeout=110)
        with np.load(path) as z:
            res[name] = {k: z[k] for k in z.files}
    assert any(k.startswith("irl_kernel<5,7,1,112,4,2>") for k in res["default"]["kernels"]), res["default"]["kernels"]
    assert not any(k.startswith("irl_kernel<5,7,1,112,4,2>") for k in res["no_irl2"]["kernels"])
    for k in res["default"]:
        if k != "kernels":
            assert np.array_equal(res["default"][k], res["no_irl2"][k]), (k, float(np.abs(res["default"][k] - res["no_irl2"][k]).max()))


# FaceMesh V2's bottleneck blocks in one launch (form "bneck": the C -> C/2 reduction, the 3x3
# depthwise, the 1x1 back to C and the residual; 128^2 / 64^2 / 32^2 planes) at a small batch and
# at the face_next line's sub-batch (512 frames in 3 sub-batches).
BNECK_CHILD = r"""
import sys, ctypes as C, numpy as np
sys.path.insert(0, sys.argv[1])
from zaru_amd.nn import NeuralNetwork, model_bytes
from zaru_amd._lib import lib, check
out, kernels = {}, []
net = NeuralNetwork.from_onnx(model_bytes("face_landmarks_detector")).load()
check(lib().zr_profile_enable(net._h, 1))
for b in (7, 171):
    x = np.random.default_rng(b).uniform(-1.0, 1.0, size=(b, 3, 256, 256)).astype(np.float32)
    for i, o in enumerate(net.estimate(x)):
        out[f"{b}/{i}"] = o
need = C.c_size_t()
buf = C.create_string_buffer(1 << 20)
check(lib().zr_profile_read(net._h, buf, len(buf), C.byref(need)))
kernels += [l.split()[0] for l in buf.value.decode().splitlines() if l.strip()]
np.savez(sys.argv[2], kernels=np.array(kernels), **out)
"""


def test_bneck_form_is_bitwise_neutral(tmp_path):
    res = {}
    for name, env in (("default", ""), ("no_bneck", "-bneck")):
        path = str(tmp_path / f"{name}.npz")
        subprocess.run([sys.executable, "-c", BNECK_CHILD, REPO, path], env=dict(os.environ, ZARU_HIP_FORMS=env),
                       check=True, timeout=110)
        with np.load(path) as z:
            res[name] = {k: z[k] for k in z.files}
    used = {k for k in res["default"]["kernels"] if k.startswith("bneck_kernel")}
    assert used == {"bneck_kernel<16,128>", "bneck_kernel<32,64>"}, used
    assert not any(k.startswith("bneck_kernel") for k in res["no_bneck"]["kernels"])
    for other in ("no_bneck",):
        for k in res["default"]:
            if k != "kernels":
                assert np.array_equal(res["default"][k], res[other][k]), (other, k, float(np.abs(res["default"][k] - res[other][k]).max()))
