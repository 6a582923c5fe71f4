"""The kernel forms the launchers choose between compute the same arithmetic in the same order,
so switching a form off (its ZR_* switch, read once per process) must not change one bit of any
model output.  Each configuration runs in a child process (the switches are process-wide); the
batch is large enough that every form the default build picks is exercised (LDS-DMA staged
VALU and MFMA forms, the windowed V4 taps, the image-row head GEMM).
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

# each switch turns one form off; "all" turns every one off together
SWITCHES = {
    "default": {},
    "no_valu_db": {"ZR_VALU_DB": "0"},
    "no_dma": {"ZR_DWPW_DMA": "0"},
    "no_v4": {"ZR_DWPW_V4": "0", "ZR_DWPW_DMA": "0"},
    "no_rows": {"ZR_GEMM_ROWS": "0"},
    "dma_chunk32": {"ZR_DWPW_FKC": "32"},  # not an off-switch: the other DMA chunk size
    "no_chain": {"ZARU_HIP_FUSE": "0"},    # the layer-per-launch plan (no chain.hip)
}


@pytest.fixture(scope="module")
def outputs(tmp_path_factory):
    d = tmp_path_factory.mktemp("forms")
    res = {}
    for name, env in SWITCHES.items():
        path = str(d / f"{name}.npz")
        e = dict(os.environ)
        for k in ("ZR_VALU_DB", "ZR_DWPW_DMA", "ZR_DWPW_V4", "ZR_GEMM_ROWS", "ZR_DWPW_FKC", "ZARU_HIP_FUSE"):
            e.pop(k, None)
        e.update(env)
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
