"""CPU-side checks of the HIP C ABI library: it loads, exports every symbol the header
declares, and compiles every hot-path model into a fused launch plan (no GPU needed)."""
import os
import re

import pytest

from zaru_amd import _lib


def _header_symbols():
    txt = open(_lib.HEADER).read()
    return sorted(set(re.findall(r"\b(zr_[a-z_]+)\s*\(", txt)))


def test_library_exports_header_symbols():
    L = _lib.lib()
    syms = _header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(L, s), s
    assert {s for s, _, _ in _lib.SIGNATURES} == set(syms)


@pytest.mark.parametrize("model,launches", [
    ("face_detection_short_range", 21), ("face_landmark", 25),
    ("palm_detection_lite", 32), ("hand_landmark_lite", 37)])
def test_plan_compiles_and_fuses(models_dir, model, launches):
    data = open(os.path.join(models_dir, model + ".onnx"), "rb").read()
    txt = _lib.plan_describe(data)
    steps = [l for l in txt.splitlines() if l.split(" ")[0] in
             ("gemm", "dw", "direct", "elt", "resize", "gap", "dwpw")]
    assert len(steps) == launches
    # no standalone element-wise pass survives: residual/pad/pool/act are all fused
    assert not [l for l in steps if l.startswith("elt")]


def test_plan_output_selection(models_dir):
    data = open(os.path.join(models_dir, "face_landmark.onnx"), "rb").read()
    full = _lib.plan_describe(data)
    flag_only = _lib.plan_describe(data, outputs=[1])
    assert "output conv2d_31" in flag_only and "conv2d_21" not in flag_only
    assert flag_only.count("\n") < full.count("\n")


def test_malformed_model_is_an_error():
    with pytest.raises(_lib.ZaruError) as e:
        _lib.plan_describe(b"\x08\x01garbage")
    assert e.value.code == -2


def test_unsupported_operator_is_an_error(models_dir):
    # iris_landmark-like ops are not part of the hot path; a hand-made graph with an
    # unknown op must be refused with a model error (Loader::load's "unimplemented
    # operations", crates/zaru/src/nn/mod.rs:255-258)
    def field(num, payload):
        return bytes([(num << 3) | 2, len(payload)]) + payload
    node = field(1, b"x") + field(2, b"y") + field(4, b"Softmax")
    vi = field(1, b"x")
    graph = field(1, node) + field(11, vi) + field(12, field(1, b"y"))
    model = field(7, graph)
    with pytest.raises(_lib.ZaruError) as e:
        _lib.plan_describe(model)
    assert e.value.code == -2 and "Softmax" in str(e.value)
