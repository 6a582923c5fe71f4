"""CPU-side checks of the HIP C ABI library: it loads, exports every symbol the header
declares, and compiles every hot-path model into a fused launch plan (no GPU needed)."""
import os
import re
import subprocess
import sys

import pytest

from zaru_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    txt = open(_lib.HEADER).read()
    return sorted(set(re.findall(r"\b(zr_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_header_symbols():
    L = _lib.lib()
    syms = _header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(L, s), s
    assert {s for s, _, _ in _lib.SIGNATURES} == set(syms)


KINDS = ("gemm", "dw", "direct", "elt", "resize", "gap", "dwpw", "dwgap")


@pytest.mark.parametrize("model,launches", [
    ("face_detection_short_range", 21), ("face_landmark", 25),
    ("palm_detection_lite", 32), ("hand_landmark_lite", 36)])
def test_plan_compiles_and_fuses(models_dir, model, launches):
    path = os.path.join(models_dir, model + ".onnx")
    txt = _lib.plan_describe(open(path, "rb").read())
    steps = [l for l in txt.splitlines() if l.split(" ")[0] in KINDS]
    assert len(steps) == launches
    # no standalone element-wise pass survives: residual/pad/pool/act are all fused
    assert not [l for l in steps if l.startswith("elt")]


@pytest.mark.parametrize("model,pairs", [
    ("hand_landmark_lite", 14), ("face_detection_short_range", 0), ("face_landmark", 0),
    ("palm_detection_lite", 0)])
def test_inverted_residual_pairs(models_dir, model, pairs):
    """mark_inverted_residuals: an expand 1x1 (gemm) is marked (ir=1) exactly when the next step is
    the depthwise -> 1x1 that is the only reader of its output (the fused ir / irl launches)."""
    txt = _lib.plan_describe(open(os.path.join(models_dir, model + ".onnx"), "rb").read())
    steps = [dict(kv.split("=", 1) for kv in l.split() if "=" in kv) | {"kind": l.split()[0]}
             for l in txt.splitlines() if l.split(" ")[0] in KINDS]
    marked = [i for i, s in enumerate(steps) if s["ir"] == "1"]
    assert len(marked) == pairs
    for i in marked:
        e, d = steps[i], steps[i + 1]
        assert e["kind"] == "gemm" and d["kind"] == "dwpw" and d["in"] == e["out"]
        readers = [s for s in steps if s["in"] == e["out"] or s.get("in2") == e["out"]]
        assert readers == [d]


@pytest.mark.parametrize("model,outputs", [
    ("face_detection_full_range", ["reshaped_regressor_face_4", "reshaped_classifier_face_4"]),
    ("face_landmarks_detector", None),
    # whole-plane AveragePool / ReduceMean(W, then H) -> GAP, and the channel
    # Concat of the pooled vectors written in place by their producers
    ("iris_landmark", ["output_eyes_contours_and_brows", "output_iris"]),
    ("landmarks_68_pfld", ["output"]),
    ("slim_160_latest", ["output1"])])
def test_next_models_compile(models_dir, model, outputs):
    """BlazeFace full range (Resize linear FPN) and FaceMesh V2 (fp16 weights)
    lower to the same fused kernels, with no standalone element-wise pass."""
    txt = _lib.plan_describe(open(os.path.join(models_dir, model + ".onnx"), "rb").read())
    steps = [l for l in txt.splitlines() if l.split(" ")[0] in KINDS]
    assert steps and not [l for l in steps if l.startswith("elt")]
    for o in outputs or []:
        assert f"output {o}" in txt
    if model == "face_landmarks_detector":
        assert txt.count("\noutput ") == 3 or txt.count("output ") >= 3


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


# ---------------------------------------------------------------- untrusted ONNX input
# A minimal ModelProto (one 1x1 Conv, x[1,3,8,8] -> y) written with the protobuf wire
# format, then corrupted one field at a time: every variant must come back as a model error
# (zr_plan_describe parses and compiles like zr_session_create, without a GPU), never a crash
# or an over-read.
def _varint(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        out.append(b | (0x80 if v else 0))
        if not v:
            return bytes(out)


def _fld(num, payload):
    return _varint((num << 3) | 2) + _varint(len(payload)) + payload


def _vfld(num, v):
    return _varint(num << 3) + _varint(v & ((1 << 64) - 1))


def _tensor(name, dims, dtype, raw):
    return b"".join(_vfld(1, d) for d in dims) + _vfld(2, dtype) + _fld(8, name) + _fld(9, raw)


def _value_info(name, dims):
    shape = b"".join(_fld(1, _vfld(1, d)) for d in dims)
    return _fld(1, name) + _fld(2, _fld(1, _vfld(1, 1) + _fld(2, shape)))


def _model(w_tensor, strides=(1, 1)):
    attr = _fld(1, b"strides") + b"".join(_vfld(8, s) for s in strides) + _vfld(20, 7)
    # NodeProto: inputs = field 1 repeated (x, w), output = field 2 (y), op_type = field 4
    node = _fld(1, b"x") + _fld(1, b"w") + _fld(2, b"y") + _fld(4, b"Conv") + _fld(5, attr)
    graph = (_fld(1, node) + _fld(5, w_tensor) + _fld(11, _value_info(b"x", [1, 3, 8, 8])) +
             _fld(12, _value_info(b"y", [1, 4, 8, 8])))
    return _fld(7, graph)


def _w(dims=(4, 3, 1, 1), dtype=1, nbytes=None):
    import numpy as np
    n = int(np.prod(dims)) if dims else 1
    size = {1: 4, 6: 4, 7: 8, 10: 2}[dtype]
    raw = b"\x00" * (n * size if nbytes is None else nbytes)
    return _tensor(b"w", dims, dtype, raw)


def test_minimal_model_compiles():
    txt = _lib.plan_describe(_model(_w()))
    assert "gemm" in txt.splitlines()[-1]


@pytest.mark.parametrize("case", ["truncated", "raw_short", "raw_long", "fp16_short",
                                  "int32_short", "int64_short", "negative_dim", "huge_dims",
                                  "zero_stride", "double_weights", "wrong_rank"])
def test_malformed_tensor_is_a_model_error(case):
    if case == "truncated":
        m = _model(_w())[:-7]
    elif case == "raw_short":
        m = _model(_w(nbytes=47))
    elif case == "raw_long":
        m = _model(_w(nbytes=4 * 12 + 4))
    elif case == "fp16_short":
        m = _model(_w(dtype=10, nbytes=23))
    elif case == "int32_short":
        m = _model(_w(dtype=6, nbytes=5))
    elif case == "int64_short":
        m = _model(_w(dtype=7, nbytes=9))
    elif case == "negative_dim":
        m = _model(_tensor(b"w", [4, -3, 1, 1], 1, b""))
    elif case == "huge_dims":  # numel overflows int64 without the bound
        m = _model(_tensor(b"w", [1 << 40, 1 << 40, 1, 1], 1, b"\x00" * 16))
    elif case == "zero_stride":
        m = _model(_w(), strides=(0, 1))
    elif case == "double_weights":  # dtype 11 carries no f32 data
        m = _model(_tensor(b"w", [4, 3, 1, 1], 11, b"\x00" * 96))
    else:
        m = _model(_w(dims=(4, 3)))
    with pytest.raises(_lib.ZaruError) as e:
        _lib.plan_describe(m)
    assert e.value.code == -2, str(e.value)


@pytest.mark.parametrize("model", ["face_detection_short_range", "face_landmark", "palm_detection_lite",
                                   "hand_landmark_lite", "face_detection_full_range",
                                   "face_landmarks_detector", "iris_landmark", "landmarks_68_pfld",
                                   "slim_160_latest"])
def test_plan_reads_only_produced_tensors(models_dir, model):
    """Every launch reads tensors (its input and its fused shortcut) that an earlier launch wrote.
    BlazeFace full range fuses an FPN Add into a conv that precedes, in ONNX order, the Resize
    producing its shortcut; the compiler must run that conv after the Resize."""
    import re
    txt = _lib.plan_describe(open(os.path.join(models_dir, model + ".onnx"), "rb").read())
    produced = set()
    for line in txt.splitlines():
        if line.split(" ")[0] not in KINDS:
            continue
        reads = [re.search(r" in=(\S+)", line).group(1)]
        m = re.search(r" in2=(\S+)", line)
        if m and m.group(1) != "-":
            reads.append(m.group(1))
        for r in reads:
            t = r.split("[")[0]
            assert t == "in0" or t in produced, (model, line)
        produced.add(re.search(r" out=(\S+)", line).group(1).split("[")[0])


def _steps(txt):
    return [l for l in txt.splitlines() if l.split(" ")[0] in KINDS]


def _field(line, key):
    return re.search(rf"\b{key}=(\S+)", line).group(1)


def _tname(ref):
    return ref.split("[")[0]


def test_sibling_steps_share_launches(models_dir):
    """the FaceMesh flag and mesh branches after the 6^2 trunk (t28) run as
    shared launches, layer by layer, and the hand network's four heads as one; a group's members
    never read each other's outputs."""
    fm = _steps(_lib.plan_describe(open(os.path.join(models_dir, "face_landmark.onnx"), "rb").read()))
    first = next(i for i, l in enumerate(fm) if _field(l, "in").startswith("t28["))
    tail = fm[first:]
    launches = [l for l in tail if _field(l, "grp") != "0"]
    assert len(launches) <= 6, "\n".join(tail)
    heads = [l for l in tail if _field(l, "out").startswith("out")]
    assert [_field(l, "grp") for l in heads] == ["2", "0"]
    hand = _steps(_lib.plan_describe(open(os.path.join(models_dir, "hand_landmark_lite.onnx"), "rb").read()))
    hheads = [l for l in hand if _field(l, "out").startswith("out")]
    assert [_field(l, "grp") for l in hheads] == ["4", "0", "0", "0"]
    for steps in (fm, hand):
        for i, l in enumerate(steps):
            g = int(_field(l, "grp"))
            members = steps[i:i + g] if g >= 2 else []
            outs = {_tname(_field(m, "out")) for m in members}
            for m in members:
                assert _tname(_field(m, "in")) not in outs
                assert _tname(_field(m, "in2")) not in outs


def test_groups_switch_off(models_dir):
    code = ("import sys; sys.path.insert(0, sys.argv[1]); from zaru_amd import _lib; "
            "print(_lib.plan_describe(open(sys.argv[2], 'rb').read()))")
    r = subprocess.run([sys.executable, "-c", code, REPO, os.path.join(models_dir, "face_landmark.onnx")],
                       env=dict(os.environ, ZARU_HIP_FORMS="-groups"), capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert all(_field(l, "grp") == "1" for l in _steps(r.stdout))
