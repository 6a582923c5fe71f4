"""Pin the CPU oracle (oracle/) against the reference's own tests, re-expressed as data.

Every case here comes from a #[test] in /root/reference (see tools/make_golden.py for the
file:line of each).  The oracle is the checker for the HIP path, so it is pinned first.
"""
import math
import os

import numpy as np
import pytest

import oracle as O

COL = {"NONE": 0, "BLACK": 0xFF000000, "WHITE": 0xFFFFFFFF, "RED": 0xFF0000FF,
       "GREEN": 0xFF00FF00, "YELLOW": 0xFF00FFFF}


def f32(v):
    return float(np.float32(v))


def test_color_mapper(kat):
    for c in kat["color_mapper"]:
        img = np.full((1, 1, 4), c["code"], np.uint8)
        v = O.preproc(img, O.view_full(1, 1), 1, 1, c["lo"], c["hi"])
        assert v.reshape(-1).tolist() == [c["want"]] * 3


def _det(conf, r):
    d = O.Det()
    d.conf = conf
    d.rect = O.Rect(*r)
    return d


def test_nms_kat(kat):
    for c in kat["nms"]:
        dets = [_det(conf, r) for conf, r in c["dets"]]
        out = O.nms(dets, c["iou"], 0 if c["mode"] == "remove" else 1)
        if "want_len" in c:
            assert len(out) == c["want_len"], c["name"]
        else:
            assert len(out) == len(c["want"]), c["name"]
            for d, (conf, r) in zip(out, c["want"]):
                assert d.conf == f32(conf)
                assert d.rect.tuple() == tuple(f32(v) for v in r), c["name"]


def test_rect_kat(kat):
    for c in kat["iou"]:
        assert O.iou(O.Rect(*c["a"]), O.Rect(*c["b"])) == c["want"]
    for c in kat["intersection"]:
        a, b = O.Rect.from_top_left(*c["a_tl"]), O.Rect.from_top_left(*c["b_tl"])
        r = O.intersection(a, b)
        if "want_area" in c:
            assert (0.0 if r is None else r.w * r.h) == c["want_area"]
        else:
            assert r.tuple() == O.Rect.from_top_left(*c["want_tl"]).tuple()
    for c in kat["fit_aspect"]:
        r = O.grow_to_fit_aspect(O.Rect(*c["r"]), *c["aspect"])
        assert r.tuple() == tuple(float(v) for v in c["want"])
    for c in kat["transform"]:
        rr = O.RRect(O.Rect.from_top_left(*c["tl"]), c["rad"])
        fn = O.transform_in if c["dir"] == "in" else O.transform_out
        got = fn(rr, *c["p"])
        if c.get("tol"):  # assert_approx_eq!: f32::EPSILON abs/rel (approx.rs:58-62)
            assert all(abs(g - w) <= 4 * np.finfo(np.float32).eps + 1e-6 for g, w in
                       zip(got, c["want"])), (c, got)
        else:
            assert got == tuple(float(v) for v in c["want"]), (c, got)
    for c in kat["rrect_bounding"]:
        rr = O.rrect_bounding(c["rad"], c["pts"])
        want = O.Rect.from_top_left(*c["want_tl"]).tuple()
        if c["exact"]:
            assert rr.rect.tuple() == want and rr.rad == f32(c["rad"])
        else:
            assert np.allclose(rr.rect.tuple(), want, atol=1e-6)


def _mkimage(rows):
    return np.array([[[(COL[c] >> (8 * i)) & 0xFF for i in range(4)] for c in row]
                     for row in rows], np.uint8)


def test_view_kat(kat):
    for c in kat["views"]:
        img = _mkimage(c["image"])
        h, w = img.shape[:2]
        v = O.view_full(w, h)
        for tl, rad in c["chain"]:
            v = O.view_compose(v, O.RRect(O.Rect.from_top_left(*tl), rad))
        if "size" in c:
            assert (v.rect.w, v.rect.h) == tuple(float(s) for s in c["size"])
        for x, y, col in c["get"]:
            assert O.view_get(img, v, x, y) == COL[col], (c["name"], x, y)
    for c in kat["view_data"]:
        v = O.view_full(*c["image"])
        for tl in c["chain"]:
            v = O.view_compose(v, O.Rect.from_top_left(*tl))
        assert v.rect.tuple() == O.Rect.from_top_left(*c["want_tl"]).tuple()


def test_detects_face(kat, golden_dir, models_dir):
    """face/detection.rs:164-173 on the committed sad_linus.jpg input codes."""
    g = np.load(f"{golden_dir}/sad_linus_face.npz")
    x = g["codes"].astype(np.float32) * np.float32(np.float32(2.0) / np.float32(255.0)) - 1.0
    net = O.Net(f"{models_dir}/face_detection_short_range.onnx", f64=True)
    reg, cls = net.run(x[None].astype(np.float32))
    w, h = (int(v) for v in g["image_wh"])
    dets = O.detect_post(O.FACE, reg[0], cls[0], w, h, 128, 128)
    m = kat["models"]["detects_face"]
    assert dets and dets[0].conf >= m["min_conf"]
    assert abs(math.degrees(dets[0].angle)) < m["max_abs_angle_deg"]
    assert np.allclose(reg, g["regressors"], atol=2e-4)


def test_facemesh_rotations(kat, golden_dir, models_dir):
    """mediapipe.rs:603-624 (confidence and eye-line angle; Procrustes is out of scope)."""
    g = np.load(f"{golden_dir}/sad_linus_mesh.npz")
    net = O.Net(f"{models_dir}/face_landmark.onnx", f64=False)
    m = kat["models"]["facemesh"]
    adj = np.float32(np.float32(2.0) / np.float32(255.0))
    for i, case in enumerate(m["cases"]):
        x = g["codes"][i].astype(np.float32) * adj - np.float32(1.0)
        lm, flag = net.run(x[None])
        lm = lm.reshape(468, 3)
        assert O.sigmoid(float(flag.reshape(-1)[0])) > m["min_conf"]
        ang = math.degrees(O.signed_angle_to(tuple(lm[263, :2] - lm[33, :2]), (1.0, 0.0)))
        assert abs(ang - case["expect_deg"]) < m["angle_tol_deg"]
        assert np.abs(lm - g["landmarks"][i]).max() < 1e-3


def test_decode_cases_self_consistent(golden_dir):
    g = np.load(f"{golden_dir}/decode_cases.npz")
    keys = sorted({k.split("/")[0] for k in g.files})
    for key in keys:
        kind = O.PALM if key.startswith("palm") else O.FACE
        s = 128 if kind == O.FACE else 192
        iw, ih = (int(v) for v in g[f"{key}/img"])
        dets = O.detect_post(kind, g[f"{key}/boxes"], g[f"{key}/confs"], iw, ih, s, s)
        want = g[f"{key}/want"]
        assert len(dets) == len(want)
        for d, w in zip(dets, want):
            assert d.conf == w[0] and d.angle == w[1] and d.rect.tuple() == tuple(w[2:6])


# ---------------------------------------------------------------- SURVEY 8(f)-1 networks
def test_full_range_detects_face(kat, golden_dir, models_dir):
    """face/detection.rs:164-173's bar applied to FullRangeNetwork (face/detection.rs:61-94:
    one 48x48 anchor layer, 192^2 input) on the same sad_linus.jpg letterbox."""
    g = np.load(f"{golden_dir}/next_models.npz")
    x = g["full_linus/codes"].astype(np.float32) * np.float32(np.float32(2.0) / np.float32(255.0)) - 1.0
    net = O.Net(f"{models_dir}/face_detection_full_range.onnx", f64=True)
    reg, cls = net.run(x[None].astype(np.float32))
    assert reg.shape == (1, 2304, 16) and cls.shape == (1, 2304, 1)
    w, h = (int(v) for v in g["full_linus/image_wh"])
    dets = O.detect_post(O.FACE_FULL, reg[0], cls[0], w, h, 192, 192)
    m = kat["models"]["detects_face"]
    assert dets and dets[0].conf >= m["min_conf"]
    assert abs(math.degrees(dets[0].angle)) < m["max_abs_angle_deg"]
    assert np.allclose(reg, g["full_linus/regressors"], atol=2e-4)


def test_facemesh_v2_rotations(kat, golden_dir, models_dir):
    """mediapipe.rs:603-624's bars applied to FaceMeshV2 (mediapipe.rs:81-116): the fp16
    initializers (upcast exactly) give a confident mesh whose eye line follows the view."""
    g = np.load(f"{golden_dir}/next_models.npz")
    net = O.Net(f"{models_dir}/face_landmarks_detector.onnx", f64=False)
    m = kat["models"]["facemesh"]
    adj = np.float32(np.float32(2.0) / np.float32(255.0))
    for i, case in enumerate(m["cases"]):
        x = g["v2_linus/codes"][i].astype(np.float32) * adj - np.float32(1.0)
        lm, flag, tongue = net.run(x[None])
        lm = lm.reshape(478, 3)
        assert O.landmark_confidence(O.FACEMESH_V2, (lm, flag)) > m["min_conf"]
        ang = math.degrees(O.landmark_angle(O.FACEMESH_V2, lm))
        assert abs(ang - case["expect_deg"]) < m["angle_tol_deg"]
        assert np.abs(lm - g["v2_linus/landmarks"][i]).max() < 1e-3
        assert 0.0 <= float(tongue.reshape(-1)[0]) <= 1.0  # sigmoid inside the graph


def test_fp16_initializers_upcast_exactly(models_dir):
    """The f32 and f64 interpreters read the same fp16 weights: their outputs differ only by
    f32 evaluation noise, far below any fp16 rounding step of the weights (2^-11 relative)."""
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "next_models.npz"))
    x = g["face_landmarks_detector/0/codes"].astype(np.float32) * np.float32(2.0 / 255.0) - 1.0
    lo = O.Net(f"{models_dir}/face_landmarks_detector.onnx", f64=False).run(x[None].astype(np.float32))
    for oi, o in enumerate(lo):
        want = g[f"face_landmarks_detector/0/out{oi}"]
        assert np.abs(o - want).max() <= 2e-4 * max(1.0, float(np.abs(want).max())), oi


ASAN_CHILD = r"""
import sys
sys.path.insert(0, sys.argv[1])
import numpy as np
import oracle as O
O.LIB_PATH = sys.argv[2]
sizes = {"face_detection_short_range": 128, "face_landmark": 192, "palm_detection_lite": 192,
         "hand_landmark_lite": 224, "face_detection_full_range": 192, "face_landmarks_detector": 256}
for m, s in sizes.items():
    n = O.Net(f"{sys.argv[1]}/zaru_amd/models/{m}.onnx", f64=False)
    for k in range(2):
        n.run(np.random.default_rng(k).uniform(-1, 1, (1, 3, s, s)).astype(np.float32))
import io
from PIL import Image
from zaru_amd import jpeg
for shape, sub in (((37, 53, 3), 2), ((40, 24, 3), 1), ((16, 16, 3), 0), ((21, 30), 0)):
    b = io.BytesIO()
    Image.fromarray(np.random.default_rng(1).integers(0, 256, size=shape, dtype=np.uint8)).save(
        b, "JPEG", quality=80, subsampling=sub)
    O.jpeg_pixels(*reversed(jpeg.coefficients(b.getvalue())))
print("clean")
"""


def test_oracle_interpreter_is_memory_clean(tmp_path):
    """The checker itself under AddressSanitizer (host code only): every model, two runs each.
    (A value-table realloc once left tensor pointers dangling mid-operator.)"""
    import shutil
    import subprocess
    import sys
    asan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    if not shutil.which("gcc") or not os.path.isabs(asan):
        pytest.skip("no gcc/libasan")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = str(tmp_path / "liboracle_asan.so")
    subprocess.run(["gcc", "-shared", "-fPIC", "-O1", "-g", "-fsanitize=address", "-fno-omit-frame-pointer",
                    "-ffp-contract=off", "-o", lib, f"{repo}/oracle/geom.c", f"{repo}/oracle/nnexec.c",
                    f"{repo}/oracle/jpeg.c", "-lm"],
                   check=True)
    env = dict(os.environ, LD_PRELOAD=asan, ASAN_OPTIONS="detect_leaks=0")
    r = subprocess.run([sys.executable, "-c", ASAN_CHILD, repo, lib], env=env, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0 and "clean" in r.stdout, r.stderr[-3000:]
