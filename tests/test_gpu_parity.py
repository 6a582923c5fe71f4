"""GPU parity of the HIP path against the oracle and the committed golden fixtures.

Tolerances: preprocessing is bit-exact; network outputs are f32 on the GPU
against the f64 oracle, bounded by the measured f32 noise floor with margin
(|err| <= 2e-3 absolute on raw outputs whose magnitude reaches ~180, landmark L2 <= 1e-3 px).
"""
import math
import os

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

MODELS = {
    "face_detection_short_range": (128, -1.0, 1.0),
    "face_landmark": (192, -1.0, 1.0),
    "palm_detection_lite": (192, 0.0, 1.0),
    "hand_landmark_lite": (224, 0.0, 1.0),
    # SURVEY 8(f)-1 (fixtures in next_models.npz)
    "face_detection_full_range": (192, -1.0, 1.0),
    "face_landmarks_detector": (256, -1.0, 1.0),
    # EyeNetwork and the two 68-point networks
    "iris_landmark": (64, -1.0, 1.0),
    "landmarks_68_pfld": (112, 0.0, 1.0),
    "slim_160_latest": (160, -1.0, 1.0),
}
NEXT = ("face_detection_full_range", "face_landmarks_detector", "iris_landmark", "landmarks_68_pfld",
        "slim_160_latest")
ABS_TOL = 2e-3


@pytest.fixture(scope="module")
def nets():
    from zaru_amd.nn import NeuralNetwork, model_bytes
    return {m: NeuralNetwork.from_onnx(model_bytes(m)).load() for m in MODELS}


def codes_to_input(codes, lo, hi):
    adj = np.float32((np.float32(hi) - np.float32(lo)) / np.float32(255.0))
    return codes.astype(np.float32) * adj + np.float32(lo)


@pytest.mark.parametrize("model", list(MODELS))
def test_model_vs_f64_golden(nets, golden_dir, model):
    g = np.load(os.path.join(golden_dir, "next_models.npz" if model in NEXT else "models_f64.npz"))
    s, lo, hi = MODELS[model]
    x = np.stack([codes_to_input(g[f"{model}/{k}/codes"], lo, hi) for k in range(2)])
    outs = nets[model].estimate(x)
    for oi, o in enumerate(outs):
        want = np.concatenate([g[f"{model}/{k}/out{oi}"] for k in range(2)])
        err = float(np.abs(o - want).max())
        print(f"{model} out{oi}: max|gpu - f64| = {err:.3e}")
        assert err <= ABS_TOL, (model, oi, err)
    if model in ("face_landmark", "hand_landmark_lite", "face_landmarks_detector", "iris_landmark"):
        lm = outs[0].reshape(2, -1, 3)
        want = np.stack([g[f"{model}/{k}/out0"].reshape(-1, 3) for k in range(2)])
        l2 = np.sqrt(((lm[..., :2] - want[..., :2]) ** 2).sum(-1)).max()
        assert l2 <= 1e-3, l2
    if model in ("landmarks_68_pfld", "slim_160_latest"):
        # (x, y) relative to the input side (multipie68.rs:71-80): L2 in network pixels
        lm = outs[0].reshape(2, -1)[:, :136].reshape(2, 68, 2) * s
        want = np.stack([g[f"{model}/{k}/out0"].reshape(-1)[:136].reshape(68, 2) for k in range(2)]) * s
        l2 = np.sqrt(((lm - want) ** 2).sum(-1)).max()
        assert l2 <= 1e-3, l2


@pytest.mark.parametrize("model", list(MODELS))
def test_batch_independence(nets, model):
    """Each image's result does not depend on the batch it runs in (bitwise)."""
    s, lo, hi = MODELS[model]
    rng = np.random.default_rng(11)
    x = codes_to_input(rng.integers(0, 256, size=(3, 3, s, s), dtype=np.uint8), lo, hi)
    one = nets[model].estimate(x[1:2])
    many = nets[model].estimate(np.concatenate([x, x[1:2], x]))
    for a, b in zip(one, many):
        assert np.array_equal(a[0], b[1]) and np.array_equal(a[0], b[3])


@pytest.mark.parametrize("model", list(MODELS))
def test_large_batch_matches_single_images(nets, model):
    """Kernel layouts are chosen per launch from the batch size (fused.hip launch_dwpw), so a
    production-size batch runs different tilings than the small parity batches.  Every
    tiling keeps each column's arithmetic order, so results must match bit for bit."""
    s, lo, hi = MODELS[model]
    rng = np.random.default_rng(13)
    n = 520
    x = codes_to_input(rng.integers(0, 256, size=(n, 3, s, s), dtype=np.uint8), lo, hi)
    many = nets[model].estimate(x)
    for i in (0, 1, 257, n - 1):
        one = nets[model].estimate(x[i:i + 1])
        for a, b in zip(one, many):
            assert np.array_equal(a[0], b[i]), (model, i)


def test_detects_face(nets, golden_dir, kat):
    """face/detection.rs:164-173 through the HIP runner."""
    g = np.load(os.path.join(golden_dir, "sad_linus_face.npz"))
    x = codes_to_input(g["codes"], -1.0, 1.0)[None]
    reg, cls = nets["face_detection_short_range"].estimate(x)
    assert np.abs(reg - g["regressors"]).max() <= ABS_TOL
    w, h = (int(v) for v in g["image_wh"])
    dets = O.detect_post(O.FACE, reg[0], cls[0], w, h, 128, 128)
    m = kat["models"]["detects_face"]
    assert dets and dets[0].conf >= m["min_conf"]
    assert abs(math.degrees(dets[0].angle)) < m["max_abs_angle_deg"]


def test_facemesh_rotations(nets, golden_dir, kat):
    """mediapipe.rs:603-624 (confidence + eye-line angle) through the HIP runner."""
    g = np.load(os.path.join(golden_dir, "sad_linus_mesh.npz"))
    x = codes_to_input(g["codes"], -1.0, 1.0)
    lms, flags = nets["face_landmark"].estimate(x)
    m = kat["models"]["facemesh"]
    for i, case in enumerate(m["cases"]):
        lm = lms[i].reshape(468, 3)
        assert O.sigmoid(float(flags[i].reshape(-1)[0])) > m["min_conf"]
        d = lm[263, :2] - lm[33, :2]
        ang = math.degrees(O.signed_angle_to((float(d[0]), float(d[1])), (1.0, 0.0)))
        assert abs(ang - case["expect_deg"]) < m["angle_tol_deg"]
        l2 = np.sqrt(((lm[:, :2] - g["landmarks"][i][:, :2]) ** 2).sum(-1)).max()
        assert l2 <= 1e-3, l2


def test_detects_face_full_range(nets, golden_dir, kat):
    """face/detection.rs:164-173's bar applied to FullRangeNetwork (face/detection.rs:61-94) on
    the same image, letterboxed to 192^2, through the HIP runner."""
    g = np.load(os.path.join(golden_dir, "next_models.npz"))
    x = codes_to_input(g["full_linus/codes"], -1.0, 1.0)[None]
    reg, cls = nets["face_detection_full_range"].estimate(x)
    assert np.abs(reg - g["full_linus/regressors"]).max() <= ABS_TOL
    assert np.abs(cls - g["full_linus/classificators"]).max() <= ABS_TOL
    w, h = (int(v) for v in g["full_linus/image_wh"])
    dets = O.detect_post(O.FACE_FULL, reg[0], cls[0], w, h, 192, 192)
    m = kat["models"]["detects_face"]
    assert dets and dets[0].conf >= m["min_conf"]
    assert abs(math.degrees(dets[0].angle)) < m["max_abs_angle_deg"]


def test_facemesh_v2_rotations(nets, golden_dir, kat):
    """mediapipe.rs:603-624's bars (confidence, eye-line angle) applied to FaceMeshV2
    (mediapipe.rs:81-116, 478 points, fp16 weights upcast at load), plus tongue_out and the
    landmark L2 against the f64 oracle."""
    g = np.load(os.path.join(golden_dir, "next_models.npz"))
    x = codes_to_input(g["v2_linus/codes"], -1.0, 1.0)
    lms, flags, tongue = nets["face_landmarks_detector"].estimate(x)
    m = kat["models"]["facemesh"]
    for i, case in enumerate(m["cases"]):
        lm = lms[i].reshape(478, 3)
        assert O.sigmoid(float(flags[i].reshape(-1)[0])) > m["min_conf"]
        d = lm[263, :2] - lm[33, :2]
        ang = math.degrees(O.signed_angle_to((float(d[0]), float(d[1])), (1.0, 0.0)))
        assert abs(ang - case["expect_deg"]) < m["angle_tol_deg"]
        l2 = np.sqrt(((lm[:, :2] - g["v2_linus/landmarks"][i][:, :2]) ** 2).sum(-1)).max()
        assert l2 <= 1e-3, l2
        assert abs(float(tongue[i].reshape(-1)[0]) - float(g["v2_linus/tongue_out"][i])) <= 1e-5


def _random_views(rng, n, w, h):
    views = []
    for i in range(n):
        kind = i % 4
        if kind == 0:  # letterbox of the whole frame
            r = O.grow_to_fit_aspect(O.Rect.from_top_left(0, 0, w, h), 1, 1)
            v = O.view_compose(O.view_full(w, h), r)
        else:
            side = float(rng.uniform(0.5, 1.5 * max(w, h) + 8))
            cx, cy = float(rng.uniform(-0.3 * w, 1.3 * w)), float(rng.uniform(-0.3 * h, 1.3 * h))
            rad = float(rng.choice([0.0, math.pi / 2, -math.pi / 2, math.pi,
                                    rng.uniform(-math.pi, math.pi)]))
            if kind == 3:
                rad = float(np.float32(10.0) * (np.float32(math.pi) / np.float32(180.0)))
            v = O.view_compose(O.view_full(w, h), O.RRect(O.Rect(cx, cy, side, side * 1.1), rad))
        views.append(v)
    return views


def test_preproc_bit_exact():
    from zaru_amd._lib import DeviceBuffer, Frame, synchronize
    from zaru_amd.nn import preprocess_views_device
    rng = np.random.default_rng(5)
    frames, bufs, all_views, view_frame = [], [], [], []
    shapes = [(61, 97), (1080, 1920), (1, 1), (480, 640)]
    for fi, (h, w) in enumerate(shapes):
        img = rng.integers(0, 256, size=(h, w, 4), dtype=np.uint8)
        b = DeviceBuffer.from_array(img)
        bufs.append((b, img))
        frames.append(Frame(b.ptr, w, h, w * 4))
        vs = _random_views(rng, 24, w, h)
        all_views += vs
        view_frame += [fi] * len(vs)
    for ow, oh, lo, hi in ((128, 128, -1.0, 1.0), (192, 192, 0.0, 1.0), (33, 17, 1.0, 2.0)):
        out = DeviceBuffer(len(all_views) * 3 * oh * ow * 4)
        preprocess_views_device(frames, [(v.rect.cx, v.rect.cy, v.rect.w, v.rect.h, v.rad)
                                         for v in all_views], view_frame, ow, oh, lo, hi, out.ptr)
        synchronize()
        got = out.download((len(all_views), 3, oh, ow), np.float32)
        for i, v in enumerate(all_views):
            img = bufs[view_frame[i]][1]
            want = O.preproc(img, v, ow, oh, lo, hi)
            assert np.array_equal(got[i].view(np.uint32), want.view(np.uint32)), (i, ow, oh)


def test_cnn_estimate_views_matches_session(nets):
    """Cnn::estimate path (preproc fused in front of the network) == preproc + estimate."""
    from zaru_amd.nn import Cnn, ColorMapper
    rng = np.random.default_rng(9)
    img = rng.integers(0, 256, size=(300, 400, 4), dtype=np.uint8)
    cnn = Cnn(nets["face_landmark"], ColorMapper.linear(-1.0, 1.0))
    views = _random_views(rng, 6, 400, 300)
    got = cnn.estimate_views(img, [(v.rect.cx, v.rect.cy, v.rect.w, v.rect.h, v.rad) for v in views])
    x = np.stack([O.preproc(img, v, 192, 192, -1.0, 1.0) for v in views])
    want = nets["face_landmark"].estimate(x)
    for a, b in zip(got, want):
        assert np.array_equal(a, b)
