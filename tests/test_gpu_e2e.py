"""End-to-end parity on synthetic 1080p frames (config 3 / config 4 shapes): the batched HIP
pipeline against the oracle's f32 restatement of the reference chain, with the parity
definitions of SURVEY.md §8a:

(ii)  the set of selected anchor indices (conf >= 0.5) is identical, except inside the boundary
      band |conf - 0.5| < 1e-5, whose cases are counted and reported (expected 0);
      the detections after NMS agree in count, and in confidence / box within the f32 noise;
(iii) landmarks agree within L2 <= 1e-3 in the network-input pixel space (192 px FaceMesh,
      224 px hand), i.e. frame-pixel error / (view side / input side).

Detection -> NMS -> mapping is bit-exact when fed the same raw tensors (test_host_cpu.py); here
the raw tensors come from two different f32 evaluation orders, so (ii)/(iii) are the bar.
"""
import math
import os

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MODELS = os.path.join(REPO, "zaru_amd", "models")
BAND = 1e-5
W, H = 1920, 1080

CASES = {
    # kind: detector, landmark net, det input, landmark input, colour lo, NMS kind, grow, padding
    "face": ("face_detection_short_range", "face_landmark", 128, 192, -1.0, O.FACE, 0.0, 0.3),
    "hand": ("palm_detection_lite", "hand_landmark_lite", 192, 224, 0.0, O.PALM, 1.5, 0.4),
}


def face_patch():
    codes = np.load(os.path.join(REPO, "tests", "golden", "sad_linus_mesh.npz"))["codes"][0]
    img = np.full((192, 192, 4), 255, np.uint8)
    img[..., :3] = codes.transpose(1, 2, 0)
    return np.repeat(np.repeat(img, 3, axis=0), 3, axis=1)


def frames_for(kind, n, seed):
    rng = np.random.default_rng(seed)
    frames = rng.integers(0, 256, size=(n, H, W, 4), dtype=np.uint8)
    patch = face_patch()
    for i in range(n):
        if kind == "face" or i % 2 == 0:  # hand frames: half noise-only (forced ROIs)
            y, x = int(rng.integers(0, H - 576)), int(rng.integers(0, W - 576))
            frames[i, y:y + 576, x:x + 576] = patch
    forced = []
    for _ in range(n):
        k = 1 if kind == "face" else 4
        rois = []
        for _ in range(k):
            side = float(rng.uniform(150, 400))
            rad = 0.0 if kind == "face" else float(rng.uniform(-math.pi, math.pi))
            rois.append((float(rng.uniform(side / 2, W - side / 2)),
                         float(rng.uniform(side / 2, H - side / 2)), side, side, rad))
        forced.append(rois)
    return frames, forced


@pytest.fixture(scope="module")
def H_():
    import zaru_amd.host as Hm
    return Hm


@pytest.mark.parametrize("kind", ["face", "hand"])
def test_pipeline_vs_oracle_1080p(H_, kind):
    from zaru_amd._lib import DeviceBuffer
    from zaru_amd.nn import Cnn, ColorMapper, NeuralNetwork, model_bytes

    det_m, lm_m, din, lin, lo, okind, grow, pad = CASES[kind]
    n = 4
    frames, forced = frames_for(kind, n, 101 if kind == "face" else 102)
    bufs = [DeviceBuffer.from_array(f) for f in frames]
    flist = [(b.ptr, W, H, W * 4) for b in bufs]
    p = H_.DetectTrackPipeline(kind, 0, 4, 1 if kind == "face" else 4)
    p.run(flist, forced)

    det_gpu = Cnn(NeuralNetwork.from_onnx(model_bytes(det_m)).load(), ColorMapper.linear(lo, 1.0))
    det_cpu = O.Net(os.path.join(MODELS, det_m + ".onnx"), f64=False)
    lm_cpu = O.Net(os.path.join(MODELS, lm_m + ".onnx"), f64=False)

    boundary = 0
    worst_lm = 0.0
    for f in range(n):
        img = frames[f]
        r = O.grow_to_fit_aspect(O.Rect.from_top_left(0, 0, W, H), din, din)
        v = O.view_compose(O.view_full(W, H), r)
        reg_g, cls_g = det_gpu.estimate_views(img, [(v.rect.cx, v.rect.cy, v.rect.w, v.rect.h, v.rad)])
        reg_c, cls_c = det_cpu.run(O.preproc(img, v, din, din, lo, 1.0)[None])
        # (ii) anchor selection: identical outside the boundary band
        cg = np.array([O.sigmoid(float(t)) for t in cls_g.reshape(-1)], np.float32)
        cc = np.array([O.sigmoid(float(t)) for t in cls_c.reshape(-1)], np.float32)
        sel_g, sel_c = cg >= 0.5, cc >= 0.5
        near = np.abs(cc - 0.5) < BAND
        boundary += int(near.sum())
        assert np.array_equal(sel_g[~near], sel_c[~near]), (kind, f, np.nonzero(sel_g != sel_c))
        # detections after NMS (frame px): the pipeline's vs the oracle chain's
        want = O.detect_post(okind, reg_c[0], cls_c[0], W, H, din, din)
        got = p.detections()[f]
        assert len(got) == len(want), (kind, f)
        scale = W / din  # letterbox px per network px
        for a, b in zip(got, want):
            assert abs(a.confidence() - b.conf) <= 1e-4
            assert np.allclose(a.bounding_rect().tuple(), b.rect.tuple(), atol=2e-3 * scale)
    print(f"{kind}: anchors within the {BAND:g} boundary band: {boundary}")
    assert boundary == 0

    # (iii) landmarks of every tracked ROI, recomputed by the oracle from the same ROI
    checked = 0
    for i in range(p.num_rois()):
        rr = p.roi(i)
        img = frames[rr["frame"]]
        roi = rr["roi"]
        cx, cy, w, h = roi.rect().tuple()
        rad = roi.rotation_radians()
        vr = O.RRect(O.grow_to_fit_aspect(O.Rect(cx, cy, w, h), 1, 1), rad)
        view = O.view_compose(O.view_full(W, H), vr)
        lrect = O.grow_to_fit_aspect(O.Rect.from_top_left(0, 0, view.rect.w, view.rect.h), 1, 1)
        v2 = O.view_compose(view, lrect)
        outs = lm_cpu.run(O.preproc(img, v2, lin, lin, lo, 1.0)[None])
        pos = O.estimator_map(outs[0].reshape(-1, 3), lrect, lin)
        want, _, _ = O.tracker_update(pos, vr, rad, 0.0, pad)
        per_px = lrect.w / lin  # frame px per network-input px
        l2 = np.sqrt(((rr["landmarks"][:, :2] - want[:, :2]) ** 2).sum(-1)).max() / per_px
        worst_lm = max(worst_lm, float(l2))
        assert l2 <= 1e-3, (kind, i, l2)
        checked += 1
    print(f"{kind}: {checked} ROIs, worst landmark L2 = {worst_lm:.2e} network px")
    assert checked >= n
