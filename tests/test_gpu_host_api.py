"""The reference's host-level call chains through the HIP backend (zaru_amd.host):
Detector::detect, Estimator::estimate, LandmarkTracker::track and the batched
DetectTrackPipeline, checked against the reference's own expectations and against each other."""
import math
import os

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


def codes_image(codes):
    """An RGBA image whose identity view reproduces the committed network input exactly."""
    c, h, w = codes.shape
    img = np.full((h, w, 4), 255, np.uint8)
    img[..., :3] = codes.transpose(1, 2, 0)
    return img


@pytest.fixture(scope="module")
def H():
    import zaru_amd.host as H
    return H


def test_detector_detects_face(H, golden_dir, kat):
    """face/detection.rs:164-173 via Detector::detect on the HIP backend."""
    g = np.load(os.path.join(golden_dir, "sad_linus_face.npz"))
    img = codes_image(g["codes"])
    det = H.Detector("face")
    dets = det.detect(img)
    m = kat["models"]["detects_face"]
    assert len(dets) >= 1
    assert dets[0].confidence() >= m["min_conf"]
    assert abs(math.degrees(dets[0].angle())) < m["max_abs_angle_deg"]
    # same selection as the oracle decode of the f64 outputs (128 px space: identity letterbox)
    want = O.detect_post(O.FACE, g["regressors"][0], g["classificators"][0], 128, 128, 128, 128)
    assert len(want) == len(dets)
    assert np.allclose(dets[0].bounding_rect().tuple(), want[0].rect.tuple(), atol=1e-2)


def test_estimator_facemesh(H, golden_dir, kat):
    g = np.load(os.path.join(golden_dir, "sad_linus_mesh.npz"))
    m = kat["models"]["facemesh"]
    est = H.Estimator("facemesh")
    for i, case in enumerate(m["cases"]):
        r = est.estimate_image(codes_image(g["codes"][i]))
        assert r["confidence"] > m["min_conf"]
        ang = math.degrees(est.angle_radians(r["landmarks"]))
        assert abs(ang - case["expect_deg"]) < m["angle_tol_deg"]
        l2 = np.sqrt(((r["landmarks"][:, :2] - g["landmarks"][i][:, :2]) ** 2).sum(-1)).max()
        assert l2 <= 1e-3, l2


@pytest.mark.parametrize("net,model,side,lo", [("eye", "iris_landmark", 64, -1.0),
                                               ("face68_pfld", "landmarks_68_pfld", 112, 0.0),
                                               ("face68_peppa", "slim_160_latest", 160, -1.0)])
def test_estimator_eye_and_68_point(H, models_dir, net, model, side, lo):
    """Estimator over the SURVEY 8(f)-4 networks on a rotated view of a seeded image against the
    oracle chain: preprocessing, f32 network, extract (eye.rs:47-64: iris first, then the
    contour; multipie68.rs:71-80: (x, y) * input resolution, z = 0) and the map-out
    (landmark.rs:336-345)."""
    import oracle as O
    rng = np.random.default_rng(21)
    img = rng.integers(0, 256, size=(150, 210, 4), dtype=np.uint8)
    est = H.Estimator(net)
    roi = O.RRect(O.Rect(100.0, 70.0, 120.0, 96.0), 0.25)
    view = O.view_compose(O.view_full(210, 150), roi)
    hv = H.ViewData.full(210, 150).view(H.RotatedRect(H.Rect.from_center(100.0, 70.0, 120.0, 96.0), 0.25))
    r = est.estimate(img, hv)
    lrect = O.grow_to_fit_aspect(O.Rect.from_top_left(0, 0, view.rect.w, view.rect.h), side, side)
    x = O.preproc(img, O.view_compose(view, lrect), side, side, lo, 1.0)
    outs = O.Net(os.path.join(models_dir, model + ".onnx"), f64=False).run(x[None])
    if net == "eye":
        pos = np.concatenate([outs[1].reshape(5, 3), outs[0].reshape(71, 3)])
    else:
        xy = outs[0].reshape(-1)[:136].reshape(68, 2) * np.float32(side)
        pos = np.concatenate([xy, np.zeros((68, 1), np.float32)], 1).astype(np.float32)
    want = O.estimator_map(pos, lrect, side)
    assert r["landmarks"].shape == want.shape
    per_px = lrect.w / side
    l2 = np.sqrt(((r["landmarks"][:, :2] - want[:, :2]) ** 2).sum(-1)).max() / per_px
    assert l2 <= 1e-3, l2
    assert r["confidence"] == 1.0  # no Confidence impl in the reference outputs


def test_tracker_follows_face(H, golden_dir):
    """LandmarkTracker::track (landmark.rs:463-501): seeded with the whole crop, tracking holds
    and the next ROI stays on the face."""
    g = np.load(os.path.join(golden_dir, "sad_linus_mesh.npz"))
    img = codes_image(g["codes"][0])
    t = H.LandmarkTracker("facemesh")
    t.set_roi_rect(H.Rect.from_top_left(0, 0, 192, 192))
    r = t.track(img)
    assert r is not None and r["confidence"] > 0.9
    roi = t.roi()
    assert roi is not None
    cx, cy = roi.rect().center
    assert 40 < cx < 150 and 40 < cy < 150
    # a second pass from the updated ROI keeps tracking
    assert t.track(img) is not None


def test_tracker_loses_on_noise(H):
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, size=(300, 300, 4), dtype=np.uint8)
    t = H.LandmarkTracker("facemesh")
    t.set_roi_rect(H.Rect.from_top_left(20, 20, 200, 200))
    r = t.track(img)
    if r is None:
        assert t.roi() is None  # lost -> ROI cleared (landmark.rs:468-477)


@pytest.mark.parametrize("kind", ["face", "hand"])
def test_pipeline_equals_per_frame_api(H, kind):
    """Batched DetectTrackPipeline == Detector::detect + one LandmarkTracker pass per frame,
    bit for bit (every kernel's per-image result is independent of the batch)."""
    from zaru_amd._lib import DeviceBuffer
    rng = np.random.default_rng(21 if kind == "face" else 22)
    frames = [rng.integers(0, 256, size=(h, w, 4), dtype=np.uint8)
              for h, w in ((240, 320), (360, 640), (300, 300), (480, 200), (256, 256))]
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "sad_linus_face.npz"))
    frames[2][:128, :128, :3] = g["codes"].transpose(1, 2, 0)  # one real face
    bufs = [DeviceBuffer.from_array(f) for f in frames]
    flist = [(b.ptr, f.shape[1], f.shape[0], f.shape[1] * 4) for b, f in zip(bufs, frames)]
    forced = [[(f.shape[1] / 2, f.shape[0] / 2, 150.0, 150.0, 0.3 if kind == "hand" else 0.0)]
              for f in frames]
    p = H.DetectTrackPipeline(kind, 0, 4, 4)
    p.run(flist, forced)
    det = H.Detector("face" if kind == "face" else "palm")
    for f, img in enumerate(frames):
        want = det.detect(img)
        got = p.detections()[f]
        assert len(got) == len(want)
        for a, b in zip(got, want):
            assert a.confidence() == b.confidence() and a.angle() == b.angle()
            assert a.bounding_rect() == b.bounding_rect()
    for i in range(p.num_rois()):
        r = p.roi(i)
        t = H.LandmarkTracker("facemesh" if kind == "face" else "hand")
        t.set_roi_padding(0.3 if kind == "face" else 0.4)
        t.set_roi(r["roi"])
        res = t.track(frames[r["frame"]])
        assert (res is not None) == r["tracked"]
        if res is not None:
            assert np.array_equal(res["landmarks"], r["landmarks"])
            assert res["updated_roi"].rect() == r["updated_roi"].rect()


def test_repeated_runs_equal_single_run(H):
    """run_frames_repeated overlaps one run's landmark mapping with the next run's detection;
    each run must still produce exactly what one run_frames() produces."""
    from zaru_amd._lib import DeviceBuffer
    rng = np.random.default_rng(31)
    frames = [rng.integers(0, 256, size=(360, 640, 4), dtype=np.uint8) for _ in range(6)]
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "sad_linus_face.npz"))
    frames[1][:128, :128, :3] = g["codes"].transpose(1, 2, 0)
    bufs = [DeviceBuffer.from_array(f) for f in frames]
    flist = [(b.ptr, f.shape[1], f.shape[0], f.shape[1] * 4) for b, f in zip(bufs, frames)]
    forced = [[(320.0, 180.0, 160.0, 160.0, 0.0)] for _ in frames]
    p = H.DetectTrackPipeline("face", 0, 4, 4, 3)
    p.set_frames(flist, forced)
    n1 = p.run_frames()
    want = [(r["frame"], r["landmarks"].copy(), r["tracked"]) for r in (p.roi(i) for i in range(n1))]
    want_det = [[(d.confidence(), d.bounding_rect().tuple()) for d in ds] for ds in p.detections()]
    tracked = p.run_frames_repeated(3)
    assert p.times()["rois"] == 3 * n1 and p.num_rois() == n1
    assert tracked == 3 * sum(tr for _, _, tr in want)

    def same():
        for i, (f, lm, tr) in enumerate(want):
            r = p.roi(i)
            assert r["frame"] == f and r["tracked"] == tr and np.array_equal(r["landmarks"], lm)
        assert [[(d.confidence(), d.bounding_rect().tuple()) for d in ds] for ds in p.detections()] == want_det
    same()
    # the step-at-a-time form (multi-GPU bench: all-gather between steps): every step's results
    p.begin_steps()
    for k in range(3):
        p.step(k < 2)
        same()


@pytest.mark.parametrize("kind,nets", [("face", {}), ("hand", {}),
                                       ("face", {"detector": "face_full", "landmarker": "facemesh_v2"})])
def test_device_post_equals_host_post(H, kind, nets):
    """The device-resident post-processing (decode + NMS + map, ROI seeding, tracker update on
    the GPU: PipelineConfig::device_post) gives the host restatement's results bit for bit:
    detections, seeds, views, tracked flags, confidences, updated / next ROIs, landmarks and the
    hand extras -- over frames with real faces, noise and forced ROIs, three steps."""
    from zaru_amd._lib import DeviceBuffer
    rng = np.random.default_rng(61)
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "sad_linus_mesh.npz"))
    face = np.repeat(np.repeat(g["codes"][0].transpose(1, 2, 0), 2, axis=0), 2, axis=1)
    frames = [rng.integers(0, 256, size=(480, 640, 4), dtype=np.uint8) for _ in range(10)]
    for i in range(0, 10, 2):
        y, x = int(rng.integers(0, 480 - 384)), int(rng.integers(0, 640 - 384))
        frames[i][y:y + 384, x:x + 384, :3] = face
    bufs = [DeviceBuffer.from_array(f) for f in frames]
    flist = [(b.ptr, 640, 480, 640 * 4) for b in bufs]
    R = 4 if kind == "hand" else 2
    forced = [[(float(rng.uniform(150, 490)), float(rng.uniform(150, 330)), float(rng.uniform(120, 300)),
                float(rng.uniform(120, 300)), float(rng.uniform(-3, 3)) if kind == "hand" else 0.0)
               for _ in range(R)] for _ in frames]

    def results(device_post):
        p = H.DetectTrackPipeline(kind, 0, 4, R, 3, True, 0.5 if kind == "face" else 0.0,
                                  device_post=device_post, **nets)
        p.set_frames(flist, forced)
        p.begin_steps()
        out = []
        for k in range(3):
            p.step(k < 2)
            dets = [[(d.confidence(), d.angle(), d.bounding_rect().tuple(), tuple(d.keypoints())) for d in ds]
                    for ds in p.detections()]
            rois = []
            for i in range(p.num_rois()):
                r = p.roi(i)
                row = [r["frame"], r["from_detection"], r["tracked"], r["confidence"], r["roi"].rect().tuple(),
                       r["roi"].rotation_radians(), r["view_rect"].rect().tuple(), r["view_rect"].rotation_radians()]
                if r["tracked"]:
                    row += [r["landmarks"].tobytes(), r["updated_roi"].rect().tuple(),
                            r["updated_roi"].rotation_radians(), r["next_roi"].rect().tuple()]
                    for extra in ("raw_handedness", "tongue_out", "world"):
                        if extra in r:
                            v = r[extra]
                            row.append(v.tobytes() if hasattr(v, "tobytes") else v)
                rois.append(tuple(row))
            out.append((dets, rois))
        return out

    host, dev = results(False), results(True)
    for k in range(3):
        assert dev[k][0] == host[k][0], ("detections", k)
        assert len(dev[k][1]) == len(host[k][1])
        for a, b in zip(dev[k][1], host[k][1]):
            assert a == b, ("roi", k, a[:4], b[:4])
    assert any(len(d) for d in host[0][0]) or kind == "hand"
    assert sum(r[2] for r in host[0][1]) >= 1  # something was tracked
