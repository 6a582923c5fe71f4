"""HandTracker (crates/zaru/src/hand/tracking.rs:115-219) on the HIP backend.

CPU tests pin the two pure steps (detection filtering against tracked ROIs, and the
swap_remove de-duplication sweep) against a direct Python restatement of the Rust loops.
GPU tests check that the batched tracker gives each hand exactly what the reference's per-hand
worker (a LandmarkTracker with padding 0.4) computes, bit for bit, and follow the redetection
schedule."""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def H():
    import zaru_amd.host as H
    return H


def ref_dedupe(rects, iou, thresh):
    """tracking.rs:197-208 verbatim: for i in (0..len).rev() { for j in 0..i { if iou >= t
    { swap_remove(i); break } } }"""
    hands = list(range(len(rects)))
    for i in reversed(range(len(hands))):
        for j in range(i):
            if iou(rects[hands[i]], rects[hands[j]]) >= thresh:
                hands[i] = hands[-1]
                hands.pop()
                break
    return hands


def test_dedupe_matches_swap_remove_sweep(H):
    rng = np.random.default_rng(3)
    for _ in range(200):
        n = int(rng.integers(0, 7))
        rects = [H.Rect.from_center(float(rng.uniform(0, 300)), float(rng.uniform(0, 300)),
                                    float(rng.uniform(20, 200)), float(rng.uniform(20, 200)))
                 for _ in range(n)]
        want = ref_dedupe(rects, lambda a, b: a.iou(b), 0.3)
        assert H.HandTracker.dedupe_rois(rects, 0.3) == want


def test_filter_detections(H):
    rois = [H.Rect.from_center(100, 100, 120, 120)]
    near = H.Detection(0.9, H.Rect.from_center(105, 100, 30, 30))  # grown to 120 px: overlaps
    far = H.Detection(0.9, H.Rect.from_center(400, 400, 30, 30))
    assert H.HandTracker.filter_detections(rois, [near, far], 0.3) == [False, True]
    assert H.HandTracker.filter_detections([], [near, far], 0.3) == [True, True]


def _frames(n, seed):
    rng = np.random.default_rng(seed)
    return [rng.integers(0, 256, size=(360, 480, 4), dtype=np.uint8) for _ in range(n)]


@pytest.mark.gpu
def test_tracker_matches_per_hand_landmark_tracker(H):
    """A tracked hand's landmarks equal a standalone LandmarkTracker('hand') seeded with
    RotatedRect(det.rect.grow_rel(1.5), det.angle) and padding 0.4 (tracking.rs:158-181)."""
    frames = _frames(4, 5)
    det = H.Detection(0.9, H.Rect.from_center(200.0, 180.0, 40.0, 44.0), 0.3)
    t = H.HandTracker()
    t.set_loss_threshold(-1.0)  # keep tracking on noise frames
    t.set_redetect_interval(1e9)
    t.inject_detections([det])
    ref = H.LandmarkTracker("hand")
    ref.set_loss_threshold(-1.0)
    ref.set_roi_padding(0.4)
    ref.set_roi(H.RotatedRect(det.bounding_rect().grow_rel(1.5), det.angle()))
    want = []
    for k, f in enumerate(frames):
        t.track(f, now_ms=float(k))
        if k > 0:  # hands() reports the previous frame's results
            h = [x for x in t.hands() if x["id"] == 0]
            assert len(h) == 1
            assert np.array_equal(h[0]["landmarks"], want[k - 1]["landmarks"])
            assert h[0]["view_rect"].rect() == want[k - 1]["updated_roi"].rect()
        want.append(ref.track(f))


@pytest.mark.gpu
def test_overlapping_detections_keep_one_hand(H):
    frames = _frames(2, 6)
    t = H.HandTracker()
    t.set_loss_threshold(-1.0)
    t.set_redetect_interval(1e9)
    a = H.Detection(0.9, H.Rect.from_center(200.0, 180.0, 40.0, 40.0), 0.0)
    b = H.Detection(0.8, H.Rect.from_center(204.0, 182.0, 40.0, 40.0), 0.0)
    t.inject_detections([a, b])
    t.track(frames[0], now_ms=0.0)
    assert t.num_tracked() == 1
    t.track(frames[1], now_ms=1.0)
    assert [h["id"] for h in t.hands()] == [0]


@pytest.mark.gpu
def test_redetection_schedule(H):
    """No hands: a detection starts on every track() while none runs; with hands, only once
    the redetect interval has elapsed (tracking.rs:210-218)."""
    frames = _frames(4, 7)
    t = H.HandTracker()
    t.set_redetect_interval(300.0)
    t.track(frames[0], now_ms=0.0)  # clock starts at 0; no hands -> detect, next due 300
    assert t.detection_running()
    t.wait_detection()
    t.set_loss_threshold(-1.0)
    t.inject_detections([H.Detection(0.9, H.Rect.from_center(200.0, 180.0, 40.0, 40.0), 0.0)])
    t.track(frames[1], now_ms=10.0)  # takes the finished detection; hands present, not due
    assert t.num_tracked() >= 1 and not t.detection_running()
    t.track(frames[2], now_ms=100.0)
    assert not t.detection_running()
    t.track(frames[3], now_ms=400.0)
    assert t.detection_running()
