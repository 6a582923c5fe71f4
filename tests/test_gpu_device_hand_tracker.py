"""SURVEY §8f-3 (HandTracker part): the device-resident hand tracker (zr_hand_manage_async +
the hand LandmarkTracker update + BlazePalm post-processing on the device, DeviceHandTracker)
against the host HandTracker, which restates crates/zaru/src/hand/tracking.rs:115-219 call for
call (its filter and swap_remove sweep are pinned against a Python restatement of the Rust loops
in tests/test_hand_tracker.py).

Schedule: the device tracker takes a palm detection requested at step t at step t + 1; the host
tracker does the same when wait_detection() precedes every track() call (the reference's
`!handle.will_block()` with every detection finishing within a frame).  Both trackers get the
same injected detections (overlapping pairs: the IoU filter against tracked hands and the
de-duplication sweep both fire), the same noise frames (loss threshold -1: tracking never drops
on them) and the same clock; hands (ids, ROIs, landmarks) must agree bit for bit every step.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def H():
    import zaru_amd.host as H
    return H


def _frames(n, seed, h=360, w=480):
    rng = np.random.default_rng(seed)
    return [rng.integers(0, 256, size=(h, w, 4), dtype=np.uint8) for _ in range(n)]


def test_device_hand_tracker_matches_host(H):
    from zaru_amd._lib import DeviceBuffer
    S, STEPS = 3, 7
    frames = [_frames(STEPS, 10 + s) for s in range(S)]
    D = H.Detection
    R = H.Rect.from_center
    # per step, per stream: detections handed to both trackers
    inject = {
        0: {0: [D(0.9, R(200.0, 180.0, 40.0, 44.0), 0.3)],
            1: [D(0.9, R(100.0, 100.0, 30.0, 30.0), 0.0), D(0.8, R(104.0, 101.0, 30.0, 30.0), 0.1)],
            2: [D(0.9, R(300.0, 200.0, 50.0, 40.0), -0.2), D(0.7, R(120.0, 260.0, 36.0, 36.0), 0.5)]},
        2: {0: [D(0.9, R(203.0, 182.0, 40.0, 44.0), 0.3),   # overlaps the tracked hand: filtered
                D(0.9, R(380.0, 90.0, 30.0, 30.0), 0.0)],
            1: [D(0.6, R(330.0, 250.0, 44.0, 44.0), 1.0)]},
        4: {2: [D(0.9, R(128.0, 262.0, 36.0, 36.0), 0.5),   # on top of stream 2's second hand
                D(0.9, R(300.0, 60.0, 30.0, 30.0), 0.0)]},
    }
    hosts = []
    for s in range(S):
        t = H.HandTracker()
        t.set_loss_threshold(-1.0)
        t.set_redetect_interval(40.0)
        hosts.append(t)
    dev = H.DeviceHandTracker(S, 4)
    dev.set_loss_threshold(-1.0)
    dev.set_redetect_interval(40.0)
    bufs = [DeviceBuffer.from_array(np.stack([frames[s][k] for s in range(S)])) for k in range(STEPS)]
    fb = 360 * 480 * 4
    checked = 0
    for k in range(STEPS):
        now = 15.0 * k
        for s in range(S):
            dets = inject.get(k, {}).get(s, [])
            if dets:
                hosts[s].inject_detections(dets)
                dev.inject_detections(s, dets)
            hosts[s].wait_detection()
            hosts[s].track(frames[s][k], now_ms=now)
        dev.step([(bufs[k].ptr + s * fb, 480, 360, 480 * 4) for s in range(S)], now)
        dev.synchronize()
        pend = dev.detection_pending()
        counts = dev.hand_counts()
        for s in range(S):
            assert counts[s] == hosts[s].num_tracked(), (k, s, counts[s], hosts[s].num_tracked())
            assert bool(pend[s]) == hosts[s].detection_running(), (k, s)
            want, got = hosts[s].hands(), dev.hands(s)
            assert [h["id"] for h in got] == [h["id"] for h in want], (k, s)
            for g, w in zip(got, want):
                assert g["view_rect"].rect() == w["view_rect"].rect(), (k, s, g["id"])
                assert g["view_rect"].rotation_radians() == w["view_rect"].rotation_radians(), (k, s)
                assert np.array_equal(g["landmarks"], w["landmarks"]), (k, s, g["id"])
                checked += 1
    assert checked >= 10, checked


def _many_hands(H):
    """six palm detections far apart (all kept) plus one on top of the first (filtered on the next
    detection pass only when tracked -- here both arrive together, so the sweep removes it)"""
    R = H.Rect.from_center
    dets = [H.Detection(0.9, R(50.0 + 75.0 * i, 60.0 + 40.0 * (i % 2), 16.0, 16.0), 0.1 * i) for i in range(6)]
    dets.append(H.Detection(0.8, R(52.0, 61.0, 16.0, 16.0), 0.0))
    return dets


@pytest.mark.parametrize("slots", [8, 3])
def test_device_hand_tracker_capacity_against_host(H, slots):
    """More kept palm detections than a small slot count: the device keeps the first `slots` hands
    exactly as the host HandTracker orders them and reports the rest as dropped (the reference's
    hand list grows instead, tracking.rs:158-194); with enough slots it equals the host outright."""
    from zaru_amd._lib import DeviceBuffer
    f = _frames(3, 21)
    host = H.HandTracker()
    host.set_loss_threshold(-1.0)
    dev = H.DeviceHandTracker(1, slots)
    dev.set_loss_threshold(-1.0)
    host.inject_detections(_many_hands(H))
    dev.inject_detections(0, _many_hands(H))
    bufs = [DeviceBuffer.from_array(f[k]) for k in range(3)]
    # with enough slots the two agree on every step; with fewer, on the step that started the
    # hands (later de-duplication sweeps may swap_remove a host hand past the device's slots into
    # an earlier position, which the capped device list cannot mirror)
    steps = 3 if slots >= 7 else 1
    dropped = []
    for k in range(steps):
        host.wait_detection()
        host.track(f[k], now_ms=10.0 * k)
        dev.step([(bufs[k].ptr, 480, 360, 480 * 4)], 10.0 * k)
        dev.synchronize()
        dropped.append(dev.dropped_hands()[0])
        n_host = host.num_tracked()
        assert dev.hand_counts()[0] == min(n_host, slots), (k, n_host)
        want = host.hands()[:slots]
        got = dev.hands(0)
        assert [h["id"] for h in got] == [h["id"] for h in want], k
        for g, w in zip(got, want):
            assert g["view_rect"].rect() == w["view_rect"].rect(), (k, g["id"])
            assert np.array_equal(g["landmarks"], w["landmarks"]), (k, g["id"])
    # the step that consumed the seven detections: all 7 pass the filter (no hand yet); the sweep
    # runs after the slots are filled, so 7 - slots found no slot when slots < 7
    assert dropped[0] == max(0, 7 - slots), dropped
    assert host.num_tracked() == 6 or steps > 1  # the sweep removed the overlapping seventh
    assert dev.dropped_detections() == [0]
    assert dev.detection_capacity() == 2016


def test_device_hand_tracker_capacity_and_rejects(H):
    # more kept detections than slots: the extra ones are counted as dropped, ids stay dense
    from zaru_amd._lib import DeviceBuffer
    dev = H.DeviceHandTracker(1, 2)
    dev.set_loss_threshold(-1.0)
    f = _frames(2, 3)
    dets = [H.Detection(0.9, H.Rect.from_center(60.0 + 120.0 * i, 100.0, 30.0, 30.0), 0.0) for i in range(3)]
    dev.inject_detections(0, dets)
    drops = []
    for k in range(2):
        b = DeviceBuffer.from_array(f[k])
        dev.step([(b.ptr, 480, 360, 480 * 4)], 10.0 * k)
        dev.synchronize()
        drops.append(dev.dropped_hands()[0])
    assert dev.hand_counts() == [2]
    assert [h["id"] for h in dev.hands(0)] == [0, 1]
    assert drops[0] == 1
    with pytest.raises(Exception):
        dev.step([], 0.0)
