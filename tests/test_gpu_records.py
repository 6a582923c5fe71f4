"""The device-resident record path of the multi-GPU pipeline and the detection
post-processing options of Detector (crates/zaru/src/detection.rs:44-111,186-202):

* the all-gather records the post-processing kernel writes on the device equal, bit for bit, the
  records the host packs from the pipeline's detections (`pack_detection_records`, the record
  layout of zaru_amd/shard.py), for face and palm frames;
* a one-rank communicator (zr_comm_*, RCCL) gathers exactly this rank's records, step after step;
  a world that is not the communicator's rank count is refused (the gather would write past the
  receive block), and a HIP error pending from earlier work is reported by the next zr_comm_*
  call instead of being cleared with RCCL's own stale status;
* SuppressionMode::Remove (nms.rs:70-76) on the device equals the host restatement;
* the default detection capacity keeps every NMS output (the reference's Detections is a Vec),
  and a smaller cap reports what it drops.

Palm detections on noise frames need a low threshold (Detector::set_threshold): at 0.05 the oracle
puts 33-76 anchors of such frames above it, which exercises grouping, ordering and capacity."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

W, H, NF = 1920, 1080, 6


@pytest.fixture(scope="module")
def frames():
    from configs import face_patch
    from zaru_amd._lib import DeviceBuffer
    rng = np.random.default_rng(44)
    f = rng.integers(0, 256, size=(NF, H, W, 4), dtype=np.uint8)
    big = np.repeat(np.repeat(face_patch(), 3, axis=0), 3, axis=1)
    for i in range(0, NF, 2):  # faces on every other frame
        y, x = int(rng.integers(0, H - 576)), int(rng.integers(0, W - 576))
        f[i, y:y + 576, x:x + 576] = big
    buf = DeviceBuffer.from_array(f)
    fb = H * W * 4
    flist = [(buf.ptr + i * fb, W, H, W * 4) for i in range(NF)]
    forced = [[(500.0, 400.0, 300.0, 300.0, 0.0)] for _ in range(NF)]
    return buf, flist, forced


def _pipe(H_, kind, **kw):
    rois = 1 if kind == "face" else 4
    return H_.DetectTrackPipeline(kind, 0, 4, rois, 3, True, **kw)


def _dets(p):
    return [[(d.confidence(), d.angle(), d.bounding_rect().tuple(), tuple(d.keypoints())) for d in ds]
            for ds in p.detections()]


@pytest.mark.parametrize("kind,thresh", [("face", 0.5), ("hand", 0.05)])
def test_device_records_equal_host_packed(frames, kind, thresh):
    import zaru_amd.host as H_
    _, flist, forced = frames
    p = _pipe(H_, kind, det_threshold=thresh)
    p.set_frames(flist, forced if kind == "face" else [[] for _ in range(NF)])
    first, stride = 7, 3
    p.enable_records(8, first, stride)
    p.begin_steps()
    total = 0
    for k in range(3):
        p.step(k + 1 < 3)
        dev = p.records()
        ids = [first + i * stride for i in range(NF)]
        host = H_.pack_detection_records(p.detections(), ids, 8)
        assert dev.shape == host.shape == (NF, 2 + 20 * 8)
        assert np.array_equal(dev.view(np.uint32), host.view(np.uint32)), (kind, k)
        total += int(dev[:, 1].view(np.uint32).sum())
    assert total >= (NF // 2 * 3 if kind == "face" else 3 * NF), total  # the records carry detections


def test_one_rank_communicator_gathers_the_records(frames):
    import zaru_amd.host as H_
    from zaru_amd._lib import Comm
    _, flist, forced = frames
    comm = Comm(Comm.unique_id(), 1, 0, 0)
    p = _pipe(H_, "face")
    p.set_frames(flist, forced)
    p.enable_records(8, 0, 1, comm.ptr, 1)
    p.begin_steps()
    for k in range(4):  # both record sets, each reused once
        p.step(k + 1 < 4)
        assert np.array_equal(p.gathered().view(np.uint32), p.records().view(np.uint32)), k
    del p
    comm.close()


def test_records_world_must_match_the_communicator(frames):
    import zaru_amd.host as H_
    from zaru_amd._lib import Comm
    _, flist, forced = frames
    comm = Comm(Comm.unique_id(), 1, 0, 0)
    assert comm.size() == 1
    p = _pipe(H_, "face")
    p.set_frames(flist, forced)
    with pytest.raises(Exception, match="rank count"):
        p.enable_records(8, 0, 1, comm.ptr, 2)
    del p
    comm.close()


def _hip():
    import ctypes as C
    h = C.CDLL(os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib", "libamdhip64.so"))
    h.hipGetErrorName.restype = C.c_char_p
    return h


def test_comm_reports_a_pending_hip_error(frames):
    # in the suite's own process: the library's own failed HIP calls are
    # returned once and leave nothing pending; an error another library left on this thread is
    # reported by the next zr_comm_* call, once
    from zaru_amd._lib import Comm, DeviceBuffer, ZaruError, lib, synchronize
    import ctypes as C
    hip = _hip()
    comm = Comm(Comm.unique_id(), 1, 0, 0)
    sp = C.c_void_p()
    assert lib().zr_stream_create(C.byref(sp)) == 0
    st = sp.value
    src, dst = DeviceBuffer(256), DeviceBuffer(256)
    # a HIP call of the library's own runtime that fails (pitch < width): returned, and consumed
    assert lib().zr_memcpy2d_async(dst.ptr, 4, src.ptr, 256, 256, 1, 2, None) == -3
    assert hip.hipPeekAtLastError() == 0
    comm.all_gather_async(src.ptr, dst.ptr, 256, st)  # not reported a second time
    # HIP work outside the library that failed and was never checked: pending on this thread
    assert hip.hipSetDevice(9999) != 0
    with pytest.raises(ZaruError, match="pending HIP error") as ei:
        comm.all_gather_async(src.ptr, dst.ptr, 256, st)
    assert ei.value.code == -3
    comm.all_gather_async(src.ptr, dst.ptr, 256, st)  # taken once: the next call runs
    synchronize(st)
    comm.close()
    assert lib().zr_stream_destroy(st) == 0
    assert hip.hipPeekAtLastError() == 0, hip.hipGetErrorName(hip.hipPeekAtLastError())


def test_comm_rejects_the_null_stream():
    # the gather runs on the caller's stream; the legacy NULL stream (which synchronises with
    # every blocking stream of the device) is refused
    from zaru_amd._lib import Comm, DeviceBuffer, ZaruError
    comm = Comm(Comm.unique_id(), 1, 0, 0)
    src, dst = DeviceBuffer(256), DeviceBuffer(256)
    with pytest.raises(ZaruError, match="stream"):
        comm.all_gather_async(src.ptr, dst.ptr, 256, None)
    comm.close()


def test_gather_then_remove_pipeline_in_one_process(frames):
    # the one-rank gather on a real stream, then a device-post Remove pipeline, in this process:
    # no error of the communicator's work may surface in the pipeline's launch checks
    import ctypes as C
    import zaru_amd.host as H_
    from zaru_amd._lib import Comm, DeviceBuffer, lib, synchronize
    _, flist, _ = frames
    hip = _hip()
    comm = Comm(Comm.unique_id(), 1, 0, 0)
    sp = C.c_void_p()
    assert lib().zr_stream_create(C.byref(sp)) == 0
    src, dst = DeviceBuffer.from_array(np.arange(64, dtype=np.uint32)), DeviceBuffer(256)
    for _ in range(3):
        comm.all_gather_async(src.ptr, dst.ptr, 256, sp.value)
    synchronize(sp.value)
    assert np.array_equal(dst.download((64,), np.uint32), np.arange(64, dtype=np.uint32))
    comm.close()
    assert lib().zr_stream_destroy(sp.value) == 0
    assert hip.hipPeekAtLastError() == 0, hip.hipGetErrorName(hip.hipPeekAtLastError())
    p = _pipe(H_, "hand", nms_mode="remove", det_threshold=0.05, device_post=True)
    p.set_frames(flist, [[] for _ in range(NF)])
    p.run_frames()
    assert sum(len(d) for d in p.detections()) >= NF


def test_nms_remove_device_equals_host(frames):
    import zaru_amd.host as H_
    _, flist, _ = frames
    empty = [[] for _ in range(NF)]
    got = []
    for device_post in (True, False):
        p = _pipe(H_, "hand", nms_mode="remove", det_threshold=0.05, device_post=device_post)
        p.set_frames(flist, empty)
        p.run_frames()
        got.append(_dets(p))
    assert got[0] == got[1]
    assert sum(len(d) for d in got[0]) >= NF
    # Remove keeps seeds as decoded, Average merges groups: the two modes really differ here
    p = _pipe(H_, "hand", det_threshold=0.05)
    p.set_frames(flist, empty)
    p.run_frames()
    assert _dets(p) != got[0]


def test_detection_capacity(frames):
    import zaru_amd.host as H_
    _, flist, _ = frames
    empty = [[] for _ in range(NF)]
    full = _pipe(H_, "hand", det_threshold=0.05)  # default capacity: the 2016 anchors
    full.set_frames(flist, empty)
    full.run_frames()
    counts = [len(d) for d in full.detections()]
    assert full.times()["dropped_detections"] == 0
    assert max(counts) > 4, counts  # more than any small cap: the default keeps them all
    host = _pipe(H_, "hand", det_threshold=0.05, device_post=False)
    host.set_frames(flist, empty)
    host.run_frames()
    assert _dets(full) == _dets(host)
    capped = _pipe(H_, "hand", det_threshold=0.05, det_cap=4)
    capped.set_frames(flist, empty)
    capped.run_frames()
    assert capped.times()["dropped_detections"] == sum(max(0, c - 4) for c in counts)
    assert _dets(capped) == [d[:4] for d in _dets(full)]
