"""Config 5 on one GPU: the face pipeline (C3: BlazeFace -> FaceMesh V1) and
the hand pipeline (C4: palm lite -> hand landmark lite) running concurrently, each from its own
host thread on its own HIP streams, over the same HBM-resident 1080p camera frames -- the
examples' two loops (examples/facemesh.rs:35-56, examples/hand_tracking.rs:19-62) sharing one
GPU.  Every step of each pipeline must be bitwise equal to the same pipeline run alone: the
detections, the combined detection records the multi-GPU all-gather ships, the ROIs and every
landmark."""
import os
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, H, NF, STEPS = 1920, 1080, 12, 3


def camera_frames():
    rng = np.random.default_rng(5)  # C5 seed
    codes = np.load(os.path.join(REPO, "tests", "golden", "sad_linus_mesh.npz"))["codes"][0]
    patch = np.full((192, 192, 4), 255, np.uint8)
    patch[..., :3] = codes.transpose(1, 2, 0)
    patch = np.repeat(np.repeat(patch, 3, axis=0), 3, axis=1)
    frames = rng.integers(0, 256, size=(NF, H, W, 4), dtype=np.uint8)
    for f in range(NF):
        y, x = int(rng.integers(0, H - 576)), int(rng.integers(0, W - 576))
        frames[f, y:y + 576, x:x + 576] = patch
    face_forced = [[(float(rng.uniform(200, W - 200)), float(rng.uniform(200, H - 200)), 300.0, 300.0, 0.0)]
                   for _ in range(NF)]
    hand_forced = [[(float(rng.uniform(200, W - 200)), float(rng.uniform(200, H - 200)),
                     float(rng.uniform(150, 400)), float(rng.uniform(150, 400)), float(rng.uniform(-3, 3)))
                    for _ in range(4)] for _ in range(NF)]
    return frames, face_forced, hand_forced


def snapshot(p):
    dets = [[(d.confidence(), d.angle(), d.bounding_rect().tuple(), tuple(d.keypoints())) for d in ds]
            for ds in p.detections()]
    rois = []
    for i in range(p.num_rois()):
        r = p.roi(i)
        rois.append((r["frame"], r["tracked"], r["confidence"], r["roi"].rect().tuple(),
                     r["roi"].rotation_radians(), r["landmarks"].tobytes() if r["tracked"] else b"",
                     r["next_roi"].rect().tuple() if r["tracked"] else None))
    return dets, rois, p.detection_records(8, 0, 1).tobytes()


def run(H_, pipes, flist, forced, concurrent):
    for p, fc in zip(pipes, forced):
        p.set_frames(flist, fc)
        p.begin_steps()
    out = [[] for _ in pipes]

    def loop(j):
        for k in range(STEPS):
            pipes[j].step(k + 1 < STEPS)
            out[j].append(snapshot(pipes[j]))

    if concurrent:
        ths = [threading.Thread(target=loop, args=(j,)) for j in range(len(pipes))]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
    else:
        for j in range(len(pipes)):
            loop(j)
    return out


def test_face_and_hand_concurrently_equal_solo():
    import zaru_amd.host as H_
    from zaru_amd._lib import DeviceBuffer
    frames, face_forced, hand_forced = camera_frames()
    buf = DeviceBuffer.from_array(frames)
    fb = H * W * 4
    flist = [(buf.ptr + f * fb, W, H, W * 4) for f in range(NF)]
    forced = [face_forced, hand_forced]

    def pipes():
        return [H_.DetectTrackPipeline("face", 0, 4, 1, 3, True), H_.DetectTrackPipeline("hand", 0, 4, 4, 3, True)]

    solo = [run(H_, [p], flist, [fc], False)[0] for p, fc in zip(pipes(), forced)]
    both = run(H_, pipes(), flist, forced, True)
    for j, name in enumerate(("face", "hand")):
        assert len(both[j]) == STEPS
        for k in range(STEPS):
            assert both[j][k][0] == solo[j][k][0], (name, k, "detections")
            assert both[j][k][1] == solo[j][k][1], (name, k, "rois / landmarks")
            assert both[j][k][2] == solo[j][k][2], (name, k, "detection records")
    # the workload really ran: faces detected on the patched frames, every ROI evaluated
    assert sum(len(d) for d in solo[0][0][0]) >= NF // 2
    assert len(solo[1][0][1]) >= 4 * NF
