"""CPU baseline worker for bench.py -- TEST INFRASTRUCTURE ONLY (the timed CPU baseline leg).

Label: "reference-semantics C restatement (ORT/tract unavailable)".  One worker = one
single-threaded instance of the reference CPU path (ORT runs 1 intra- + 1 inter-op thread,
crates/zaru/src/nn/mod.rs:342-346), restated by this oracle in f32:

  face (config 3):  letterbox view + ColorMapper (nn/mod.rs:54-73) -> BlazeFace (direct f32
  convolutions, oracle/nnexec_impl.h) -> decode + weighted NMS + map (detection.rs:216-270)
  -> per detection (or the forced ROI when none) one LandmarkTracker pass: ROI view +
  preprocessing -> FaceMesh -> Estimator map-out (landmark.rs:314-348) -> loss check and
  tracker update with the estimate's angle (landmark.rs:463-501).
  hand (config 4): the same with BlazePalm lite / hand landmark lite, ROI grow 1.5 and
  padding 0.4 (hand/tracking.rs:34,136-159).

bench.py starts P of these (P = the host cores it may use) BEFORE it touches the GPU; worker w
takes frames w, w + P, ... of the bench's own synthetic frames (same seeds) until its time
budget ends, and prints one JSON line: objects tracked, frames, seconds and per-stage ms,
mirroring Detector / Estimator timers (detection.rs:273-275, landmark.rs:289-291).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=["face", "hand"], default="face")
    ap.add_argument("--worker", type=int, default=0)
    ap.add_argument("--workers", type=int, default=1)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--seed", type=int, default=3)
    args = ap.parse_args()
    os.environ["OMP_NUM_THREADS"] = "1"

    import numpy as np

    import oracle as O
    from bench import FrameSet, forced_rois, load_patch

    face = args.workload == "face"
    rng = np.random.default_rng(args.seed)
    fs = FrameSet(rng, args.batch, patch=load_patch() if face else None)
    forced = forced_rois(rng, args.batch, args.workload)
    models = os.path.join(REPO, "zaru_amd", "models")
    if face:
        det = O.Net(os.path.join(models, "face_detection_short_range.onnx"), f64=False)
        lm = O.Net(os.path.join(models, "face_landmark.onnx"), f64=False)
        din, lin, lo, kind, lkind, grow, pad = 128, 192, -1.0, O.FACE, O.FACEMESH, 0.0, 0.3
    else:
        det = O.Net(os.path.join(models, "palm_detection_lite.onnx"), f64=False)
        lm = O.Net(os.path.join(models, "hand_landmark_lite.onnx"), f64=False)
        din, lin, lo, kind, lkind, grow, pad = 192, 224, 0.0, O.PALM, O.HAND, 1.5, 0.4
    stage = {"preproc_ms": 0.0, "det_infer_ms": 0.0, "extract_nms_ms": 0.0,
             "lm_infer_ms": 0.0, "lm_map_ms": 0.0}
    clk = time.perf_counter
    # per-stage figures in process CPU time: with more processes than the cgroup's cores, wall
    # spans of a stage would include the time the process waited for a core
    sclk = time.process_time
    nframes = nrois = ntracked = 0
    t_start = clk()
    f = args.worker
    while clk() - t_start < args.seconds:
        img = fs.frame(f % args.batch)
        h, w = img.shape[:2]
        t = sclk()
        r = O.grow_to_fit_aspect(O.Rect.from_top_left(0, 0, w, h), din, din)
        v = O.view_compose(O.view_full(w, h), r)
        x = O.preproc(img, v, din, din, lo, 1.0)
        t1 = sclk()
        reg, cls = det.run(x[None])
        t2 = sclk()
        dets = O.detect_post(kind, reg[0], cls[0], w, h, din, din)
        if dets:
            rois = [O.RRect(O.grow_rel(d.rect, grow) if grow else d.rect, 0.0 if face else d.angle)
                    for d in dets[:1 if face else 4]]  # max_rois_per_frame of the GPU pipeline
        else:
            rois = [O.RRect(O.Rect(*fr[:4]), fr[4]) for fr in forced[f % args.batch]]
        t3 = sclk()
        stage["preproc_ms"] += (t1 - t) * 1e3
        stage["det_infer_ms"] += (t2 - t1) * 1e3
        stage["extract_nms_ms"] += (t3 - t2) * 1e3
        for roi in rois:
            t = sclk()
            vr = O.RRect(O.grow_to_fit_aspect(roi.rect, 1, 1), roi.rad)
            view = O.view_compose(O.view_full(w, h), vr)
            lrect = O.grow_to_fit_aspect(O.Rect.from_top_left(0, 0, view.rect.w, view.rect.h), 1, 1)
            xl = O.preproc(img, O.view_compose(view, lrect), lin, lin, lo, 1.0)
            t1 = sclk()
            outs = lm.run(xl[None])
            t2 = sclk()
            pos = O.estimator_map(outs[0].reshape(-1, 3), lrect, lin)  # Estimator maps first
            if O.landmark_confidence(lkind, outs) >= 0.5:  # then the tracker's loss check
                O.tracker_update(pos, vr, roi.rad, O.landmark_angle(lkind, pos), pad)
                ntracked += 1
            t3 = sclk()
            stage["preproc_ms"] += (t1 - t) * 1e3
            stage["lm_infer_ms"] += (t2 - t1) * 1e3
            stage["lm_map_ms"] += (t3 - t2) * 1e3
            nrois += 1
        nframes += 1
        f += args.workers
    dt = clk() - t_start
    print(json.dumps({"worker": args.worker, "frames": nframes, "rois": nrois,
                      "tracked": ntracked, "seconds": dt, "stage_ms": stage}))


if __name__ == "__main__":
    main()
