#!/usr/bin/env python3
"""Benchmark: end-to-end faces/sec (BlazeFace detect + 468-pt FaceMesh) on synthetic 1080p
frames, one process per GPU (BASELINE.json metric, config 3; config 5's frame sharding for
N > 1).

A step = one batch of `--batch` 1920x1080 RGBA8 frames per GPU, already resident in HBM,
through the whole reference call chain (crates/zaru/src/detection.rs:216-270 then one
LandmarkTracker pass per face, landmark.rs:463-501): GPU letterbox preprocessing + BlazeFace,
exact host decode + weighted NMS, GPU ROI preprocessing + FaceMesh, host landmark mapping and
ROI update.  With N > 1 every rank all-gathers its fixed-size detection records over RCCL
(the single collective of SURVEY.md §8e) inside the timed region.

Synthetic data: seeded uniform-noise frames, each carrying one face patch (the reference's
own FaceMesh test image, upscaled; see load_patch) at a seeded position; frames whose detector
finds nothing are tracked on a seeded square ROI ("forced-ROI mode") so every
frame runs FaceMesh at least once.

Prints ONE JSON line (rank 0).  `--workload hand` runs config 4 (palm + 4 hand ROIs) instead.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E (MI355X_MICROARCH.md chip table)
FP32_PEAK_TFLOPS = 157.3   # f32 MFMA = f32 VALU peak


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=1024, help="frames per step per GPU")
    ap.add_argument("--workload", choices=["face", "hand"], default="face")
    ap.add_argument("--threads", type=int, default=16, help="host decode/map threads per rank")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--sub-batches", type=int, default=3)
    ap.add_argument("--streams", choices=["multi", "single"], default="multi")
    ap.add_argument("--no-cross-step", action="store_true",
                    help="one pipeline call per step (no overlap across step boundaries)")
    ap.add_argument("--no-traffic", action="store_true",
                    help="skip the rocprofv3 FETCH_SIZE/WRITE_SIZE passes behind roofline.traffic")
    return ap.parse_args()


def kernel_symbol(name: str) -> str:
    """rocprofv3's demangled kernel name -> the symbol the runtime's profiler reports
    ("void zr::dwpw_kernel<3, 1, 1, 1, 1>(zr::DwPwParams, int)" -> "dwpw_kernel<3,1,1,1,1>")."""
    name = name.split("(")[0]
    name = name.split("zr::", 1)[-1] if "zr::" in name else name.split(" ")[-1]
    return name.replace(" ", "")


def roofline_of(kernels, traffic):
    """Roofline of the dominant kernel symbol (most total time; one symbol may serve both
    networks, so records aggregate by symbol): algorithmic bytes (or FLOPs) per launch over
    its average HIP-event launch duration, against HBM or f32-MFMA peak."""
    by_symbol = {}
    for k in kernels:
        sym = k["kernel"].split("/", 1)[-1]
        a = by_symbol.setdefault(sym, {"kernel": sym, "launches": 0, "ms": 0.0, "bytes": 0.0, "flops": 0.0})
        for f in ("launches", "ms", "bytes", "flops"):
            a[f] += k[f]
    if not by_symbol:
        return None
    dom = max(by_symbol.values(), key=lambda k: k["ms"])
    avg_s = dom["ms"] / dom["launches"] / 1e3
    gbs = dom["bytes"] / dom["launches"] / avg_s / 1e9
    tfl = dom["flops"] / dom["launches"] / avg_s / 1e12
    if tfl / FP32_PEAK_TFLOPS > gbs / HBM_PEAK_GBS:
        r = {"bound": "mfma", "achieved": round(tfl, 3), "peak": FP32_PEAK_TFLOPS,
             "unit": "TFLOP/s", "frac": round(tfl / FP32_PEAK_TFLOPS, 4)}
    else:
        r = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
             "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4)}
    r["traffic"] = round(traffic[dom["kernel"]]) if traffic and dom["kernel"] in traffic else None
    r["kernel"] = dom["kernel"]
    r["avg_launch_us"] = round(avg_s * 1e6, 2)
    r["algorithmic_bytes_per_launch"] = round(dom["bytes"] / dom["launches"])
    r["kernel_share"] = round(dom["ms"] / sum(k["ms"] for k in kernels), 3)
    return r


def measure_traffic(args):
    """HBM bytes per launch of every kernel symbol, from two rocprofv3 --pmc passes (one counter
    each, no other trace domain) over a short child run of this same benchmark.  Per
    MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are KiB, and on gfx950 FETCH_SIZE counts
    half of a wide coalesced read, so it is doubled.  Runs before this process touches the GPU."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    if not shutil.which("rocprofv3"):
        return None
    child = [sys.executable, os.path.abspath(__file__), "--steps", "2", "--warmup", "1",
             "--no-cpu-baseline", "--no-profile", "--no-traffic", "--batch", str(args.batch),
             "--workload", args.workload, "--sub-batches", str(args.sub_batches),
             "--streams", args.streams]
    kib, launches = {}, {}
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with tempfile.TemporaryDirectory(dir=os.path.join(REPO, "gpurun_out")) as d:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            cmd = ["rocprofv3", "--pmc", ctr, "--kernel-trace", "--output-format", "csv",
                   "-d", d, "-o", ctr.lower(), "--"] + child
            try:
                subprocess.run(cmd, timeout=240, stdout=subprocess.DEVNULL,
                               stderr=subprocess.DEVNULL, check=True, env=dict(os.environ, TMPDIR="/tmp"))
            except (subprocess.SubprocessError, OSError):
                return None
            files = glob.glob(os.path.join(d, "**", f"{ctr.lower()}_counter_collection.csv"), recursive=True)
            if not files:
                return None
            seen = set()
            for row in csv.DictReader(open(files[0])):
                sym = kernel_symbol(row["Kernel_Name"])
                v = float(row["Counter_Value"]) * (2.0 if ctr == "FETCH_SIZE" else 1.0) * 1024.0
                kib[sym] = kib.get(sym, 0.0) + v
                key = (sym, row["Dispatch_Id"])
                if ctr == "FETCH_SIZE" and key not in seen:
                    seen.add(key)
                    launches[sym] = launches.get(sym, 0) + 1
    return {k: kib[k] / launches[k] for k in launches if launches[k]}


def make_frames(rng, n, h=1080, w=1920, patch=None):
    """n frames: one of 16 seeded uniform-noise backgrounds each, with the face patch pasted at
    a seeded position (generating 8 GB of fresh noise per run would dominate the run time)."""
    base = rng.integers(0, 256, size=(min(n, 16), h, w, 4), dtype=np.uint8)
    frames = np.empty((n, h, w, 4), np.uint8)
    centers = []
    for i in range(n):
        frames[i] = base[i % len(base)]
        if patch is not None:
            ph, pw = patch.shape[:2]
            y = int(rng.integers(0, h - ph))
            x = int(rng.integers(0, w - pw))
            frames[i, y:y + ph, x:x + pw] = patch
            centers.append((x + pw / 2, y + ph / 2, pw))
        else:
            centers.append(None)
    return frames, centers


def forced_rois(rng, n, workload, h=1080, w=1920):
    out = []
    for _ in range(n):
        k = 1 if workload == "face" else 4
        rois = []
        for _ in range(k):
            side = float(rng.uniform(150, 400))
            cx = float(rng.uniform(side / 2, w - side / 2))
            cy = float(rng.uniform(side / 2, h - side / 2))
            rad = 0.0 if workload == "face" else float(rng.uniform(-math.pi, math.pi))
            rois.append((cx, cy, side, side, rad))
        out.append(rois)
    return out


def load_patch():
    """A face to paste into the noise frames: the reference's own FaceMesh test image
    (tests/golden/sad_linus_mesh.npz, the 192x192 colour codes of sad_linus_cropped.jpg),
    upscaled 3x to 576x576, so the face spans ~400 px of the 1920-px frame and BlazeFace's
    128-px letterbox sees it at ~27 px (the size its own test image has)."""
    p = os.path.join(REPO, "tests", "golden", "sad_linus_mesh.npz")
    codes = np.load(p)["codes"][0]  # [3, 192, 192] uint8
    img = np.full((192, 192, 4), 255, np.uint8)
    img[..., :3] = codes.transpose(1, 2, 0)
    return np.repeat(np.repeat(img, 3, axis=0), 3, axis=1)


# ---------------------------------------------------------------- CPU baseline (oracle)
def cpu_baseline(frames, forced, workload, budget_s):
    """The reference path restated on the host (oracle/, single thread): same frames, same
    stages.  Label: reference-semantics C restatement, ORT/tract unavailable."""
    import oracle as O
    models = os.path.join(REPO, "zaru_amd", "models")
    if workload == "face":
        det = O.Net(os.path.join(models, "face_detection_short_range.onnx"), f64=False)
        lm = O.Net(os.path.join(models, "face_landmark.onnx"), f64=False)
        din, lin, dlo, llo, kind = 128, 192, -1.0, -1.0, O.FACE
    else:
        det = O.Net(os.path.join(models, "palm_detection_lite.onnx"), f64=False)
        lm = O.Net(os.path.join(models, "hand_landmark_lite.onnx"), f64=False)
        din, lin, dlo, llo, kind = 192, 224, 0.0, 0.0, O.PALM
    t0 = time.perf_counter()
    nframes = nfaces = 0
    for i in range(len(frames)):
        img = frames[i]
        h, w = img.shape[:2]
        r = O.grow_to_fit_aspect(O.Rect.from_top_left(0, 0, w, h), din, din)
        v = O.view_compose(O.view_full(w, h), r)
        x = O.preproc(img, v, din, din, dlo, 1.0)
        reg, cls = det.run(x[None])
        dets = O.detect_post(kind, reg[0], cls[0], w, h, din, din)
        if dets:
            grow = 0.0 if workload == "face" else 1.5
            rois = [O.RRect(O.grow_rel(d.rect, grow) if grow else d.rect,
                            d.angle if workload == "hand" else 0.0) for d in dets]
        else:
            rois = [O.RRect(O.Rect(*f[:4]), f[4]) for f in forced[i]]
        for roi in rois:
            vr = O.RRect(O.grow_to_fit_aspect(roi.rect, 1, 1), roi.rad)
            view = O.view_compose(O.view_full(w, h), vr)
            lrect = O.grow_to_fit_aspect(O.Rect.from_top_left(0, 0, view.rect.w, view.rect.h), 1, 1)
            v2 = O.view_compose(view, lrect)
            xl = O.preproc(img, v2, lin, lin, llo, 1.0)
            outs = lm.run(xl[None])
            pos = O.estimator_map(outs[0].reshape(-1, 3), lrect, lin)
            O.tracker_update(pos, vr, roi.rad, 0.0, 0.3)
            nfaces += 1
        nframes += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": nfaces / dt, "unit": "faces/s" if workload == "face" else "hands/s",
            "cores": 1, "kind": "port",
            "sample": f"{nframes} synthetic 1080p frames / {nfaces} ROIs through oracle/ "
                      f"(C restatement, f32, naive ONNX interpreter, 1 thread) in {dt:.1f} s"}


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # PMC traffic passes first: child processes, while this one has not touched the GPU
    traffic = measure_traffic(args) if (world == 1 and not args.no_traffic and not args.no_profile) else None
    import torch
    import torch.distributed as dist
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    device = local if world > 1 else 0
    torch.cuda.set_device(device)

    import zaru_amd.host as H

    B = args.batch
    rng = np.random.default_rng(3 + 1000 * rank)
    patch = load_patch() if args.workload == "face" else None
    frames_np, _ = make_frames(rng, B, patch=patch)
    forced = forced_rois(rng, B, args.workload)
    frames_t = torch.from_numpy(frames_np).to(f"cuda:{device}")
    torch.cuda.synchronize()
    fp = frames_t.data_ptr()
    fbytes = 1080 * 1920 * 4
    flist = [(fp + i * fbytes, 1920, 1080, 1920 * 4) for i in range(B)]

    pipe = H.DetectTrackPipeline(args.workload, device, args.threads,
                                 1 if args.workload == "face" else 4, args.sub_batches,
                                 args.streams == "multi")
    from zaru_amd import shard
    gather_in = torch.zeros((B, shard.record_width()), dtype=torch.float32, device=f"cuda:{device}")

    pipe.set_frames(flist, forced)

    def step():
        pipe.run_frames()
        if world > 1:
            # one RCCL all-gather of fixed-size detection records per step;
            # this rank's frames are global frames rank, rank + world, ... (shard.frames_of_rank)
            recs = pipe.detection_records(shard.REC_DETS, rank, world)
            gather_in.copy_(torch.from_numpy(recs))
            shard.all_gather_records(gather_in)
        return pipe.num_rois()

    # N = 1: the steps run back to back in one call that overlaps each step's host tail
    # (landmark mapping) with the next step's detection on the GPU (run_frames_repeated).
    # N > 1 keeps one call per step: every step ends in the all-gather of its detections.
    repeated = world == 1 and not args.no_cross_step
    if repeated:
        pipe.run_frames_repeated(args.warmup)
    else:
        for _ in range(args.warmup):
            step()
    if not args.no_profile:
        pipe.profile_read()  # drop warmup records
        pipe.profile(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    faces = 0
    stage = {"detect_gpu_ms": 0.0, "decode_nms_ms": 0.0, "landmark_gpu_ms": 0.0, "map_ms": 0.0}
    dets_total = 0
    if repeated:
        faces = pipe.run_frames_repeated(args.steps)
        t = pipe.times()
        for k in stage:
            stage[k] = t[k]
        dets_total = t["detections"]
    else:
        for _ in range(args.steps):
            faces += step()
            t = pipe.times()
            for k in stage:
                stage[k] += t[k]
            dets_total += t["detections"]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    prof = pipe.profile_read() if not args.no_profile else ""
    pipe.profile(False)

    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{device}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        c = torch.tensor([faces], dtype=torch.float64, device=f"cuda:{device}")
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        faces_all = int(c.item())
    else:
        faces_all = faces

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    # ---- roofline of the dominant kernel, from the HIP-event records of the timed region
    kernels = []
    for line in prof.splitlines():
        name, n, ms, by, fl = line.rsplit(" ", 4)
        k = {"kernel": name, "launches": int(n), "ms": float(ms), "bytes": float(by), "flops": float(fl)}
        sym = name.split("/", 1)[-1]
        if traffic and sym in traffic:
            k["traffic_per_launch_symbol_avg"] = round(traffic[sym])
        kernels.append(k)
    roofline = roofline_of(kernels, traffic)
    # The timed region runs the sub-batches on concurrent streams, so a launch shares the GPU
    # with the other stream's kernels and its HIP-event duration overstates the kernel's own.
    # The same frames once more on ONE stream give each kernel's uncontended launch time.
    roofline_isolated = None
    if not args.no_profile and world == 1:
        pipe1 = H.DetectTrackPipeline(args.workload, device, args.threads,
                                      1 if args.workload == "face" else 4, args.sub_batches, False)
        pipe1.set_frames(flist, forced)
        pipe1.run_frames_repeated(2)
        pipe1.profile_read()
        pipe1.profile(True)
        pipe1.run_frames_repeated(max(3, args.steps // 2))
        iso = []
        for line in pipe1.profile_read().splitlines():
            name, n, ms, by, fl = line.rsplit(" ", 4)
            iso.append({"kernel": name, "launches": int(n), "ms": float(ms), "bytes": float(by), "flops": float(fl)})
        pipe1.profile(False)
        roofline_isolated = roofline_of(iso, traffic)
        if roofline_isolated:
            roofline_isolated["note"] = "same frames, sub-batches on one HIP stream (no cross-stream overlap)"
    st = pipe.stats()
    frames_per_s = world * B * args.steps / elapsed
    bytes_frame = st["detector_bytes_per_image"] + st["landmarker_bytes_per_image"] * faces / (B * args.steps)
    pipeline_gbs_per_gpu = frames_per_s / world * bytes_frame / 1e9

    cpu = None
    if not args.no_cpu_baseline and world == 1:
        cpu = cpu_baseline(frames_np, forced, args.workload, args.cpu_baseline_seconds)

    unit = "faces/s" if args.workload == "face" else "hands/s"
    out = {
        "metric": "end-to-end faces/sec (detect+468-pt mesh), 1080p synthetic, 1/2/4/8 GPU"
        if args.workload == "face" else "end-to-end hands/sec (palm detect + 21-pt hand landmarks, 4 ROIs/frame)",
        "value": round(faces_all / elapsed, 1),
        "unit": unit,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: seeded uniform-noise 1920x1080 RGBA8 frames"
                + (" + one 576x576 face patch each (reference test image, upscaled)" if args.workload == "face" else "")
                + "; forced seeded ROI when no detection; ONNX weights from the reference",
        "config": {"workload": "face pipeline BlazeFace->FaceMesh V1 (config 3/5)" if args.workload == "face"
                   else "palm lite + hand landmark lite, 4 ROIs/frame (config 4)",
                   "frames_per_gpu_per_step": B, "frame": "1920x1080 RGBA8",
                   "parallelism": f"frame-sharded x{world}" + (", RCCL all-gather of detections" if world > 1 else "")},
        "frames_per_s": round(frames_per_s, 1),
        "detections_per_step": round(dets_total / args.steps, 1),
        "stage_ms_per_step": {k: round(v / args.steps, 3) for k, v in stage.items()},
        "pipeline_algorithmic_GBs_per_gpu": round(pipeline_gbs_per_gpu, 1),
        "roofline": roofline,
        "roofline_isolated": roofline_isolated,
        "kernels": sorted(kernels, key=lambda k: -k["ms"]),
        "cpu_baseline": cpu,
    }
    print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
