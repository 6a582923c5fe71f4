#!/usr/bin/env python3
"""Benchmark: end-to-end faces/sec (BlazeFace detect + 468-pt FaceMesh) on synthetic 1080p
frames, one process per GPU (BASELINE.json metric, config 3; config 5's frame sharding with
the RCCL all-gather of detections for N > 1).

A step = one batch of `--batch` 1920x1080 RGBA8 frames per GPU, already resident in HBM,
through the whole reference call chain (crates/zaru/src/detection.rs:216-270, then one
LandmarkTracker pass seeded from the best detection, examples/facemesh.rs:40-54 /
landmark.rs:463-501): GPU letterbox preprocessing + BlazeFace, exact host decode + weighted NMS,
GPU ROI preprocessing + FaceMesh, host landmark mapping, loss check and ROI update.  Steps run
back to back, software-pipelined (the next step's detections are enqueued before this step's
landmark mapping).  With N > 1 the post-processing kernel writes each step's fixed-size
detection records straight into a device buffer and every rank all-gathers them over RCCL (the
single collective of SURVEY.md §8e, zr_comm_all_gather_async) on the pipeline's own gather
stream, overlapped with the following steps, inside the timed region: no host copy per step.
torch.distributed (gloo) is the control plane only (the communicator id, barriers, the max of
the per-rank times).

`value` = tracked faces (face_flag >= the 0.5 loss threshold) per second over all ranks.

Synthetic data: seeded uniform-noise frames (16 backgrounds), each carrying one face patch (the
reference's own FaceMesh test image, upscaled; see load_patch) at a seeded position; frames
whose detector finds nothing are tracked on a seeded square ROI ("forced-ROI mode", SURVEY.md
§8d C3).

Prints ONE JSON line (rank 0).  At N = 1 it also carries:
  * "hand": config 4 (palm lite + hand landmark lite, 4 ROIs per frame, 256 frames per step);
  * "cpu_baseline": the oracle's C restatement of the same pipeline, P single-threaded
    processes on the host cores, timed before the GPU is touched;
  * "roofline": the dominant kernel, from an uncontended (one-stream) profiled pass, with the
    rocprofv3 PMC traffic of that kernel; "pipeline_roofline": SURVEY §8d's per-frame model.
`--workload hand` benchmarks config 4 alone; `--workload both` runs face and hand pipelines
concurrently on their own HIP streams with one combined all-gather (config 5).
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

# Hardware queues per process (read by the HIP runtime at initialisation, so set before anything
# here touches the GPU).  The face line runs 4 sub-batch streams + 1 gather stream; with HIP's
# default of 4 queues (which the GPU boxes also export), streams beyond that share a queue and
# independent sub-batches serialise behind each other.  8 queues with 4 face sub-batches:
# 255.7 k vs 247.7-251.4 k faces/s with 4 queues and 3, and 216-218 k with 4 queues and 4
# (profiles/r05_hwqueues_ab.txt).  ZARU_BENCH_HW_QUEUES picks another count for A/B runs.
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("ZARU_BENCH_HW_QUEUES", "8")

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E (MI355X_MICROARCH.md chip table)
FP32_PEAK_TFLOPS = 157.3   # f32 MFMA = f32 VALU peak
METRIC = "end-to-end faces/sec (detect+468-pt mesh), 1080p synthetic, 1/2/4/8 GPU"

# SURVEY.md §8d roofline model: algorithmic bytes per image at layer boundaries (fp32, fused
# epilogues, weights excluded) and per preprocessed view (4 B gathered + 12 B written / pixel)
SURVEY_BYTES = {"face_detection_short_range": 11.02e6, "face_landmark": 16.56e6,
                "palm_detection_lite": 51.58e6, "hand_landmark_lite": 37.20e6}
SURVEY_FLOPS = {"face_detection_short_range": 61.52e6, "face_landmark": 69.96e6,
                "palm_detection_lite": 566.34e6, "hand_landmark_lite": 291.21e6}
# SURVEY §8f-1 networks have no §8d figure: their compiled plans' own per-image bytes at fused
# kernel boundaries and FLOPs (zr_plan_describe; for the four §8d networks these plan bytes
# are 0.64-0.65x the §8d layer-boundary model, so this is the stricter denominator)
SURVEY_BYTES.update({"face_detection_full_range": 30.08e6, "face_landmarks_detector": 39.93e6})
SURVEY_FLOPS.update({"face_detection_full_range": 211.34e6, "face_landmarks_detector": 225.73e6})

WORKLOADS = {
    # kind: detector, landmark net, det input, landmark input, ROIs per frame, seed (§8d)
    "face": ("face_detection_short_range", "face_landmark", 128, 192, 1, 3),
    "hand": ("palm_detection_lite", "hand_landmark_lite", 192, 224, 4, 4),
    # BlazeFace full range -> FaceMesh V2 (478 points) on config 3's frames
    "face_next": ("face_detection_full_range", "face_landmarks_detector", 192, 256, 1, 3),
}
# pipeline kind and network overrides of each workload (DetectTrackPipeline arguments)
PIPELINE = {"face": ("face", "", ""), "hand": ("hand", "", ""),
            "face_next": ("face", "face_full", "facemesh_v2")}


def sub_batches(args, kind):
    """Sub-batches per step: --sub-batches, else 4 for the face line (with 8 hardware queues,
    profiles/r05_hwqueues_ab.txt) and 3 for the others (the hand line's 341-ROI sub-batches:
    91.8 k ROIs/s against 81.6 k with 4, profiles/r05_bench_hand_subbatches.txt)."""
    if args.sub_batches:
        return args.sub_batches
    return 4 if kind == "face" and int(os.environ["GPU_MAX_HW_QUEUES"]) >= 8 else 3


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); N > 1 without WORLD_SIZE set: this process starts the N ranks "
                         "itself (zaru_amd/launch.py), under torchrun WORLD_SIZE must equal N")
    ap.add_argument("--rank-timeout", type=float, default=1500.0,
                    help="launcher only: seconds before the N ranks are stopped and the run fails")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=1024, help="frames per step per GPU")
    ap.add_argument("--workload", choices=["face", "hand", "both", "face_next"], default="face")
    ap.add_argument("--threads", type=int, default=16, help="host decode/map threads per rank")
    ap.add_argument("--sub-batches", type=int, default=None,
                    help="software-pipelined sub-batches per step (default: face 4, others 3)")
    ap.add_argument("--streams", choices=["multi", "single"], default="multi")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="skip the per-kernel profiled pass")
    ap.add_argument("--no-traffic", action="store_true",
                    help="skip the rocprofv3 FETCH_SIZE/WRITE_SIZE passes behind roofline.traffic")
    ap.add_argument("--no-hand", action="store_true", help="skip the config-4 line at N = 1")
    ap.add_argument("--hand-steps", type=int, default=30)
    ap.add_argument("--hand-batch", type=int, default=256)
    ap.add_argument("--no-next", action="store_true",
                    help="skip the SURVEY §8f-1 line (full range + FaceMesh V2) at N = 1")
    ap.add_argument("--next-steps", type=int, default=30)
    ap.add_argument("--no-tracking", action="store_true",
                    help="skip the SURVEY §8f-3 device-tracker line at N = 1")
    ap.add_argument("--tracking-steps", type=int, default=50)
    ap.add_argument("--no-jpeg", action="store_true", help="skip the SURVEY §8f-2 JPEG-source line at N = 1")
    ap.add_argument("--next-batch", type=int, default=512)
    ap.add_argument("--no-c5", action="store_true", help="skip the config-5 line (face + hand concurrently) at N = 1")
    ap.add_argument("--c5-steps", type=int, default=8)
    ap.add_argument("--host-post", action="store_true",
                    help="decode/NMS/map and the tracker update on host threads (the host restatement) "
                         "instead of on the device")
    ap.add_argument("--self-gather", action="store_true",
                    help="N = 1 only: run the N > 1 data path (device records + an RCCL all-gather per step "
                         "over a one-rank communicator), to price it on one GPU")
    ap.add_argument("--prime-seconds", type=float, default=0.6,
                    help="untimed pipeline priming before the warmup steps (see prime())")
    return ap.parse_args()


# ---------------------------------------------------------------- synthetic frames
class FrameSet:
    """n 1080p RGBA8 frames: one of 16 seeded uniform-noise backgrounds each, with the face
    patch pasted at a seeded position (generating 8 GB of fresh noise per run would dominate
    the run time).  Frames are composed on demand (host) or on the GPU (to_device)."""

    def __init__(self, rng, n, h=1080, w=1920, patch=None):
        self.n, self.h, self.w, self.patch = n, h, w, patch
        self.base = rng.integers(0, 256, size=(min(n, 16), h, w, 4), dtype=np.uint8)
        self.pos = []
        for _ in range(n):
            if patch is None:
                self.pos.append(None)
                continue
            ph, pw = patch.shape[:2]
            y = int(rng.integers(0, h - ph))
            x = int(rng.integers(0, w - pw))
            self.pos.append((y, x))

    def frame(self, i):
        f = self.base[i % len(self.base)].copy()
        if self.pos[i] is not None:
            y, x = self.pos[i]
            ph, pw = self.patch.shape[:2]
            f[y:y + ph, x:x + pw] = self.patch
        return f

    def to_device(self, device):
        import torch
        base = torch.from_numpy(self.base).to(device)
        out = torch.empty((self.n, self.h, self.w, 4), dtype=torch.uint8, device=device)
        patch = torch.from_numpy(self.patch).to(device) if self.patch is not None else None
        for i in range(self.n):
            out[i].copy_(base[i % len(self.base)])
            if self.pos[i] is not None:
                y, x = self.pos[i]
                out[i, y:y + patch.shape[0], x:x + patch.shape[1]] = patch
        torch.cuda.synchronize(device)
        return out


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


# ---------------------------------------------------------------- rocprofv3 evidence
def kernel_symbol(name: str) -> str:
    """rocprofv3's demangled kernel name -> the symbol the runtime's profiler reports
    ("void zr::dwpw_kernel<3, 1, 1, 1, 1>(zr::DwPwParams, int)" -> "dwpw_kernel<3,1,1,1,1>")."""
    name = name.split("(")[0]
    name = name.split("zr::", 1)[-1] if "zr::" in name else name.split(" ")[-1]
    return name.replace(" ", "")


def measure_traffic(args, kind, batch=None):
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
             "--no-cpu-baseline", "--no-profile", "--no-traffic", "--no-hand", "--no-next", "--no-tracking",
             "--no-jpeg", "--no-c5"] + (["--host-post"] if args.host_post else []) + [
             "--batch", str(batch or args.batch), "--workload", kind,
             "--sub-batches", str(sub_batches(args, kind)), "--streams", args.streams]
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


def parse_profile(txt):
    out = []
    for line in txt.splitlines():
        name, n, ms, by, fl = line.rsplit(" ", 4)
        out.append({"kernel": name, "launches": int(n), "ms": float(ms), "bytes": float(by), "flops": float(fl)})
    return out


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
    r["timing"] = "uncontended: sub-batches on one HIP stream, HIP events around every launch"
    return r


# ---------------------------------------------------------------- CPU baseline (oracle)
def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_quota():
    """CPUs this process may really use: the cgroup v2 quota (cpu.max), else its affinity."""
    n = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, round(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    return n


def cpu_baseline(kind, seconds, batch, seed, P=None):
    """The reference path restated on the host (oracle/cpu_baseline.py): P single-threaded
    worker processes (ORT's 1 intra + 1 inter thread per session, nn/mod.rs:342-346) over the
    bench's own frames; P = nproc by default (one instance per host core).
    Runs before this process touches the GPU."""
    import subprocess
    P = P or os.cpu_count() or 1
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, os.path.join(REPO, "oracle", "cpu_baseline.py"), "--workload", kind,
           "--workers", str(P), "--seconds", str(seconds), "--batch", str(batch), "--seed", str(seed)]
    procs = [subprocess.Popen(cmd + ["--worker", str(w)], stdout=subprocess.PIPE,
                              stderr=subprocess.DEVNULL, env=env) for w in range(P)]
    res = []
    for p in procs:
        out, _ = p.communicate(timeout=seconds + 180)
        if p.returncode == 0 and out.strip():
            res.append(json.loads(out.decode().strip().splitlines()[-1]))
    if not res:
        return None
    frames = sum(r["frames"] for r in res)
    stage = {k: round(sum(r["stage_ms"][k] for r in res) / max(1, frames), 3) for k in res[0]["stage_ms"]}
    value = sum(r["tracked"] / r["seconds"] for r in res)
    # cores: the hardware threads the P processes really ran on (on the GPU box nproc shows the
    # whole machine, but the cgroup quota is the per-GPU share)
    return {"value": round(value, 2), "unit": "faces/s" if kind == "face" else "tracked hands/s",
            "cores": min(len(res), cpu_quota()), "kind": "port", "processes": len(res),
            "nproc": os.cpu_count(), "cpu_quota": cpu_quota(),
            "rois_per_s": round(sum(r["rois"] / r["seconds"] for r in res), 2),
            "frames_per_s": round(sum(r["frames"] / r["seconds"] for r in res), 2),
            "cpu": cpu_model(), "stage_ms_per_frame": stage,
            "stage_clock": "process CPU time per frame (the processes share the cgroup's cores)",
            "label": "reference-semantics C restatement (ORT/tract unavailable): oracle/ direct f32 "
                     "convolutions, glibc-exact geometry, 1 thread per process",
            "sample": f"{frames} synthetic 1080p frames ({sum(r['rois'] for r in res)} ROIs) of the "
                      f"bench's own frames over {len(res)} processes x {seconds:g} s"}


# ---------------------------------------------------------------- the GPU pipelines
class Workload:
    """One DetectTrackPipeline over its resident synthetic frames."""

    device_post = True  # bench.py --host-post sets False

    def __init__(self, H, kind, device, batch, rank, threads, sub_batches, multi_stream, shared=None):
        det, lm, din, lin, rois, seed = WORKLOADS[kind]
        self.kind, self.batch, self.det, self.lm = kind, batch, det, lm
        rng = np.random.default_rng(seed + 1000 * rank)
        base, dnet, lnet = PIPELINE[kind]
        if shared is None:
            self.fs = FrameSet(rng, batch, patch=load_patch() if base == "face" else None)
            self.frames = self.fs.to_device(f"cuda:{device}")
        else:  # config 5: the other pipeline's frames (the same camera streams)
            self.fs, self.frames = shared.fs, shared.frames
        forced = forced_rois(rng, batch, base)
        fp, fb = self.frames.data_ptr(), 1080 * 1920 * 4
        self.flist = [(fp + i * fb, 1920, 1080, 1920 * 4) for i in range(batch)]
        self.forced = forced
        self.args = (base, device, threads, rois, sub_batches)
        self.nets = {"detector": dnet, "landmarker": lnet}
        self.pipe = H.DetectTrackPipeline(base, device, threads, rois, sub_batches, multi_stream,
                                          device_post=Workload.device_post, **self.nets)
        self.pipe.set_frames(self.flist, forced)

    def profiled(self, H, steps):
        """Per-kernel HIP-event times with the sub-batches on one stream (uncontended)."""
        kind, device, threads, rois, sub_batches = self.args
        p = H.DetectTrackPipeline(kind, device, threads, rois, sub_batches, False,
                                  device_post=Workload.device_post, **self.nets)
        p.set_frames(self.flist, self.forced)
        p.run_frames_repeated(2)
        p.profile_read()
        p.profile(True)
        p.run_frames_repeated(steps)
        txt = p.profile_read()
        p.profile(False)
        return parse_profile(txt), p.times()


def prime(workloads, seconds, pool):
    """Untimed steps before the warmup, until `seconds` have passed (at least 3 steps): the
    first launches of every kernel load their code objects and the GPU leaves its idle clocks,
    which makes the first ~10 steps up to 2.3x slower than steady state
    (profiles/r03_probe_steps.jsonl).  The W warmup and K timed steps follow unchanged."""
    import torch
    t0 = time.perf_counter()
    n = 0
    while n < 3 or time.perf_counter() - t0 < seconds:
        run_steps(workloads, 1, None, 0, 1, pool)
        n += 1
    torch.cuda.synchronize()
    return {"steps": n, "seconds": round(time.perf_counter() - t0, 3),
            "why": "first-launch code-object loads and GPU clock ramp before the warmup steps"}


def run_steps(workloads, steps, gather, rank, world, pool):
    """`steps` software-pipelined steps of every workload (concurrently when there are two).  With
    N > 1 each pipeline all-gathers its device-written records itself (RCCL, enable_records);
    `gather` is only the shared-GPU dry run's stand-in (gloo has no device path: the records are
    copied to the host and gathered there)."""
    for w in workloads:
        w.pipe.begin_steps()
    for k in range(steps):
        more = k + 1 < steps
        if pool is None:
            for w in workloads:
                w.pipe.step(more)
        else:
            list(pool.map(lambda w: w.pipe.step(more), workloads))
        if gather is not None:
            recs = [w.pipe.records() for w in workloads]
            gather.submit(np.concatenate(recs) if len(recs) > 1 else recs[0])
    if gather is not None:
        gather.finish()
    return [w.pipe.times() for w in workloads]


def main():
    args = parse()
    from zaru_amd import launch
    try:
        world = launch.world_from_env(args.gpus)
    except ValueError as e:
        print(f"bench.py: {e}", file=sys.stderr)
        sys.exit(2)
    if world is None:
        # --gpus N > 1 without an outside launcher: start the N ranks here (child processes,
        # before this process touches the GPU) and exit with their verdict
        sys.exit(launch.run_ranks([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                  args.gpus, args.rank_timeout))
    Workload.device_post = not args.host_post
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    primary = args.workload if args.workload in ("hand", "face_next") else "face"
    # child processes first, while this one has not touched the GPU: PMC traffic passes,
    # then the CPU baseline (its workers would otherwise compete with the pipeline's threads)
    traffic, side_traffic = None, {}
    if world == 1 and not args.no_traffic and not args.no_profile:
        traffic = measure_traffic(args, primary)
        # the side lines' dominant kernels, at the side lines' own batch sizes
        if args.workload == "face" and not args.no_hand:
            side_traffic["hand"] = measure_traffic(args, "hand", args.hand_batch)
        if args.workload == "face" and not args.no_next:
            side_traffic["face_next"] = measure_traffic(args, "face_next", args.next_batch)
    cpu = None
    if world == 1 and not args.no_cpu_baseline and primary in ("face", "hand"):
        seed = WORKLOADS[primary][5]
        cpu = cpu_baseline(primary, args.cpu_baseline_seconds, args.batch, seed)
        if cpu is not None and (os.cpu_count() or 1) > 16:  # the GPU box's per-GPU CPU share
            c16 = cpu_baseline(primary, args.cpu_baseline_seconds, args.batch, seed, P=16)
            if c16 is not None:
                cpu["p16"] = {k: c16[k] for k in ("value", "cores", "processes", "frames_per_s", "sample")}

    import torch
    import torch.distributed as dist
    # ZARU_BENCH_SHARE_GPU=1: a dry run of the N > 1 path on a one-GPU box -- every rank on
    # cuda:0 and the record gather over gloo (RCCL refuses two ranks on one device)
    share = world > 1 and os.environ.get("ZARU_BENCH_SHARE_GPU") == "1"
    device = 0 if (share or world == 1) else local
    torch.cuda.set_device(device)
    if world > 1:
        # one node: the RCCL bootstrap needs no network interface beyond loopback
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        from zaru_amd._lib import _StdoutToStderr
        with _StdoutToStderr():  # gloo's connection notices: stdout carries the one JSON line
            dist.init_process_group("gloo")  # control plane only (ids, barriers, max / sum)
            dist.barrier()

    import zaru_amd.host as H
    from zaru_amd import shard
    from zaru_amd._lib import Comm

    kinds = ["face", "hand"] if args.workload == "both" else [primary]
    threads = args.threads if len(kinds) == 1 else max(2, args.threads // 2)
    wls = []
    for k in kinds:  # config 5: the hand pipeline runs on the face pipeline's frames
        wls.append(Workload(H, k, device, args.batch, rank, threads, sub_batches(args, k),
                            args.streams == "multi", shared=wls[0] if wls else None))
    comms, gather = [], None
    if world > 1:
        if not share:
            # the data-path communicators: RCCL over xGMI, one rank per GPU; one per pipeline, since
            # config 5's two pipelines step from two host threads and a communicator's collectives
            # must be issued in the same order on every rank
            for _ in wls:
                uid = torch.zeros(128, dtype=torch.uint8)
                if rank == 0:
                    uid.copy_(torch.frombuffer(bytearray(Comm.unique_id()), dtype=torch.uint8))
                dist.broadcast(uid, 0)
                comms.append(Comm(bytes(uid.numpy().tobytes()), world, rank, device))
        else:
            gather = shard.RecordGather(args.batch * len(wls), shard.record_width())
    if world == 1 and args.self_gather:  # the N > 1 data path on one GPU: a one-rank communicator
        comms = [Comm(Comm.unique_id(), 1, 0, device) for _ in wls]
    if world > 1 or comms:
        # global frame ids: rank + world * i, the second workload's after the first's
        for j, w in enumerate(wls):
            w.pipe.enable_records(shard.REC_DETS, rank + j * world * w.batch, world,
                                  comms[j].ptr if comms else 0, world)
    pool = None
    if len(wls) > 1:
        from concurrent.futures import ThreadPoolExecutor
        pool = ThreadPoolExecutor(len(wls))

    primed = prime(wls, args.prime_seconds, pool)
    run_steps(wls, args.warmup, gather, rank, world, pool)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    times = run_steps(wls, args.steps, gather, rank, world, pool)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    counts = np.array([[t["tracked"], t["rois"], t["frames"], t["detections"]] for t in times], np.float64)
    gather_check = None
    if comms:  # the last step's gathered records: every rank's frames, ids as assigned
        g = wls[0].pipe.gathered()
        ids = np.sort(g[:, 0].view(np.uint32))
        gather_check = bool(np.array_equal(ids, np.arange(world * args.batch, dtype=np.uint32)))
    elif gather is not None:  # the shared-GPU dry run: the gloo gather of the last step
        g = gather.result(gather.steps - 1).numpy()
        ids = np.sort(g[:, 0].view(np.uint32))
        gather_check = bool(np.array_equal(ids, np.arange(world * args.batch * len(wls), dtype=np.uint32)))
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)  # gloo control group: host tensors
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        c = torch.from_numpy(counts)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        counts = c.numpy()
    if rank != 0:
        if world > 1:
            torch.cuda.synchronize()
            for c in comms:
                c.close()
            dist.destroy_process_group()
        return

    wl = wls[0]
    tracked, rois, frames, dets = counts[0]
    stage = {k: round(times[0][k] / args.steps, 3)
             for k in ("detect_gpu_ms", "decode_nms_ms", "landmark_gpu_ms", "map_ms")}
    if Workload.device_post:  # device mode: the stages are kernels (names as the reference's timers)
        stage = {"infer_detector_ms": stage["detect_gpu_ms"], "extract_nms_map_seed_ms": stage["decode_nms_ms"],
                 "infer_landmarks_ms": stage["landmark_gpu_ms"], "track_update_ms": stage["map_ms"]}
    frames_per_s_gpu = frames / elapsed / world
    # SURVEY §8d pipeline model: detector + (landmark net per ROI) + both preprocessings
    din, lin = WORKLOADS[wl.kind][2], WORKLOADS[wl.kind][3]
    rois_per_frame = rois / frames
    bytes_frame = (SURVEY_BYTES[wl.det] + 16.0 * din * din
                   + rois_per_frame * (SURVEY_BYTES[wl.lm] + 16.0 * lin * lin))
    flops_frame = SURVEY_FLOPS[wl.det] + rois_per_frame * SURVEY_FLOPS[wl.lm]
    pipe_gbs = frames_per_s_gpu * bytes_frame / 1e9
    out = {
        "metric": {"face": METRIC, "face_next": NEXT_METRIC,
                   "hand": "end-to-end hand landmark ROIs/sec (palm detect + 21-pt hand landmarks, "
                           "4 ROIs/frame)"}[wl.kind],
        "value": round(rois / elapsed, 1) if wl.kind == "hand" else round(tracked / elapsed, 1),
        "unit": "hand ROIs/s" if wl.kind == "hand" else "faces/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: seeded uniform-noise 1920x1080 RGBA8 frames"
                + (" + one 576x576 face patch each (reference test image, upscaled)" if wl.kind != "hand" else "")
                + "; forced seeded ROI when no detection; ONNX weights from the reference",
        "config": {"workload": {"face": "config 3: BlazeFace -> FaceMesh V1 face pipeline",
                                "hand": "config 4: palm lite + hand landmark lite, 4 ROIs/frame",
                                "face_next": NEXT_WORKLOAD}[wl.kind]
                   + (" + config 4 hand pipeline concurrently on its own streams (config 5)" if len(wls) > 1 else ""),
                   "frames_per_gpu_per_step": args.batch, "frame": "1920x1080 RGBA8",
                   "sub_batches": sub_batches(args, wl.kind), "streams": args.streams,
                   "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
                   "parallelism": f"frame-sharded x{world}"
                   + ((", device-written detection records copied to the host and all-gathered over gloo "
                       "each step (shared-GPU dry run: gloo has no device path)" if share
                       else ", one RCCL all-gather per step of the detection records the post-processing "
                       "kernel writes on the device, on the pipeline's gather stream") if world > 1
                      else (", with the N > 1 data path (device records + an RCCL all-gather per step over a "
                            "one-rank communicator)" if comms else ""))},
        "prime": primed,
        "gather_check": gather_check,
        "rccl_ranks": comms[0].size() if comms else None,
        "launcher": ("bench.py --gpus" if os.environ.get("ZARU_BENCH_LAUNCHED") == "1" else "external")
                    if world > 1 else None,
        "frames_per_s": round(frames / elapsed, 1),
        "rois_per_s": round(rois / elapsed, 1),
        "tracked_per_step": round(tracked / args.steps / world, 2),
        "detections_per_step": round(dets / args.steps / world, 2),
        "stage_ms_per_step": stage,
        "stage_timing": ("HIP-event spans of each stage on the sub-batch streams, summed over the "
                         "concurrent sub-batches (detector / decode+NMS+map+ROI seeding / landmark "
                         "network / tracker update)") if Workload.device_post else "host waits and host work",
        "host_wait_ms_per_step": round(times[0]["host_wait_ms"] / args.steps, 3),
        # NMS candidates (confidence >= threshold) whose exact confidence another candidate of the
        # frame shares: nms.rs:66's unstable sort pins their order only up to 20 candidates
        "nms_ties": {"candidates": int(times[0]["nms_candidates"]), "tied": int(times[0]["nms_tied"]),
                     "unpinned_frames": int(times[0]["nms_unpinned_frames"]), "frames": int(frames)},
        "pipeline_roofline": {
            "model": "SURVEY.md §8d: fixed algorithmic bytes per frame (detector + preprocessing + "
                     "landmark net per ROI), fp32 activations at layer boundaries",
            "bytes_per_frame": round(bytes_frame), "flops_per_frame": round(flops_frame),
            "achieved_GBs_per_gpu": round(pipe_gbs, 1), "peak": HBM_PEAK_GBS,
            "frac": round(pipe_gbs / HBM_PEAK_GBS, 4),
            "flop_frac": round(frames_per_s_gpu * flops_frame / 1e12 / FP32_PEAK_TFLOPS, 4)},
    }
    if len(wls) > 1:
        ht, hr = counts[1][0], counts[1][1]
        out["hand_rois_per_s"] = round(hr / elapsed, 1)
        out["hand_tracked_per_s"] = round(ht / elapsed, 1)
    if not args.no_profile and world == 1:
        kernels, _ = wl.profiled(H, max(3, args.steps // 4))
        if traffic:
            for k in kernels:
                sym = k["kernel"].split("/", 1)[-1]
                if sym in traffic:
                    k["traffic_per_launch_symbol_avg"] = round(traffic[sym])
        out["roofline"] = roofline_of(kernels, traffic)
        out["kernels"] = sorted(kernels, key=lambda k: -k["ms"])
    if world == 1 and args.workload == "face" and not args.no_hand:
        out["hand"] = hand_line(H, args, device, side_traffic.get("hand"))
    if world == 1 and args.workload == "face" and not args.no_next:
        out["face_next"] = next_line(H, args, device, side_traffic.get("face_next"))
    if world == 1 and args.workload == "face" and not args.no_tracking:
        out["tracking"] = tracking_line(H, args, device, wl)
        out["face_loop"] = face_loop_line(H, args, device, wl)
        out["hand_tracking"] = hand_tracking_line(H, args, device, wl)
    if world == 1 and args.workload == "face" and not args.no_c5:
        out["config5"] = c5_line(H, args, device, wl)
    if world == 1 and args.workload == "face" and not args.no_jpeg:
        out["jpeg_source"] = jpeg_line(args, device)
    out["cpu_baseline"] = cpu
    print(json.dumps(out))
    if world > 1:
        torch.cuda.synchronize()
        for c in comms:
            c.close()
        dist.destroy_process_group()


NEXT_METRIC = "end-to-end faces/sec (full-range detect + 478-pt FaceMesh V2), 1080p synthetic"
NEXT_WORKLOAD = "SURVEY 8f-1: BlazeFace full range -> FaceMesh V2 face pipeline (config 3 frames)"


def next_line(H, args, device, traffic=None):
    """SURVEY §8f-1 on the same GPU after the face line: BlazeFace full range (192^2, 2304
    anchors) -> FaceMesh V2 (256^2, 478 points) over config 3's frame generator."""
    import torch
    w = Workload(H, "face_next", device, args.next_batch, 0, args.threads, sub_batches(args, "face_next"),
                 args.streams == "multi")
    run_steps([w], 5, None, 0, 1, None)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    t = run_steps([w], args.next_steps, None, 0, 1, None)[0]
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    fps = t["frames"] / elapsed
    bpf = SURVEY_BYTES[w.det] + 16.0 * 192 * 192 + (t["rois"] / t["frames"]) * (
        SURVEY_BYTES[w.lm] + 16.0 * 256 * 256)
    out = {"metric": NEXT_METRIC, "value": round(t["tracked"] / elapsed, 1), "unit": "faces/s",
           "workload": NEXT_WORKLOAD, "frames_per_s": round(fps, 1),
           "tracked_per_step": round(t["tracked"] / args.next_steps, 2),
           "ms_per_step": round(1e3 * elapsed / args.next_steps, 3), "steps": args.next_steps,
           "frames_per_step": args.next_batch,
           "pipeline_roofline": {"model": "plan fused-boundary bytes per image (zr_plan_describe)",
                                 "bytes_per_frame": round(bpf),
                                 "achieved_GBs": round(fps * bpf / 1e9, 1),
                                 "frac": round(fps * bpf / 1e9 / HBM_PEAK_GBS, 4)}}
    if not args.no_profile:
        kernels, _ = w.profiled(H, 5)
        out["roofline"] = roofline_of(kernels, traffic)
        out["kernels"] = sorted(kernels, key=lambda k: -k["ms"])[:8]
    del w
    return out


def tracking_line(H, args, device, wl):
    """the video loop of LandmarkTracker with its state on the device
    (DeviceTracker): every frame of the face workload is one stream, seeded with an RoI on its
    face patch; each step = FaceMesh on the views the previous update wrote + the update kernel,
    no host round trip.  value = tracked faces (active ROIs) per second."""
    import torch
    fs = wl.fs
    rng = np.random.default_rng(77)
    rois = []
    for (y, x) in fs.pos:
        side = float(rng.uniform(380, 440))
        rois.append((x + 288.0 + float(rng.uniform(-8, 8)), y + 288.0 + float(rng.uniform(-8, 8)), side, side, 0.0))
    tr = H.DeviceTracker("facemesh", device, 0.3, 0.5)
    tr.set_rois(rois, [(fs.w, fs.h)] * len(rois))
    for _ in range(3):
        tr.step(wl.flist)
    tr.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.tracking_steps):
        tr.step(wl.flist)
    tr.synchronize()
    elapsed = time.perf_counter() - t0
    active = sum(1 for st in tr.states() if st["active"])
    bpf = SURVEY_BYTES["face_landmark"] + 16.0 * 192 * 192
    fps = active * args.tracking_steps / elapsed
    return {"metric": "tracked faces/sec, LandmarkTracker video loop with device-resident state "
                      "(FaceMesh V1 per frame, no detection)",
            "value": round(fps, 1), "unit": "faces/s", "streams": len(rois), "active_streams": active,
            "steps": args.tracking_steps, "ms_per_step": round(1e3 * elapsed / args.tracking_steps, 3),
            "pipeline_roofline": {"model": "SURVEY.md §8d FaceMesh bytes + 192^2 preprocessing per face",
                                  "bytes_per_face": round(bpf), "achieved_GBs": round(fps * bpf / 1e9, 1),
                                  "frac": round(fps * bpf / 1e9 / HBM_PEAK_GBS, 4)}}


def face_loop_line(H, args, device, wl, streams=256, sets=8):
    """The reference demo's face video loop (examples/facemesh.rs:35-56: BlazeFace short range +
    FaceMesh V2, track and detect only when tracking is lost, re-seed from the most confident
    face) with its state on the device (DeviceFaceLoop).  `streams` camera streams
    over a `sets`-frame synthetic video of 1080p frames, cycled: each stream's face patch drifts
    4/6 px per frame, and on every other stream the face leaves one frame of the cycle (a
    different frame per stream), so the tracker loses it, the detector runs on that frame (no
    face) and the next one (face found: re-seeded), and tracking resumes on the frame after.
    No host decision between frames.  value = tracked faces (FaceMesh results) per second."""
    import torch
    fs = wl.fs
    dev = f"cuda:{device}"
    patch = torch.from_numpy(load_patch()).to(dev)
    base = torch.from_numpy(fs.base).to(dev)
    ph, pw = patch.shape[:2]
    video = torch.empty((sets, streams, fs.h, fs.w, 4), dtype=torch.uint8, device=dev)
    hidden = 0
    for v in range(sets):
        for s in range(streams):
            video[v, s].copy_(base[s % len(fs.base)])
            if s % 2 == 0 and (s // 2) % sets == v:
                hidden += 1
                continue
            y, x = fs.pos[s]
            y, x = min(fs.h - ph, y + 4 * v), min(fs.w - pw, x + 6 * v)
            video[v, s, y:y + ph, x:x + pw] = patch
    torch.cuda.synchronize(device)
    lists = [[(video[v, s].data_ptr(), fs.w, fs.h, fs.w * 4) for s in range(streams)] for v in range(sets)]
    loop = H.DeviceFaceLoop("face", "facemesh_v2", streams, device)
    for k in range(2 * sets):  # first frame: every stream detects (no RoI yet), then the cycle
        loop.step(lists[k % sets])
    loop.synchronize()
    d0, r0 = loop.detections_run(), loop.reacquisitions()
    steps = max(sets, args.tracking_steps // sets * sets)
    t0 = time.perf_counter()
    for k in range(steps):
        loop.step(lists[k % sets])
    loop.synchronize()
    elapsed = time.perf_counter() - t0
    dets, reacq = loop.detections_run() - d0, loop.reacquisitions() - r0
    tracked = streams * steps - dets  # a stream detects exactly when its track() returned None
    del loop, video
    return {"metric": "tracked faces/sec, the face demo's video loop on the device (examples/facemesh.rs:35-56: "
                      "FaceMesh V2 tracking, BlazeFace short range only on lost streams, re-seed from the best face)",
            "value": round(tracked / elapsed, 1), "unit": "faces/s", "streams": streams, "steps": steps,
            "ms_per_step": round(1e3 * elapsed / steps, 3),
            "video": f"{sets}-frame 1080p cycle; {hidden} of {streams * sets} stream-frames without the face",
            "detections_run": int(dets), "reacquisitions": int(reacq),
            "tracked_results": int(tracked)}


def hand_tracking_line(H, args, device, wl, streams=256, slots=4):
    """SURVEY §8f-3 (HandTracker): DeviceHandTracker over `streams` video streams (the face
    workload's 1080p frames), 4 hand slots each, seeded with 4 injected palm detections per
    stream; each step = the hand landmark update + the bookkeeping kernel (filter, new hands,
    swap_remove de-duplication, redetection schedule) + hand landmarks on every slot + BlazePalm
    with device post-processing on every frame, no host round trip.  Loss threshold -1 keeps
    the synthetic hands tracked.  value = tracked hands per second."""
    import torch
    fs = wl.fs
    frames = wl.flist[:streams]
    tr = H.DeviceHandTracker(len(frames), slots, device)
    tr.set_loss_threshold(-1.0)
    for s, (y, x) in enumerate(fs.pos[:len(frames)]):
        tr.inject_detections(s, [H.Detection(0.9, H.Rect.from_center(x + 96.0 + 384.0 * (k % 2), y + 96.0 + 384.0 * (k // 2),
                                                                     60.0, 60.0), 0.0) for k in range(slots)])
    ms = 1000.0 / 30.0
    for k in range(3):
        tr.step(frames, k * ms)
    tr.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.tracking_steps):
        tr.step(frames, (3 + k) * ms)
    tr.synchronize()
    elapsed = time.perf_counter() - t0
    hands = int(sum(tr.hand_counts()))
    return {"metric": "tracked hands/sec, HandTracker video loop with device-resident state (hand landmarks "
                      "per hand + BlazePalm per frame + bookkeeping on the device)",
            "value": round(hands * args.tracking_steps / elapsed, 1), "unit": "hands/s", "streams": len(frames),
            "slots": slots, "hands": hands, "steps": args.tracking_steps,
            "ms_per_step": round(1e3 * elapsed / args.tracking_steps, 3)}


RST_MCUS = 4  # restart interval of the JPEG-source frames (MCUs): 2040 intervals per 1080p 4:2:0 frame


def jpeg_line(args, device, n_distinct=32, n_decodes=2048, threads=16, batch=16):
    """1080p JPEG -> RGBA8 frames in HBM, byte-identical to the reference's
    libjpeg-turbo backend.  `threads` host threads (camera ingest workers) each own a decoder
    and a HIP stream (ctypes releases the GIL) and decode `batch` frames per call
    (zr_jpeg_decode_batch_async: one Huffman launch for the batch).  The frames carry restart
    markers every RST_MCUS MCUs (an encoder option MJPEG cameras use), so the Huffman stage runs
    on the GPU, one lane per interval, and only the unstuffed scan bytes cross PCIe.  Beside
    them: the same frames one per call (zr_jpeg_decode_async), the same frames without restart
    markers (the self-synchronising device Huffman decoder, jpeg_sync.hip, batched the same way),
    and libjpeg-turbo itself (Pillow) on one core, the reference's CPU decode."""
    import io
    import threading
    import torch
    from PIL import Image
    from zaru_amd import jpeg
    from zaru_amd._lib import check, lib
    import ctypes as C
    rng = np.random.default_rng(55)
    fs = FrameSet(rng, n_distinct, patch=load_patch())

    def encode(i, **kw):
        b = io.BytesIO()
        Image.fromarray(fs.frame(i)[..., :3]).save(b, "JPEG", quality=90, **kw)
        return b.getvalue()

    rst = [encode(i, restart_marker_blocks=RST_MCUS) for i in range(n_distinct)]
    plain = [encode(i) for i in range(n_distinct)]
    w, h = jpeg.info(rst[0])
    out = torch.empty((threads, batch, h, w, 4), dtype=torch.uint8, device=f"cuda:{device}")
    decs, streams = [], []
    for t in range(threads):
        decs.append(jpeg.JpegDecoder(device))
        sp = C.c_void_p()
        check(lib().zr_stream_create(C.byref(sp)))
        streams.append(sp.value)

    def work(t, count, datas, nb):
        ptrs = [out[t, j].data_ptr() for j in range(nb)]
        for k in range(0, count, nb):
            frames = [datas[(t * 7 + k + j) % n_distinct] for j in range(nb)]
            if nb == 1:
                decs[t].decode_into(frames[0], ptrs[0], w * 4, streams[t])
            else:
                decs[t].decode_batch_into(frames, ptrs, [w * 4] * nb, streams[t])
        check(lib().zr_stream_synchronize(streams[t]))

    def run(total, datas, nb):
        per = total // threads // nb * nb
        ths = [threading.Thread(target=work, args=(t, per, datas, nb)) for t in range(threads)]
        t0 = time.perf_counter()
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        return per * threads, time.perf_counter() - t0

    run(threads * batch * 2, rst, batch)
    n, el = run(n_decodes, rst, batch)
    # every frame of the last batches equals libjpeg-turbo's decode (spot check of the timed path)
    ok = True
    per = n_decodes // threads // batch * batch
    for t in (0, threads - 1):
        for j in range(batch):
            k = per - batch + j
            want = np.asarray(Image.open(io.BytesIO(rst[(t * 7 + k) % n_distinct])).convert("RGBA"))
            ok &= bool(np.array_equal(out[t, j].cpu().numpy(), want))
    run(threads * 2, rst, 1)
    n1, el1 = run(n_decodes // 2, rst, 1)
    run(threads * batch * 2, plain, batch)
    n_p, el_p = run(n_decodes, plain, batch)
    ok_p = True
    for t in (0, threads - 1):
        for j in range(batch):
            k = per - batch + j
            want = np.asarray(Image.open(io.BytesIO(plain[(t * 7 + k) % n_distinct])).convert("RGBA"))
            ok_p &= bool(np.array_equal(out[t, j].cpu().numpy(), want))
    gpu_dec = sum(d.status()[0] for d in decs)
    host_dec = sum(d.status()[1] for d in decs)
    corrupt = any(d.status()[2] for d in decs)
    t0 = time.perf_counter()
    cpu_n = 0
    while time.perf_counter() - t0 < 3.0:
        Image.open(io.BytesIO(rst[cpu_n % n_distinct])).convert("RGBA").load()
        cpu_n += 1
    cpu_el = time.perf_counter() - t0
    for t in range(threads):
        check(lib().zr_stream_destroy(streams[t]))
        decs[t].close()
    mb = sum(len(d) for d in rst) / len(rst) / 1e6
    return {"metric": "1080p JPEG frames/sec decoded into HBM (RGBA8, byte-identical to libjpeg-turbo)",
            "value": round(n / el, 1), "unit": "frames/s", "host_threads": threads, "decodes": n,
            "frames_per_call": batch,
            "entropy": f"GPU, one lane per restart interval (restart_marker_blocks={RST_MCUS})",
            "gpu_entropy_decodes": gpu_dec, "host_entropy_decodes": host_dec, "corrupt": bool(corrupt),
            "equal_libjpeg_turbo": ok,
            "jpeg_MB_per_frame": round(mb, 3), "quality": 90, "subsampling": "4:2:0",
            "one_frame_per_call": {"value": round(n1 / el1, 1), "unit": "frames/s", "decodes": n1},
            "no_restart_markers": {"value": round(n_p / el_p, 1), "unit": "frames/s", "decodes": n_p,
                                   "frames_per_call": batch, "equal_libjpeg_turbo": ok_p,
                                   "entropy": "GPU, self-synchronising (4096-bit segments, one lane each)",
                                   "jpeg_MB_per_frame": round(sum(len(d) for d in plain) / len(plain) / 1e6, 3),
                                   "note": "same frames without restart markers (host Huffman before round 4: 1.9 k)"},
            "cpu_libjpeg_turbo_1core": {"value": round(cpu_n / cpu_el, 1), "unit": "frames/s",
                                        "note": "Pillow's libjpeg-turbo (the reference's libjpeg-turbo backend), one core"}}


def c5_line(H, args, device, wl):
    """Config 5 on one GPU: the face pipeline (config 3, the main line's own)
    and a hand pipeline (config 4: palm lite + 4 hand ROIs per frame) over the SAME resident
    1080p frames, each stepping from its own host thread on its own HIP streams
    (examples/facemesh.rs:35-56 and examples/hand_tracking.rs:19-62 sharing the GPU).  At N > 1
    the same pair runs per rank with one combined record all-gather (--workload both)."""
    import torch
    from concurrent.futures import ThreadPoolExecutor
    threads = max(2, args.threads // 2)
    face = Workload(H, "face", device, args.batch, 0, threads, sub_batches(args, "face"), args.streams == "multi",
                    shared=wl)
    hand = Workload(H, "hand", device, args.batch, 0, threads, sub_batches(args, "hand"), args.streams == "multi",
                    shared=wl)
    pool = ThreadPoolExecutor(2)
    prime([face, hand], 0.3, pool)
    run_steps([face, hand], 2, None, 0, 1, pool)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tf, th = run_steps([face, hand], args.c5_steps, None, 0, 1, pool)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    pool.shutdown()
    del face, hand
    return {"metric": "config 5 on one GPU: face pipeline + hand pipeline concurrently over the same 1080p frames",
            "faces_per_s": round(tf["tracked"] / el, 1), "hand_rois_per_s": round(th["rois"] / el, 1),
            "frames_per_s": round(tf["frames"] / el, 1), "frames_per_step": args.batch,
            "steps": args.c5_steps, "ms_per_step": round(1e3 * el / args.c5_steps, 3),
            "rois_per_frame": {"face": round(tf["rois"] / max(1, tf["frames"]), 3),
                               "hand": round(th["rois"] / max(1, th["frames"]), 3)},
            "streams": "each pipeline: its own host thread and sub-batch HIP streams",
            "multi_gpu": "bench.py --workload both: per rank, one combined face+palm record all-gather per step"}


def hand_line(H, args, device, traffic=None):
    """Config 4 on the same GPU after the face line: palm lite on every frame + hand landmark
    lite on 4 ROIs per frame (detection-derived when the palm detector fires, else seeded
    rotated ROIs).  The frames hold no hands, so the figure is landmark-ROI throughput."""
    import torch
    w = Workload(H, "hand", device, args.hand_batch, 0, args.threads, sub_batches(args, "hand"),
                 args.streams == "multi")
    run_steps([w], 5, None, 0, 1, None)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    t = run_steps([w], args.hand_steps, None, 0, 1, None)[0]
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    rpf = t["rois"] / max(1, t["frames"])
    bpf = (SURVEY_BYTES[w.det] + 16.0 * 192 * 192 + rpf * (SURVEY_BYTES[w.lm] + 16.0 * 224 * 224))
    gbs = t["frames"] / elapsed * bpf / 1e9
    out = {"value": round(t["rois"] / elapsed, 1), "unit": "hand ROIs/s",
           "pipeline_roofline": {"model": "SURVEY.md §8d bytes per frame: palm + 192^2 preprocessing + "
                                          "hand landmark + 224^2 preprocessing per ROI",
                                 "bytes_per_frame": round(bpf), "achieved_GBs_per_gpu": round(gbs, 1),
                                 "peak": HBM_PEAK_GBS, "frac": round(gbs / HBM_PEAK_GBS, 4)},
           "frames_per_s": round(t["frames"] / elapsed, 1),
           "tracked_per_s": round(t["tracked"] / elapsed, 1),
           "ms_per_step": round(1e3 * elapsed / args.hand_steps, 3), "steps": args.hand_steps,
           "frames_per_step": args.hand_batch}
    if not args.no_profile:
        kernels, _ = w.profiled(H, 5)
        out["roofline"] = roofline_of(kernels, traffic)
        out["kernels"] = sorted(kernels, key=lambda k: -k["ms"])[:8]
    del w
    return out


if __name__ == "__main__":
    main()
