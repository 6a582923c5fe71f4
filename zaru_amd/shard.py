"""Frame sharding and the single collective of the multi-GPU path.

The reference has no multi-device code. Frames, and ROI crops within a frame, are
independent: nothing crosses frames except tracker ROIs (crates/zaru/src/landmark.rs:364,
hand/tracking.rs:22). So the path shards by frame. Each rank (one process per GPU) runs the
whole detect→track pipeline on its own frames. Frame i goes to rank i mod G, which is weak
scaling: per-rank work stays fixed as G grows. The only exchange is one all-gather per step of
fixed-size detection records. On GPUs it runs natively: the post-processing kernel writes the
records on the device and the pipeline all-gathers them over RCCL itself
(``DetectTrackPipeline.enable_records`` → ``zr_comm_all_gather_async``); nothing in this module
is on that path. What lives here is the host side of the same exchange over a gloo group: the
record layout, the frame → rank map, and the gather the CPU tests and the shared-GPU dry run use.
Landmarks stay rank-local.

Record layout (``zaru_amd.host.pack_detection_records``, width 2 + 20·rmax f32):
``[frame id (u32 bits), count (u32 bits), rmax × {conf, angle, cx, cy, w, h, 7 × (kx, ky)}]``.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np

REC_DETS = 8
DET_FIELDS = 20


def record_width(rmax: int = REC_DETS) -> int:
    return 2 + DET_FIELDS * rmax


def frames_of_rank(n_frames: int, rank: int, world: int) -> List[int]:
    """Round-robin frame → rank assignment (frame i on rank i mod world)."""
    return list(range(rank, n_frames, world))


def unpack_records(recs: np.ndarray, rmax: int = REC_DETS) -> Dict[int, List[Tuple[float, ...]]]:
    """frame id -> list of (conf, angle, cx, cy, w, h, *keypoints) tuples (first rmax kept)."""
    recs = np.ascontiguousarray(recs, dtype=np.float32)
    ids = recs[:, 0].view(np.uint32)
    counts = recs[:, 1].view(np.uint32)
    out: Dict[int, List[Tuple[float, ...]]] = {}
    for row, fid, cnt in zip(recs, ids, counts):
        dets = []
        for k in range(min(int(cnt), rmax)):
            e = row[2 + DET_FIELDS * k: 2 + DET_FIELDS * (k + 1)]
            dets.append(tuple(float(v) for v in e))
        out[int(fid)] = dets
    return out


def all_gather_records(local, group=None):
    """All-gather one [B, W] f32 CPU tensor of records from every rank of a gloo group into
    [world·B, W] (rank-major)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    out = torch.empty((world * local.shape[0], local.shape[1]), dtype=local.dtype)
    dist.all_gather(list(out.chunk(world)), local.contiguous(), group=group)
    return out


class RecordGather:
    """The per-step all-gather of host records over a gloo group, overlapped with the next steps
    (the shared-GPU dry run of bench.py and the CPU tests; GPU ranks gather on the device).

    ``submit(recs)`` takes one step's records ([B, W] f32), copies them into a slot and starts the
    all-gather asynchronously (``async_op=True``: gloo runs it on its own thread), then returns at
    once, so the pipeline's next step starts while the collective is in flight.  Two slots
    alternate; a slot is reused only after its previous gather completed.  ``finish()`` waits for
    the collectives still in flight; ``result(step)`` is the [world * B, W] gathered tensor of a
    finished step (rank-major, frames of rank r first).  One collective per step and no other:
    SURVEY.md §8e.
    """

    def __init__(self, rows: int, width: int, group=None):
        import torch
        import torch.distributed as dist
        if dist.get_backend(group) != "gloo":
            raise ValueError("RecordGather is the gloo (host) gather; GPU ranks use enable_records")
        self.group = group
        self.world = dist.get_world_size(group)
        self.inp = [torch.empty((rows, width), dtype=torch.float32) for _ in range(2)]
        self.out = [torch.empty((self.world * rows, width), dtype=torch.float32) for _ in range(2)]
        self.work = [None, None]
        self.step_of = [-1, -1]
        self.steps = 0

    def _wait(self, k):
        if self.work[k] is not None:
            self.work[k].wait()
            self.work[k] = None

    def submit(self, recs: np.ndarray) -> None:
        import torch.distributed as dist
        k = self.steps & 1
        self._wait(k)
        self.inp[k].numpy()[...] = recs
        self.work[k] = dist.all_gather(list(self.out[k].chunk(self.world)), self.inp[k],
                                       group=self.group, async_op=True)
        self.step_of[k] = self.steps
        self.steps += 1

    def finish(self) -> None:
        for k in range(2):
            self._wait(k)

    def result(self, step: int):
        for k in range(2):
            if self.step_of[k] == step:
                self._wait(k)
                return self.out[k]
        raise KeyError(f"step {step} is no longer held (only the last two are)")
