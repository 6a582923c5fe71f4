"""Frame sharding and the single collective of the multi-GPU path.

The reference has no multi-device code. Frames, and ROI crops within a frame, are
independent: nothing crosses frames except tracker ROIs (crates/zaru/src/landmark.rs:364,
hand/tracking.rs:22). So the path shards by frame. Each rank (one process per GPU) runs the
whole detect→track pipeline on its own frames. Frame i goes to rank i mod G, which is weak
scaling: per-rank work stays fixed as G grows. The only exchange is one all-gather per step of
fixed-size detection records (RCCL over xGMI with the "nccl" backend; gloo in the CPU tests).
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
    """All-gather one [B, W] f32 tensor of records from every rank into [world·B, W] (rank-major).
    Uses all_gather_into_tensor on RCCL; gloo lacks it, so there it gathers a list."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    out = torch.empty((world * local.shape[0], local.shape[1]), dtype=local.dtype, device=local.device)
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, local.contiguous(), group=group)
    else:
        dist.all_gather(list(out.chunk(world)), local.contiguous(), group=group)
    return out
