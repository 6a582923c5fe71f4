"""The multi-GPU path on the CPU: frame sharding and the detection-record all-gather with the
gloo backend at world size 2 (the GPU run uses the same code over RCCL)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from zaru_amd import shard


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _frame_detections(H, fid):
    """A deterministic, frame-specific detection list (0 to 9 detections, some beyond rmax)."""
    rng = np.random.default_rng(1000 + fid)
    out = []
    for _ in range(int(rng.integers(0, 10))):
        r = H.Rect.from_center(*[float(v) for v in rng.uniform(10, 500, 4)])
        kps = [tuple(float(v) for v in rng.uniform(0, 640, 2)) for _ in range(7)]
        out.append(H.Detection(float(rng.uniform(0.5, 1)), r, float(rng.uniform(-3, 3)), kps))
    return out


def _worker(rank, world, port, n_frames, q):
    import torch
    import torch.distributed as dist
    import zaru_amd.host as H
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = shard.frames_of_rank(n_frames, rank, world)
        recs = H.pack_detection_records([_frame_detections(H, f) for f in mine], mine, 8)
        got = shard.all_gather_records(torch.from_numpy(recs))
        q.put((rank, got.numpy()))
    finally:
        dist.destroy_process_group()


def test_frames_of_rank_partition():
    for world in (1, 2, 3, 8):
        seen = sorted(f for r in range(world) for f in shard.frames_of_rank(37, r, world))
        assert seen == list(range(37))


def test_pack_unpack_roundtrip():
    import zaru_amd.host as H
    dets = [_frame_detections(H, f) for f in range(6)]
    recs = H.pack_detection_records(dets, [10, 11, 12, 13, 14, 15], 8)
    assert recs.shape == (6, shard.record_width(8)) and recs.dtype == np.float32
    back = shard.unpack_records(recs)
    for f, ds in enumerate(dets):
        got = back[10 + f]
        assert recs[f, 1].view(np.uint32) == len(ds)
        assert len(got) == min(len(ds), 8)
        for g, d in zip(got, ds):
            assert g[0] == np.float32(d.confidence()) and g[1] == np.float32(d.angle())
            assert g[2:6] == tuple(np.float32(v) for v in d.bounding_rect().tuple())
            assert g[6:] == tuple(np.float32(v) for p in d.keypoints() for v in p)


def test_all_gather_world2_gloo():
    world, n_frames = 2, 10
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_frames, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import zaru_amd.host as H
    want = {f: [tuple(float(np.float32(v)) for v in
                      (d.confidence(), d.angle(), *d.bounding_rect().tuple(),
                       *[c for kp in d.keypoints() for c in kp]))
                for d in _frame_detections(H, f)][:8] for f in range(n_frames)}
    for rank in range(world):
        assert np.array_equal(results[rank], results[0])  # every rank holds the same records
        got = shard.unpack_records(results[rank])
        assert sorted(got) == list(range(n_frames))
        for f in range(n_frames):
            assert got[f] == want[f]


def _gather_worker(rank, world, port, steps, q):
    """A stand-in pipeline: step k yields frame records whose ids encode (step, rank); the
    gather of every step must hold every rank's records, while the loop never waits for it."""
    import time

    import torch.distributed as dist
    import zaru_amd.host as H
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        B = 6
        g = shard.RecordGather(B, shard.record_width())
        got = []
        t0 = time.perf_counter()
        for k in range(steps):
            mine = shard.frames_of_rank(B * world, rank, world)
            recs = H.pack_detection_records([_frame_detections(H, f) for f in mine],
                                            [1000 * k + f for f in mine], 8)
            time.sleep(0.01)  # the pipeline step
            g.submit(recs)
            if k >= 1:  # the previous step's gather has had a whole step to finish
                got.append(g.result(k - 1).numpy().copy())
        g.finish()
        got.append(g.result(steps - 1).numpy().copy())
        q.put((rank, got, time.perf_counter() - t0))
    finally:
        dist.destroy_process_group()


def test_record_gather_overlaps_steps_world2_gloo():
    world, steps = 2, 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    for _ in range(world):
        r, got, dt = q.get(timeout=180)
        results[r] = (got, dt)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import zaru_amd.host as H
    for rank in range(world):
        got, dt = results[rank]
        assert len(got) == steps
        for k in range(steps):
            assert np.array_equal(got[k], results[0][0][k])
            recs = shard.unpack_records(got[k])
            assert sorted(recs) == [1000 * k + f for f in range(6 * world)]
            for f in range(6 * world):
                want = [tuple(float(np.float32(v)) for v in
                              (d.confidence(), d.angle(), *d.bounding_rect().tuple(),
                               *[c for kp in d.keypoints() for c in kp]))
                        for d in _frame_detections(H, f)][:8]
                assert recs[1000 * k + f] == want


def _combined_worker(rank, world, port, steps, q):
    """Config 5's gather: each step packs the face pipeline's records and the hand pipeline's
    palm records of the rank's frames into one [2B, W] block (bench.py run_steps: face ids
    rank + world*i, hand ids rank + world*(B + i)) and ships both in the one collective."""
    import torch.distributed as dist
    import zaru_amd.host as H
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        B = 5
        g = shard.RecordGather(2 * B, shard.record_width())
        got = []
        for k in range(steps):
            face_ids = [rank + world * i for i in range(B)]
            hand_ids = [rank + world * (B + i) for i in range(B)]
            face = H.pack_detection_records([_frame_detections(H, 100 * k + f)[:3] for f in face_ids],
                                            face_ids, 8)
            palm = H.pack_detection_records([_frame_detections(H, 5000 + 100 * k + f) for f in hand_ids],
                                            hand_ids, 8)
            g.submit(np.concatenate([face, palm]))
            got.append(None)
        g.finish()
        got = [g.result(k).numpy().copy() for k in range(max(0, steps - 2), steps)]
        q.put((rank, got))
    finally:
        dist.destroy_process_group()


def test_combined_face_palm_gather_world2_gloo():
    world, steps, B = 2, 4, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_combined_worker, args=(r, world, port, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import zaru_amd.host as H

    def tup(d):
        return tuple(float(np.float32(v)) for v in (d.confidence(), d.angle(), *d.bounding_rect().tuple(),
                                                     *[c for kp in d.keypoints() for c in kp]))
    for rank in range(world):
        for j, k in enumerate(range(steps - 2, steps)):
            blk = results[rank][j]
            assert blk.shape == (world * 2 * B, shard.record_width())
            assert np.array_equal(blk, results[0][j])
            recs = shard.unpack_records(blk)
            assert sorted(recs) == list(range(2 * B * world))  # every face and hand frame of every rank
            for fid, dets in recs.items():
                src = (100 * k + fid) if fid < B * world else (5000 + 100 * k + fid)
                want = [tup(d) for d in _frame_detections(H, src)]
                want = want[:3] if fid < B * world else want[:8]
                assert dets == want, (rank, k, fid)
