"""One process per GPU for `bench.py --gpus N` (frames shard across the GPUs of
one node, one rank each, RCCL for the record all-gather).

`bench.py --gpus N` with N > 1 and no `WORLD_SIZE` in its environment is the launcher: before
anything touches the GPU it starts N children of the same command line, each with `RANK`,
`LOCAL_RANK`, `WORLD_SIZE`, `MASTER_ADDR` (127.0.0.1) and a free `MASTER_PORT`, as
`torch.distributed.run` would.  The children are `subprocess` children in process groups of
their own (never an exec from this process).  Rank 0's stdout (the one JSON line) is forwarded;
the other ranks' stdout goes to stderr.  If any rank exits non-zero or the deadline passes, the
other ranks' process groups are terminated and the launcher exits non-zero.  Under an outside
launcher (`torchrun`), `WORLD_SIZE` is already set and must equal `--gpus`.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from typing import Dict, List, Optional, Sequence

RANK_VARS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")


def free_port(host: str = "127.0.0.1") -> int:
    with socket.socket() as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def world_from_env(gpus: int, env=None) -> Optional[int]:
    """The world an already-launched rank belongs to, or None when this process must launch.

    Raises ValueError when an outside launcher's WORLD_SIZE disagrees with --gpus."""
    env = os.environ if env is None else env
    if "WORLD_SIZE" not in env:
        return None if gpus > 1 else 1
    world = int(env["WORLD_SIZE"])
    if world != gpus:
        raise ValueError(f"WORLD_SIZE={world} from the launcher but --gpus {gpus}")
    return world


def rank_plan(n: int, port: int, base_env: Dict[str, str], addr: str = "127.0.0.1") -> List[Dict[str, str]]:
    """The environment of each of the n ranks (one node, rank = local rank = GPU index)."""
    if n < 1:
        raise ValueError("at least one rank")
    plan = []
    for r in range(n):
        env = {k: v for k, v in base_env.items() if k not in RANK_VARS}
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR=addr, MASTER_PORT=str(port), ZARU_BENCH_LAUNCHED="1")
        plan.append(env)
    return plan


def _kill_group(p: subprocess.Popen, sig) -> None:
    try:
        os.killpg(p.pid, sig)  # the child's own process group (start_new_session)
    except (ProcessLookupError, PermissionError):
        pass


def run_ranks(cmd: Sequence[str], n: int, timeout: float, env=None, out=None, err=None,
              poll: float = 0.2) -> int:
    """Start `cmd` as n ranks, forward rank 0's stdout to `out`, and return 0 only if every rank
    exits 0 before `timeout` seconds.  On the first failure (or the deadline) the remaining
    ranks get SIGTERM, then SIGKILL 10 s later; the return code is then the failing rank's code
    (or 124 for the deadline, 128 + s for a rank killed by signal s)."""
    out = out if out is not None else sys.stdout
    err = err if err is not None else sys.stderr
    plan = rank_plan(n, free_port(), dict(os.environ if env is None else env))
    procs = []
    for r, e in enumerate(plan):
        procs.append(subprocess.Popen(list(cmd), env=e, start_new_session=True,
                                      stdout=subprocess.PIPE if r == 0 else err.fileno(),
                                      stderr=err.fileno()))
    # rank 0's stdout drains on a thread so a long line never blocks the child
    import threading
    chunks: List[bytes] = []
    reader = threading.Thread(target=lambda: chunks.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    deadline = time.monotonic() + timeout
    rc = 0
    while True:
        codes = [p.poll() for p in procs]
        failed = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
        if failed:
            r, rc = failed[0]
            print(f"launch: rank {r} exited with {rc}; stopping the other ranks", file=err)
            break
        if all(c == 0 for c in codes):
            break
        if time.monotonic() > deadline:
            rc = 124
            print(f"launch: ranks still running after {timeout:g} s; stopping them", file=err)
            break
        time.sleep(poll)
    if rc != 0:
        for p in procs:
            if p.poll() is None:
                _kill_group(p, signal.SIGTERM)
        t_end = time.monotonic() + 10.0
        for p in procs:
            try:
                p.wait(max(0.1, t_end - time.monotonic()))
            except subprocess.TimeoutExpired:
                _kill_group(p, signal.SIGKILL)
                p.wait()
    reader.join(timeout=10.0)
    text = b"".join(chunks).decode(errors="replace")
    if text:
        out.write(text)
        out.flush()
    return rc if rc >= 0 else 128 - rc  # a signal -s: the shell's 128 + s
