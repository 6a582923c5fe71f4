"""`bench.py --gpus N` starts its N ranks itself (zaru_amd/launch.py; SURVEY.md §8e, BASELINE.json
metric "1/2/4/8 GPU"): the rank plan, rank 0's line forwarded, and failures propagated."""
import json
import os
import subprocess
import sys

import pytest

from zaru_amd import launch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys, time
r, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
assert os.environ["LOCAL_RANK"] == str(r) and os.environ["MASTER_ADDR"] == "127.0.0.1"
if os.environ.get("FAIL_RANK") == str(r):
    sys.exit(7)
if os.environ.get("HANG_RANK") == str(r):
    time.sleep(600)
time.sleep(0.3 * r)
print("rank", r, "stdout", flush=True)
if r == 0:
    print(json.dumps({"n_gpus": n, "port": os.environ["MASTER_PORT"]}))
"""


def test_rank_plan():
    base = {"PATH": "/bin", "RANK": "5", "WORLD_SIZE": "9", "GPU_MAX_HW_QUEUES": "8"}
    plan = launch.rank_plan(4, 29123, base)
    assert [e["RANK"] for e in plan] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in plan] == ["0", "1", "2", "3"]
    for e in plan:
        assert e["WORLD_SIZE"] == "4" and e["MASTER_PORT"] == "29123" and e["MASTER_ADDR"] == "127.0.0.1"
        assert e["PATH"] == "/bin" and e["GPU_MAX_HW_QUEUES"] == "8" and e["ZARU_BENCH_LAUNCHED"] == "1"
    with pytest.raises(ValueError):
        launch.rank_plan(0, 1, {})


def test_world_from_env():
    assert launch.world_from_env(1, {}) == 1
    assert launch.world_from_env(8, {}) is None  # launch the 8 ranks here
    assert launch.world_from_env(2, {"WORLD_SIZE": "2"}) == 2  # torchrun started this rank
    with pytest.raises(ValueError):
        launch.world_from_env(8, {"WORLD_SIZE": "2"})


def _run(tmp_path, n, timeout=60, **env):
    out, err = open(tmp_path / "out", "w+"), open(tmp_path / "err", "w+")
    rc = launch.run_ranks([sys.executable, "-c", CHILD], n, timeout, env=dict(os.environ, **env), out=out, err=err)
    out.seek(0)
    err.seek(0)
    return rc, out.read(), err.read()


def test_run_ranks_forwards_rank0(tmp_path):
    rc, out, err = _run(tmp_path, 3)
    assert rc == 0
    line = json.loads(out.strip().splitlines()[-1])
    assert line["n_gpus"] == 3 and int(line["port"]) > 0
    assert "rank 0 stdout" in out and "rank 1 stdout" not in out  # other ranks' stdout -> stderr
    assert "rank 1 stdout" in err and "rank 2 stdout" in err


def test_run_ranks_propagates_failure(tmp_path):
    rc, out, err = _run(tmp_path, 3, FAIL_RANK="1", HANG_RANK="2")
    assert rc == 7 and "rank 1 exited with 7" in err


def test_run_ranks_deadline(tmp_path):
    rc, _, err = _run(tmp_path, 2, timeout=3, HANG_RANK="1")
    assert rc == 124 and "still running" in err


def test_bench_rejects_a_world_that_is_not_gpus():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


def test_bench_launcher_fails_when_its_ranks_fail():
    # no GPU here: both ranks fail at their first device call, and the launcher must say so
    env = {k: v for k, v in os.environ.items() if k not in launch.RANK_VARS}
    env.update(ZARU_BENCH_SHARE_GPU="1")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--warmup", "0", "--no-cpu-baseline", "--rank-timeout", "240"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "launch: rank" in r.stderr, r.stderr[-2000:]
    assert r.stdout.strip() == ""
