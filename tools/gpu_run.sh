#!/bin/bash
# One GPU-box session through gpurun: usage  bash tools/gpu_run.sh <tag> <step>[,<step>...] [bench args]
# steps: tests (pytest -m gpu), smoke, bench (default bench line), quick (face line only, no side
# lines), both (config 5), n2 (shared-GPU N = 2 dry run, bench.py's own launcher, gloo gather; n2run:
# the same via torchrun), probe (comm pending-error replay), replay5 (the
# round-5 build's failing sequence, alt/r05), prof
# (rocprofv3 --kernel-trace --stats of the face line).  Each step has its own time limit; the
# chain stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r04}; STEPS=${2:-tests,smoke}; shift 2
O=gpurun_out/$TAG && mkdir -p $O || exit 1
NOSIDE="--no-hand --no-next --no-tracking --no-jpeg --no-c5"
for s in ${STEPS//,/ }; do
  case $s in
    tests) timeout -k 10 500 python -u -m pytest tests -m gpu -v -rP --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 ;;
    smoke) timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 ;;
    bench) timeout -k 10 700 python bench.py "$@" > $O/bench.json 2> $O/bench.err ;;
    quick) timeout -k 10 300 python bench.py --no-cpu-baseline --no-traffic $NOSIDE "$@" > $O/quick.json 2> $O/quick.err ;;
    hand) timeout -k 10 300 python bench.py --workload hand --batch 256 --steps 30 --warmup 5 --no-cpu-baseline --no-traffic "$@" > $O/hand.json 2> $O/hand.err ;;
    both) timeout -k 10 300 python bench.py --workload both --steps 30 --warmup 5 --no-cpu-baseline --no-traffic --no-profile "$@" > $O/both.json 2> $O/both.err ;;
    n1) timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-traffic --no-profile $NOSIDE "$@" > $O/n1.json 2> $O/n1.err ;;
    n1g) timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-traffic --no-profile --self-gather $NOSIDE "$@" > $O/n1g.json 2> $O/n1g.err ;;
    n2) ZARU_BENCH_SHARE_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --steps 50 --warmup 10 --no-cpu-baseline \
          --no-traffic --no-profile $NOSIDE "$@" > $O/n2.json 2> $O/n2.err ;;
    n2run) ZARU_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
          --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 50 --warmup 10 --no-cpu-baseline \
          --no-traffic --no-profile $NOSIDE "$@" > $O/n2run.json 2> $O/n2run.err ;;
    probe) timeout -k 10 300 python -u tools/debug/comm_pending_probe.py --stream real --force-pending --repeat 6 \
          > $O/probe.log 2>&1 ;;
    replay5) for k in 1 2 3; do (cd alt/r05 && timeout -k 10 200 python -u -m pytest -v -p no:cacheprovider \
          --timeout 120 --timeout-method thread test_records_r05.py) >> $O/replay_r05.log 2>&1; echo "replay $k rc=$?" \
          >> $O/replay_r05.log; done; ZARU_PROBE_ROOT=alt/r05 timeout -k 10 300 python -u \
          tools/debug/comm_pending_probe.py --stream null --repeat 12 > $O/replay_r05_probe.log 2>&1 ;;
    n2half) ZARU_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
          --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --batch 512 --steps 50 --warmup 10 \
          --no-cpu-baseline --no-traffic --no-profile $NOSIDE "$@" > $O/n2half.json 2> $O/n2half.err ;;
    jpeg) timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-traffic --no-profile \
          --no-hand --no-next --no-tracking --no-c5 "$@" > $O/jpeg.json 2> $O/jpeg.err ;;
    prof) timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py \
          --steps 20 --warmup 5 --no-cpu-baseline --no-traffic $NOSIDE "$@" > $O/bench_prof.json 2> $O/prof.err ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  rc=$?
  echo "$s rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
