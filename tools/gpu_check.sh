#!/bin/bash
# One GPU-box session: GPU tests, the default bench line (with its PMC traffic passes and CPU
# baseline), variants, and a rocprofv3 kernel trace + stats of the bench command.
# Usage: bash tools/gpu_check.sh <tag> [extra bench args]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
TAG=${1:-r01}; shift
O=gpurun_out/$TAG && mkdir -p $O &&
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 600 python bench.py "$@" > $O/bench.json 2> $O/bench.err &&
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-traffic --streams single "$@" > $O/bench_single.json 2>> $O/bench.err &&
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-traffic --no-cross-step "$@" > $O/bench_nocross.json 2>> $O/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-traffic "$@" > $O/bench_prof.json 2>> $O/bench.err &&
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-traffic --workload hand --batch 256 "$@" > $O/bench_hand.json 2>> $O/bench.err
