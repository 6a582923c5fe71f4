#!/bin/bash
# One GPU-box session (run through gpurun): the GPU tests, smoke, the default bench line (with
# its PMC traffic passes, CPU baseline and hand line), the config-5 line, and a rocprofv3
# kernel trace + stats of the bench command.  Every step has its own time limit; the chain
# stops at the first failure.  Usage: bash tools/gpu_session.sh <tag> [extra bench args]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r02}; shift
O=gpurun_out/$TAG && mkdir -p $O &&
timeout -k 10 400 python -u -m pytest tests -m gpu -v -rP --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
echo "pytest ok" &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
echo "smoke ok" &&
timeout -k 10 600 python bench.py "$@" > $O/bench.json 2> $O/bench.err &&
echo "bench ok" &&
timeout -k 10 300 python bench.py --workload both --steps 30 --warmup 5 --no-cpu-baseline --no-traffic --no-profile "$@" > $O/bench_both.json 2>> $O/bench.err &&
echo "both ok" &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-hand --no-next --no-tracking --no-jpeg --no-c5 "$@" > $O/bench_prof.json 2>> $O/bench.err &&
echo "rocprof ok"
