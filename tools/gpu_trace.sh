#!/bin/bash
# kernel trace of the face bench line: bash tools/gpu_trace.sh <tag> "<bench args>"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1 && mkdir -p $O &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-hand --no-next --no-tracking --no-jpeg --no-c5 --no-profile $2 > $O/bench_prof.json 2>> $O/err.txt && echo prof ok
