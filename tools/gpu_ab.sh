#!/bin/bash
# GPU tests, then an A/B of the face bench line: bash tools/gpu_ab.sh <tag> "<bench args A>" "<bench args B>"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1 && mkdir -p $O &&
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -rP --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 ; echo "pytest rc=$?" &&
F="--no-cpu-baseline --no-traffic --no-hand --no-next --no-tracking --no-jpeg --no-c5 --steps 100 --warmup 20" &&
timeout -k 10 200 python3 bench.py $F $2 > $O/bench_a.json 2> $O/err.txt && echo a ok &&
timeout -k 10 200 python3 bench.py $F $3 > $O/bench_b.json 2>> $O/err.txt && echo b ok
