#!/bin/bash
# diagnostics: HIP last-error semantics, one pytest selection with HIP error logging, then an
# A/B of the face bench line on the same box: bash tools/gpu_diag.sh <tag> "<-k expr>" "<bench A>" "<bench B>"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1 && mkdir -p $O &&
timeout -k 10 60 ./tools/hip_lasterr.bin > $O/lasterr.txt 2>&1 ; echo "lasterr rc=$?"
AMD_LOG_LEVEL=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -rP --timeout 120 --timeout-method thread -k "$2" > $O/pytest.log 2>&1 ; echo "pytest rc=$?"
F="--no-cpu-baseline --no-traffic --no-hand --no-next --no-tracking --no-jpeg --no-c5 --steps 100 --warmup 20"
timeout -k 10 200 python3 bench.py $F $3 > $O/bench_a.json 2> $O/err.txt && echo a ok &&
timeout -k 10 200 python3 bench.py $F $4 > $O/bench_b.json 2>> $O/err.txt && echo b ok
