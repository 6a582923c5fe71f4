#!/bin/bash
# GPU tests, then the run-to-run spread of the concurrent bench line per sub-batch count, and
# one single-stream line (per-kernel times).  Usage: bash tools/gpu_var.sh <tag> [counts...]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
O=gpurun_out/${1:-var}; shift; mkdir -p $O
SB=${*:-2 3}
F="bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-profile"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-traffic --streams single > $O/single.json 2>> $O/err.log &&
for i in 1 2 3; do
  for b in $SB; do
    timeout -k 10 200 python $F --sub-batches $b > $O/sb${b}_$i.json 2>> $O/err.log || exit 1
  done
done
