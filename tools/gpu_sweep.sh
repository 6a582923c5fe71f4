#!/bin/bash
# GPU tests, then the face bench line under a list of environment settings:
#   bash tools/gpu_sweep.sh <tag> "ENV=a" "ENV=b" ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1 && mkdir -p $O && shift &&
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -rP --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 ; echo "pytest rc=$?"
F="--no-cpu-baseline --no-traffic --no-hand --no-next --no-tracking --no-jpeg --no-c5 --steps 100 --warmup 20"
i=0
for E in "$@"; do
  env $E timeout -k 10 200 python3 bench.py $F > $O/bench_$i.json 2>> $O/err.txt || exit 1
  echo "$i $E ok"; i=$((i+1))
done
