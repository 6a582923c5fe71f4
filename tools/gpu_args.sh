#!/bin/bash
# The face bench line under a list of bench.py argument sets (no tests):
#   bash tools/gpu_args.sh <tag> "--sub-batches 1" "--sub-batches 2" ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1 && mkdir -p $O && shift
F="--no-cpu-baseline --no-traffic --no-hand --no-next --no-tracking --no-jpeg --no-c5 --no-profile --steps 100 --warmup 20"
i=0
for A in "$@"; do
  timeout -k 10 200 python3 bench.py $F $A > $O/bench_$i.json 2>> $O/err.txt || exit 1
  echo "$i [$A] $(python3 -c "import json,sys; d=json.loads([l for l in open('$O/bench_$i.json') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'])")"; i=$((i+1))
done
