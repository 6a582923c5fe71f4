#!/bin/bash
# A quick GPU check after a kernel change: the parity/forms tests named by a pytest -k
# expression, then the face bench line under a list of bench.py argument sets.
#   bash tools/gpu_check.sh <tag> "<pytest -k expr>" "--sub-batches 3" "ZARU_HIP_DFKC=32 |" ...
# (an item "ENV=a ENV2=b | args" sets environment variables for that bench run)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1 && mkdir -p $O && K=$2 && shift 2
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread ${K:+-k "$K"} > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
F="--no-cpu-baseline --no-traffic --no-hand --no-next --no-tracking --no-jpeg --no-c5 --steps 100 --warmup 20"
i=0
for A in "$@"; do
  E=""; case "$A" in *"|"*) E=${A%%|*}; A=${A#*|};; esac
  env $E timeout -k 10 300 python3 bench.py $F $A > $O/bench_$i.json 2>> $O/err.txt || exit 1
  echo "$i [$E|$A] $(python3 -c "import json,sys; d=json.loads([l for l in open('$O/bench_$i.json') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'])")"; i=$((i+1))
done
