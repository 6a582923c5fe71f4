#!/bin/bash
# GPU tests named by a pytest -k expression, then the hand (config 4) bench line under a list of
# environment settings, then per-layer traces of the hand networks.
#   bash tools/gpu_hand.sh <tag> "<pytest -k expr>" "ENV=a" ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1 && mkdir -p $O && K=$2 && shift 2
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread ${K:+-k "$K"} > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
i=0
for E in "$@"; do
  env $E timeout -k 10 300 python3 bench.py --workload hand --batch 256 --steps 30 --warmup 5 --no-cpu-baseline --no-traffic --no-next --no-tracking --no-jpeg --no-c5 > $O/hand_$i.json 2>> $O/err.txt || exit 1
  echo "$i [$E] $(python3 -c "import json; d=json.loads([l for l in open('$O/hand_$i.json') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'])")"; i=$((i+1))
done
