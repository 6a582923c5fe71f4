#!/bin/bash
# A/B/... of one env switch over several values (100-step face lines, alternated 2x) plus one
# single-stream line per value (per-kernel times).  Usage: bash tools/gpu_abn.sh <tag> <VAR> <values...>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
TAG=$1 VAR=$2; shift 2
O=gpurun_out/$TAG && mkdir -p $O &&
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
F="bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-traffic" &&
for i in 1 2; do
  for V in "$@"; do
    env $VAR=$V timeout -k 10 200 python $F > $O/face_${V}_$i.json 2>> $O/err.log || exit 1
  done
done &&
for V in "$@"; do
  env $VAR=$V timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-traffic --streams single > $O/single_$V.json 2>> $O/err.log || exit 1
done
