#!/bin/bash
# Kernel-trace stats of tools/kernel_probe.py for the listed models under several env settings.
# Usage: bash tools/probe_times.sh <tag> "<env A>" ["<env B>" ...]
# (models: $MODELS, default BlazeFace and FaceMesh; batch $BATCH, default 341)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; shift
i=0
for E in "$@"; do
  for M in ${MODELS:-face_detection_short_range face_landmark}; do
    O=gpurun_out/$TAG/$i/$M; mkdir -p $O
    env $E timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o trace -- python3 tools/kernel_probe.py $M ${BATCH:-341} 5 > /dev/null 2> $O/err.txt || exit 1
  done
  i=$((i+1))
done
echo "probe_times ok"
