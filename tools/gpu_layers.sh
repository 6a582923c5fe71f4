#!/bin/bash
# Per-layer kernel times (rocprofv3 kernel trace of tools/kernel_probe.py) of the four hot-path
# networks at their bench batch sizes, once per listed environment setting (a space-separated
# list of VAR=value, e.g. "ZARU_HIP_FORMS=-ws ZARU_HIP_DMA_NBUF=2"; "" = defaults).
# Usage: bash tools/gpu_layers.sh <tag> "<env A>" ["<env B>" ...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; shift
MODELS=${LAYER_MODELS:-hand_landmark_lite:1024 palm_detection_lite:256 face_landmark:341 face_detection_short_range:341}
i=0
for F in "$@"; do
  for MB in $MODELS; do
    M=${MB%%:*}; B=${MB##*:}
    O=gpurun_out/$TAG/$i/${M}_$B; mkdir -p $O
    ( [ -n "$F" ] && export $F; timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o trace -- \
      python3 tools/kernel_probe.py $M $B 5 > /dev/null 2> $O/err.txt ) || { echo "probe $M failed ($F)"; exit 1; }
  done
  echo "$i: '$F' ok"
  i=$((i+1))
done
