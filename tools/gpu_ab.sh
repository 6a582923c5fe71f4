#!/bin/bash
# Same-box A/B of prebuilt library variants: alt/libzaru_hip_<V>.so is copied over the in-tree
# zaru_amd/lib/libzaru_hip.so before each run.  Usage:
#   bash tools/gpu_ab.sh <tag> <quick|hand|layers> <V> [<V> ...]     (e.g. A B A B)
# quick / hand: the face / config-4 line, value per run appended to gpurun_out/<tag>/summary.txt;
# layers: tools/gpu_layers.sh per variant (LAYER_MODELS as there), into gpurun_out/<tag>_<i>/.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; STEP=$2; shift 2
mkdir -p gpurun_out/$TAG || exit 1
LIB=zaru_amd/lib/libzaru_hip.so
cp $LIB gpurun_out/$TAG/.orig.so || exit 1
i=0
for V in "$@"; do
  cp alt/libzaru_hip_$V.so $LIB || exit 1
  case $STEP in
    quick|hand)
      bash tools/gpu_run.sh $TAG $STEP --no-profile || { cp gpurun_out/$TAG/.orig.so $LIB; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" \
        gpurun_out/$TAG/$STEP.json "$i:$V" >> gpurun_out/$TAG/summary.txt ;;
    layers)
      bash tools/gpu_layers.sh ${TAG}_$i "" || { cp gpurun_out/$TAG/.orig.so $LIB; exit 1; } ;;
  esac
  i=$((i+1))
done
cp gpurun_out/$TAG/.orig.so $LIB && rm gpurun_out/$TAG/.orig.so
