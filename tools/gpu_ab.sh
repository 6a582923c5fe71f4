#!/bin/bash
# GPU parity tests, then an A/B of one env switch on the face and hand workloads
# (single stream, with a rocprofv3 kernel-stats pass per side).
# Usage: bash tools/gpu_ab.sh <tag> <VAR> <value-A> <value-B>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
TAG=$1 VAR=$2 A=$3 B=$4
O=gpurun_out/$TAG && mkdir -p $O &&
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
F="bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-traffic" &&
for V in $A $B; do
  env $VAR=$V timeout -k 10 200 python $F > $O/face_$V.json 2>> $O/err.log &&
  env $VAR=$V timeout -k 10 200 python $F --streams single > $O/face_single_$V.json 2>> $O/err.log &&
  env $VAR=$V timeout -k 10 200 python $F --workload hand --batch 256 > $O/hand_$V.json 2>> $O/err.log || exit 1
done &&
export $VAR=$B &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $F --streams single > $O/prof_face.json 2>> $O/err.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profh -o run -- python3 $F --workload hand --batch 256 --streams single > $O/prof_hand.json 2>> $O/err.log
