#!/bin/bash
# Serialized kernel time per step of the default plan vs a ZARU_HIP_FORMS setting (rocprofv3
# kernel-trace stats of a short bench run each).  Usage: bash tools/form_cost.sh <tag> <forms>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; F=$2
O=gpurun_out/$TAG && mkdir -p $O &&
B="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-profile --no-traffic --no-hand --no-next --no-tracking --no-jpeg"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/a -o run -- $B > $O/a.json 2> $O/a.err &&
ZARU_HIP_FORMS="$F" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/b -o run -- $B > $O/b.json 2> $O/b.err &&
echo "form_cost ok"
