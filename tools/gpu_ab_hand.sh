#!/bin/bash
# A/B of depthwise forms on the hand workload (palm 5x5 blocks, hand inverted residuals).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
O=gpurun_out/${1:-ab}; mkdir -p $O
B="python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-traffic --workload hand --batch 256 --streams single"
timeout -k 10 200 $B > $O/hand_default.json 2> $O/err.log &&
ZR_DWPW_IMG=5 timeout -k 10 200 $B > $O/hand_img5.json 2>> $O/err.log &&
ZR_DWPW_IMG=1 timeout -k 10 200 $B > $O/hand_img.json 2>> $O/err.log &&
ZR_DWPW_ROWS=1 timeout -k 10 200 $B > $O/hand_rows.json 2>> $O/err.log
