#!/bin/bash
# Hardware-counter passes over a short bench run (one rocprofv3 --pmc pass per counter group,
# never combined with other trace domains).  Usage: bash tools/gpu_pmc.sh <tag> [bench args]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
TAG=${1:-r01}; shift
O=gpurun_out/$TAG/pmc && mkdir -p $O &&
timeout -k 10 60 rocprofv3 -L > $O/avail.txt 2>&1
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile $*"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O -o fetch -- $B > $O/fetch.json 2> $O/fetch.err &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O -o write -- $B > $O/write.json 2> $O/write.err &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU --kernel-trace --output-format csv -d $O -o sq -- $B > $O/sq.json 2> $O/sq.err
