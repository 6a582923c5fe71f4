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
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU --kernel-trace --output-format csv -d $O -o sq -- $B > $O/sq.json 2> $O/sq.err&&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_SMEM --kernel-trace --output-format csv -d $O -o sq2 -- $B > $O/sq2.json 2> $O/sq2.err &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_ADDR_CONFLICT --kernel-trace --output-format csv -d $O -o sq3 -- $B > $O/sq3.json 2> $O/sq3.err
