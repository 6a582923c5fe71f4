#!/bin/bash
# Kernel trace + PMC passes of tools/kernel_probe.py for one model (one counter group per pass).
# Usage: bash tools/probe_pmc.sh <tag> <model> [batch]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; M=$2; B=${3:-341}
O=gpurun_out/$TAG && mkdir -p $O &&
P="python3 tools/kernel_probe.py $M $B 5"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o trace -- $P > /dev/null 2> $O/trace.err &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d $O -o sq1 -- $P > /dev/null 2> $O/sq1.err &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d $O -o sq2 -- $P > /dev/null 2> $O/sq2.err &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH --kernel-trace --output-format csv -d $O -o sq3 -- $P > /dev/null 2> $O/sq3.err &&
echo "probe ok"
