#!/bin/bash
# Per-workload hardware-counter tables: the four rocprofv3 --pmc passes of
# tools/gpu_pmc.sh over tools/kernel_probe.py of ONE network at a time, so every table holds only
# that network's kernels.  Each pass runs alone under its own hard limit.  Summarise each
# directory with tools/pmc_table.py.
# Usage: bash tools/gpu_pmc_models.sh <tag> model:batch [model:batch ...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; shift
for MB in "$@"; do
  M=${MB%%:*}; B=${MB##*:}
  O=gpurun_out/$TAG/${M}_$B && mkdir -p $O || exit 1
  P="python3 tools/kernel_probe.py $M $B 3"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O -o fetch -- $P > /dev/null 2> $O/fetch.err &&
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O -o write -- $P > /dev/null 2> $O/write.err &&
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d $O -o sq1 -- $P > /dev/null 2> $O/sq1.err &&
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU --kernel-trace --output-format csv -d $O -o sq2 -- $P > /dev/null 2> $O/sq2.err || { echo "pmc $MB failed"; exit 1; }
  echo "$MB ok"
done
