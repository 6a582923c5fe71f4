#!/bin/bash
# Hardware-counter passes over a short bench run: one rocprofv3 --pmc pass per counter group,
# never combined with other trace domains, each under its own hard time limit.  Summarise with
# tools/pmc_table.py (per-kernel traffic, MFMA-busy, wave states, LDS conflicts).  Usage: bash tools/gpu_pmc.sh <tag> [bench args]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r02}; shift
O=gpurun_out/$TAG/pmc && mkdir -p $O &&
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-traffic --no-hand --no-next --no-tracking --no-jpeg $*"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O -o fetch -- $B > $O/fetch.json 2> $O/fetch.err &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O -o write -- $B > $O/write.json 2> $O/write.err &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d $O -o sq1 -- $B > $O/sq1.json 2> $O/sq1.err &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU --kernel-trace --output-format csv -d $O -o sq2 -- $B > $O/sq2.json 2> $O/sq2.err &&
echo "pmc ok"
