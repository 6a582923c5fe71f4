#!/bin/bash
# The device Huffman probe (tools/debug/jpeg_huff_probe.py) + a kernel trace and one PMC pass.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1 && mkdir -p $O
timeout -k 10 200 python3 tools/debug/jpeg_huff_probe.py > $O/probe.txt 2>&1 && cat $O/probe.txt &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/debug/jpeg_huff_probe.py > /dev/null 2>&1 && echo prof ok &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU --output-format csv -d $O/pmc -o run -- python3 tools/debug/jpeg_huff_probe.py 4 > /dev/null 2>&1 && echo pmc ok
