#!/bin/bash
# bench.py's JPEG line at several (threads, frames per call) settings.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/jsweep
for tb in "16 8" "16 16" "8 16" "32 8"; do
set -- $tb
timeout -k 10 200 python3 -c "
import sys, json; sys.argv=['bench.py']; sys.path.insert(0,'.')
import bench, argparse
r = bench.jpeg_line(argparse.Namespace(), 0, threads=$1, batch=$2, n_decodes=4096)
print('threads $1 batch $2', r['value'], r['equal_libjpeg_turbo'], flush=True)
" > gpurun_out/jsweep/t$1_b$2.txt 2>&1 || exit 1
grep threads gpurun_out/jsweep/t$1_b$2.txt
done
