#!/bin/bash
# two independent single-rank bench processes on the one GPU at the same time
# (no torchrun, no gloo, no gather), with and without the device-record RCCL self-gather, beside
# the shared-GPU N = 2 dry run: if the pair of independent processes loses as much aggregate
# throughput as the dry run, the loss is the two processes time-slicing the card, not the N > 1
# data path.  Usage: bash tools/gpu_two_procs.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r05}; O=gpurun_out/$TAG && mkdir -p $O || exit 1
B="python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-traffic --no-profile --no-hand --no-next --no-tracking --no-jpeg --no-c5"
for g in "" "--self-gather"; do
  tagg=${g:+_gather}
  timeout -k 10 300 $B $g > $O/proc_a$tagg.json 2> $O/proc_a$tagg.err & pa=$!
  timeout -k 10 300 $B $g > $O/proc_b$tagg.json 2> $O/proc_b$tagg.err & pb=$!
  wait $pa; ra=$?; wait $pb; rb=$?
  echo "two procs $g: rc $ra $rb"
  [ $ra -eq 0 ] && [ $rb -eq 0 ] || exit 1
done
