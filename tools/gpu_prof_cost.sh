#!/bin/bash
# Cost of the in-region HIP-event profiling: the bench line with and without it, alternated.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
O=gpurun_out/${1:-pc}; mkdir -p $O
F="bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic"
for i in 1 2; do
  timeout -k 10 200 python $F > $O/prof_$i.json 2>> $O/err.log || exit 1
  timeout -k 10 200 python $F --no-profile > $O/noprof_$i.json 2>> $O/err.log || exit 1
done
