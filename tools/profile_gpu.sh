#!/bin/bash
# Collect the rocprofv3 evidence for profiles/ (run on the GPU box via gpurun).
#   1) kernel trace + stats of the benchmark command
#   2) separate PMC passes (FETCH_SIZE, WRITE_SIZE) on a shorter run of the same command
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 500 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT -o trace -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench.json
echo "trace done"
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T --output-format csv -d $OUT -o fetch -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $OUT/bench_fetch.json
echo "fetch done"
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T --output-format csv -d $OUT -o write -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $OUT/bench_write.json
echo "write done"
find $OUT -name "*.csv" | head -20
