#!/bin/bash
# usage: ab.sh tag "ENV_A" "ENV_B" reps [bench args]
TAG=$1; A=$2; B=$3; N=$4; shift 4
O=gpurun_out/$TAG; mkdir -p $O
for i in $(seq 1 $N); do
  for v in A B; do
    E=$A; [ $v = B ] && E=$B
    env $E timeout -k 10 200 python bench.py --no-traffic --no-cpu-baseline --no-hand --no-profile "$@" > $O/${v}_$i.json 2>> $O/err.txt || exit 1
  done
done
echo ab ok
