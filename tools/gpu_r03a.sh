cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03a && mkdir -p $O &&
timeout -k 10 120 python -u tools/probe_steps.py 12 30 5 > $O/probe.jsonl 2> $O/probe.err &&
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err &&
timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-traffic --no-hand --no-next --no-tracking --no-jpeg > $O/bench_100.json 2>> $O/bench_driver.err &&
echo done
