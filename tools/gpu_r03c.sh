cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03c && mkdir -p $O &&
{ nproc; python3 -c "import os; print(len(os.sched_getaffinity(0)), os.cpu_count())"; cat /sys/fs/cgroup/cpu.max; free -g; } > $O/box.txt 2>&1;
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -rP --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 &&
echo "pytest ok" &&
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err &&
echo "bench ok"
