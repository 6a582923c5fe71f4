cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1 && mkdir -p $O &&
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -rP --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 ; echo "pytest rc=$?" &&
F="--no-cpu-baseline --no-traffic --no-hand --no-next --no-tracking --no-jpeg --no-c5 --steps 100 --warmup 20" &&
timeout -k 10 200 python3 bench.py $F > $O/bench_a.json 2> $O/err.txt && echo a ok &&
timeout -k 10 200 python3 bench.py $F --host-post > $O/bench_b.json 2>> $O/err.txt && echo b ok &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-hand --no-next --no-tracking --no-jpeg --no-c5 --no-profile > $O/bench_prof.json 2>> $O/err.txt && echo prof ok
