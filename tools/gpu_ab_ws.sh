cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-ws1} && mkdir -p $O &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_forms.py tests/test_gpu_parity.py -x -v -rP --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 ; echo "pytest rc=$?" &&
F="--no-cpu-baseline --no-traffic --no-hand --no-next --no-tracking --no-jpeg --no-c5 --steps 100 --warmup 20" &&
timeout -k 10 200 python3 bench.py $F > $O/bench_ws.json 2> $O/err.txt && echo ws ok &&
ZARU_HIP_FORMS=-ws timeout -k 10 200 python3 bench.py $F > $O/bench_nows.json 2>> $O/err.txt && echo nows ok
