# round 6: irl step timeline (trace build, tools/debug/irl_trace.py) + forms test of the final irl layouts
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06n && \
timeout -k 10 120 python -u tools/debug/irl_trace.py 341 > gpurun_out/r06n/irl_trace.txt 2> gpurun_out/r06n/irl_trace.err && \
ZARU_HIP_IRL_LDS=0 timeout -k 10 120 python -u tools/debug/irl_trace.py 341 > gpurun_out/r06n/irl_trace_plain.txt 2>> gpurun_out/r06n/irl_trace.err && \
timeout -k 10 500 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_forms.py > gpurun_out/r06n/forms.log 2>&1
