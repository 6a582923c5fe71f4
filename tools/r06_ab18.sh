# round 6: irl LV 3 (double-buffered window rows, reads kept ahead by sched_barrier) vs LV 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06v && \
timeout -k 10 500 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_forms.py > gpurun_out/r06v/forms.log 2>&1 && \
timeout -k 10 120 python -u tools/debug/irl_trace.py 341 > gpurun_out/r06v/irl_trace.txt 2> gpurun_out/r06v/irl_trace.err && \
LAYER_MODELS="hand_landmark_lite:341" bash tools/gpu_layers.sh r06v_l "" "ZARU_HIP_IRL_LDS=2" && \
bash tools/gpu_run.sh r06v_h3a hand && ZARU_HIP_IRL_LDS=2 bash tools/gpu_run.sh r06v_h2a hand && \
bash tools/gpu_run.sh r06v_h3b hand && ZARU_HIP_IRL_LDS=2 bash tools/gpu_run.sh r06v_h2b hand
