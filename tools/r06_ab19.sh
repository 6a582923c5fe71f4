# round 6: irl LV 4 (double-buffered staging registers) vs LV 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06w && \
timeout -k 10 500 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_forms.py > gpurun_out/r06w/forms.log 2>&1 && \
timeout -k 10 120 python -u tools/debug/irl_trace.py 341 > gpurun_out/r06w/irl_trace.txt 2> gpurun_out/r06w/irl_trace.err && \
LAYER_MODELS="hand_landmark_lite:341" bash tools/gpu_layers.sh r06w_l "" "ZARU_HIP_IRL_LDS=3" && \
bash tools/gpu_run.sh r06w_h4a hand && ZARU_HIP_IRL_LDS=3 bash tools/gpu_run.sh r06w_h3a hand && \
bash tools/gpu_run.sh r06w_h4b hand && ZARU_HIP_IRL_LDS=3 bash tools/gpu_run.sh r06w_h3b hand
