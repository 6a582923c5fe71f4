# round 6: 4-wide row tasks for the 5x5 MTW-1 DMA dwpw layouts (16-byte reads) vs ZARU_HIP_RT_CAP=2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06t && \
timeout -k 10 500 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_forms.py > gpurun_out/r06t/forms.log 2>&1 && \
LAYER_MODELS="hand_landmark_lite:341 palm_detection_lite:85 palm_detection_lite:256" bash tools/gpu_layers.sh r06t_l "" "ZARU_HIP_RT_CAP=2" && \
bash tools/gpu_run.sh r06t_h1 hand && bash tools/gpu_run.sh r06t_h2 hand
