cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06c && \
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_forms.py > gpurun_out/r06c/forms.log 2>&1 && \
LAYER_MODELS="palm_detection_lite:85 palm_detection_lite:256" bash tools/gpu_layers.sh r06c_palm "" "ZARU_HIP_FORMS=-wsp" && \
bash tools/gpu_run.sh r06c_wsp hand && ZARU_HIP_FORMS=-wsp bash tools/gpu_run.sh r06c_nowsp hand && bash tools/gpu_run.sh r06c_wsp2 hand && \
LAYER_MODELS="face_landmark:256 face_detection_short_range:256" bash tools/gpu_layers.sh r06c_face "" "ZARU_HIP_RT_CAP=4" "ZARU_HIP_RT_CAP=2" && \
ZARU_BENCH_HW_QUEUES=4 bash tools/gpu_run.sh r06c_jq4 jpeg && ZARU_BENCH_HW_QUEUES=8 bash tools/gpu_run.sh r06c_jq8 jpeg
