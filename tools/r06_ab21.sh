# round 6: padded LDS channel stride of the pin layouts (default) vs ZARU_HIP_DMA_PAD=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06y && \
timeout -k 10 500 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_forms.py > gpurun_out/r06y/forms.log 2>&1 && \
LAYER_MODELS="face_landmark:256 face_detection_short_range:256 face_detection_full_range:171 palm_detection_lite:256" bash tools/gpu_layers.sh r06y_l "" "ZARU_HIP_DMA_PAD=0" && \
bash tools/gpu_pmc_models.sh r06y_pmc face_landmark:256 face_detection_short_range:256 && \
bash tools/gpu_run.sh r06y_a1 quick && ZARU_HIP_DMA_PAD=0 bash tools/gpu_run.sh r06y_b1 quick && \
bash tools/gpu_run.sh r06y_a2 quick && ZARU_HIP_DMA_PAD=0 bash tools/gpu_run.sh r06y_b2 quick && \
bash tools/gpu_run.sh r06y_h1 hand && ZARU_HIP_DMA_PAD=0 bash tools/gpu_run.sh r06y_h0 hand
