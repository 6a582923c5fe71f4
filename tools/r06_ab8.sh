# round 6: form "pin" (full-width ds_read_b64 / ds_read_b128 row-task window reads in the DMA dwpw)
# and ZARU_HIP_DMA_PAD (LDS channel strides padded by the bank model) against the old reads
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06k && \
timeout -k 10 500 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_forms.py > gpurun_out/r06k/forms.log 2>&1 && \
LAYER_MODELS="face_landmark:256 face_detection_short_range:256 palm_detection_lite:256 palm_detection_lite:85 hand_landmark_lite:341" \
  bash tools/gpu_layers.sh r06k_l "" "ZARU_HIP_DMA_PAD=1" "ZARU_HIP_FORMS=-pin" && \
bash tools/gpu_pmc_models.sh r06k_pmc face_landmark:256 face_detection_short_range:256 && \
ZARU_HIP_DMA_PAD=1 bash tools/gpu_pmc_models.sh r06k_pmcpad face_landmark:256 face_detection_short_range:256 && \
bash tools/gpu_run.sh r06k_a1 quick && ZARU_HIP_FORMS=-pin bash tools/gpu_run.sh r06k_b1 quick && \
ZARU_HIP_DMA_PAD=1 bash tools/gpu_run.sh r06k_c1 quick && \
bash tools/gpu_run.sh r06k_a2 quick && ZARU_HIP_FORMS=-pin bash tools/gpu_run.sh r06k_b2 quick && \
ZARU_HIP_DMA_PAD=1 bash tools/gpu_run.sh r06k_c2 quick && \
bash tools/gpu_run.sh r06k_h1 hand && ZARU_HIP_FORMS=-pin bash tools/gpu_run.sh r06k_h0 hand
