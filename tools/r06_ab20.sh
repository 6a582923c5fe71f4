# round 6: FaceMesh's 48^2 -> 24^2 3x3 block on the DMA form with 8-channel chunks (pin) vs register-staged
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06x && \
timeout -k 10 500 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_forms.py > gpurun_out/r06x/forms.log 2>&1 && \
LAYER_MODELS="face_landmark:256 face_detection_full_range:171 face_landmarks_detector:171" bash tools/gpu_layers.sh r06x_l "" "ZARU_HIP_FORMS=-pin" && \
bash tools/gpu_run.sh r06x_q1 quick && bash tools/gpu_run.sh r06x_q2 quick
