# round 6: 8-channel chunks for the 16-output VALU dwpw at >= 96-wide planes (default) vs 4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06zb && \
timeout -k 10 500 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_forms.py > gpurun_out/r06zb/forms.log 2>&1 && \
LAYER_MODELS="face_detection_full_range:171 hand_landmark_lite:341" bash tools/gpu_layers.sh r06zb_l "" "ZARU_HIP_VALU16_VF8=0" && \
NX="--no-cpu-baseline --no-traffic --no-profile --no-hand --no-tracking --no-jpeg --no-c5" && \
bash tools/gpu_run.sh r06zb_a1 bench $NX && ZARU_HIP_VALU16_VF8=0 bash tools/gpu_run.sh r06zb_b1 bench $NX && \
bash tools/gpu_run.sh r06zb_h1 hand && ZARU_HIP_VALU16_VF8=0 bash tools/gpu_run.sh r06zb_h0 hand
