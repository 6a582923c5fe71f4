# round 6: 32-channel chunks for the 32-column stride-1 3x3 DMA dwpw tiles (default) vs ZARU_HIP_DFKC=16
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06s && \
timeout -k 10 500 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_forms.py > gpurun_out/r06s/forms.log 2>&1 && \
LAYER_MODELS="face_detection_full_range:171 face_landmarks_detector:171 hand_landmark_lite:341" bash tools/gpu_layers.sh r06s_l "" "ZARU_HIP_DFKC=16" && \
NX="--no-cpu-baseline --no-traffic --no-profile --no-hand --no-tracking --no-jpeg --no-c5" && \
bash tools/gpu_run.sh r06s_a1 bench $NX && ZARU_HIP_DFKC=16 bash tools/gpu_run.sh r06s_b1 bench $NX && \
bash tools/gpu_run.sh r06s_a2 bench $NX && ZARU_HIP_DFKC=16 bash tools/gpu_run.sh r06s_b2 bench $NX && \
bash tools/gpu_run.sh r06s_a3 bench $NX && ZARU_HIP_DFKC=16 bash tools/gpu_run.sh r06s_b3 bench $NX
