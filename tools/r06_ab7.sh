# round 6: dwpair (BlazeFace full range's dwpw -> dwpw + residual double blocks in one launch)
# against the two separate dwpw launches: forms test, per-layer times, face_next line
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06j && \
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_forms.py > gpurun_out/r06j/forms.log 2>&1 && \
LAYER_MODELS="face_detection_full_range:171" bash tools/gpu_layers.sh r06j_fr "" "ZARU_HIP_FORMS=-dwpair" && \
NX="--no-cpu-baseline --no-traffic --no-profile --no-hand --no-tracking --no-jpeg --no-c5" && \
bash tools/gpu_run.sh r06j_a1 bench $NX && ZARU_HIP_FORMS=-dwpair bash tools/gpu_run.sh r06j_b1 bench $NX && \
bash tools/gpu_run.sh r06j_a2 bench $NX && ZARU_HIP_FORMS=-dwpair bash tools/gpu_run.sh r06j_b2 bench $NX
