# round 6: vres5 (32-channel vres dwpw at 5 waves per SIMD), 8-channel chunks for the 48-channel vres
# blocks, ring3 (three LDS-DMA buffers in the palm 12^2 / 6^2 MFMA dwpw), face sub-batch sweep
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06h gpurun_out/r06i && \
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_forms.py > gpurun_out/r06h/forms.log 2>&1 && \
LAYER_MODELS="face_landmark:256 face_detection_short_range:256" bash tools/gpu_layers.sh r06h_face "" "ZARU_HIP_FORMS=-vres5" "ZARU_HIP_VRES48_VF8=1" && \
bash tools/gpu_run.sh r06h_a1 quick && ZARU_HIP_FORMS=-vres5 bash tools/gpu_run.sh r06h_b1 quick && \
bash tools/gpu_run.sh r06h_a2 quick && ZARU_HIP_FORMS=-vres5 bash tools/gpu_run.sh r06h_b2 quick && \
ZARU_HIP_VRES48_VF8=1 bash tools/gpu_run.sh r06h_c1 quick && \
LAYER_MODELS="palm_detection_lite:85 palm_detection_lite:256" bash tools/gpu_layers.sh r06i_palm "" "ZARU_HIP_FORMS=-ring3" && \
bash tools/gpu_run.sh r06i_h1 hand && ZARU_HIP_FORMS=-ring3 bash tools/gpu_run.sh r06i_h0 hand && \
bash tools/gpu_run.sh r06i_h2 hand && ZARU_HIP_FORMS=-ring3 bash tools/gpu_run.sh r06i_h3 hand && \
bash tools/gpu_run.sh r06i_s4 quick && bash tools/gpu_run.sh r06i_s6 quick --sub-batches 6 && \
ZARU_BENCH_HW_QUEUES=12 bash tools/gpu_run.sh r06i_s8 quick --sub-batches 8 && \
ZARU_BENCH_HW_QUEUES=12 bash tools/gpu_run.sh r06i_s6q quick --sub-batches 6
