# round 6: ring3 (three LDS-DMA buffers in the palm 12^2 / 6^2 MFMA dwpw), face sub-batch sweep
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06i && \
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_forms.py > gpurun_out/r06i/forms.log 2>&1 && \
LAYER_MODELS="palm_detection_lite:85 palm_detection_lite:256" bash tools/gpu_layers.sh r06i_palm "" "ZARU_HIP_FORMS=-ring3" && \
bash tools/gpu_run.sh r06i_h1 hand && ZARU_HIP_FORMS=-ring3 bash tools/gpu_run.sh r06i_h0 hand && \
bash tools/gpu_run.sh r06i_h2 hand && ZARU_HIP_FORMS=-ring3 bash tools/gpu_run.sh r06i_h3 hand && \
bash tools/gpu_run.sh r06i_s4 quick && bash tools/gpu_run.sh r06i_s6 quick --sub-batches 6 && \
ZARU_BENCH_HW_QUEUES=12 bash tools/gpu_run.sh r06i_s8 quick --sub-batches 8 && \
ZARU_BENCH_HW_QUEUES=12 bash tools/gpu_run.sh r06i_s6q quick --sub-batches 6
