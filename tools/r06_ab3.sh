# round 6: bneck (128^2 / 64^2 only) + gpf forms, FaceMesh V2 layers, face_next A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06e && \
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_forms.py tests/test_gpu_configs.py tests/test_gpu_parity.py > gpurun_out/r06e/forms.log 2>&1 && \
LAYER_MODELS="face_landmarks_detector:171 face_detection_full_range:171" bash tools/gpu_layers.sh r06e_fn "" "ZARU_HIP_FORMS=-gpf" && \
timeout -k 10 300 python bench.py --workload face_next --batch 512 --steps 30 --warmup 5 --no-cpu-baseline --no-traffic > gpurun_out/r06e/fn.json 2> gpurun_out/r06e/fn.err && \
ZARU_HIP_FORMS=-gpf timeout -k 10 300 python bench.py --workload face_next --batch 512 --steps 30 --warmup 5 --no-cpu-baseline --no-traffic --no-profile > gpurun_out/r06e/fn_nogpf.json 2> gpurun_out/r06e/fn_nogpf.err && \
timeout -k 10 300 python bench.py --workload face_next --batch 512 --steps 30 --warmup 5 --no-cpu-baseline --no-traffic --no-profile > gpurun_out/r06e/fn2.json 2> gpurun_out/r06e/fn2.err
