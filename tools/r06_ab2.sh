# round 6: bneck forms + face_next A/B, face line after the row-task cap
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06d && \
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_forms.py > gpurun_out/r06d/forms.log 2>&1 && \
LAYER_MODELS="face_landmarks_detector:171" bash tools/gpu_layers.sh r06d_fn "" "ZARU_HIP_FORMS=-bneck" && \
timeout -k 10 300 python bench.py --workload face_next --batch 512 --steps 30 --warmup 5 --no-cpu-baseline --no-traffic > gpurun_out/r06d/fn_bneck.json 2> gpurun_out/r06d/fn_bneck.err && \
ZARU_HIP_FORMS=-bneck timeout -k 10 300 python bench.py --workload face_next --batch 512 --steps 30 --warmup 5 --no-cpu-baseline --no-traffic > gpurun_out/r06d/fn_nobneck.json 2> gpurun_out/r06d/fn_nobneck.err && \
timeout -k 10 300 python bench.py --workload face_next --batch 512 --steps 30 --warmup 5 --no-cpu-baseline --no-traffic --no-profile > gpurun_out/r06d/fn_bneck2.json 2> gpurun_out/r06d/fn_bneck2.err && \
bash tools/gpu_run.sh r06d_q1 quick && bash tools/gpu_run.sh r06d_q2 quick
