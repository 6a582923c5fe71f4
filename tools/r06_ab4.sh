# round 6: vres3 (three staging buffers in the vres dwpw), irlpad (hand 14^2 irl depthwise tasks on
# 16 lane slots), VALU 8-channel chunks for 16-out layers -- bitwise forms, layers, line A/Bs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06f && \
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_forms.py > gpurun_out/r06f/forms.log 2>&1 && \
LAYER_MODELS="face_landmark:256 face_detection_short_range:256" bash tools/gpu_layers.sh r06f_face "" "ZARU_HIP_FORMS=-vres3" && \
bash tools/gpu_run.sh r06f_a1 quick && ZARU_HIP_FORMS=-vres3 bash tools/gpu_run.sh r06f_b1 quick && \
bash tools/gpu_run.sh r06f_a2 quick && ZARU_HIP_FORMS=-vres3 bash tools/gpu_run.sh r06f_b2 quick && \
LAYER_MODELS="hand_landmark_lite:341" bash tools/gpu_layers.sh r06g_hand "" "ZARU_HIP_FORMS=-irlpad" && \
LAYER_MODELS="face_detection_full_range:171 face_detection_short_range:256" bash tools/gpu_layers.sh r06g_fr "" "ZARU_HIP_VALU_WIDE=1" && \
bash tools/gpu_run.sh r06g_h1 hand && ZARU_HIP_FORMS=-irlpad bash tools/gpu_run.sh r06g_h0 hand && \
mkdir -p gpurun_out/r06g && ZARU_HIP_VALU_WIDE=1 timeout -k 10 300 python bench.py --workload face_next --batch 512 --steps 30 --warmup 5 --no-cpu-baseline --no-traffic --no-profile > gpurun_out/r06g/fn_wide.json 2> gpurun_out/r06g/fn_wide.err && \
timeout -k 10 300 python bench.py --workload face_next --batch 512 --steps 30 --warmup 5 --no-cpu-baseline --no-traffic --no-profile > gpurun_out/r06g/fn.json 2> gpurun_out/r06g/fn.err
