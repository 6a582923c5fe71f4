# round 6: irl's LDS layouts (ZARU_HIP_IRL_LDS 0 plain / 1 padded for 8-byte reads / 2 padded +
# 16-byte window reads, the default) and the pin form restricted to 16-byte steps
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06m && \
timeout -k 10 500 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_forms.py > gpurun_out/r06m/forms.log 2>&1 && \
LAYER_MODELS="hand_landmark_lite:341 face_landmark:256" bash tools/gpu_layers.sh r06m_l "" "ZARU_HIP_IRL_LDS=0" "ZARU_HIP_IRL_LDS=1" && \
bash tools/gpu_pmc_models.sh r06m_pmc hand_landmark_lite:341 && \
ZARU_HIP_IRL_LDS=0 bash tools/gpu_pmc_models.sh r06m_pmc0 hand_landmark_lite:341 && \
bash tools/gpu_run.sh r06m_h2a hand && ZARU_HIP_IRL_LDS=0 bash tools/gpu_run.sh r06m_h0a hand && \
ZARU_HIP_IRL_LDS=1 bash tools/gpu_run.sh r06m_h1a hand && \
bash tools/gpu_run.sh r06m_h2b hand && ZARU_HIP_IRL_LDS=0 bash tools/gpu_run.sh r06m_h0b hand && \
bash tools/gpu_run.sh r06m_q quick
