# round 6: the measured layout tuner (ZARU_HIP_TUNE=1) against the heuristic on the face, hand and face_next lines
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
NX="--no-cpu-baseline --no-traffic --no-profile --no-hand --no-tracking --no-jpeg --no-c5" && \
bash tools/gpu_run.sh r06q_a1 bench $NX && ZARU_HIP_TUNE=1 bash tools/gpu_run.sh r06q_t1 bench $NX && \
bash tools/gpu_run.sh r06q_a2 bench $NX && ZARU_HIP_TUNE=1 bash tools/gpu_run.sh r06q_t2 bench $NX && \
bash tools/gpu_run.sh r06q_h1 hand && ZARU_HIP_TUNE=1 bash tools/gpu_run.sh r06q_ht hand
