# round 6: one descriptor upload per network launch (views + frames in one block) -- GPU suite,
# face line, kernel stats
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
bash tools/gpu_run.sh r06u tests && bash tools/gpu_run.sh r06u_q1 quick && bash tools/gpu_run.sh r06u_q2 quick && \
bash tools/gpu_run.sh r06u_p prof
