# round 6: irl step timeline with the expand / projection and staging / depthwise split
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r06o && \
timeout -k 10 120 python -u tools/debug/irl_trace.py 341 > gpurun_out/r06o/irl_trace.txt 2> gpurun_out/r06o/irl_trace.err
