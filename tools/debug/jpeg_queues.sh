cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/jq
for q in 4 16; do
GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 -c "
import sys, json; sys.argv=['bench.py']; sys.path.insert(0,'.')
import bench, argparse
r = bench.jpeg_line(argparse.Namespace(), 0)
print('queues $q', r['value'], r['host_entropy']['value'], flush=True)
" > gpurun_out/jq/q$q.txt 2>&1 || exit 1
cat gpurun_out/jq/q$q.txt | grep queues
done
