#!/bin/bash
# The JPEG-source side line alone (bench.py's jpeg_line) + a rocprofv3 kernel trace of it.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1 && mkdir -p $O
timeout -k 10 300 python3 -c "
import sys, json; sys.argv=['bench.py']; sys.path.insert(0,'.')
import bench, argparse
print(json.dumps(bench.jpeg_line(argparse.Namespace(), 0)))
" > $O/jpeg.json 2> $O/err.txt && tail -1 $O/jpeg.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -c "
import sys, json; sys.argv=['bench.py']; sys.path.insert(0,'.')
import bench, argparse
print(json.dumps(bench.jpeg_line(argparse.Namespace(), 0, n_decodes=256)))
" > $O/jpeg_prof.json 2>> $O/err.txt && echo prof ok
