# round 6 evidence on the final build: GPU tests, smoke, the default bench, rocprofv3 kernel stats of
# the face line, the shared-GPU N = 2 run through bench.py's own launcher, per-network PMC passes
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && O=gpurun_out/${1:-r06z} && mkdir -p $O && \
NOSIDE="--no-hand --no-next --no-tracking --no-jpeg --no-c5" && \
timeout -k 10 600 python -u -m pytest tests -m gpu -v -rP --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 700 python bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py \
  --steps 20 --warmup 5 --no-cpu-baseline --no-traffic $NOSIDE > $O/bench_prof.json 2> $O/prof.err && \
ZARU_BENCH_SHARE_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --steps 50 --warmup 10 --no-cpu-baseline \
  --no-traffic --no-profile $NOSIDE > $O/n2.json 2> $O/n2.err && \
ZARU_BENCH_SHARE_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --workload both --steps 10 --warmup 3 \
  --no-cpu-baseline --no-traffic --no-profile > $O/n2_both.json 2> $O/n2_both.err && \
bash tools/gpu_pmc_models.sh ${1:-r06z}_pmc face_detection_short_range:256 face_landmark:256 hand_landmark_lite:341 palm_detection_lite:256
