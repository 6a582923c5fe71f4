#!/bin/bash
# GPU tests + smoke on the box; usage: bash tools/gpu_tests.sh <tag> [pytest -k expr]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r03}; K=${2:-}
O=gpurun_out/$TAG && mkdir -p $O &&
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -rP --timeout 120 --timeout-method thread ${K:+-k "$K"} > $O/pytest.log 2>&1 &&
echo "pytest ok" &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
echo "smoke ok"
