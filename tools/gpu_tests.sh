#!/bin/bash
# GPU test suite (or a -k subset) on the box, one process, hang-bounded.
# usage: tools/gpu_tests.sh <tag> [pytest -k expression] [timeout seconds]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-tests}; K=${2:-}; T=${3:-1100}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
ARGS=(tests -m gpu -x -v --timeout 300 --timeout-method thread)
[ -n "$K" ] && ARGS+=(-k "$K")
timeout -k 10 $T python -u -m pytest "${ARGS[@]}" > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
