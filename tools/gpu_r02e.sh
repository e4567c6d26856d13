#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02e
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_api.py tests/test_gpu_features.py tests/test_gpu_cg.py > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "Error|assert" $O/tests.log | head -20; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
