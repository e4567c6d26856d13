#!/bin/bash
# round 2: new headline/estimator tests, bench with walk roofline + MFMA leg, FETCH_SIZE calibration, host CPU probe
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02a
mkdir -p $O
{ nproc; python3 -c "import os; print('cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; } > $O/cpu.txt 2>&1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_estimator.py tests/test_gpu_headline.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
timeout -k 10 120 $R/tools/fetch_calib > $R/$O/calib.txt 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $R/$O/calib_fetch -o run --output-format csv -- $R/tools/fetch_calib > $R/$O/calib_fetch.log 2>&1 || { echo "pmc failed"; exit 1; }
echo ok
