#!/bin/bash
# walk_phi with the modulator's LDS trimmed to Lf entries: C5 / C4 timing + parity of the walk tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    -k "walk_phi or steps_and_phi" > gpurun_out/wl_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/walkphi_ab.py c5 count,count > gpurun_out/wlc5.json 2>&1 && \
timeout -k 10 200 python -u tools/walkphi_ab.py c4 count,count > gpurun_out/wlc4.json 2>&1
rc=$?; tail -2 gpurun_out/wl_tests.log; tail -n1 gpurun_out/wlc5.json gpurun_out/wlc4.json; exit $rc
