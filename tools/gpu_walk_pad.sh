#!/bin/bash
# walk_phi occupancy A/B on one box: extra LDS per source (GRF_PHI_LDS_PAD) at C5 and C4
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "walk_phi or steps_and_phi or sharded or column_block" > gpurun_out/wpad_tests.log 2>&1 || exit 1
: > gpurun_out/wpad.log
for pad in 0 504 0 504 256; do
  GRF_PHI_LDS_PAD=$pad timeout -k 10 200 python -u tools/walkphi_ab.py c5 count > gpurun_out/wpad_c5.json 2>&1 || exit 1
  GRF_PHI_LDS_PAD=$pad timeout -k 10 200 python -u tools/walkphi_ab.py c4 count > gpurun_out/wpad_c4.json 2>&1 || exit 1
  echo "pad=$pad $(tail -n1 gpurun_out/wpad_c5.json) $(tail -n1 gpurun_out/wpad_c4.json)" >> gpurun_out/wpad.log
done
cat gpurun_out/wpad.log
