#!/bin/bash
# register/shuffle bitonic sort vs the all-LDS sort in walk_phi / phi_fused: parity, then C5 / C4 timing A/B
set -o pipefail
mkdir -p gpurun_out/sort
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    -k "walk_phi or steps_and_phi or degenerate or cora or sharded or snap" > gpurun_out/sort/tests.log 2>&1 || exit 1
: > gpurun_out/sort/ab.log
for v in 0 1 0 1; do
  GRF_PHI_SORT_LDS=$v timeout -k 10 200 python -u tools/walkphi_ab.py c5 count > gpurun_out/sort/c5.json 2>&1 || exit 1
  GRF_PHI_SORT_LDS=$v timeout -k 10 200 python -u tools/walkphi_ab.py c4 count > gpurun_out/sort/c4.json 2>&1 || exit 1
  echo "lds=$v $(tail -n1 gpurun_out/sort/c5.json) $(tail -n1 gpurun_out/sort/c4.json)" >> gpurun_out/sort/ab.log
done
cat gpurun_out/sort/ab.log
