#!/bin/bash
# C5 walk_phi decomposition: with / without bucket counting, without the augmented matrix, slots-only walk
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/walkphi_ab.py c5 count,nocount,noaug,walk > gpurun_out/wc5.json 2>&1 && \
GRF_PHI_THREADS=128 timeout -k 10 200 python -u tools/walkphi_ab.py c5 count > gpurun_out/wc5_t128.json 2>&1 && \
timeout -k 10 200 python -u tools/walkphi_ab.py c4 count,nocount,noaug,walk > gpurun_out/wc4.json 2>&1
rc=$?; tail -n1 gpurun_out/wc5.json gpurun_out/wc5_t128.json gpurun_out/wc4.json; exit $rc
