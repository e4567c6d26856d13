#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 120 python tools/dense_sweep.py 2708 4096 10000 16384 || exit 1
GRF_DENSE_TILE=128 timeout -k 10 120 python tools/dense_sweep.py 2708 10000 || exit 1
GRF_DENSE_TILE=64 timeout -k 10 120 python tools/dense_sweep.py 10000 || exit 1
GRF_DENSE_TILE=128 GRF_DENSE_BK=32 timeout -k 10 120 python tools/dense_sweep.py 10000 16384 || exit 1
