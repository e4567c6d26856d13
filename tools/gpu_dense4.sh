#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for sp in 1 2 3 4 6; do GRF_DENSE_SPLIT=$sp timeout -k 10 120 python tools/dense_sweep.py 2708 4096 6000 8192 | sed "s/^/S=$sp /" || exit 1; done
