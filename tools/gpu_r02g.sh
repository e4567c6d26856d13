#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02g
timeout -k 10 300 python tools/window_exp.py > gpurun_out/r02g/window.txt 2>&1 || { tail -20 gpurun_out/r02g/window.txt; exit 1; }
cat gpurun_out/r02g/window.txt
