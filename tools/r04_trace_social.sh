#!/bin/bash
# Kernel traces of the social-graph benches (Enron, Facebook) on the round-4 tree.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r04_social
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for g in enron facebook; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$g -o run --output-format csv -- \
      python3 $R/bench.py --graph $g --steps 10 --warmup 2 --no-cpu-baseline --no-mfma-leg > $O/$g.log 2>&1 || { echo "$g trace failed"; tail $O/$g.log; exit 1; }
  echo "$g ok"
done
