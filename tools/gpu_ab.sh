#!/bin/bash
# Same-box A/B of environment configurations over one python command, each config run twice
# interleaved (A B ... A B ...), one JSON line per run.
# usage: tools/gpu_ab.sh <tag> "<script and args>" "<ENV=v ...>" "<ENV=v ...>" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1; CMD=$2; shift 2
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for rep in 1 2; do
  i=0
  for cfg in "$@"; do
    env $cfg timeout -k 10 300 python3 $CMD > $O/ab_${i}_$rep.json 2> $O/ab_${i}_$rep.err || { echo "cfg '$cfg' failed"; tail -5 $O/ab_${i}_$rep.err; exit 1; }
    echo "[$cfg] $(tail -1 $O/ab_${i}_$rep.json)" | tee -a $O/ab.txt
    i=$((i+1))
  done
done
