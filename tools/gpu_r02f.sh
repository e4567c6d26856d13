#!/bin/bash
# symmetric Gram band-width x waves sweep (C4), K digests must agree
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02f
mkdir -p $O
for bw in 4096 3584 4608 5120 6144; do
  for wv in 4 8; do
    GRF_BW=$bw GRF_GRAM_WAVES=$wv timeout -k 10 120 python tools/gram_time.py 100000 4 sym > $O/gt_${bw}_${wv}.json 2>> $O/err.log || { echo "fail $bw $wv"; tail -5 $O/err.log; exit 1; }
    echo "bw=$bw waves=$wv $(cat $O/gt_${bw}_${wv}.json)"
  done
done
