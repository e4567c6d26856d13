#!/bin/bash
# gram kernel knob sweep (env knobs are read once per process -> one process per setting)
# usage: tools/gram_sweep.sh <tag> <bands,csv> [xcd values] [wave values]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-sweep}
BWS=${2:-1024,2048,4096}
XS=${3:-"0 1"}
WS=${4:-"1 4"}
mkdir -p $O
for x in $XS; do for w in $WS; do
  GRF_GRAM_XCD=$x GRF_GRAM_WAVES=$w timeout -k 10 300 python3 $R/tools/gram_sweep.py 100000 $BWS > $O/x${x}_w${w}.json 2> $O/x${x}_w${w}.err || { echo "x$x w$w failed"; tail $O/x${x}_w${w}.err; exit 1; }
  echo "xcd=$x waves=$w $(cat $O/x${x}_w${w}.json)"
done; done
