#!/bin/bash
# C5 column-block Gram: waves per tile / gathers in flight (GRF_GRAM_WAVES / GRF_GRAM_UNROLL), interleaved twice
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/c5knobs
mkdir -p $O
cd $R
for rep in 1 2; do
for cfg in "0 8" "4 8" "8 4" "4 4"; do
  set -- $cfg
  GRF_GRAM_WAVES=$1 GRF_GRAM_UNROLL=$2 timeout -k 10 200 python bench.py --workload c5 --steps 8 --warmup 2 --no-cpu-baseline \
      > $O/w$1u$2_$rep.json 2> $O/w$1u$2_$rep.err || { echo "$cfg failed"; tail $O/w$1u$2_$rep.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],3), 'gram', round(d['roofline']['kernel_ms'],3))" $O/w$1u$2_$rep.json "waves=$1 unroll=$2 rep=$rep"
done
done
