#!/bin/bash
# C3 dense leg with the split-K rule (2 slices below 384 tiles) against 4 slices forced, interleaved twice;
# then the dense parity tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/c3split
mkdir -p $O
cd $R
for rep in 1 2; do
for s in 0 4; do
  GRF_DENSE_SPLIT=$s timeout -k 10 200 python bench.py --workload c3 --steps 50 --warmup 5 --no-cpu-baseline > $O/s${s}_$rep.json 2> $O/s${s}_$rep.err || { echo "split $s failed"; tail $O/s${s}_$rep.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], round(d['ms_per_step'],4), 'gram', round(r['kernel_ms'],4), 'frac', round(r['frac'],3))" $O/s${s}_$rep.json "split=$s(0=rule) rep=$rep"
done
done
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "dense or c3 or cora" > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
