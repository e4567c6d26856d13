#!/bin/bash
# Round 4: VALU ceiling (+ its PMC pass), headline / C3 / C2 / C5 bench lines, the walk's SQ pass.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r04_run1
mkdir -p $O
cd $R
timeout -k 10 120 ./tools/valu_ceiling > $O/valu_ceiling.txt 2>&1 || { echo valu failed; tail $O/valu_ceiling.txt; exit 1; }
cat $O/valu_ceiling.txt
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES \
    -d $O/valu_pmc -o run --output-format csv -- $R/tools/valu_ceiling > $O/valu_pmc.log 2>&1) || { echo valu pmc failed; tail $O/valu_pmc.log; exit 1; }
echo valu pmc ok
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
echo bench ok; tail -c 600 $O/bench.json
for w in c3 c2 c5; do
  timeout -k 10 400 python3 -u bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { echo $w failed; tail $O/bench_$w.err; exit 1; }
  echo $w ok; tail -c 300 $O/bench_$w.json
done
PASSES=sq timeout -k 10 500 $R/tools/pmc_passes.sh $O/pmc_c4 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-mfma-leg || exit 1

bash tools/r04_ab11.sh || exit 1
timeout -k 10 400 python3 -u tools/c5_hub_model.py > $O/c5_hub_model.txt 2>&1 || { echo c5 model failed; tail $O/c5_hub_model.txt; exit 1; }
tail -9 $O/c5_hub_model.txt
