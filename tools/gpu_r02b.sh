#!/bin/bash
# mirror A/B: LDS tile (GRF_MIRROR_REG=0) vs register 4x4 transposes (=1): parity tests, K digest, timings, bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02b
mkdir -p $O
GRF_MIRROR_REG=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_headline.py -k c4 tests/test_gpu_parity.py -k "gram or heavy or degenerate or c4" > $O/tests_reg.log 2>&1 || { echo "tests failed"; tail -30 $O/tests_reg.log; exit 1; }
for r in 0 3 0 3; do
  GRF_MIRROR_REG=$r timeout -k 10 120 python tools/gram_time.py 100000 5 sym,mirror > $O/gt_$r.json 2>> $O/err.log || exit 1
  echo "reg=$r $(cat $O/gt_$r.json)"
done
for r in 0 3 0 3; do
  GRF_MIRROR_REG=$r timeout -k 10 200 python bench.py --no-cpu-baseline --no-mfma-leg --steps 20 > $O/bench_$r.json 2>> $O/err.log || exit 1
  echo "bench reg=$r $(python -c "import json;d=json.loads(open('$O/bench_$r.json').read().splitlines()[-1]);print(round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), round(d['serial_ms_per_step'],2), round(d['roofline_walk']['kernel_ms'],3))")"
done
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
for r in 0 3; do
GRF_MIRROR_REG=$r timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $R/$O/pmc_lds_$r -o run --output-format csv -- python3 $R/tools/gram_time.py 100000 2 mirror > $R/$O/pmc_lds_$r.log 2>&1 || exit 1
done
echo done
