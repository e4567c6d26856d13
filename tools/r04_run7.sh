#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r04_run7
mkdir -p $O
bash tools/gpu_tests.sh r04_run7_tests "laplacian or snap or golden or degenerate or headline or star or api" 900 || exit 1
for w in "--workload c5" "--graph enron"; do
  tag=$(echo "x$w" | tr -d ' -')
  timeout -k 10 300 python3 -u bench.py $w --no-cpu-baseline > $O/bench_$tag.json 2> $O/bench_$tag.err || { echo "$w bench failed"; exit 1; }
  echo "$w: $(python3 -c "import json,sys; d=json.loads(open('$O/bench_$tag.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('serial_ms_per_step'), d['parity']['ok'])")"
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/c5trace -o run --output-format csv -- python3 $R/bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $R/$O/c5trace.log 2>&1) || { echo c5 trace failed; exit 1; }
echo done
