#!/bin/bash
# full GPU suite + smoke + bench (round 2 checkpoint)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02c
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|error" $O/tests.log | head -20; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench.json').read().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline_walk']['kernel_ms'], d['cpu_baseline']['value'], d['cpu_baseline']['cores'])"
