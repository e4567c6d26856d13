#!/bin/bash
# C5: serial steps vs the next front issued beside the Gram (--overlap)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02h
mkdir -p $O
for ov in "" "--overlap" "" "--overlap"; do
  timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline --steps 10 $ov > $O/c5.json 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "c5 $ov $(python -c "import json;d=json.loads(open('$O/c5.json').read().splitlines()[-1]);print(round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), round(d['roofline_walk']['kernel_ms'],2), round(d['serial_ms_per_step'],2))")"
done
