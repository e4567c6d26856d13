#!/bin/bash
# PCIe hand-over of the drop-in boundary (H2D of A, D2H of K) beside the device-resident step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/xfer
mkdir -p $O
timeout -k 10 300 python bench.py --transfers --no-cpu-baseline --no-mfma-leg --steps 10 > $O/c4.json 2> $O/c4.err || { tail $O/c4.err; exit 1; }
python -c "import json;d=json.loads(open('$O/c4.json').read().splitlines()[-1]);print(d['ms_per_step'], d['transfers'])"
timeout -k 10 300 python bench.py --workload c5 --transfers --no-cpu-baseline --steps 5 > $O/c5.json 2> $O/c5.err || { tail $O/c5.err; exit 1; }
python -c "import json;d=json.loads(open('$O/c5.json').read().splitlines()[-1]);print(d['ms_per_step'], d['transfers'])"
