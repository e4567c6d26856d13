#!/bin/bash
# multi-GPU path checks on one GPU: sharded gloo parity tests + bench rehearsals (2 and 3 ranks, balanced shards)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02d
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "sharded or column_block" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
export GRF_DIST_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > $O/reh2.json 2> $O/reh2.err || { echo reh2 failed; tail -20 $O/reh2.err; exit 1; }
echo "reh2 $(tail -1 $O/reh2.json | cut -c1-300)"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 3 --steps 3 --warmup 1 --no-cpu-baseline --balance phi > $O/reh3.json 2> $O/reh3.err || { echo reh3 failed; tail -20 $O/reh3.err; exit 1; }
echo "reh3 $(python -c "import json;d=json.loads(open('$O/reh3.json').read().splitlines()[-1]);print(d['config']['shard'], d['config']['balance'], d['ms_per_step'])")"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline --workload c5 --balance phi > $O/reh2c5.json 2> $O/reh2c5.err || { echo reh2c5 failed; tail -20 $O/reh2c5.err; exit 1; }
echo "reh2c5 $(tail -1 $O/reh2c5.json | cut -c1-200)"
