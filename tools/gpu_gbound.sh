#!/bin/bash
# exact Phi all-gather bound: the N > 1 parity tests (gloo ranks on one GPU) and the bench's N = 2
# C4 / C5 rehearsal with the exact and the capacity bound
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/gbound
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread \
    -k "exact_gather or sharded" > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
export GRF_DIST_BACKEND=gloo
for gb in exact cap; do
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29551 \
    bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --gather-bound $gb > $O/c4_$gb.json 2> $O/c4_$gb.err \
    || { echo c4 $gb failed; tail $O/c4_$gb.err; exit 1; }
echo c4 $gb ok; cut -c1-200 $O/c4_$gb.json
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29552 \
    bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline --workload c5 > $O/c5.json 2> $O/c5.err \
    || { echo c5 failed; tail $O/c5.err; exit 1; }
echo c5 ok; cut -c1-200 $O/c5.json
