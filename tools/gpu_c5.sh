set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "walk_phi or heavy or sharded or snap or full_pipeline or transpose" > gpurun_out/gpu_c5tests.log 2>&1 && echo TESTS_OK && \
bash tools/trace_c5.sh
