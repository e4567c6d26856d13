#!/bin/bash
# A sequence of GPU steps on the box, each under its own time limit, stopping at the first failure
# (no retries).  Outputs go to gpurun_out/<tag>/.  One argument per step:
#   tests:<seconds>:<pytest -k expression>        -> <tag>/tests_<i>/gpu_tests.log (tools/gpu_tests.sh)
#   bench:<name>:<seconds>:<bench.py args>        -> <tag>/<name>.json, <name>.err
#   trace:<name>:<seconds>:<bench.py args>        -> rocprofv3 --kernel-trace --stats under <tag>/<name>/
#   pmc:<name>:<passes>:<bench.py args>           -> tools/pmc_passes.sh + tools/pmc_summary.py (passes:
#                                                    space-separated subset of "fetch write sq lds ta")
#   py:<name>:<seconds>:<python script and args>  -> <tag>/<name>.txt
#   dist:<name>:<seconds>:<world>:<bench.py args> -> bench.py under torch.distributed.run (gloo, one GPU)
# usage: tools/gpu_steps.sh <tag> <step> [<step> ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
i=0
for st in "$@"; do
    i=$((i + 1))
    kind=${st%%:*}; rest=${st#*:}
    case $kind in
    tests)
        t=${rest%%:*}; k=${rest#*:}
        bash tools/gpu_tests.sh "$TAG/tests_$i" "$k" "$t" || exit 1 ;;
    bench)
        name=${rest%%:*}; rest=${rest#*:}; t=${rest%%:*}; args=${rest#*:}
        timeout -k 10 "$t" python3 -u bench.py $args > "$O/$name.json" 2> "$O/$name.err" \
            || { echo "bench $name failed"; tail -20 "$O/$name.err"; exit 1; }
        echo "bench $name ok: $(tail -c 600 "$O/$name.json")" ;;
    trace)
        name=${rest%%:*}; rest=${rest#*:}; t=${rest%%:*}; args=${rest#*:}
        (cd /tmp && export TMPDIR=/tmp && timeout -k 10 "$t" rocprofv3 --kernel-trace --stats -d "$O/$name" -o run \
            --output-format csv -- python3 "$R/bench.py" $args > "$O/$name.log" 2>&1) \
            || { echo "trace $name failed"; tail -20 "$O/$name.log"; exit 1; }
        python3 - "$O/$name" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:16]:
    print(f"{float(r['AverageNs'])/1e6:8.4f} ms x{r['Calls']:>4}  {r['Name'][:100]}")
PY
        ;;
    pmc)
        name=${rest%%:*}; rest=${rest#*:}; passes=${rest%%:*}; args=${rest#*:}
        PASSES="$passes" bash tools/pmc_passes.sh "$O/$name" "$R/bench.py" $args || exit 1
        python3 tools/pmc_summary.py "$O/$name" > "$O/$name.json" && echo "pmc $name ok" ;;
    py)
        name=${rest%%:*}; rest=${rest#*:}; t=${rest%%:*}; args=${rest#*:}
        timeout -k 10 "$t" python3 -u $args > "$O/$name.txt" 2>&1 || { echo "py $name failed"; tail -30 "$O/$name.txt"; exit 1; }
        echo "py $name ok"; tail -20 "$O/$name.txt" ;;
    dist)
        name=${rest%%:*}; rest=${rest#*:}; t=${rest%%:*}; rest=${rest#*:}; w=${rest%%:*}; args=${rest#*:}
        GRF_DIST_BACKEND=gloo timeout -k 10 "$t" python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$w" \
            --master-addr 127.0.0.1 --master-port $((29500 + i)) bench.py --gpus "$w" $args \
            > "$O/$name.json" 2> "$O/$name.err" || { echo "dist $name failed"; tail -30 "$O/$name.err"; exit 1; }
        echo "dist $name ok: $(tail -c 600 "$O/$name.json")" ;;
    *)
        echo "unknown step '$st'"; exit 2 ;;
    esac
done
echo "all steps ok"
