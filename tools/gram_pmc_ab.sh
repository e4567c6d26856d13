#!/bin/bash
# Gram-lever A/B with PMC bytes: for each "ENV=v ..." config, the HIP-event time of the symmetric Gram
# tiles (tools/gram_time.py upper) and rocprofv3 --pmc passes (FETCH_SIZE; WRITE_SIZE + L2 hit/miss)
# of the same command, summarised per config for gram_sparse_kernel (bytes per launch).
# usage: tools/gram_pmc_ab.sh <tag> "<config>" "<config>" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
i=0
for cfg in "$@"; do
  ( export $cfg
    cd $R && timeout -k 10 300 python3 tools/gram_time.py 100000 5 upper > $O/time_$i.json 2> $O/time_$i.err ) || { echo "time '$cfg' failed"; tail -5 $O/time_$i.err; exit 1; }
  ( export $cfg PASSES="fetch write"
    $R/tools/pmc_passes.sh $O/pmc_$i $R/tools/gram_time.py 100000 1 upper ) || exit 1
  python3 - "$cfg" $O/time_$i.json $O/pmc_$i <<'PY' >> $O/ab.txt
import json, subprocess, sys
cfg, tj, pdir = sys.argv[1:]
t = json.loads(open(tj).read().strip().splitlines()[-1])
s = json.loads(subprocess.run([sys.executable, "tools/pmc_summary.py", pdir, "gram_sparse_kernel"], capture_output=True,
                              text=True, cwd=__import__("os").environ.get("GRAFT_REPO_ROOT", "/root/repo")).stdout)
(k, m), = s.items()
print(json.dumps({"config": cfg, "upper_ms": round(t["upper_ms"], 3), "t_rec_MB": t["t_rec_MB"],
                  "fetch_GB": round(2 * m["FETCH_SIZE"] * 1024 / 1e9, 2), "write_GB": round(m["WRITE_SIZE"] * 1024 / 1e9, 2),
                  "traffic_GB": round(m["hbm_bytes_per_launch"] / 1e9, 2), "l2_hit": round(m["l2_hit_rate"], 3),
                  "kernel": k}))
PY
  tail -1 $O/ab.txt
  i=$((i+1))
done
