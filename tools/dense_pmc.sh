#!/bin/bash
# PMC of the dense MFMA Gram kernels (tools/dense_ab.py at the given n), one rocprofv3 --pmc run per counter group:
# MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs), HBM bytes = 2 FETCH_SIZE + WRITE_SIZE
# (KiB; tools/pmc_summary.py), L2 hit rate.  Knobs (GRF_DENSE_XCD, GRF_DENSE_PLANES, ...) come from the environment.
# usage: tools/dense_pmc.sh <outdir> <n> [<n> ...]   -> <outdir>/summary.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$1; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {
    local name=$1; shift
    timeout -k 10 300 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- \
        python3 "$R/tools/dense_ab.py" --reps 3 "${NS[@]}" > "$OUT/$name.log" 2>&1 \
        || { echo "pass $name failed"; tail -20 "$OUT/$name.log"; exit 1; }
    echo "pass $name ok"
}
NS=("$@")
run mfma SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES
run fetch FETCH_SIZE
run write WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
python3 "$R/tools/pmc_summary.py" "$OUT" gram_ > "$OUT/summary.json" || exit 1
python3 - "$OUT/summary.json" > "$OUT/summary.txt" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, m in sorted(d.items()):
    busy = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / max(1.0, m.get("GRBM_GUI_ACTIVE", 0.0) / 8 * 1024)
    print(f"{k[:52]:52s} MFMA busy {busy:.3f}  HBM {m.get('hbm_bytes_per_launch', 0) / 1e9:7.3f} GB"
          f"  L2 hit {m.get('l2_hit_rate', 0):.3f}  wait_any/wave_cycles "
          f"{m.get('SQ_WAIT_ANY', 0) / max(1.0, m.get('SQ_WAVE_CYCLES', 1)):.3f}")
PY
cat "$OUT/summary.txt"
