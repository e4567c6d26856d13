#!/bin/bash
# Same-box A/B of configurations over one python command, each config run twice interleaved
# (A B ... A B ...), one JSON line per run.  A config is "ENV=v ..." or "ENV=v ... :: --extra --args"
# (either part may be empty; "X=0" is a harmless placeholder).
# usage: tools/gpu_ab.sh <tag> "<script and args>" "<config>" "<config>" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1; CMD=$2; shift 2
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for rep in 1 2; do
  i=0
  for cfg in "$@"; do
    envp="$cfg"; argp=""
    case "$cfg" in *::*) envp="${cfg%%::*}"; argp="${cfg#*::}";; esac
    env $envp timeout -k 10 300 python3 $CMD $argp > $O/ab_${i}_$rep.json 2> $O/ab_${i}_$rep.err || { echo "cfg '$cfg' failed"; tail -5 $O/ab_${i}_$rep.err; exit 1; }
    echo "[$cfg] $(tail -1 $O/ab_${i}_$rep.json | cut -c1-2000)" >> $O/ab.txt
    python3 - "$cfg" $O/ab_${i}_$rep.json <<'PY'
import json, sys
try:
    d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
except Exception:
    print(f"[{sys.argv[1]}] (no JSON)"); sys.exit(0)
keys = ("ms_per_step", "value", "serial_ms_per_step", "upper_ms", "sym_ms", "mirror_ms", "rows_ms")
print(f"[{sys.argv[1]}] " + " ".join(f"{k}={d[k]:.4g}" for k in keys if isinstance(d.get(k), (int, float)))
      + (f" kernel_ms={d['roofline']['kernel_ms']:.4g}" if isinstance(d.get("roofline"), dict) else "")
      + (f" parity={d['parity']['max_ratio']:.3g}" if isinstance(d.get("parity"), dict) else ""))
PY
    i=$((i+1))
  done
done
