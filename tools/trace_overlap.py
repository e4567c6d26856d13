"""Per-kernel durations from a rocprofv3 kernel trace, split by whether another kernel ran at the same time
(e.g. the pipelined bench's front beside the Gram) -- the 'alone' column is the kernel's own time.
usage: python tools/trace_overlap.py <run_kernel_trace.csv> [name-substring ...]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
keys = sys.argv[2:]
alone, shared = defaultdict(list), defaultdict(list)
for i, (s, e, name) in enumerate(ev):
    short = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:70]
    if keys and not any(k in name for k in keys):
        continue
    ov = any(s2 < e and e2 > s for j, (s2, e2, _) in enumerate(ev) if j != i and abs(j - i) < 64)
    (shared if ov else alone)[short].append((e - s) / 1e3)
for k in sorted(set(alone) | set(shared), key=lambda k: -sum(alone.get(k, [])) - sum(shared.get(k, []))):
    a, b = alone.get(k, []), shared.get(k, [])
    fa = f"{sum(a) / len(a):9.2f} us alone x{len(a):<4}" if a else " " * 25
    fb = f"{sum(b) / len(b):9.2f} us shared x{len(b):<4}" if b else ""
    print(f"{fa} {fb} {k}")
