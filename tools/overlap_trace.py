"""From a rocprofv3 kernel trace: per-kernel busy time inside the last step's gram/mirror window
and how much of the mirror time overlaps gram kernels."""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
ks.sort()
gram = [(s, e) for s, e, n in ks if "gram_sparse_kernel" in n]
mir = [(s, e) for s, e, n in ks if "mirror" in n]
# the last step: gram launches after the last non-gram, non-mirror kernel before them
last_other = max(s for s, e, n in ks if "gram" not in n and "mirror" not in n)
g = [(s, e) for s, e in gram if s > last_other]
m = [(s, e) for s, e in mir if s > last_other]
t0 = min(s for s, e in g + m)
t1 = max(e for s, e in g + m)
print(f"window {(t1 - t0) / 1e6:.2f} ms: {len(g)} gram launches busy {sum(e - s for s, e in g) / 1e6:.2f} ms, "
      f"{len(m)} mirror launches busy {sum(e - s for s, e in m) / 1e6:.2f} ms")
ov = 0
for ms, me in m:
    for gs, ge in g:
        ov += max(0, min(me, ge) - max(ms, gs))
print(f"mirror time overlapping gram: {ov / 1e6:.2f} ms")
for s, e in (g + m)[:0]:
    pass
for (gs, ge), (ms, me) in list(zip(g, m))[:6]:
    print(f"  gram {(gs - t0) / 1e6:7.3f}-{(ge - t0) / 1e6:7.3f}  mirror {(ms - t0) / 1e6:7.3f}-{(me - t0) / 1e6:7.3f}")
