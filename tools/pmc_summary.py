"""Summarise tools/pmc_passes.sh output: per-kernel mean counters + HBM traffic per launch.

traffic (bytes) = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024: FETCH_SIZE / WRITE_SIZE are in KiB and
on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced read (MI355X_MICROARCH.md, HBM); the same
factor 2 holds for 12-B buffer_load_dwordx3 streams and line-aligned 12-B gathers (tools/fetch_calib.hip,
profiles/r02_fetch_calib.json).
usage: python tools/pmc_summary.py <outdir> [kernel-substring] > summary.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(outdir):
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [values per dispatch]
    for f in glob.glob(os.path.join(outdir, "*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            per[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return per


def main():
    outdir = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    per = load(outdir)
    res = {}
    for k, cs in per.items():
        if pat and pat not in k:
            continue
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            m["hbm_bytes_per_launch"] = 2 * m["FETCH_SIZE"] * 1024 + m["WRITE_SIZE"] * 1024
        if "TCC_HIT_sum" in m:
            m["l2_hit_rate"] = m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
        res[k.replace("(anonymous namespace)::", "").split("(")[0]] = m
    json.dump(res, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main()
