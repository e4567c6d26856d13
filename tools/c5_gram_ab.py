"""C5 column-block Gram alone (bench.py --workload c5's K assembly: 1M rows x the 8192-column slot block),
under a list of kernel knob settings read per call by the library (GRF_GRAM_PIPE, GRF_GRAM_PIPE_G,
GRF_GRAM_PIPE_ABLATE): HIP-event ms per launch (mean of reps, alternating rounds) and the K block's
fingerprint (tools/gram_hash.py; identical = identical bits; ablations are timing-only).
usage: c5_gram_ab.py [reps] [rounds] [cfg ...]   cfg = comma-separated VAR=value list ("base" = none)"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "efficient-gaussian-process-on-graphs_amd")]
import bench  # noqa: E402
from grf_amd import pipeline as P  # noqa: E402
from grf_amd.engine import DeviceCSR, GRFEngine  # noqa: E402
from grf_amd.graphs import powerlaw_graph  # noqa: E402
from tools.gram_hash import fingerprint  # noqa: E402

KNOBS = ("GRF_GRAM_PIPE", "GRF_GRAM_PIPE_G", "GRF_GRAM_PIPE_ABLATE")


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    cfgs = sys.argv[3:] or ["GRF_GRAM_PIPE=0", "base"]
    eng = GRFEngine("cuda:0")
    n, m, L, p = 1_000_000, 64, 8, 0.1
    f = bench.diffusion_modulator(L, 1.0)
    A = DeviceCSR.from_scipy(powerlaw_graph(n, 10.0, 2.5, seed=0), eng.device)
    pl = P.plan_step(n, m, L, p, f, k_rows=8192)
    fr = P.front(eng, A, pl)
    K = P.alloc_k(eng, pl)
    res = {c: [] for c in cfgs}
    prints = {}
    for _ in range(rounds):
        for c in cfgs:
            for k in KNOBS:
                os.environ.pop(k, None)
            if c != "base":
                for kv in c.split(","):
                    k, v = kv.split("=")
                    os.environ[k] = v
            P.k_assembly(eng, fr, pl, K)  # (warm)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(reps):
                P.k_assembly(eng, fr, pl, K)
            ev[1].record()
            ev[1].synchronize()
            res[c].append(ev[0].elapsed_time(ev[1]) / reps)
            if "ABLATE" not in c and c not in prints:
                prints[c] = fingerprint(P.k_view(K, pl))
    for c in cfgs:
        print(json.dumps({"cfg": c, "ms": [round(x, 4) for x in res[c]], "best_ms": round(min(res[c]), 4),
                          "fingerprint": prints.get(c)}), flush=True)


if __name__ == "__main__":
    main()
