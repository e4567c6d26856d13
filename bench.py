"""Headline benchmark: GRF kernel matrices / s on a 100k-node, 1M-edge graph, m = 128.

One step = one full pass of the hot path with the adjacency CSR already resident
in HBM: normalised Laplacian -> 12.8M Philox random walks (L = 8, p_halt = 0.1)
-> Phi = sum_l f_l M_l (diffusion modulator, beta = 1) -> K = Phi Phi^T as a
dense float32 N x N matrix in HBM (40 GB at N = 100k).  With --gpus N (launched
by torch.distributed.run) every rank walks its source range, the Phi rows are
all-gathered over RCCL and each rank writes its row block of K (strong scaling:
one K per step for the whole job).  On one GPU the steps are pipelined over two HIP
streams: step s+1's front (Laplacian, walks, Phi, transpose) starts when step s's Gram
tiles finish and runs beside step s's HBM-bound mirror pass; every step still runs its
whole path, and `serial_ms_per_step` reports the un-pipelined latency beside `value`.

Prints ONE JSON line on rank 0 (contract in the task description) with a
`roofline` object for the dominant kernel (gram_sparse) and a `cpu_baseline`
object (the C oracle -- a restatement of the reference's CPU algorithm -- on the
host cores, bounded sample, extrapolated; rank 0 at N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "efficient-gaussian-process-on-graphs_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

from grf_amd.graphs import er_graph_exact_edges, powerlaw_graph, snap_graph  # noqa: E402,F401

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# rocprofv3 PMC summary of this workload (tools/gpu_profile.sh -> tools/pmc_summary.py), committed
PMC_SUMMARY = os.path.join(ROOT, "profiles", "r06_pmc_summary.json")
# ... and of the C5 workload (bench.py --workload c5; tools/gpu_steps.sh pmc step)
PMC_SUMMARY_C5 = os.path.join(ROOT, "profiles", "r06_c5_pmc_summary.json")
DEFAULT_WORKLOAD = (100_000, 1_000_000, 128, 8, 0.1)


def pmc_traffic(kernels, path=PMC_SUMMARY):
    """HBM bytes per launch of the named kernels from the committed PMC summary
    (2 * FETCH_SIZE + WRITE_SIZE KiB, the gfx950 FETCH_SIZE correction of MI355X_MICROARCH.md)."""
    import json as _json
    try:
        d = _json.load(open(path))
    except (OSError, ValueError):
        return None
    total = 0.0
    for k in kernels:
        hits = [v for name, v in d.items() if name.split("<")[0].replace("void ", "") == k]
        if not hits or "hbm_bytes_per_launch" not in hits[0]:
            return None
        total += hits[0]["hbm_bytes_per_launch"]
    return total


def pmc_counter(kernel, counter, path=PMC_SUMMARY):
    """One counter's per-launch value of the named kernel from the committed PMC summary (None if absent)."""
    import json as _json
    try:
        d = _json.load(open(path))
    except (OSError, ValueError):
        return None
    hits = [v for name, v in d.items() if name.split("<")[0].replace("void ", "") == kernel]
    return hits[0].get(counter) if hits else None


# VALU issue ceiling per SIMD: one wave64 (non-packed) VALU instruction per 4 cycles, measured on this part
# (tools/valu_ceiling.hip, profiles/r04_valu_ceiling.txt: independent v_fma_f32 / v_xad_u32 / v_mul_hi_u32 /
# v_fma_f64 chains at 4 waves per SIMD issue every 3.8-4.2 shader cycles by s_memtime, and the PMC formula
# this line uses, SQ_INSTS_VALU / (GRBM_GUI_ACTIVE / 8 x 1024), reads 0.23-0.26 on them)
VALU_PEAK_PER_SIMD_CYCLE = 0.25
N_SIMDS = 256 * 4


def auto_hubs(eng, A_dev, m, p, L, f, share: float = 0.13):
    """(hub columns worth a dense panel, skewed) from one setup walk (untimed): a column in c of the n rows
    saves ~c^2 / 2 gathered records and costs n^2 / 2 MFMA multiply-adds, ~60x cheaper each, so it pays from
    c / n ~ 1 / sqrt(60) = 0.13 (measured: Enron's best split is 128 columns, whose c reaches 13 % of n;
    Facebook's 64th column is in 9 % of the rows and the split loses there, profiles/r02_hubs_sweep.txt);
    with the split (bf16) panel the count is then taken at engine.HUB_EXTEND_SHARE (Enron 192 columns).
    Multiples of 32 (the panel's width).  skewed: the Gram's waves take pair-balanced shares
    (engine.row_cuts)."""
    from grf_amd.dist import setup_phi
    return eng.column_stats(setup_phi(eng, A_dev, m, p, L, f, seed=42), share, extend=eng.hub_extend_share())


def _device_tensors(obj, depth: int = 3):
    """The CUDA tensors held by a front (its attributes, theirs, ... to ``depth`` levels; the engine skipped)."""
    import torch

    from grf_amd.engine import GRFEngine
    if torch.is_tensor(obj):
        return [obj] if obj.is_cuda else []
    if depth == 0 or obj is None or isinstance(obj, (GRFEngine, int, float, str, bool)):
        return []
    out = []
    for v in (vars(obj).values() if hasattr(obj, "__dict__") else []):
        out += _device_tensors(v, depth - 1)
    return out


def init_distributed(local_rank: int) -> int:
    """One process per GPU over RCCL (backend "nccl").  GRF_DIST_BACKEND=gloo rehearses the same
    multi-process path with several ranks on one GPU (device tensors staged through host memory
    in grf_amd.dist); the returned device index is local_rank modulo the visible GPUs."""
    import torch
    import torch.distributed as dist

    backend = os.environ.get("GRF_DIST_BACKEND", "nccl")
    dev = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    else:
        dist.init_process_group(backend)
    return dev


def make_graph(args):
    """The adjacency of the configured workload (scipy CSR, unit weights)."""
    if args.graph == "er":
        return er_graph_exact_edges(args.n, args.edges, seed=0)
    if args.graph == "powerlaw":
        return powerlaw_graph(args.n, args.avg_degree, 2.5, seed=0)
    return snap_graph(args.graph)


def workload_name(args, A):
    n, nnz = A.shape[0], A.nnz
    if args.graph == "er":
        return {"short": f"N={n // 1000}k ER graph" if n % 1000 == 0 else f"N={n} ER graph",
                "long": (f"{'C4: ' if (n, args.edges) == DEFAULT_WORKLOAD[:2] else 'C2: ' if (n, args.edges) == C2_DENSE else ''}"
                         f"ER N={n}, {args.edges} undirected edges"
                         + (" (CSR sparse path)" if (n, args.edges) == C2_DENSE else "")),
                "data": "synthetic Erdos-Renyi graph (seed 0), unit weights"}
    if args.graph == "powerlaw":
        return {"short": f"N={n // 1000}k power-law graph",
                "long": f"C5: Chung-Lu power-law N={n}, exponent 2.5, mean degree {nnz / n:.2f} "
                        f"(max {int(np.diff(A.indptr).max())})",
                "data": "synthetic Chung-Lu power-law graph (seed 0), unit weights"}
    return {"short": f"{args.graph} N={n}",
            "long": f"SNAP {args.graph} social graph shipped with the reference, N={n}, {nnz} adjacency entries",
            "data": f"real graph: the reference's {args.graph} edge list (tests/golden/snap.npz)"}


def diffusion_modulator(L: int, beta: float = 1.0) -> np.ndarray:
    import math
    return np.array([(-beta) ** l / (2 ** l * math.factorial(l)) for l in range(L)])


def cpu_baseline(A, f, m, p, L, budget_rows: int, n_threads: int, k_rows: int = 0):
    """Reference algorithm on the host (C oracle, PCG64 reference stream), bounded sample.
    k_rows: the unit is K rows (Phi of all nodes + k_rows rows of K per step) instead of whole K's."""
    from oracle import oracle as O

    n = A.shape[0]
    t0 = time.perf_counter()
    Ls, _ = O.laplacian_sparse(A)
    t1 = time.perf_counter()
    ip, ix, dx = O._csr_arrays(Ls)
    node, load = O.walk_slots(ip, ix, dx, m, p, L, rng=O.RNG_PCG64, n_chunks=n_threads, seed=42,
                              n_threads=n_threads)
    t2 = time.perf_counter()
    mats = O.reduce_steps(node, load, O.NORM_MUL_RECIP, n_threads=n_threads)
    del node, load
    phi = O.phi_sparse(mats, f, n_threads=n_threads)
    del mats
    t3 = time.perf_counter()
    rows = min(budget_rows, n)
    O.gram_rows(phi, 0, rows, n_threads=n_threads)
    t4 = time.perf_counter()
    target = min(k_rows, n) if k_rows else n
    t_full = (t1 - t0) + (t2 - t1) + (t3 - t2) + (t4 - t3) * target / rows
    return {
        "value": (target if k_rows else 1.0) / t_full,
        "unit": "K-rows/s" if k_rows else "K-matrices/s",
        "cores": n_threads,
        "kind": "port",
        "sample": (f"C oracle (reference algorithm: PCG64 stream, {n_threads} chunks) on {n_threads} host threads: "
                   f"full Laplacian+walks+step reduction+Phi ({t3 - t0:.2f} s) + K rows 0..{rows} "
                   f"({t4 - t3:.2f} s) extrapolated x{target / rows:.2f} to {target} rows; fp64"),
        "stages_s": {"laplacian": t1 - t0, "walks": t2 - t1, "phi": t3 - t2,
                     "gram_extrapolated": (t4 - t3) * target / rows},
    }


def cpu_baseline_predict(phi_csr, tr, te, y, noise, S, iters):
    """SparseGraphGP.predict restated on the host (oracle/cg.py, scipy sparse, fp64, 1 thread):
    setup + 1 and + 2 CG iterations timed, extrapolated to the GPU's iteration count."""
    from oracle import cg as OCG

    r = np.random.default_rng(1)
    e1 = r.standard_normal((S, phi_csr.shape[0]))
    e2 = np.sqrt(noise) * r.standard_normal((S, len(tr)))
    t = []
    for mi in (1, 2):
        t0 = time.perf_counter()
        OCG.pathwise_predict(phi_csr, tr, te, y, noise, e1, e2, max_iter=mi)
        t.append(time.perf_counter() - t0)
    per_iter = max(t[1] - t[0], 1e-9)
    setup = max(t[0] - per_iter, 0.0)
    t_full = setup + iters * per_iter
    return {
        "value": 1.0 / t_full,
        "unit": "posterior-sample-batches/s",
        "cores": 1,
        "kind": "port",
        "sample": (f"oracle/cg.py pathwise_predict (scipy sparse, fp64, 1 thread) at the same size: setup "
                   f"{setup:.2f} s + {iters} CG iterations x {per_iter:.2f} s (timed at max_iter 1 and 2, "
                   f"extrapolated)"),
    }


def main_predict(args):
    """Pathwise-conditioning posterior samples (models/sparse_grf_model.py:21-45) at C4 scale:
    Phi of the headline workload resident in HBM, 60/20 % train/test split (the reference's
    scaling experiment, run_scaling_experiment.py splits=[0.6, 0.2, 0.2]), n_samples = 64.
    One step = eps draws + Phi_train^T CSR + priors + linear_cg (cg_tolerance 1) + K_test,train V.
    Multi-GPU: independent sample batches per rank (weak scaling, no collective)."""
    import torch

    from grf_amd.engine import DeviceCSR, GRFEngine

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist

        from grf_amd.dist import all_reduce as dist_all_reduce
        local_rank = init_distributed(local_rank)
    eng = GRFEngine(f"cuda:{local_rank}")
    A = make_graph(args)
    n, m, L, p, S = A.shape[0], args.walks, args.length, args.p_halt, args.samples
    f = diffusion_modulator(L, 1.0)
    G = eng.laplacian(DeviceCSR.from_scipy(A, eng.device))
    phi = eng.compact(eng.walk_phi(G, m, p, L, f, seed=42, want64=False), want64=False)
    perm = np.random.default_rng(0).permutation(n)
    n_tr, n_te = int(0.6 * n), int(0.2 * n)
    tr = torch.from_numpy(perm[:n_tr]).to(eng.device)
    te = torch.from_numpy(perm[n_tr:n_tr + n_te]).to(eng.device)
    y = torch.randn(n_tr, device=eng.device, generator=torch.Generator(eng.device).manual_seed(5))
    noise = 0.01  # (the scaling experiment's noise_std 0.1)
    dtype = torch.float64 if args.cg_dtype == "f64" else torch.float32
    gen = torch.Generator(eng.device).manual_seed(1000 + rank)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    cg_ms, its = [], [0]

    def step(record):
        e1 = torch.randn(S, n, device=eng.device, generator=gen)
        e2 = noise ** 0.5 * torch.randn(S, n_tr, device=eng.device, generator=gen)
        E = e1.to(dtype).t().contiguous()
        f_train = eng.spmm(phi, E, tr)
        f_test = eng.spmm(phi, E, te)
        B = (y.to(dtype)[:, None] - (f_train + e2.to(dtype).t())).contiguous()
        phi_t = eng.csr_transpose(phi, tr)
        if record:
            ev[0].record()
        V, it = eng.cg_solve(phi, B, noise, tr, phi_t)
        if record:
            ev[1].record()
            ev[1].synchronize()
            cg_ms.append(ev[0].elapsed_time(ev[1]))
        its[0] = it
        return f_test + eng.spmm(phi, eng.spmm(phi_t, V), te)

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([t], dtype=torch.float64, device=eng.device)
        dist_all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt.item())
    nnz_tr = int((phi.ptr[tr + 1] - phi.ptr[tr]).sum().item())
    elem = 8 if dtype == torch.float64 else 4
    per_it_ms = float(np.mean(cg_ms)) / max(its[0], 1)
    # one CG iteration = Phi_t^T P (n x S out) + Phi_t W (n_tr x S out): CSR entries (col + val)
    # streamed twice, the dense inputs read once and outputs written once; gathers re-read rows
    alg = 2 * 8.0 * nnz_tr + elem * S * (n_tr + n + n + 3 * n_tr)
    gathers = 2.0 * nnz_tr * S * elem
    out = {
        "metric": (f"GRF pathwise-conditioning posterior sample batches/s (SparseGraphGP.predict, "
                   f"{workload_name(args, A)['short']}, {S} samples)"),
        "value": world * args.steps / t,
        "unit": "posterior-sample-batches/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1000.0 * t / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": ("fp64" if elem == 8 else "fp32") + " CG vectors, fp32 Phi",
        "data": workload_name(args, A)["data"] + "; random targets, torch.randn draws",
        "config": {"workload": f"{workload_name(args, A)['long']} predict: m={m}, L={L}, p_halt={p}; "
                               f"{n_tr} train / {n_te} test nodes, n_samples={S}, noise {noise}, cg_tolerance 1",
                   "cg_iterations": its[0], "nnz_phi_train": nnz_tr,
                   "parallelism": f"independent sample batches x{world}"},
        "roofline": {"bound": "hbm", "achieved": alg / (per_it_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": alg / (per_it_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "traffic": None,
                     "kernel": "CG iteration (2 column-tiled spmm_kernel passes + 3 cg_* kernels)",
                     "kernel_ms": per_it_ms, "algorithmic_bytes": alg,
                     "gather_TBps": gathers / (per_it_ms * 1e-3) / 1e12,
                     "gather_note": "X rows gathered per CSR entry (L2/Infinity-Cache served; MI355X_MICROARCH.md "
                                    "'Indexed rows': ~17 TB/s L2-resident, ~8.6 TB/s Infinity Cache)"},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_predict(_phi_host(phi), perm[:n_tr], perm[n_tr:n_tr + n_te],
                                                   y.cpu().numpy().astype(np.float64), noise, S, its[0])
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


MFMA_F32_PEAK_TFS = 157.3  # MI355X_MICROARCH.md: FP32 matrix (v_mfma_f32_32x32x2_f32), dense
MFMA_BF16_PEAK_TFS = 2500.0  # MI355X_MICROARCH.md: BF16 MFMA ~2.5 PF dense (v_mfma_f32_32x32x16_bf16 = 16x the fp32 rate)
SPLIT_PRODUCTS = 6  # grf_gram_dense_split: bf16 plane products per fp32 multiply-add (p + q <= 2 of 3 x 3)


def dense_gram_roofline(precision: str, flops: float, ms: float) -> dict:
    """The dense Gram's roofline for the arithmetic it ran on: 'fp32' = v_mfma_f32_32x32x2_f32 against the
    fp32 matrix peak; 'split' = the bf16 three-plane split (SPLIT_PRODUCTS bf16 products per fp32 term on
    v_mfma_f32_32x32x16_bf16) against the bf16 peak, with the fp32-equivalent rate beside it."""
    tfs = flops / (ms * 1e-3) / 1e12
    if precision == "split":
        return {"bound": "mfma", "achieved": SPLIT_PRODUCTS * tfs, "peak": MFMA_BF16_PEAK_TFS, "unit": "TFLOP/s",
                "frac": SPLIT_PRODUCTS * tfs / MFMA_BF16_PEAK_TFS, "traffic": None,
                "kernel": "gram_split_mfma_kernel (128x128 tiles, fp32 LDS-DMA staging, the exact three-plane bf16 "
                          "split in registers; n <= 8064) / gram_planes_wide_kernel (256x128 items of 8 waves, "
                          "XCD-ordered whole-item rounds + stream-K, the planes split once by the front and staged "
                          "as they are) -- v_mfma_f32_32x32x16_bf16, 6 products per term",
                "kernel_ms": ms, "algorithmic_flops": flops, "bf16_flops": SPLIT_PRODUCTS * flops,
                "fp32_equivalent_tflops": tfs, "fp32_equivalent_vs_fp32_peak": tfs / MFMA_F32_PEAK_TFS}
    return {"bound": "mfma", "achieved": tfs, "peak": MFMA_F32_PEAK_TFS, "unit": "TFLOP/s",
            "frac": tfs / MFMA_F32_PEAK_TFS, "traffic": None,
            "kernel": "gram_dense_mfma_kernel / gram_dense_sk_kernel (LDS-DMA staged 128x128 upper tiles, "
                      "v_mfma_f32_32x32x2f32, both triangles written)",
            "kernel_ms": ms, "algorithmic_flops": flops}


def cora_adjacency() -> np.ndarray:
    """Cora (experiments/dense/cora/data/cora/cora.cites, 2,708 nodes) as the symmetric 0/1 dense
    adjacency of tests/golden/cora.npz (made by tests/golden/make_golden.py from the reference's file)."""
    d = np.load(os.path.join(ROOT, "tests", "golden", "cora.npz"), allow_pickle=False)
    n = len(d["A_indptr"]) - 1
    return sp.csr_matrix((d["A_data"], d["A_indices"], d["A_indptr"]), shape=(n, n)).toarray()


C2_DENSE = (10_000, 49_995)  # G(10k, 0.001) (E[M] = 49,995), run through the dense path


def dense_workload(name: str):
    """(dense adjacency, description, data) of a dense-path workload: C3 = Cora, C2 = ER N = 10k with
    49,995 edges (graph seed 0), both as the reference's dense path takes them (an ndarray)."""
    if name == "c2":
        n, edges = C2_DENSE
        W = er_graph_exact_edges(n, edges, seed=0).toarray()
        return W, f"C2: ER N={n}, {edges} undirected edges, dense adjacency", \
            "synthetic Erdos-Renyi graph (seed 0), unit weights"
    return cora_adjacency(), "C3: Cora N=2708 dense adjacency", \
        "real graph: Cora citation graph shipped with the reference (tests/golden/cora.npz)"


def main_c3(args):
    """C3 (C2 with --workload c2): the reference's DENSE path on Cora (graph_kernels/fast_grf_kernel_general.py:11-39) --
    numpy-semantics dense Laplacian of the dense adjacency (resident in HBM) -> Philox walks
    (m = 128, L = 8) -> step rows (dense sampler's divide-by-m rule) -> Phi = F f -> dense
    float32 Phi -> K = Phi Phi^T on the MFMA (gram_dense_kernel, v_mfma_f32_32x32x2_f32).
    The roofline is the MFMA Gram's (+ its mirror pass): N (N + 1) k flops (the symmetric
    product's unique entries) against the fp32 matrix peak."""
    import torch

    from grf_amd import _lib as C
    from grf_amd.engine import GRFEngine

    eng = GRFEngine("cuda:0")
    W, wdesc, wdata = dense_workload(args.workload)
    n, m, L, p = W.shape[0], args.walks, args.length, args.p_halt
    f = diffusion_modulator(L, 1.0)
    Wt = torch.from_numpy(W).to(eng.device)
    nnz_w = int(np.count_nonzero(W))  # (setup: sizes every step's walk matrix without a device count)
    gram_ev = []        # the Gram in the timed (pipelined) steps
    gram_ev_alone = []  # the Gram in the serial steps (nothing beside it): the roofline's time
    # the next step's front runs here beside this step's Gram (--side-priority high: the stream's workgroups
    # are dispatched ahead of the Gram's when both wait for a CU slot)
    side = torch.cuda.Stream(eng.device, priority=-1 if args.side_priority == "high" else 0)
    main = torch.cuda.current_stream(eng.device)

    def front():
        G = eng.walk_matrix_dense(Wt, C.LAP_NUMPY, nnz_w=nnz_w)
        # fused Philox walks -> Phi rows with the dense sampler's divide-by-m rule, written straight into
        # the dense fp32 Phi the Gram reads (no compaction, no memset: grf_densify_padded)
        return eng.densify_padded(eng.walk_phi(G, m, p, L, f, seed=42, norm=C.NORM_DIV, want64=False),
                                  planes=use_planes)

    # the split Gram's planes written by the front itself (grf_densify_padded_planes) where the planes path runs
    use_planes = (args.gram_precision or eng.dense_precision) == "split" and eng.use_planes(n)

    def front_on_side():
        # independent of `main`: a front reads only the resident adjacency and writes fresh buffers
        with torch.cuda.stream(side):
            dense = front()
            done = torch.cuda.Event()
            done.record(side)
        return dense, done

    def back(dense, record):
        if record:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        K = eng.gram_dense(dense, n, precision=args.gram_precision or None)
        if record:
            ev[1].record()
            (gram_ev if record is True else gram_ev_alone).append(ev)
        return K

    def run(steps, record, pipelined):
        """`steps` whole steps.  Pipelined (the default; --no-overlap: serial): step s+1's front is
        issued on the side stream before step s's Gram, so the latency-bound walks run beside the
        MFMA tiles; every step still runs its whole path, and the call's first front is not
        overlapped (nothing is carried across the call's boundary)."""
        if not pipelined:
            for _ in range(steps):
                back(front(), record)
            return
        cur = front_on_side()
        for s_ in range(steps):
            dense, done = cur
            main.wait_event(done)
            dense.record_stream(main)  # (allocated on `side`, read on `main`)
            cur = front_on_side() if s_ + 1 < steps else None
            back(dense, record)

    # pipelined by default only while the front is a real share of the step: at C3 (the Gram 0.205 ms, the front
    # ~0.09 ms alone) 0.291-0.301 vs 0.295-0.298 serial; at C2 the front's 800 MB read of W slows the 7.4 ms MFMA
    # Gram more than it hides (8.13-8.79 vs 7.76-8.48 serial; profiles/r05_dense_overlap_ab.txt)
    pipelined = args.overlap if args.overlap is not None else n < 4096
    run(args.warmup, False, pipelined)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps, True, pipelined)
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    # latency of one un-pipelined step (reported beside the throughput; not part of `value`)
    run(2, False, False)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    run(5, "alone", False)
    torch.cuda.synchronize()
    serial_ms = 1000.0 * (time.perf_counter() - t1) / 5
    gram_ms_pipe = float(np.mean([a.elapsed_time(b) for a, b in gram_ev]))
    # the roofline's time: the Gram alone (the serial steps); pipelined it shares the GPU with the next front
    gram_ms = float(np.mean([a.elapsed_time(b) for a, b in gram_ev_alone]))
    # the symmetric product's unique entries, 2 k flops each (the kernel computes the tiles on and
    # above the diagonal and mirrors them; counting 2 n^2 k would credit work it does not do; k = n,
    # the zero padding of the k range is not counted either)
    flops = 1.0 * n * (n + 1) * n
    prec = args.gram_precision or eng.dense_precision
    split = prec == "split"
    roof = dense_gram_roofline(prec, flops, gram_ms)
    roof.update({"kernel_ms": gram_ms,
                 "kernel_ms_note": "HIP events around the Gram in the serial steps (alone on the GPU)",
                 "kernel_ms_pipelined": gram_ms_pipe})
    out = {
        "metric": (f"GRF kernel-matrices/sec ({'Cora N=2708' if args.workload == 'c3' else f'ER N={n}'}, dense path, "
                   f"m={m} walks; MFMA utilisation of the Gram)"),
        "value": args.steps / t,
        "unit": "K-matrices/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1000.0 * t / args.steps,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": ("fp64 walk loads, fp32 Phi, fp32 Gram on the bf16 MFMA (exact three-plane split, fp32 accumulation)"
                  if split else "fp64 walk loads, fp32 Phi, fp32 MFMA Gram"),
        "data": wdata,
        "config": {"workload": f"{wdesc} resident in HBM, dense numpy-semantics Laplacian, "
                               f"walks_per_node={m}, max_walk_length={L}, p_halt={p}, diffusion modulator beta=1, "
                               f"Philox seed 42, dense fp32 Phi and K", "n_nodes": n},
        "roofline": roof,
        "pipelined": pipelined,
        "serial_ms_per_step": serial_ms,
    }
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_dense(W, f, m, p, L,
                                                 host_threads())
    print(json.dumps(out), flush=True)


def cpu_baseline_dense(W, f, m, p, L, n_threads):
    """The reference's dense path restated on the host (C oracle: numpy Laplacian, PCG64 pool walks
    on n_threads chunks, step tensor F, Phi = F f, K = Phi Phi^T with numpy's BLAS)."""
    from oracle import oracle as O

    t0 = time.perf_counter()
    Ld = O.laplacian_dense(W, 0)
    F = O.dense_random_walk(Ld, m, p, L, n_processes=n_threads, n_threads=n_threads)
    phi = F @ np.asarray(f)
    K = phi @ phi.T
    t = time.perf_counter() - t0
    del K
    return {"value": 1.0 / t, "unit": "K-matrices/s", "cores": n_threads, "kind": "port",
            "sample": f"C oracle dense path (reference algorithm, PCG64 stream, {n_threads} chunks) on {n_threads} "
                      f"host threads, the whole K ({t:.2f} s); fp64"}


def _phi_host(phi):
    n = phi.n_rows
    return sp.csr_matrix((phi.val32.cpu().numpy().astype(np.float64), phi.idx.cpu().numpy(), phi.ptr.cpu().numpy()),
                         shape=(n, phi.n_cols))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", "--n-nodes", dest="n", type=int, default=100_000)
    ap.add_argument("--edges", type=int, default=1_000_000)
    ap.add_argument("--walks", type=int, default=128)
    ap.add_argument("--length", type=int, default=8)
    ap.add_argument("--p-halt", type=float, default=0.1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--transfers", action="store_true",
                    help="also time the host hand-over of the drop-in boundary (SURVEY.md §8d: H2D of the CSR "
                         "adjacency, D2H of the K block into pinned host memory) and report the PCIe-inclusive "
                         "rate beside the device-resident value (never as `value`)")
    ap.add_argument("--cpu-rows", type=int, default=2048)
    ap.add_argument("--no-sym", action="store_true", help="compute every K tile (one GPU: no symmetric mode; N > 1 "
                    "column blocks: no symmetric square K[b:e, b:e])")
    ap.add_argument("--mode", choices=["cols", "rows", "allreduce"], default="cols",
                    help="cols (default; N > 1): K column blocks K[:, R_r] (= the row blocks, K symmetric) from a "
                         "transpose of the rank's own Phi rows after a Phi all-gather; rows: K row blocks from a "
                         "transpose of all of Phi (one GPU always runs rows / symmetric); allreduce: the north star's literal "
                         "option -- per-rank partial K over an inner-dimension slice + bucketed RCCL all-reduce, "
                         "K replicated on every rank (SURVEY.md §8e)")
    ap.add_argument("--workload", choices=["kernel", "predict", "c5", "c3", "c2"], default="kernel",
                    help="kernel: K = Phi Phi^T (headline); predict: pathwise-conditioning posterior samples; "
                         "c5: SURVEY.md C5 -- N=1M power-law graph, m=64, Phi + a K row block per GPU; "
                         "c3: Cora dense path with the MFMA Gram; c2: ER N=10k through the dense path (MFMA Gram)")
    ap.add_argument("--graph", choices=["er", "powerlaw", "facebook", "enron"], default="er",
                    help="er: Erdos-Renyi with --edges edges (C4); powerlaw: Chung-Lu, exponent 2.5, mean degree "
                         "--avg-degree (C5); facebook / enron: the reference's shipped social graphs")
    ap.add_argument("--avg-degree", type=float, default=10.0, help="powerlaw: expected mean degree")
    ap.add_argument("--band-width", type=int, default=0,
                    help="transpose band width of the single-GPU Gram (a multiple of 64, <= 8192; default: 4096 for "
                         "the symmetric mode, 8192 for row modes)")
    ap.add_argument("--k-rows", type=int, default=0,
                    help="compute only the first R rows of every rank's K row block (0 = all rows); "
                         "the unit becomes K rows/s")
    ap.add_argument("--overlap", dest="overlap", action="store_true", default=None,
                    help="pipeline the steps on two HIP streams: step s+1's Laplacian/walks/Phi/transpose start "
                         "when step s's Gram tiles finish and run beside its HBM-bound mirror pass (default for "
                         "the single-GPU symmetric K: 24.3 vs 26.5 ms per step); with N > 1 (default) the next "
                         "front, with its RCCL collectives, runs beside this step's Gram; single-GPU row modes "
                         "gain ~1 % and default to serial steps")
    ap.add_argument("--no-overlap", dest="overlap", action="store_false", help="serial steps")
    ap.add_argument("--front-at", type=float, default=None,
                    help="pipelined: the next front starts after this fraction of the Gram tiles (1 = at the mirror, "
                         "0 = with the tiles); default: 0 when the front outlasts the mirror (n < 400 m: Facebook "
                         "2.78 -> 2.45 ms per K), else 1 (C4: the front beside the Gram tiles loses)")
    ap.add_argument("--mirror-wgs", type=int, default=1024,
                    help="pipelined symmetric K: the mirror pass's workgroups beside the next front (0 = one per block)")
    ap.add_argument("--balance", choices=["nodes", "phi"], default="nodes",
                    help="N > 1 source shards: equal node ranges (default), or ranges of equal estimated step work "
                         "from the per-source Phi row counts of one setup walk (dist.balanced_shards)")
    ap.add_argument("--hubs", type=lambda v: -1 if v == "auto" else int(v), default=-1,
                    help="one GPU, whole K: split Phi's densest HUBS columns off into a dense panel whose MFMA Gram "
                         "the sparse Gram adds to (hub-heavy graphs: enron; 0 = no split; auto, the default = the columns "
                         "in at least 13%% of the rows, from a setup walk, in multiples of 32: C4 / Facebook 0, Enron 96)")
    ap.add_argument("--gather-bound", choices=["exact", "cap"], default="exact",
                    help="N > 1 Phi all-gather size per rank: the rank's Phi entries from the setup walk "
                         "(default; checked on the device, a larger step raises after the loop) or its rows x "
                         "the padded row capacity")
    ap.add_argument("--no-mfma-leg", action="store_true",
                    help="skip the C3 dense MFMA Gram leg that adds roofline_mfma to the headline line")
    ap.add_argument("--path", choices=["dense", "sparse"], default="dense",
                    help="c2: the reference's dense path (dense adjacency, MFMA Gram; default) or its sparse path "
                         "as BASELINE config 2 names it (CSR adjacency, fused walks, transpose, symmetric sparse Gram)")
    ap.add_argument("--serial-steps", type=int, default=3,
                    help="un-pipelined steps timed after the throughput steps (serial_ms_per_step, the walk kernel "
                         "alone); 0 skips them (the all-reduce mode at the headline size under gloo: minutes per step)")
    ap.add_argument("--rank-turns", action="store_true",
                    help="N > 1: after the timed steps, re-run each rank's K assembly alone (ranks take turns between "
                         "barriers) and report gram_ms_alone_per_rank (the per-rank time of an unshared GPU when the "
                         "ranks share one GPU under GRF_DIST_BACKEND=gloo)")
    ap.add_argument("--fingerprint-dir", default=None,
                    help="write a bit-level fingerprint of every rank's K block (tools/gram_hash.py) to "
                         "DIR/rank<r>.json after the run (the multi-rank at-size parity test)")
    ap.add_argument("--gram-precision", choices=["fp32", "split"], default=None,
                    help="dense-path Gram (c3 / c2 and the MFMA legs): the fp32 MFMA, or the same product on the bf16 "
                         "MFMA from an exact three-plane bf16 split of Phi (grf_gram_dense_split); default: the "
                         "engine's (GRF_GRAM_DENSE_PRECISION, 'split')")
    ap.add_argument("--side-priority", choices=["normal", "high"], default="high",
                    help="pipelined steps: the HIP priority of the stream the next front runs on (high: its workgroups "
                         "are dispatched ahead of the Gram's; C3 0.295-0.301 vs 0.306-0.313 ms, C4 equal: "
                         "profiles/r05_dense_overlap_ab.txt)")
    ap.add_argument("--samples", type=int, default=64, help="predict: n_samples")
    ap.add_argument("--cg-dtype", choices=["f64", "f32"], default="f64", help="predict: CG vector precision")
    args = ap.parse_args()
    if args.workload == "c5":
        args.n, args.graph, args.walks = 1_000_000, "powerlaw", 64
        args.k_rows = args.k_rows or 8192
    if args.graph in ("facebook", "enron"):
        args.n = None
    if args.workload == "predict":
        return main_predict(args)
    if args.workload == "c2" and args.path == "sparse":
        args.n, args.edges = C2_DENSE  # G(10k, 0.001) through the CSR path (the headline machinery)
    elif args.workload in ("c3", "c2"):
        return main_c3(args)

    import torch
    import torch.distributed as dist

    from grf_amd import dist as D
    from grf_amd import pipeline as P
    from grf_amd.dist import all_reduce as dist_all_reduce
    from grf_amd.engine import DeviceCSR, GRFEngine
    import grf_amd.engine as engine_mod

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # GRF_DIST_FORCE=1 (under torch.distributed.run, one rank): the N > 1 path with its RCCL collectives
    # on a one-GPU box (the all-gather of one shard, the timing / parity all-reduces)
    coll = world > 1 or os.environ.get("GRF_DIST_FORCE", "0") == "1"
    if coll:
        local_rank = init_distributed(local_rank)
    eng = GRFEngine(f"cuda:{local_rank}")
    dev = eng.device
    A = make_graph(args)
    n, m, L, p = A.shape[0], args.walks, args.length, args.p_halt
    f = diffusion_modulator(L, 1.0)
    A_dev = DeviceCSR.from_scipy(A, dev)
    shards = None
    phi0 = None
    if coll:
        from grf_amd.dist import balanced_shards, setup_phi
        phi0 = setup_phi(eng, A_dev, m, p, L, f, seed=42)  # (setup, untimed: the Phi every step makes)
        if args.balance != "nodes":
            shards = balanced_shards(eng, A_dev, m, p, L, f, world, policy=args.balance, phi=phi0)
    pl = P.plan_step(n, m, L, p, f, seed=42, world=world, rank=rank, mode=args.mode, k_rows=args.k_rows,
                     band_width=args.band_width, no_sym=args.no_sym, shards=shards, collective=coll)
    if pl.mode == "sym":
        hubs_auto, pl.skewed = auto_hubs(eng, A_dev, m, p, L, f)
        pl.hubs = int(args.hubs) if args.hubs > 0 else (hubs_auto if args.hubs < 0 else 0)
    if phi0 is not None:
        if args.gather_bound == "exact":
            # the Phi all-gather moves each rank's actual entries (C4: 435 per row) instead of its rows x
            # the padded row capacity (1024); a step whose Phi outgrew it would raise after the loop
            from grf_amd.dist import shard_entries
            pl.gather_bound = max(shard_entries(phi0, pl.shards))
        del phi0
    b, e, kr_end = pl.b, pl.e, pl.kr_end
    K = P.alloc_k(eng, pl)  # resident output block, reused
    if args.overlap is None:
        # one GPU, whole K: the next front beside the mirror; N > 1 row / column blocks: the next
        # front's collectives beside this step's Gram (the compute of a front beside a Gram gains
        # ~1 %: single-GPU row modes stay serial)
        # K-row-block workloads (C5) on one GPU: serial -- the column-block Gram is a persistent kernel
        # holding every CU's LDS, so a front issued beside it only waits (16.68 vs 16.20 ms per step,
        # profiles/r06_bench_c5.json; with the tile-per-workgroup Gram it gained 0.6 ms, r02_c5_overlap.txt)
        args.overlap = pl.mode == "sym" or (coll and pl.mode != "allreduce")
    gram_ev = []  # (start, end) events around the K assembly of every timed step, read after the loop
    walk_ev = []  # (start, end) events around walk_phi in the serial-latency steps (kernel alone)
    last = [None]

    # the next step's front runs here while the Gram runs on `main` (--side-priority: see main_c3)
    side = torch.cuda.Stream(dev, priority=-1 if args.side_priority == "high" else 0)
    main = torch.cuda.current_stream(dev)

    if args.front_at is None:
        # the mirror moves 4 n^2 bytes (~6.7e-13 n^2 s), the next front ~2.7e-10 s per walk (C4: 3.5 ms for
        # 12.8 M walks): below n = 400 m the front outlasts the mirror and is issued with the Gram tiles
        # (profiles/r03_front_at_ab.txt)
        args.front_at = 0.0 if n < 400 * m else 1.0

    def front(record_walk: bool = False):
        if record_walk:
            # the walk kernel timed alone (serial steps): events around the front's walk_phi launch
            orig = eng.walk_phi

            def timed(*a, **k):
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
                out = orig(*a, **k)
                ev[1].record()
                walk_ev.append(ev)
                return out

            eng.walk_phi = timed
            try:
                return P.front(eng, A_dev, pl)
            finally:
                eng.walk_phi = orig
        return P.front(eng, A_dev, pl)

    def back(fr, record: bool, after_gram=None):
        if record:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        # (pipelined: a 1024-workgroup mirror leaves CU slots to the next front)
        P.k_assembly(eng, fr, pl, K, after_tiles=after_gram, mirror_workgroups=args.mirror_wgs if after_gram else 0,
                     front_at=args.front_at)
        if record:
            ev[1].record(main)
            gram_ev.append(ev)
        last[0] = fr

    def front_on_side(after=None, independent=False):
        # after: an event on `main`; default: everything issued on `main` so far.  independent: no
        # wait at all (a front reads only the resident adjacency and writes fresh buffers; buffers
        # freed on `main` are recorded there, so the allocator does not hand them out early)
        if independent:
            pass
        elif after is None:
            side.wait_stream(main)
        else:
            side.wait_event(after)
        with torch.cuda.stream(side):
            fr = front()
            done = torch.cuda.Event()
            done.record(side)
        return fr, done

    def back_on_main(frd, record, after_gram=None):
        fr, done = frd
        main.wait_event(done)
        # every device buffer the front allocated on `side` (Phi -- CSR or padded rows --, the transpose, the row
        # cuts, ...) is used on `main`: recorded there, so the allocator does not hand it out before `main` is done
        for v in _device_tensors(fr):
            v.record_stream(main)
        back(fr, record, after_gram)

    def run(steps: int, record: bool, record_walk: bool = False):
        """`steps` whole steps.  Pipelined (--overlap): step s+1's front is issued on the side
        stream before step s's K assembly, so the two overlap on the GPU; every step still runs
        its whole path, and the first front of the call is not overlapped (no work is carried
        across the call's boundary)."""
        if not args.overlap:
            for _ in range(steps):
                back(front(record_walk), record)
            return
        cur = front_on_side()
        for s_ in range(steps):
            if pl.mode == "sym":
                # the next front starts when this step's Gram tiles are done: it runs beside the
                # HBM-bound mirror instead of the gather-bound Gram
                nxt = [None]

                def issue_next(tiles_done, last=s_ + 1 >= steps):
                    if not last:
                        nxt[0] = front_on_side(tiles_done)

                back_on_main(cur, record, issue_next)
                cur = nxt[0]
            else:
                # row / column modes: this step's Gram is issued first, then the next front, which
                # overlaps it (with N > 1 the collectives run beside it)
                back_on_main(cur, record)
                cur = front_on_side(independent=True) if s_ + 1 < steps else None

    run(args.warmup, False)
    torch.cuda.synchronize()
    if coll:
        dist.barrier()
        D.GATHER_STATS = []  # HIP events around every Phi all-gather of the timed steps
        D.ALLREDUCE_STATS = [] if pl.mode == "allreduce" else None  # ... and every bucketed K all-reduce
    t0 = time.perf_counter()
    run(args.steps, True)
    torch.cuda.synchronize()
    if coll:
        dist.barrier()
    t = time.perf_counter() - t0
    gather_stats = D.GATHER_STATS or []
    D.GATHER_STATS = None
    allreduce_stats = D.ALLREDUCE_STATS or []
    D.ALLREDUCE_STATS = None
    if coll:
        from grf_amd.dist import check_gather_overflow
        check_gather_overflow(dev)  # (raises if a bounded all-gather truncated a rank's Phi)
    # in-run parity of the LAST TIMED step's K block (the pipelined path itself) against the Phi that
    # step gathered (every rank), before the serial steps below overwrite K
    parity = P.k_block_check(eng, last[0], pl, K)
    # latency of one un-pipelined step (reported beside the throughput; not part of `value`), with
    # the walk kernel timed alone there
    ov = args.overlap
    serial_ms = None
    if args.serial_steps > 0:
        args.overlap = False
        run(1, False)  # (warm-up of the serial order)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        run(args.serial_steps, False, record_walk=True)
        torch.cuda.synchronize()
        serial_ms = 1000.0 * (time.perf_counter() - t1) / args.serial_steps
        args.overlap = ov
    gram_ms = [a.elapsed_time(b_) for a, b_ in gram_ev]
    walk_ms = float(np.mean([a.elapsed_time(b_) for a, b_ in walk_ev])) if walk_ev else 0.0
    gram_alone = rank_turns_gram_ms(eng, last[0], pl, K, coll, rank, world) if args.rank_turns else None
    if args.fingerprint_dir:
        # bit-level fingerprint of this rank's K block (tools/gram_hash.py), for the at-size multi-rank test
        from tools.gram_hash import fingerprint
        torch.cuda.synchronize()
        h, s_ = fingerprint(P.k_view(K, pl))
        os.makedirs(args.fingerprint_dir, exist_ok=True)
        with open(os.path.join(args.fingerprint_dir, f"rank{rank}.json"), "w") as fh:
            json.dump({"rank": rank, "world": world, "mode": pl.mode, "shard": [b, e], "cols_sym": pl.cols_sym,
                       "k_rows": args.k_rows, "hash": h, "sum": s_}, fh)
    # the sparse Gram tiles' gather roofline (whole-K mode): their bucket-line gathers against the
    # guide's indexed-row rates (after the fingerprint: the timing launches rewrite K's upper tiles)
    gather_rl = gather_roofline(eng, last[0], pl, K) if pl.mode == "sym" else None
    coll_ms = float(np.mean([a.elapsed_time(b_) for a, b_, _, _ in gather_stats])) if gather_stats else 0.0
    coll_sent = float(np.mean([x for _, _, x, _ in gather_stats])) if gather_stats else 0.0
    coll_recv = float(np.mean([x for _, _, _, x in gather_stats])) if gather_stats else 0.0
    ar_ms = float(np.mean([a.elapsed_time(b_) for a, b_, _ in allreduce_stats])) if allreduce_stats else 0.0
    ar_bytes = float(np.mean([x for _, _, x in allreduce_stats])) if allreduce_stats else 0.0
    if coll:
        tt = torch.tensor([t, float(np.mean(gram_ms)), walk_ms], dtype=torch.float64, device=dev)
        dist_all_reduce(tt, op=dist.ReduceOp.MAX)
        t, gram_avg, walk_ms = (float(x) for x in tt.tolist())
        # every rank's Gram time, collective time and volume, and parity ratio (rank order)
        mine = torch.tensor([float(np.mean(gram_ms)), coll_ms, coll_sent, coll_recv, parity["max_ratio"],
                             float(pl.e - pl.b), gram_alone or 0.0, ar_ms, ar_bytes], dtype=torch.float64, device=dev)
        allr = torch.zeros(world * mine.numel(), dtype=torch.float64, device=dev)
        allr[rank * mine.numel():(rank + 1) * mine.numel()] = mine
        dist_all_reduce(allr)
        per_rank = allr.view(world, -1).cpu().numpy()
        parity = dict(parity, max_ratio=float(per_rank[:, 4].max()), ok=bool(per_rank[:, 4].max() <= 1.0),
                      per_rank=[float(x) for x in per_rank[:, 4]])
        dist_info = {"backend": dist.get_backend(), "world_size": dist.get_world_size(),
                     "rank_rows": [int(x) for x in per_rank[:, 5]],
                     "gram_ms_per_rank": [float(x) for x in per_rank[:, 0]],
                     "gram_balance": float(per_rank[:, 0].min() / max(per_rank[:, 0].max(), 1e-9)),
                     "gather_ms_per_rank": [float(x) for x in per_rank[:, 1]],
                     "gather_bytes_sent_per_rank": [int(x) for x in per_rank[:, 2]],
                     "gather_bytes_received_per_rank": [int(x) for x in per_rank[:, 3]],
                     "gather_note": "HIP events on the issuing stream around each step's Phi all-gather "
                                    "(the transfer + the wait for the slowest rank), mean over the timed steps"}
        if pl.mode == "allreduce":
            dist_info["allreduce_ms_per_rank"] = [float(x) for x in per_rank[:, 7]]
            dist_info["allreduce_bytes_per_rank"] = [int(x) for x in per_rank[:, 8]]
            dist_info["allreduce_note"] = ("HIP events on the issuing stream around each timed step's bucketed K "
                                           "all-reduce (1 GiB buckets; under gloo staged through host memory)")
        if args.rank_turns:
            dist_info["gram_ms_alone_per_rank"] = [float(x) for x in per_rank[:, 6]]
            dist_info["gram_alone_note"] = ("each rank's K assembly (its column / row block from the last front) "
                                            "re-run alone on the GPU, ranks taking turns between barriers, HIP events "
                                            "over 3 launches, the faster of two rounds of turns: the per-rank Gram time of an unshared GPU (under gloo "
                                            "the ranks share one GPU, so gram_ms_per_rank includes the others' work)")
    else:
        gram_avg = float(np.mean(gram_ms))
        dist_info = None

    ms_per_step = 1000.0 * t / args.steps
    phi_last = last[0].phi
    nnz_phi = phi_last.nnz
    local_nnz = last[0].local.nnz
    # algorithmic bytes of the K assembly (gram_sparse_kernel [+ the mirror kernel]): write this
    # rank's K rows once, read its Phi rows (col int32 + val fp32) and every Phi^T entry once
    rows = kr_end - b
    alg_bytes = 4.0 * rows * n + 8.0 * local_nnz * rows / max(e - b, 1) + 8.0 * nnz_phi
    if pl.mode == "allreduce":  # every K entry written; all of Phi scanned, the slice's share of Phi^T read
        alg_bytes = 4.0 * n * n + 8.0 * nnz_phi + 8.0 * nnz_phi * rows / n
    achieved = alg_bytes / (gram_avg * 1e-3) / 1e9
    sym = pl.mode == "sym"
    kernels = ["grf::gram_sparse_kernel", "grf::gram_mirror_swz_kernel"] if sym else ["grf::gram_sparse_kernel"]
    headline = (n, args.edges, m, L, p) == DEFAULT_WORKLOAD and args.graph == "er" and world == 1 and sym
    # the committed PMC summary of this workload: the headline's, or C5's (one GPU)
    pmc_path = PMC_SUMMARY if headline else (
        PMC_SUMMARY_C5 if getattr(args, "workload", "") == "c5" and world == 1 else None)
    traffic = pmc_traffic(kernels, pmc_path) if pmc_path else None
    # the walk kernel (phi_fused_kernel): per walk, E[moves] = (1-p)(1-(1-p)^(L-1))/p recorded moves,
    # each reading the current node's row bounds + the chosen entry's column and weight (SURVEY.md
    # §8d: 16 B per move), + the compact Phi row written (int32 column + fp32 value per entry)
    walks = float(e - b) * m
    moves = walks * (1.0 - p) * (1.0 - (1.0 - p) ** (L - 1)) / p
    walk_alg = 16.0 * moves + 8.0 * local_nnz
    walk_achieved = walk_alg / (walk_ms * 1e-3) / 1e9 if walk_ms > 0 else 0.0
    walk_traffic = pmc_traffic(["grf::phi_fused_kernel"], pmc_path) if pmc_path else None
    # the walk's VALU issue rate from ONE rocprofv3 --pmc pass (SQ_INSTS_VALU and GRBM_GUI_ACTIVE counted
    # together, tools/pmc_passes.sh "sq"): wave-instructions per SIMD-cycle, the cycles of the dispatch being
    # GRBM_GUI_ACTIVE / 8 (the counter sums the 8 XCDs, MI355X_MICROARCH.md); no clock or timer involved
    walk_valu = pmc_counter("grf::phi_fused_kernel", "SQ_INSTS_VALU", pmc_path) if pmc_path else None
    walk_gui = pmc_counter("grf::phi_fused_kernel", "GRBM_GUI_ACTIVE", pmc_path) if pmc_path else None
    walk_valu_rate = walk_valu / (walk_gui / 8.0 * N_SIMDS) if walk_valu and walk_gui else None
    wl = workload_name(args, A)
    if args.k_rows:
        metric = (f"GRF kernel rows/sec ({wl['short']}, m={m} walks: Phi of all N nodes + a {args.k_rows}-row "
                  f"fp32 K block per GPU, every step)")
        unit, value, scaling = "K-rows/s", world * rows * args.steps / t, "weak"
    else:
        metric = "GRF kernel-matrices/sec (N=100k graph, m=128 walks; + achieved HBM GB/s of the Gram kernel)"
        if args.graph != "er" or (n, args.edges, m, L, p) != DEFAULT_WORKLOAD:
            metric = f"GRF kernel-matrices/sec ({wl['short']}, m={m} walks; + achieved HBM GB/s of the Gram kernel)"
        unit, value, scaling = "K-matrices/s", args.steps / t, "strong"
    cols = pl.mode == "cols"
    out = {
        "metric": metric,
        "value": value,
        "unit": unit,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "fp64 walk loads, fp32 Phi, exact-product int64 fixed-point Gram, fp32 K",
        "data": wl["data"],
        "config": {"workload": f"{wl['long']}, walks_per_node={m}, max_walk_length={L}, p_halt={p}, diffusion "
                               f"modulator beta=1, Philox seed 42, dense fp32 K "
                               + ((f"columns [r0, r0+{args.k_rows}) (= those K rows: K is symmetric) of every "
                                   f"rank's block" if cols else f"rows [r0, r0+{args.k_rows}) of every rank's block")
                                  if args.k_rows else "")
                               + " resident in HBM",
                   "n_nodes": n, "n_edges": int(A.nnz // 2), "walks_per_node": m, "max_walk_length": L,
                   "k_rows_per_gpu": rows, "shard": [b, e], "balance": args.balance if coll else None,
                   "gather_entries_per_rank": pl.gather_bound or None,
                   "hub_columns": pl.hubs or None,
                   "pair_balanced_waves": pl.mode == "sym" and
                   (engine_mod.ROW_CUTS == "1" or (engine_mod.ROW_CUTS == "auto" and bool(pl.skewed))),
                   "parallelism": (f"source-sharded x{world}, Phi all-gather, partial K over inner slices + "
                                   f"RCCL all-reduce (K replicated)") if pl.mode == "allreduce" else
                                  (f"source-sharded x{world}, Phi all-gather, K column blocks K[:, R_r] from each "
                                   f"rank's own-rows transpose") if cols else
                                  f"source-sharded x{world}, Phi all-gather, K row blocks"
                                  + (" (one GPU: symmetric tiles + mirror)" if sym else "")},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_source": (f"rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE of the same kernels on this workload, "
                                        f"{os.path.relpath(pmc_path or PMC_SUMMARY, ROOT)} (FETCH_SIZE x the calibrated factor "
                                        f"+ WRITE_SIZE; bytes per launch)")
                     if traffic is not None else None,
                     "kernel": "+".join(k.split("::")[1] for k in kernels), "kernel_ms": gram_avg,
                     "algorithmic_bytes": alg_bytes},
        "roofline_walk": {"bound": "valu" if walk_valu_rate is not None else "hbm",
                          "achieved": walk_valu_rate if walk_valu_rate is not None else walk_achieved,
                          "peak": VALU_PEAK_PER_SIMD_CYCLE if walk_valu_rate is not None else HBM_PEAK_GBS,
                          "unit": "VALU wave-instructions per SIMD-cycle" if walk_valu_rate is not None else "GB/s",
                          "frac": (walk_valu_rate / VALU_PEAK_PER_SIMD_CYCLE) if walk_valu_rate is not None
                          else walk_achieved / HBM_PEAK_GBS,
                          "valu_insts_per_launch": walk_valu,
                          "gui_active_cycles_per_launch": walk_gui / 8.0 if walk_gui else None,
                          "valu_source": (f"one rocprofv3 --pmc pass of this workload (SQ_INSTS_VALU, GRBM_GUI_ACTIVE), "
                                          f"{os.path.relpath(pmc_path or PMC_SUMMARY, ROOT)}: SQ_INSTS_VALU / (GRBM_GUI_ACTIVE / 8 x "
                                          f"1024 SIMDs) against the measured 1 wave64 VALU instruction per 4 cycles per SIMD "
                                          f"(profiles/r04_valu_ceiling.txt; fp64 transcendentals take 16: a lower bound "
                                          f"of the VALU pipe's busy share)") if walk_valu_rate is not None else None,
                          "hbm": {"achieved": walk_achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                  "frac": walk_achieved / HBM_PEAK_GBS, "traffic": walk_traffic},
                          "kernel": "phi_fused_kernel (fused Philox walks -> Phi rows)",
                          "kernel_ms": walk_ms, "kernel_ms_note": "HIP events around the launch in this run's serial "
                                                                  "steps (the hbm rate's time; not the valu frac's)",
                          "algorithmic_bytes": walk_alg,
                          "algorithmic_note": f"16 B per expected recorded move ({moves:.4g}) + 8 B per Phi "
                                              f"entry written ({local_nnz}); timed alone in the serial steps "
                                              f"(pipelined it shares HBM with the mirror)"},
        "nnz_phi": nnz_phi,
        "parity": parity,
        "parity_note": "the last timed (pipelined) step's K block, checked after the timed region",
        "roofline_gather": gather_rl,
        "pipelined": bool(ov),
        "front_at": args.front_at,
        "serial_ms_per_step": serial_ms,
    }
    if dist_info is not None:
        out["distributed"] = dist_info
    if headline and not args.no_mfma_leg:
        # (side legs: a failure there is reported in the line and never costs the headline number)
        for key, wl in (("roofline_mfma", "c3"), ("roofline_mfma_c2", "c2")):  # C3 (Cora); C2 (ER N = 10k) dense path
            try:
                out[key] = mfma_leg(eng, args, workload=wl)
            except Exception as exc:  # noqa: BLE001
                out[key] = {"error": f"{type(exc).__name__}: {exc}"}
    if args.transfers:
        try:
            out["transfers"] = time_transfers(A, K, pl, dev, ms_per_step)
            out["transfers"]["pcie_inclusive_value"] = value * ms_per_step / out["transfers"]["pcie_inclusive_ms_per_step"]
            out["transfers"]["pcie_inclusive_unit"] = unit
        except Exception as exc:  # noqa: BLE001
            out["transfers"] = {"error": f"{type(exc).__name__}: {exc}"}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(A, f, m, p, L, args.cpu_rows, host_threads(), k_rows=args.k_rows)
            out["cpu_baseline"]["host"] = host_cpu_note()
        except Exception as exc:  # noqa: BLE001  (reported, never at the cost of the GPU line)
            out["cpu_baseline"] = {"error": f"{type(exc).__name__}: {exc}"}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if coll:
        dist.destroy_process_group()


# MI355X_MICROARCH.md "Indexed rows": chip-wide rates of rows gathered by index, by where they are served
GATHER_PEAK_IC_TBS = 8.6      # 38 MB table, uniformly random rows (Infinity Cache)
GATHER_PEAK_BEYOND_TBS = 7.4  # 151 MB table (7.4-7.9); past 256 MiB 3-9 % slower again (lower bound taken)
IC_BYTES = 256 << 20


def gather_model(phi, tr, sym: bool = True):
    """Bucket gathers of the sparse Gram tiles (gram_sparse_kernel), counted from the transpose's
    descriptors and Phi's entries, no PMC: the tile of row i gathers, for every nonzero Phi[i, k], the
    bucket (band b, column k) of every band b of its tiles (symmetric mode: b >= band(i)), so bucket
    (b, k) is read by the entries of column k in bands <= b.  Returns (128-B lines gathered, record
    bytes gathered, table bytes), or None for the slot layout (its buckets are not in t_desc)."""
    import torch

    from grf_amd import _lib as C

    if tr.rec_unit == C.REC_SLOT or phi.nnz == 0:
        return None
    n, ncol, W = tr.n_rows, tr.n_cols, tr.band_width
    nb = -(-n // W)
    desc = tr.t_desc[:2 * nb * ncol].view(nb, ncol, 2).long()
    first, pairs = desc[..., 0], desc[..., 1]
    if tr.rec_unit == C.REC_LINE:
        lines = (12 * pairs + 127) // 128
    else:  # packed: the lines a bucket's bytes span from its start
        start = first * tr.rec_unit
        lines = torch.where(pairs > 0, (start + 12 * pairs - 1) // 128 - start // 128 + 1, torch.zeros_like(pairs))
    nnz = phi.nnz
    rows = torch.repeat_interleave(torch.arange(phi.n_rows, device=phi.ptr.device), phi.ptr.diff())
    ent = torch.bincount((rows // W) * ncol + phi.idx[:nnz].long(), minlength=nb * ncol).view(nb, ncol)
    del rows
    visits = ent.cumsum(0) if sym else ent.sum(0, keepdim=True).expand(nb, ncol)
    line_visits = int((visits * lines).sum())
    rec_bytes = int((visits * pairs).sum()) * 12
    table = int(((first + (lines if tr.rec_unit == C.REC_LINE else 0)).max() * tr.rec_unit)) \
        if tr.rec_unit == C.REC_LINE else int((first * tr.rec_unit + 12 * pairs).max())
    return line_visits, rec_bytes, table


def gather_roofline(eng, fr, pl, K, reps: int = 3) -> dict:
    """roofline_gather: the sparse Gram tiles alone (no mirror, no hub panel; the
    hub columns, when split off, are already dropped from this front's transpose) timed with HIP events,
    their gathered 128-B bucket lines (gather_model) per launch / that time, against the guide's
    indexed-row rate for where the transpose is served from (Infinity Cache when it fits, else the
    larger-table rate).  HBM bytes stay in `roofline`."""
    import torch

    try:
        model = gather_model(fr.phi, fr.tr, sym=True)
        if model is None:
            return None
        lines, rec_bytes, table = model
        cuts = getattr(fr, "cuts", None)
        if cuts is None and pl.hubs > 0:
            cuts = eng.row_cuts(fr.phi, fr.tr, pl.skewed)
        eng.gram_sparse_upper(fr.phi, fr.tr, out=K, cuts=cuts)  # (warm)
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
        for _ in range(reps):
            eng.gram_sparse_upper(fr.phi, fr.tr, out=K, cuts=cuts)
        ev[1].record()
        ev[1].synchronize()
        ms = ev[0].elapsed_time(ev[1]) / reps
        peak = GATHER_PEAK_IC_TBS if table <= IC_BYTES else GATHER_PEAK_BEYOND_TBS
        ach = 128.0 * lines / (ms * 1e-3) / 1e12
        return {"bound": "gather", "achieved": ach, "peak": peak, "unit": "TB/s", "frac": ach / peak,
                "kernel": "gram_sparse_kernel (upper tiles alone)", "kernel_ms": ms,
                "lines_gathered": lines, "line_bytes_gathered": 128 * lines, "record_bytes_gathered": rec_bytes,
                "record_TBps": rec_bytes / (ms * 1e-3) / 1e12, "table_bytes": table,
                "peak_source": ("MI355X_MICROARCH.md 'Indexed rows': " +
                                ("38 MB table, uniformly random rows, Infinity Cache: 8.6 TB/s" if table <= IC_BYTES else
                                 "151 MB table 7.4-7.9 TB/s, past 256 MiB 3-9 % slower: 7.4 TB/s taken")),
                "model": "bucket (band b, column k) read by the entries of column k in bands <= b; 128-B lines "
                         "of its 12-B record pairs (line-aligned buckets, or the lines a packed bucket spans)"}
    except Exception as exc:  # noqa: BLE001  (a side leg: reported, never at the cost of the line)
        return {"error": f"{type(exc).__name__}: {exc}"}


def rank_turns_gram_ms(eng, fr, pl, K, coll: bool, rank: int, world: int, reps: int = 3) -> float:
    """This rank's K assembly (from front `fr`) timed alone: the ranks take turns between barriers, so
    on a shared GPU (gloo rehearsal) no other rank's kernels run beside it.  The all-reduce mode's
    collective needs every rank and is not re-run (0).  HIP events on this rank's stream."""
    import torch
    import torch.distributed as dist

    from grf_amd import pipeline as P

    ms = float("inf")
    for _round in range(2):  # (two rounds of turns, the faster kept: the first turn may meet a cold clock)
        for turn in range(world):
            if coll:
                dist.barrier()
            if turn == rank and pl.mode != "allreduce":
                P.k_assembly(eng, fr, pl, K)  # (warm)
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
                for _ in range(reps):
                    P.k_assembly(eng, fr, pl, K)
                ev[1].record()
                ev[1].synchronize()
                ms = min(ms, ev[0].elapsed_time(ev[1]) / reps)
            torch.cuda.synchronize()
    if coll:
        dist.barrier()
    return ms if ms != float("inf") else 0.0


def time_transfers(A, K, pl, dev, ms_per_step: float, reps: int = 3) -> dict:
    """The drop-in boundary's host hand-over, timed apart from the device-resident step (SURVEY.md
    §8d): H2D of the CSR adjacency (DeviceCSR.from_scipy: indptr, indices, data) and D2H of this
    rank's K block into pinned host memory (one async copy on a side stream, HIP events)."""
    import torch

    from grf_amd import pipeline as P
    from grf_amd.engine import DeviceCSR

    h2d = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        DeviceCSR.from_scipy(A, dev)
        torch.cuda.synchronize()
        h2d.append(1000.0 * (time.perf_counter() - t0))
    Kv = P.k_view(K, pl)
    nbytes = Kv.numel() * Kv.element_size()
    try:
        host = torch.empty(K.shape, dtype=K.dtype, pin_memory=True)
        pinned = True
    except RuntimeError:
        host = torch.empty(K.shape, dtype=K.dtype)
        pinned = False
    d2h = []
    for _ in range(2):
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
        host.copy_(K, non_blocking=pinned)
        ev[1].record()
        ev[1].synchronize()
        d2h.append(ev[0].elapsed_time(ev[1]))
    h2d_ms, d2h_ms = min(h2d), min(d2h)
    total = ms_per_step + h2d_ms + d2h_ms
    return {"h2d_adjacency_ms": h2d_ms, "h2d_adjacency_bytes": int(A.indptr.nbytes + A.indices.nbytes + A.data.nbytes),
            "d2h_k_ms": d2h_ms, "d2h_k_bytes": int(K.numel() * K.element_size()), "d2h_k_logical_bytes": int(nbytes),
            "d2h_GBps": K.numel() * K.element_size() / (d2h_ms * 1e-3) / 1e9, "pinned": pinned,
            "pcie_inclusive_ms_per_step": total,
            "note": "serial sum: device-resident step + H2D of A + D2H of the whole K buffer (ldk-padded rows); "
                    "reported beside `value`, never as it"}


def host_threads() -> int:
    """All host CPU the process is granted (the reference's pool defaults to os.cpu_count() workers):
    the CPUs it may run on, capped by the cgroup's CPU quota.  The GPU box shows 256 logical CPUs
    but grants a quota of 16 (cpu.max 1600000 100000, profiles/r02_host_cpu.txt); 256 threads there
    are throttled to 16 CPUs' time and run the oracle 25 % slower than 16 threads."""
    env = int(os.environ.get("GRF_CPU_THREADS", "0") or 0)
    if env:
        return env
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def host_cpu_note() -> str:
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = None
    try:
        quota = open("/sys/fs/cgroup/cpu.max").read().strip()
    except OSError:
        quota = "n/a"
    return f"os.cpu_count()={os.cpu_count()}, affinity={aff}, cgroup cpu.max={quota}"


def mfma_leg(eng, args, steps: int = 20, workload: str = "c3"):
    """MFMA utilisation of the Phi Phi^T kernel on the dense path (C3: Cora; C2: ER N = 10k; the
    reference's dense graph_kernels/fast_grf_kernel_general.py:11-39; the north star puts MFMA only
    on the dense contraction): grf_gram_dense (tiles + split-K combine / mirror) timed with HIP
    events over `steps` launches."""
    import torch

    from grf_amd import _lib as C

    W, wdesc, _ = dense_workload(workload)
    n, m, L, p = W.shape[0], args.walks, args.length, args.p_halt
    f = diffusion_modulator(L, 1.0)
    G = eng.walk_matrix_dense(W, C.LAP_NUMPY)  # (host W: nnz counted on the host)
    dense = eng.densify_padded(eng.walk_phi(G, m, p, L, f, seed=42, norm=C.NORM_DIV, want64=False))
    del G, W
    flops = 1.0 * n * (n + 1) * n
    # the split path's operand as the bench's front leaves it: the bf16 planes where the planes path runs
    planes = eng.split_planes(dense, n) if eng.use_planes(n) else None

    def time_gram(prec):
        op = planes if prec == "split" and planes is not None else dense
        for _ in range(3):
            eng.gram_dense(op, n, precision=prec)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(steps):
            eng.gram_dense(op, n, precision=prec)
        ev[1].record()
        ev[1].synchronize()
        return ev[0].elapsed_time(ev[1]) / steps

    prec = args.gram_precision or eng.dense_precision
    out = dense_gram_roofline(prec, flops, time_gram(prec))
    out["workload"] = (f"{wdesc} dense path, m={m}, L={L}: K = Phi Phi^T of the dense fp32 Phi "
                       f"(N (N+1) N flops: the unique entries of the symmetric product)")
    if prec != "fp32":
        # the fp32 matrix instruction's kernel on the same operand, for comparison
        f32 = dense_gram_roofline("fp32", flops, time_gram("fp32"))
        out["fp32_path"] = {k: f32[k] for k in ("kernel_ms", "achieved", "peak", "frac", "kernel")}
    return out


if __name__ == "__main__":
    main()
