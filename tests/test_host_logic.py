"""CPU-only: host-side logic of the engine (no GPU calls)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def test_shard_range_partitions():
    from grf_amd.dist import shard_range
    for n in (0, 1, 7, 100, 100_000):
        for w in (1, 2, 3, 8):
            rs = [shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            sizes = [e - b for b, e in rs]
            assert max(sizes) - min(sizes) <= 1


def test_chunk_bounds_match_numpy_array_split():
    from grf_amd import _lib
    from oracle import oracle as O
    lib = _lib.load()
    for n, c in [(10, 3), (100, 8), (5, 8), (1, 1), (100_000, 192)]:
        ours = [lib.grf_chunk_bounds(n, c, i) for i in range(c)] + [n]
        ref = [int(a[0]) if len(a) else None for a in np.array_split(np.arange(n), c)]
        assert list(O.chunk_bounds(n, c)) == ours
        assert [x for x in ref if x is not None] == [ours[i] for i in range(c) if ours[i] < ours[i + 1]]


def test_rng_mode_resolution(monkeypatch):
    from grf_amd import api
    monkeypatch.delenv("GRF_AMD_RNG", raising=False)
    assert api.resolve_rng(None) == "reference"
    monkeypatch.setenv("GRF_AMD_RNG", "philox")
    assert api.resolve_rng(None) == "philox"
    with pytest.raises(ValueError):
        api.resolve_rng("mt19937")
    assert api.resolve_processes(None) == os.cpu_count()
    with pytest.raises(ValueError):
        api.resolve_processes(0)


def test_product_path_fails_loudly_without_gpu():
    """No CPU fallback: the engine refuses to run when no GPU is visible."""
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from grf_amd.engine import GRFEngine
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        GRFEngine()
    from efficient_graph_gp_sparse.graph_kernels_sparse.fast_grf_kernel_general import fast_general_grf_kernel
    import scipy.sparse as sp
    with pytest.raises(RuntimeError):
        fast_general_grf_kernel(sp.eye(4, format="csr"), [1.0, 0.5], walks_per_node=2, max_walk_length=2)


def test_mirror_packages_import():
    import efficient_graph_gp.gpflow_kernels as gk
    import efficient_graph_gp.graph_kernels as g
    import efficient_graph_gp_sparse.gptorch_kernels_sparse as tk
    import efficient_graph_gp_sparse.preprocessor as pp
    assert callable(g.fast_diffusion_grf_kernel) and callable(gk.GraphGeneralFastGRFKernel)
    assert tk.SparseGRFKernel and pp.GraphPreprocessor
    with pytest.raises(NotImplementedError):
        g.diffusion_kernel(np.eye(2))


def test_step_cache_roundtrip_without_pickle(tmp_path):
    import scipy.sparse as sp
    from efficient_graph_gp_sparse.preprocessor.graph_preprocessor import GraphPreprocessor
    mats = [sp.random(30, 30, density=0.1, random_state=i, format="csr") for i in range(3)]
    fn = str(tmp_path / "c" / "steps.npz")
    GraphPreprocessor.save_step_matrices(mats, fn)
    back = GraphPreprocessor.load_step_matrices(fn)
    for a, b in zip(mats, back):
        assert (a != b).nnz == 0
    with pytest.raises(ValueError):
        GraphPreprocessor.load_step_matrices(str(tmp_path / "x.pkl"))


# ------------------------------------------------------------- 2-rank gloo
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gather_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import scipy.sparse as sp
        from grf_amd.dist import allgather_csr_rows, shard_range
        n = 57
        full = sp.random(n, n, density=0.2, random_state=5, format="csr")
        full.sort_indices()
        b, e = shard_range(n, rank, world)
        part = full[b:e]
        ptr = torch.from_numpy(part.indptr.astype(np.int64))
        idx = torch.from_numpy(part.indices.astype(np.int32))
        val = torch.from_numpy(part.data.astype(np.float32))
        gptr, gidx, gval = allgather_csr_rows(ptr, idx, val)
        ok = (np.array_equal(gptr.numpy(), full.indptr) and np.array_equal(gidx.numpy(), full.indices)
              and np.array_equal(gval.numpy(), full.data.astype(np.float32)))
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def _allreduce_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from grf_amd.dist import allreduce_buckets
        n, ld = 37, 40
        parts = [torch.from_numpy(np.random.default_rng(r).random((n, ld), dtype=np.float32)) for r in range(world)]
        buf = parts[rank].clone()
        view = buf[:, :n]                       # row-padded like the engine's K (leading dim > n)
        allreduce_buckets(view, bucket_bytes=3 * ld * 4)   # several buckets, last one ragged
        want = sum(p[:, :n] for p in parts)
        q.put((rank, bool(torch.allclose(view, want, rtol=0, atol=1e-6))))
    finally:
        dist.destroy_process_group()


def _gather_phi_worker(rank, world, port, q):
    """gather_phi: Phi rows all-gathered and the per-rank bucket counts summed in place."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import scipy.sparse as sp
        from grf_amd.dist import gather_phi, shard_range
        from grf_amd.engine import DEFAULT_BAND_WIDTH, DeviceCSR
        n = 5000
        full = sp.random(n, n, density=0.002, random_state=7, format="csr", dtype=np.float32)
        full.sort_indices()
        b, e = shard_range(n, rank, world)
        part = full[b:e]
        local = DeviceCSR(e - b, n, torch.from_numpy(part.indptr.astype(np.int64)),
                          torch.from_numpy(part.indices.astype(np.int32)), None,
                          torch.from_numpy(part.data.astype(np.float32)), int(part.nnz))
        nbk = -(-n // DEFAULT_BAND_WIDTH) * n
        cnt = np.zeros(nbk + 16, np.int32)  # (the workspace is longer than its count head)
        rows = np.repeat(np.arange(b, e), np.diff(part.indptr))
        np.add.at(cnt, (rows // DEFAULT_BAND_WIDTH) * n + part.indices, 1)
        ws = torch.from_numpy(cnt.view(np.uint8).copy())
        phi = gather_phi(None, local, ws)
        want = np.zeros(nbk, np.int64)
        allrows = np.repeat(np.arange(n), np.diff(full.indptr))
        np.add.at(want, (allrows // DEFAULT_BAND_WIDTH) * n + full.indices, 1)
        got = ws.numpy().view(np.int32)
        ok = (np.array_equal(phi.ptr.numpy(), full.indptr) and np.array_equal(phi.idx.numpy(), full.indices)
              and np.array_equal(phi.val32.numpy(), full.data) and np.array_equal(got[:nbk], want)
              and np.array_equal(got[nbk:], cnt[nbk:]))
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def _spawn(target, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    return sorted(res)


def _bounded_gather_worker(rank, world, port, q):
    """allgather_csr_rows_bounded: uneven shards, each rank's entries in a buffer padded to its
    rows x the row capacity (as a sync-free compaction leaves them), garbage past its nnz."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import scipy.sparse as sp
        from grf_amd.dist import allgather_csr_rows_bounded, shard_bounds
        n, cap = 61, 20
        full = sp.random(n, n, density=0.15, random_state=9, format="csr")
        full.sort_indices()
        shards = shard_bounds(np.arange(1, n + 1) ** 2, world)  # uneven on purpose
        b, e = shards[rank]
        part = full[b:e]
        ptr = torch.from_numpy(part.indptr.astype(np.int64))
        idx = torch.full(((e - b) * cap,), -7, dtype=torch.int32)
        val = torch.full(((e - b) * cap,), 9e9, dtype=torch.float32)
        idx[:part.nnz] = torch.from_numpy(part.indices.astype(np.int32))
        val[:part.nnz] = torch.from_numpy(part.data.astype(np.float32))
        rows = [s1 - s0 for s0, s1 in shards]
        gptr, gidx, gval = allgather_csr_rows_bounded(ptr, idx, val, rows, max(rows) * cap)
        nnz = int(gptr[-1])
        ok = (np.array_equal(gptr.numpy(), full.indptr) and np.array_equal(gidx[:nnz].numpy(), full.indices)
              and np.array_equal(gval[:nnz].numpy(), full.data.astype(np.float32)))
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_allgather_csr_rows_bounded_gloo(world):
    assert _spawn(_bounded_gather_worker, world) == [(r, True) for r in range(world)]


def _tight_gather_worker(rank, world, port, q):
    """The exact bound (dist.shard_entries: the largest shard's entries) gathers the same CSR; one
    entry less flags the overflow (raised by check_gather_overflow on every rank) and gathers the
    overflowing rank's rows empty, with every offset inside the buffers."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import scipy.sparse as sp
        from grf_amd.dist import allgather_csr_rows_bounded, check_gather_overflow, shard_bounds
        n, cap = 61, 20
        full = sp.random(n, n, density=0.15, random_state=11, format="csr")
        full.sort_indices()
        shards = shard_bounds(np.arange(1, n + 1) ** 2, world)
        b, e = shards[rank]
        part = full[b:e]
        ptr = torch.from_numpy(part.indptr.astype(np.int64))
        idx = torch.full(((e - b) * cap,), -7, dtype=torch.int32)
        val = torch.full(((e - b) * cap,), 9e9, dtype=torch.float32)
        idx[:part.nnz] = torch.from_numpy(part.indices.astype(np.int32))
        val[:part.nnz] = torch.from_numpy(part.data.astype(np.float32))
        rows = [s1 - s0 for s0, s1 in shards]
        ents = [int(full.indptr[s1] - full.indptr[s0]) for s0, s1 in shards]
        exact = max(ents)
        gptr, gidx, gval = allgather_csr_rows_bounded(ptr, idx, val, rows, exact)
        nnz = int(gptr[-1])
        ok = (np.array_equal(gptr.numpy(), full.indptr) and np.array_equal(gidx[:nnz].numpy(), full.indices)
              and np.array_equal(gval[:nnz].numpy(), full.data.astype(np.float32)) and gidx.numel() == world * exact)
        check_gather_overflow("cpu")  # (no overflow: must not raise)
        gptr, gidx, _ = allgather_csr_rows_bounded(ptr, idx, val, rows, exact - 1)
        over = [r for r in range(world) if ents[r] > exact - 1]
        cnt = np.diff(gptr.numpy())
        for r, (s0, s1) in enumerate(shards):
            want = 0 if r in over else np.diff(full.indptr[s0:s1 + 1])
            ok = ok and np.array_equal(cnt[s0:s1], np.broadcast_to(want, (s1 - s0,)))
        ok = ok and int(gptr[-1]) <= gidx.numel()
        try:
            check_gather_overflow("cpu")
            ok = False
        except RuntimeError:
            pass
        check_gather_overflow("cpu")  # (the flag is cleared by the raise)
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_allgather_csr_rows_tight_bound_and_overflow_gloo(world):
    assert _spawn(_tight_gather_worker, world) == [(r, True) for r in range(world)]


def test_shard_bounds_equal_weight_ranges():
    from grf_amd.dist import shard_bounds
    rng = np.random.default_rng(0)
    for n, w in [(100, 2), (1000, 3), (5000, 8), (7, 8), (3, 3)]:
        wt = rng.pareto(1.5, n) + 0.1
        sh = shard_bounds(wt, w)
        assert len(sh) == w and sh[0][0] == 0 and sh[-1][1] == n
        assert all(sh[i][1] == sh[i + 1][0] for i in range(w - 1))
        if n >= w:
            assert all(e > b for b, e in sh)
            sums = np.array([wt[b:e].sum() for b, e in sh])
            # every prefix boundary is within one row's weight of its target
            for r in range(w - 1):
                target = wt.sum() * (r + 1) / w
                assert abs(wt[:sh[r][1]].sum() - target) <= wt.max() + 1e-9 or n < 4 * w
            assert sums.max() <= wt.sum() / w + 2 * wt.max()
    assert shard_bounds(np.ones(10), 1) == [(0, 10)]
    assert shard_bounds(np.ones(12), 4) == [(0, 3), (3, 6), (6, 9), (9, 12)]


@pytest.mark.parametrize("world", [2, 3])
def test_allreduce_buckets_gloo(world):
    assert _spawn(_allreduce_worker, world) == [(r, True) for r in range(world)]


@pytest.mark.parametrize("world", [2, 3])
def test_gather_phi_sums_bucket_counts_gloo(world):
    assert _spawn(_gather_phi_worker, world) == [(r, True) for r in range(world)]


@pytest.mark.parametrize("world", [2, 3])
def test_allgather_csr_rows_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert sorted(res) == [(r, True) for r in range(world)]


def test_gptorch_kernels_fail_loudly_without_gpu(golden):
    """The GPyTorch surface runs on the HIP kernels only (tests/test_gpu_features.py): on a host
    without a GPU its forward raises instead of falling back to CPU tensor algebra."""
    from golden_util import csr
    from efficient_graph_gp_sparse.gptorch_kernels_sparse import SparseGRFKernel
    from efficient_graph_gp_sparse.preprocessor import GraphPreprocessor
    from efficient_graph_gp_sparse.utils_sparse.sparse_lo import SparseLinearOperator
    d = golden("small_graphs")
    ops = [SparseLinearOperator(GraphPreprocessor.from_scipy_csr(csr(d, f"er40_sp_n3_s7_l{l}", 40))) for l in range(4)]
    kern = SparseGRFKernel(4, ops)
    with pytest.raises(RuntimeError):
        kern(torch.tensor([0, 1]), torch.tensor([2]))


def test_record_unit_choice():
    """Line-aligned buckets for dense buckets (C4), packed pairs for sparse ones (C5)."""
    from grf_amd import _lib as C
    from grf_amd.engine import choose_rec_unit
    assert choose_rec_unit(43_484_870, 100_000, 100_000, 4096) == C.REC_LINE      # C4: ~18 entries per bucket
    assert choose_rec_unit(100_000 * 1024, 100_000, 100_000, 8192) == C.REC_LINE  # C4 bound, row mode
    assert choose_rec_unit(1_000_000 * 512, 1_000_000, 1_000_000, 8192) == C.REC_PACKED  # C5 bound: ~4 entries
    assert choose_rec_unit(0, 10, 10, 64) == C.REC_PACKED


def test_powerlaw_graph_is_simple_and_heavy_tailed():
    from grf_amd.graphs import powerlaw_graph
    A = powerlaw_graph(20_000, 10.0, 2.5, seed=1)
    assert (A != A.T).nnz == 0 and A.diagonal().sum() == 0 and A.data.min() == 1.0
    deg = np.diff(A.indptr)
    assert 8.0 < deg.mean() < 10.5 and deg.max() > 20 * deg.mean()  # hubs
    assert np.array_equal(A.indices, powerlaw_graph(20_000, 10.0, 2.5, seed=1).indices)  # seeded


def test_snap_graphs_load():
    from grf_amd.graphs import snap_graph
    fb, en = snap_graph("facebook"), snap_graph("enron")
    assert fb.shape == (22470, 22470) and en.shape == (36692, 36692)
    assert (fb != fb.T).nnz == 0 and (en != en.T).nnz == 0
    with pytest.raises(ValueError):
        snap_graph("youtube")


def test_shard_entries_from_row_pointer():
    """dist.shard_entries: every shard's Phi entries from the row pointer (the exact gather bound)."""
    from types import SimpleNamespace
    from grf_amd.dist import shard_entries, shard_range
    rng = np.random.default_rng(3)
    cnt = rng.integers(0, 40, size=57)
    ptr = torch.from_numpy(np.r_[0, np.cumsum(cnt)].astype(np.int64))
    for world in (1, 2, 3, 8):
        shards = [shard_range(57, r, world) for r in range(world)]
        got = shard_entries(SimpleNamespace(ptr=ptr), shards)
        assert got == [int(cnt[b:e].sum()) for b, e in shards] and sum(got) == int(cnt.sum())


def _empty_shard_gather_worker(rank, world, port, q):
    """gather_phi with a rank that owns no rows (n < world): every rank must take the same gather path
    (the bounded one: chosen from global information -- shards and the row capacity -- not from its
    own row count), so the collectives match and the full CSR comes back on every rank."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import scipy.sparse as sp
        from grf_amd.dist import gather_phi, shard_range
        from grf_amd.engine import DeviceCSR
        n, cap = 2, 5
        full = sp.csr_matrix(np.array([[1.0, 0.0], [2.0, 3.0]]))
        shards = [shard_range(n, r, world) for r in range(world)]
        b, e = shards[rank]
        part = full[b:e]
        ptr = torch.from_numpy(np.asarray(part.indptr, np.int64))
        idx = torch.zeros(max(1, (e - b) * cap), dtype=torch.int32)
        val = torch.zeros(max(1, (e - b) * cap), dtype=torch.float32)
        idx[:part.nnz] = torch.from_numpy(part.indices.astype(np.int32))
        val[:part.nnz] = torch.from_numpy(part.data.astype(np.float32))
        local = DeviceCSR(e - b, n, ptr, idx, None, val, None)
        local.nnz_bound = (e - b) * cap
        out = gather_phi(None, local, shards=shards, row_cap=cap)
        nnz = int(out.ptr[-1])
        ok = (np.array_equal(out.ptr.numpy(), full.indptr) and np.array_equal(out.idx[:nnz].numpy(), full.indices)
              and np.array_equal(out.val32[:nnz].numpy(), full.data.astype(np.float32)))
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def test_gather_phi_empty_shard_same_path_gloo():
    assert _spawn(_empty_shard_gather_worker, 3) == [(r, True) for r in range(3)]


def test_gather_model_counts_bucket_line_visits():
    """bench.gather_model (roofline_gather): bucket (band b, column k) is read once per entry of column
    k in bands <= b (symmetric tiles) or in any band (row tiles); lines from the descriptors' pairs
    (line-aligned) or the span of a packed bucket.  Checked against a brute-force count."""
    import types

    import scipy.sparse as sp
    import torch

    import bench
    from grf_amd import _lib as C
    r = np.random.default_rng(5)
    n, W = 37, 8
    nb = -(-n // W)
    dense = (r.random((n, n)) < 0.3) * r.standard_normal((n, n))
    A = sp.csr_matrix(dense)
    phi = types.SimpleNamespace(nnz=A.nnz, n_rows=n, ptr=torch.from_numpy(A.indptr.astype(np.int64)),
                                idx=torch.from_numpy(A.indices.astype(np.int32)))
    ent = np.zeros((nb, n), np.int64)
    for i in range(n):
        for k in A.indices[A.indptr[i]:A.indptr[i + 1]]:
            ent[i // W, k] += 1
    pairs = (ent + 1) // 2
    for unit in (C.REC_LINE, C.REC_PACKED):
        first = np.zeros((nb, n), np.int64)
        pos = 0
        for b in range(nb):
            for k in range(n):
                first[b, k] = pos
                pos += -(-12 * pairs[b, k] // 128) if unit == C.REC_LINE else pairs[b, k]
        desc = np.stack([first, pairs], -1).reshape(-1).astype(np.int32)
        tr = types.SimpleNamespace(n_rows=n, n_cols=n, band_width=W, rec_unit=unit,
                                   t_desc=torch.from_numpy(np.concatenate([desc, [0, 0]]).astype(np.int32)))
        for sym in (True, False):
            want_lines = want_rec = 0
            for b in range(nb):
                for k in range(n):
                    visits = ent[:b + 1, k].sum() if sym else ent[:, k].sum()
                    if unit == C.REC_LINE:
                        lines = -(-12 * pairs[b, k] // 128)
                    else:
                        s0 = first[b, k] * 12
                        lines = (s0 + 12 * pairs[b, k] - 1) // 128 - s0 // 128 + 1 if pairs[b, k] else 0
                    want_lines += visits * lines
                    want_rec += visits * pairs[b, k] * 12
            got = bench.gather_model(phi, tr, sym=sym)
            assert got[0] == want_lines and got[1] == want_rec, (unit, sym)


def test_hub_column_policy_extension():
    """engine.column_stats: columns in >= share of the rows, in panel widths of 32; with `extend` (the split
    panel's HUB_EXTEND_SHARE) a graph that has a panel at `share` takes its columns down to `extend`, and a
    graph without one stays unsplit (Enron 96 -> 192 columns, Facebook 0)."""
    from grf_amd.engine import HUB_EXTEND_SHARE, HUB_SHARE, DeviceCSR, GRFEngine

    def csr_with_column_counts(n_rows, counts):
        cols = np.concatenate([np.full(c, k, np.int32) for k, c in enumerate(counts)])
        ptr = torch.zeros(n_rows + 1, dtype=torch.int64)
        ptr[-1] = len(cols)  # (only the column list and nnz are read)
        return DeviceCSR(n_rows, len(counts), ptr, torch.from_numpy(cols), None, None, len(cols))

    n = 1000
    # 40 columns in 14 % of the rows, 40 more in 11 %, the rest in 1 %
    counts = [140] * 40 + [110] * 40 + [10] * 200
    phi = csr_with_column_counts(n, counts)
    assert GRFEngine.column_stats(phi, HUB_SHARE)[0] == 32
    assert GRFEngine.column_stats(phi, HUB_SHARE, extend=HUB_EXTEND_SHARE)[0] == 64
    # fewer than one panel width at the gate share: no split, extension or not
    counts = [140] * 20 + [110] * 60 + [10] * 200
    phi = csr_with_column_counts(n, counts)
    assert GRFEngine.column_stats(phi, HUB_SHARE)[0] == 0
    assert GRFEngine.column_stats(phi, HUB_SHARE, extend=HUB_EXTEND_SHARE)[0] == 0
