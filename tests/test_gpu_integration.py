"""INTEGRATION.md's reference-side ctypes stub, executed as written (only the library path is made
absolute), against the engine's own walk and the oracle (the reference's PCG64 stream)."""
import os
import re

import numpy as np
import pytest
import scipy.sparse as sp

from oracle import oracle as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "efficient-gaussian-process-on-graphs_amd", "grf_amd", "libgrf_amd.so")


def _stub_source() -> str:
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = text[text.index("### The ctypes stub"):]
    code = re.search(r"```python\n(.*?)```", sec, re.S).group(1)
    assert 'ctypes.CDLL("libgrf_amd.so")' in code
    return code.replace('ctypes.CDLL("libgrf_amd.so")', f'ctypes.CDLL({LIB!r})')


def test_integration_stub_walks_match_engine_and_reference_stream():
    import torch
    from grf_amd.engine import GRFEngine

    ns = {}
    exec(compile(_stub_source(), "INTEGRATION.md", "exec"), ns)
    r = np.random.default_rng(2)
    U = sp.random(500, 500, density=0.02, random_state=r, format="csr")
    A = ((U + U.T) > 0).astype(np.float64).tocsr()
    A.setdiag(0)
    A.eliminate_zeros()
    A.sort_indices()
    Ls, _ = O.laplacian_sparse(A)
    for n_proc, seed in ((8, None), (3, 7)):
        node, load = ns["walk_slots"](Ls, 16, 0.1, 4, seed=seed, n_processes=n_proc)
        torch.cuda.synchronize()
        eng = GRFEngine("cuda:0")
        slots = eng.walk(eng.to_device(Ls), 16, 0.1, 4, rng=0, seed=seed or 42, n_chunks=n_proc)
        assert torch.equal(node, slots.node)
        used = node >= 0  # (loads of empty slots are not written)
        assert torch.equal(load[used], slots.load[used])
        on, ol = O.walk_slots(*O._csr_arrays(Ls), 16, 0.1, 4, rng=O.RNG_PCG64, n_chunks=n_proc, seed=seed or 42)
        assert np.array_equal(node.cpu().numpy(), on)
        mask = on >= 0
        assert np.array_equal(load.cpu().numpy()[mask].view(np.uint64), ol[mask].view(np.uint64))
