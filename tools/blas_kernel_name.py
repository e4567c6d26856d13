"""Which vendor kernel does torch.matmul (fp32, A A^T) dispatch at these n?  Run under rocprofv3
--kernel-trace; prints the HIP-event time per call."""
import sys
import torch
torch.backends.cuda.matmul.allow_tf32 = False
for n in [int(a) for a in sys.argv[1:]] or [10000, 16384]:
    A = torch.rand((n, n), device="cuda")
    for _ in range(2):
        C = torch.matmul(A, A.t())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        C = torch.matmul(A, A.t())
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / 5
    print(n, f"{ms:.3f} ms", f"{2 * n**3 / ms / 1e9:.1f} TF/s", flush=True)
