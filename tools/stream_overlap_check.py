"""Do two torch streams run kernels concurrently on this GPU?  _sleep kernels on main + side."""
import time

import torch

dev = torch.device("cuda:0")
main = torch.cuda.current_stream(dev)
side = torch.cuda.Stream(dev)
cyc = 200_000_000  # ~0.1 s at ~2 GHz
torch.cuda._sleep(1000)
torch.cuda.synchronize()
t = time.perf_counter()
torch.cuda._sleep(cyc)
torch.cuda.synchronize()
one = time.perf_counter() - t
t = time.perf_counter()
torch.cuda._sleep(cyc)
with torch.cuda.stream(side):
    torch.cuda._sleep(cyc)
torch.cuda.synchronize()
two = time.perf_counter() - t
print(f"one sleep {one*1e3:.1f} ms, two streams {two*1e3:.1f} ms -> {'concurrent' if two < 1.5 * one else 'SERIALISED'}",
      flush=True)
