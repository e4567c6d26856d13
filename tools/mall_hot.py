"""Does the Infinity Cache (MALL) keep what a kernel just wrote?  Times a read of a buffer right
after writing it (hot) against the same read after a 2 GiB write to another buffer (cold), for
buffer sizes around the 256 MB MALL.  Decides whether a mirror pass that trails the Gram tiles
closely could read the upper triangle from the MALL instead of HBM.
usage: python tools/mall_hot.py  (one JSON line per size)"""
import json

import torch


def main():
    dev = torch.device("cuda:0")
    flush = torch.empty(512 << 20, dtype=torch.float32, device=dev)  # 2 GiB
    out = torch.empty(1 << 28, dtype=torch.float32, device=dev)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for mb in (32, 64, 128, 192, 256, 512, 1024):
        n = (mb << 20) // 4
        x = torch.empty(n, dtype=torch.float32, device=dev)
        res = {"mb": mb}
        for mode in ("hot", "cold", "hot", "cold"):
            x.fill_(1.0)
            if mode == "cold":
                flush.fill_(2.0)
            s.record()
            x.sum()  # read only
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e)
            res.setdefault(mode, []).append(round((mb << 20) / ms / 1e9, 3))  # TB/s
        # read-then-write (mirror-like): copy x -> out
        for mode in ("hot_copy", "cold_copy"):
            x.fill_(1.0)
            if mode == "cold_copy":
                flush.fill_(2.0)
            s.record()
            out[:n].copy_(x)
            e.record()
            torch.cuda.synchronize()
            res[mode] = round(2 * (mb << 20) / s.elapsed_time(e) / 1e9, 3)  # TB/s read + written
        print(json.dumps(res), flush=True)
        del x


if __name__ == "__main__":
    main()
