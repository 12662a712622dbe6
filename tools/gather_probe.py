"""Probe: random-gather rate vs table size (does the 256 MB MALL serve random 8/16-B gathers
faster than HBM?).  torch index_select of 10 M random rows from tables of 64 MB .. 1.6 GB."""
import torch

n = 10_000_000
g = torch.Generator(device="cuda").manual_seed(0)
for rowb in (16, 8):
    for mb in (32, 64, 128, 256, 512, 800, 1600):
        rows = mb * 2**20 // rowb
        t = torch.zeros((rows, rowb // 8), dtype=torch.float64, device="cuda")
        idx = torch.randint(0, rows, (n,), device="cuda", generator=g)
        out = torch.empty((n, rowb // 8), dtype=torch.float64, device="cuda")
        for _ in range(3):
            torch.index_select(t, 0, idx, out=out)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            torch.index_select(t, 0, idx, out=out)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        print("row %2d B table %5d MB: %.4f ms per 10 M gathers (%.1f G/s)" % (rowb, mb, ms, n / ms / 1e6), flush=True)
        del t, idx, out
