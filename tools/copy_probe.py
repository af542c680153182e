"""Calibration (not product code): device-to-device copy rate of this GPU for the roofline
discussion -- torch's copy kernel and a read-only reduction over the same 4.2 GB."""
import torch

n = 4_226_189_427
a = torch.empty(n, dtype=torch.uint8, device="cuda")
b = torch.empty(n, dtype=torch.uint8, device="cuda")
a.fill_(1)
for _ in range(3):
    b.copy_(a)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    b.copy_(a)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 10
print(f"copy {n / 1e9:.2f} GB: {ms:.3f} ms = {2 * n / ms / 1e6:.0f} GB/s read+write")
x = a.view(torch.int64)
for _ in range(3):
    s = x.sum()
torch.cuda.synchronize()
e0.record()
for _ in range(10):
    s = x.sum()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 10
print(f"read-only sum {n / 1e9:.2f} GB: {ms:.3f} ms = {n / ms / 1e6:.0f} GB/s")
