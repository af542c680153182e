"""Timing experiment: lsmblk_crc32_batch over 1 Mi synthetic ~4 KiB blocks (4.2 GB resident),
for the library named by LSMBLK_SO_OVERRIDE (tools/var_build.sh variants)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from lsm_amd import batch  # noqa: E402


def main():
    nblk = 1 << 20
    g = torch.Generator().manual_seed(5)
    sizes = torch.randint(3900, 4097, (nblk,), generator=g, dtype=torch.int64)
    off = torch.zeros(nblk + 1, dtype=torch.int64)
    off[1:] = torch.cumsum(sizes, 0)
    blocks = torch.randint(0, 256, (int(off[-1]),), dtype=torch.uint8, device="cuda")
    d_off = off.cuda()
    crc = torch.empty(nblk, dtype=torch.int32, device="cuda")
    stats = torch.zeros(16, dtype=torch.int64, device="cuda")
    for _ in range(3):
        batch.crc32_into(blocks, d_off, nblk, crc, stats)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        batch.crc32_into(blocks, d_off, nblk, crc, stats)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 10
    print(f"{os.path.basename(os.environ.get('LSMBLK_SO_OVERRIDE', 'base'))}: {ms:.3f} ms  {int(off[-1]) / ms / 1e6:.0f} GB/s")


if __name__ == "__main__":
    main()
