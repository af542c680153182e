"""Multi-GPU sharding for the block path.

Two shapes:
  * block-parallel (bench.py): every rank owns a contiguous range of blocks or segments;
    blocks decode and segments (SSTs) encode independently, so there is no data-path
    collective -- only the timing barrier and a max-reduce of the elapsed time.
  * compaction-shaped (next step): key-range sharding of L0 -> L1 batches.  The only
    exchange is the splitter keys: each rank samples the first keys of the input blocks
    it holds (BlockMeta.first_key, reference src/table.rs:22-26, 253-257: host-visible
    without decoding), the samples are all-gathered (tiny: <= world x samples x key bytes,
    latency-bound over xGMI), and every rank derives the same world-1 splitters.  Data
    never moves between GPUs; blocks straddling a splitter are read by both neighbours and
    filtered on the key range.

Works with any torch.distributed backend ("nccl" = RCCL on ROCm, "gloo" on CPU).
"""
import bisect
import struct

import torch
import torch.distributed as dist


def block_ranges(nblk: int, world: int):
    """Contiguous [lo, hi) block ranges, one per rank, sizes differing by at most one."""
    q, r = divmod(nblk, world)
    out, lo = [], 0
    for i in range(world):
        hi = lo + q + (1 if i < r else 0)
        out.append((lo, hi))
        lo = hi
    return out


def max_over_ranks(x: float, device=None) -> float:
    """Max of a scalar over all ranks (the bench's whole-job time)."""
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _pack_keys(keys, max_key_bytes):
    buf = bytearray()
    for k in keys:
        k = bytes(k)[:max_key_bytes]
        buf += struct.pack(">H", len(k)) + k.ljust(max_key_bytes, b"\0")
    return bytes(buf)


def _unpack_keys(buf, max_key_bytes):
    out, rec = [], 2 + max_key_bytes
    for i in range(0, len(buf), rec):
        (n,) = struct.unpack_from(">H", buf, i)
        out.append(bytes(buf[i + 2:i + 2 + n]))
    return out


def sample_first_keys(first_keys, samples: int):
    """Evenly spaced samples of a rank's (sorted) block first keys."""
    if not first_keys:
        return []
    n = len(first_keys)
    if n <= samples:
        return list(first_keys)
    return [first_keys[(i * n) // samples] for i in range(samples)]


def choose_splitters(all_samples, world: int):
    """world-1 splitter keys from the union of the samples (deterministic)."""
    keys = sorted(set(all_samples))
    if world <= 1 or not keys:
        return []
    return [keys[(i * len(keys)) // world] for i in range(1, world)]


def exchange_splitters(first_keys, samples: int = 64, max_key_bytes: int = 64, device=None):
    """All-gather every rank's key samples (fixed-size records in one tensor) and return
    the common splitters.  Keys longer than max_key_bytes are truncated for the sample,
    which only moves a splitter, never correctness (straddling blocks go to both ranks)."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    mine = sample_first_keys(first_keys, samples)
    rec = 2 + max_key_bytes
    payload = bytearray(_pack_keys(mine, max_key_bytes))
    payload += b"\0" * (rec * samples - len(payload))
    count = torch.tensor([len(mine)], dtype=torch.int64, device=device)
    t = torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(device)
    if world == 1:
        return choose_splitters(mine, 1)
    counts = [torch.zeros_like(count) for _ in range(world)]
    dist.all_gather(counts, count)
    bufs = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(bufs, t)
    allk = []
    for c, b in zip(counts, bufs):
        allk += _unpack_keys(bytes(b.cpu().numpy()[:int(c.item()) * rec]), max_key_bytes)
    return choose_splitters(allk, world)


def owner_of(key: bytes, splitters) -> int:
    """Rank owning `key` under the splitters (rank i owns [s_{i-1}, s_i))."""
    return bisect.bisect_right(splitters, key)
