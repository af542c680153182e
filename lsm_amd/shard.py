"""Multi-GPU sharding of the block path.

Two shapes:
  * block-parallel (bench.py configs U / Z / M): every rank owns a contiguous range of blocks or
    segments; blocks decode and segments (SSTs) encode independently, so there is no data-path
    collective -- only the timing barrier and a max-reduce of the elapsed time.
  * compaction-shaped (bench.py config C at N > 1): the L0 -> L1 compaction split by user-key range,
    one range per rank, with output byte-identical to the single-stream compact_generate_sst
    (reference src/compact.rs:223-311), SST boundaries included.  Three small exchanges:
      1. splitters: every rank contributes key samples of the input blocks it holds (BlockMeta first
         keys, src/table.rs:22-26, host-visible without decoding); one all-gather, and every rank
         derives the same world-1 splitters.  Blocks straddling a splitter are read by both
         neighbours; the merge keeps only the rank's own keys (lsmblk_compact_merge_batch's range).
      2. halo: every rank all-gathers the head of its kept stream -- the first
         lsmblk_shard_halo_entries(block_size) entries, enough to finish any block that starts
         before the next range.  A rank appends the heads of the ranks after it to its own stream.
      3. carry: the SST rotation's state entering each range -- the open SST's next block start and
         data-section size, 16 bytes -- goes rank to rank (send / recv), each rank turning its
         carry-in into its carry-out with one tiny kernel (lsmblk_shard_rotation_carry) after the
         carry-independent rotation work has run everywhere at once.
    Bulk KV data never moves between GPUs: the halo is a few KiB, the carry 16 bytes.

Works with any torch.distributed backend ("nccl" = RCCL on ROCm, "gloo" on CPU).  The device work
is liblsmblk.so's; RangeShard is its host-side driver, and the exchange drivers (compact_local,
compact_dist) only move the small messages above.
"""
import bisect
import struct

import numpy as np
import torch
import torch.distributed as dist

from . import batch
from ._lib import (LSMBLK_MERGE_RUNS, LSMBLK_MERGE_TWO_LEVEL, LSMBLK_TWO_END_ABOVE, LSMBLK_TWO_END_BELOW,
                   LSMBLK_TWO_END_IN_RANGE, LsmBlkError, lib)


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


# ---------------------------------------------------------------------------------------------
# splitters
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


def exchange_splitters(first_keys, samples: int = 64, max_key_bytes: int = 64, device=None, ranges: int = None):
    """All-gather every rank's key samples (fixed-size records in one tensor) and return
    the common splitters: ranges - 1 of them (default: one range per rank).  Keys longer than
    max_key_bytes are truncated for the sample, which only moves a splitter (any byte string
    splits the key space)."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    nr = ranges or world
    mine = sample_first_keys(first_keys, samples)
    if world == 1:
        return choose_splitters(mine, nr)
    rec = 2 + max_key_bytes
    payload = bytearray(_pack_keys(mine, max_key_bytes))
    payload += b"\0" * (rec * samples - len(payload))
    count = torch.tensor([len(mine)], dtype=torch.int64, device=device)
    t = torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(device)
    counts = [torch.zeros_like(count) for _ in range(world)]
    dist.all_gather(counts, count)
    bufs = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(bufs, t)
    allk = []
    for c, b in zip(counts, bufs):
        allk += _unpack_keys(bytes(b.cpu().numpy()[:int(c.item()) * rec]), max_key_bytes)
    return choose_splitters(allk, nr)


def owner_of(key: bytes, splitters) -> int:
    """Rank owning `key` under the splitters (rank i owns [s_{i-1}, s_i))."""
    return bisect.bisect_right(splitters, key)


def range_of(rank: int, splitters):
    """(lo, hi) key bounds of a rank (None: unbounded)."""
    lo = splitters[rank - 1] if rank > 0 else None
    hi = splitters[rank] if rank < len(splitters) else None
    return lo, hi


# ---------------------------------------------------------------------------------------------
# halo: the heads of the kept streams
def halo_entries(block_size: int) -> int:
    return int(lib().lsmblk_shard_halo_entries(block_size))


class Head:
    """The first h <= W kept entries of a range (of n in all): relative offsets int64[h+1], ts
    int64[h], key / value bytes, and (two-level merges) the loop's same_as_last_key uint8[h] --
    tensors on the exchange's device."""

    def __init__(self, n, ko, vo, ts, keys, vals, ks=None):
        self.n, self.ko, self.vo, self.ts, self.keys, self.vals = n, ko, vo, ts, keys, vals
        self.ks = ks if ks is not None else torch.zeros(ts.numel(), dtype=torch.uint8, device=ts.device)

    @property
    def h(self):
        return self.ts.numel()

    def to(self, device):
        return Head(self.n, self.ko.to(device), self.vo.to(device), self.ts.to(device), self.keys.to(device),
                    self.vals.to(device), self.ks.to(device))


def assemble_halo(heads, g: int, W: int):
    """Rank g's halo: the first W entries after its range, from the heads of the ranks after it
    (a short range contributes all of its entries and the next one continues).  Returns (keys,
    ko, vals, vo, ts, last, ks): `last` when the halo reaches the end of the whole stream, ks the
    entries' same_as_last_key (two-level merges)."""
    need, parts, taken, remaining = W, [], 0, sum(h.n for h in heads[g + 1:])
    for hd in heads[g + 1:]:
        if need == 0:
            break
        t = min(need, hd.h)
        if t:
            parts.append((hd, t))
        need -= t
        taken += t
    dev = heads[g].ts.device
    kb = [hd.keys[:int(hd.ko[t])] for hd, t in parts]
    vb = [hd.vals[:int(hd.vo[t])] for hd, t in parts]
    ko, vo, kbase, vbase = [torch.zeros(1, dtype=torch.int64, device=dev)], [torch.zeros(1, dtype=torch.int64,
                                                                                         device=dev)], 0, 0
    for hd, t in parts:
        ko.append(hd.ko[1:t + 1] + kbase)
        vo.append(hd.vo[1:t + 1] + vbase)
        kbase += int(hd.ko[t])
        vbase += int(hd.vo[t])
    cat = (lambda xs, dt: torch.cat(xs) if xs else torch.zeros(0, dtype=dt, device=dev))
    return (cat(kb, torch.uint8), torch.cat(ko), cat(vb, torch.uint8), torch.cat(vo),
            cat([hd.ts[:t] for hd, t in parts], torch.int64), taken == remaining,
            cat([hd.ks[:t] for hd, t in parts], torch.uint8))


def two_end_mode(kb, lo, hi):
    """Where b's last key kb (None: b empty everywhere) lies relative to the range [lo, hi): the
    LSMBLK_TWO_END_* of lsmblk_compact_merge_batch_ex (two-level merges)."""
    if kb is None or (lo is not None and kb < lo):
        return LSMBLK_TWO_END_BELOW
    if hi is not None and kb >= hi:
        return LSMBLK_TWO_END_ABOVE
    return LSMBLK_TWO_END_IN_RANGE


def _u32_as_i32(x: torch.Tensor) -> torch.Tensor:
    """int64 values in [0, 2^32) -> their u32 bit pattern in an int32 tensor."""
    x = x & 0xFFFFFFFF
    return torch.where(x >= (1 << 31), x - (1 << 32), x).to(torch.int32)


# ---------------------------------------------------------------------------------------------
class RangeShard:
    """One key range of a compaction on one device: the decoded input runs (kv, run_start), the
    compaction options (batch.compact_opts) and the range [lo, hi) (None: unbounded).  Phases:
    merge() -> head() -> set_halo() -> prepare() -> carry() -> encode() -> result(); buffers are kept
    for the next call with the same sizes (the bench's timed loop allocates nothing).  Every shard
    owns its library context (which holds the rotation state between prepare, carry and encode),
    so several shards can share one stream; `stream` defaults to the device's current stream."""

    def __init__(self, kv: batch.KVStream, run_start, opts: dict, lo: bytes = None, hi: bytes = None, stream=None):
        self.dev = torch.device("cuda", batch._dev_index(kv.key_off))
        self.kv, self.opts = kv, opts
        self.stream = stream if stream is not None else torch.cuda.current_stream(self.dev)
        self.ctx = batch.OwnCtx(self.dev.index)
        self.two = opts.get("merge_mode", LSMBLK_MERGE_RUNS) == LSMBLK_MERGE_TWO_LEVEL
        self.lo, self.hi = (bytes(lo) if lo is not None else None), (bytes(hi) if hi is not None else None)
        self.two_end = LSMBLK_TWO_END_IN_RANGE  # two-level: set from the whole compaction's b end (set_b_end)
        self.rs = batch._u32_table(run_start, self.dev)
        self.nrun = self.rs.numel() - 1
        self.bs, self.target = opts["block_size"], opts["target_sst_size"]
        self.W = halo_entries(self.bs)
        self._lo = self._bound(lo)
        self._hi = self._bound(hi)
        self.range_c = batch.key_range_c(self._lo, self._hi)
        # the input's capacities bound the kept stream (the input may not be decoded yet)
        self.n_in, self.K_in, self.V_in = kv.key_off.numel() - 1, kv.keys.numel(), kv.vals.numel()
        self.kept = None
        self.mstats = torch.zeros(5, dtype=torch.int64, device=self.dev)
        self.cout = torch.zeros(2, dtype=torch.int64, device=self.dev)
        self.estats = torch.zeros(8, dtype=torch.int64, device=self.dev)
        self.out = None
        self._grow_kept(self.n_in + self.W, self.K_in + 64 * self.W, self.V_in + 256 * self.W)

    def _bound(self, b):
        if b is None:
            return None
        return torch.frombuffer(bytearray(bytes(b) or b"\0"), dtype=torch.uint8)[:len(b)].to(self.dev)

    def _grow_kept(self, n, kb, vb, keep=0):
        old, old_ks = self.kept, getattr(self, "ks", None)
        self.kept = batch.KVStream.empty(n, kb, vb, self.dev)
        self.ks = torch.zeros(n + 1, dtype=torch.uint8, device=self.dev)  # same_as_last_key (two-level)
        if old_ks is not None and keep:
            self.ks[:keep].copy_(old_ks[:keep])
        if old is not None and keep:  # the first `keep` entries survive a regrow
            self.kept.keys[:self.Kk].copy_(old.keys[:self.Kk])
            self.kept.vals[:self.Vk].copy_(old.vals[:self.Vk])
            self.kept.key_off[:keep + 1].copy_(old.key_off[:keep + 1])
            self.kept.val_off[:keep + 1].copy_(old.val_off[:keep + 1])
            self.kept.ts[:keep].copy_(old.ts[:keep])

    # -- phase 0 (two-level merges): where the whole compaction's b ends
    def b_end(self):
        """The last key of this range's input b run (run nrun - 1), or None if it holds none: the
        maximum over the ranges is b's last key over the whole compaction."""
        if self.dev.type == "cuda":
            self.stream.synchronize()  # the input may have been decoded on the shard's stream
        a, b = int(self.rs[self.nrun - 1].item()) & 0xFFFFFFFF, int(self.rs[self.nrun].item()) & 0xFFFFFFFF
        if b <= a:
            return None
        k0, k1 = [int(x) & 0xFFFFFFFF for x in self.kv.key_off[b - 1:b + 1].cpu().tolist()]
        return bytes(self.kv.keys[k0:k1].cpu().numpy())

    def set_b_end(self, kb):
        self.two_end = two_end_mode(kb, self.lo, self.hi)

    # -- phase 1: merge + rules + range
    def merge(self):
        with torch.cuda.stream(self.stream):
            return self._merge()

    def _merge(self):
        k = self.kept
        k.n = 0
        batch.compact_merge_into(self.kv, self.rs, self.nrun, self.opts, self.range_c, k, self.mstats, self.stream,
                                 ctx=self.ctx, two_end=self.two_end, kept_same=self.ks if self.two else None)
        torch.cuda.synchronize(self.dev)
        s = self.mstats.cpu().tolist()
        st = lib().lsmblk_stats_status(s[3] & 0xFFFFFFFFFFFFFFFF)
        if st:
            raise LsmBlkError(st, "compact_merge")
        self.m, self.Kk, self.Vk, self.merged = s[0], s[1], s[2], s[4]
        k.n = self.m
        return self.m

    # -- phase 2: halo
    def head(self) -> Head:
        with torch.cuda.stream(self.stream):
            hd = self._head()
        self.stream.synchronize()  # the head is read on other streams (the exchange)
        return hd

    def _head(self) -> Head:
        h = min(self.W, self.m)
        ko = self.kept.key_off[:h + 1].to(torch.int64) & 0xFFFFFFFF
        vo = self.kept.val_off[:h + 1].to(torch.int64) & 0xFFFFFFFF
        kb, vb = (int(ko[h]), int(vo[h])) if h else (0, 0)
        return Head(self.m, ko, vo, self.kept.ts[:h].clone(), self.kept.keys[:kb].clone(), self.kept.vals[:vb].clone(),
                    self.ks[:h].clone())

    def set_halo(self, keys, ko, vals, vo, ts, last: bool, ks=None):
        self.stream.wait_stream(torch.cuda.current_stream(self.dev))  # the halo was assembled there
        with torch.cuda.stream(self.stream):
            self._set_halo(keys, ko, vals, vo, ts, last, ks)
        self.stream.synchronize()  # the halo tensors may be freed by the caller right after

    def _set_halo(self, keys, ko, vals, vo, ts, last: bool, ks=None):
        m, h = self.m, ts.numel()
        Kh, Vh = keys.numel(), vals.numel()
        ecap, kcap, vcap = self.kept.caps()
        if m + h > ecap or self.Kk + Kh + 16 > kcap or self.Vk + Vh + 16 > vcap:
            self._grow_kept(max(ecap, m + h), max(kcap, self.Kk + Kh + 16), max(vcap, self.Vk + Vh + 16), keep=m)
        k = self.kept
        if Kh:
            k.keys[self.Kk:self.Kk + Kh].copy_(keys.to(self.dev))
        if Vh:
            k.vals[self.Vk:self.Vk + Vh].copy_(vals.to(self.dev))
        if h:
            k.key_off[m + 1:m + 1 + h].copy_(_u32_as_i32(ko[1:].to(self.dev) + self.Kk))
            k.val_off[m + 1:m + 1 + h].copy_(_u32_as_i32(vo[1:].to(self.dev) + self.Vk))
            k.ts[m:m + h].copy_(ts.to(self.dev))
            if ks is not None:
                self.ks[m:m + h].copy_(ks.to(self.dev))
        self.h, self.Kh, self.Vh, self.last = h, Kh, Vh, bool(last)
        self.ext = batch.KVStream(k.keys, k.key_off, k.vals, k.val_off, k.ts, m + h)

    # -- phase 3: carry-independent rotation
    def prepare(self):
        n = self.m + self.h
        self.sst_cap = (self.Kk + self.Vk + self.Kh + self.Vh + 22 * n) // self.target + 3
        batch.shard_prepare(self.ext, self.m, self.last, self.bs, self.target, self.sst_cap, self.stream, ctx=self.ctx,
                            ext_same=self.ks if self.two else None)

    # -- phase 4: carry
    def carry(self, carry_in: torch.Tensor) -> torch.Tensor:
        self.carry_in = carry_in
        batch.shard_carry(carry_in, self.cout, self.stream, ctx=self.ctx)
        return self.cout

    # -- phase 5: SST cut points + blocks
    def encode(self):
        with torch.cuda.stream(self.stream):
            self._encode()

    def _encode(self):
        n = self.ext.n
        out_cap = self.Kk + self.Vk + self.Kh + self.Vh + 18 * n + 16
        blk_cap, seg_cap = n + 2, self.sst_cap + 3
        if self.out is None or self.out.numel() < out_cap or self.blk_off.numel() < blk_cap or \
                self.seg.numel() < seg_cap:
            self.out = batch._aligned_empty(out_cap, self.dev)
            self.blk_off = torch.zeros(blk_cap, dtype=torch.int64, device=self.dev)
            self.seg = torch.zeros(seg_cap, dtype=torch.int32, device=self.dev)
            self.seg_blk = torch.zeros(seg_cap, dtype=torch.int32, device=self.dev)
        batch.shard_encode_into(self.ext, self.out, out_cap, self.blk_off, blk_cap, self.seg, self.seg_blk, seg_cap,
                                self.estats, self.stream, ctx=self.ctx)

    def result(self):
        """Host view of the range's output (synchronizes): blocks, blk_off, seg_start (ext entry
        indices, nseg+1), seg_blk, and whether the first / last segment continue an SST of the
        previous / next range."""
        torch.cuda.synchronize(self.dev)
        s = self.estats.cpu().tolist()
        st = lib().lsmblk_stats_status(s[3] & 0xFFFFFFFFFFFFFFFF)
        if st:
            raise LsmBlkError(st, "shard_encode")
        nblk, nbytes, nseg = s[0], s[1], s[2]
        return dict(blocks=self.out[:nbytes], blk_off=self.blk_off[:nblk + 1],
                    seg_start=self.seg[:nseg + 1].cpu().numpy().view(np.uint32) if nseg else np.zeros(0, np.uint32),
                    seg_blk=self.seg_blk[:nseg + 1].cpu().numpy().view(np.uint32) if nseg else np.zeros(0, np.uint32),
                    nblk=nblk, nbytes=nbytes, nseg=nseg, first_continues=bool(s[4]), last_continues=bool(s[5]),
                    first=s[6], end=s[7], m=self.m, merged=self.merged,
                    carry_in=tuple(self.carry_in.cpu().tolist()), carry_out=tuple(self.cout.cpu().tolist()))


def sst_starts(results, bases):
    """Global kept-entry index of every SST start, from the ranges' results in key order (bases =
    each range's first global kept index)."""
    starts = []
    for r, base in zip(results, bases):
        if r["nseg"] == 0:
            continue
        first = 1 if r["first_continues"] else 0
        starts += [base + int(x) for x in r["seg_start"][first:-1]]
    return starts


# ---------------------------------------------------------------------------------------------
# exchange drivers
def compact_local(shards):
    """Every range of the compaction in this process (in key order), e.g. several ranges on one
    GPU: the same phases and messages as compact_dist, passed in memory."""
    if shards and shards[0].two:  # two-level: b's last key over the whole compaction
        ends = [e for e in (s.b_end() for s in shards) if e is not None]
        for s in shards:
            s.set_b_end(max(ends) if ends else None)
    for s in shards:
        s.merge()
    heads = [s.head() for s in shards]
    for g, s in enumerate(shards):
        h = assemble_halo(heads, g, s.W)
        s.set_halo(*h[:6], ks=h[6])
    for s in shards:
        s.prepare()
    c = torch.zeros(2, dtype=torch.int64, device=shards[0].dev) if shards else None
    for s in shards:
        torch.cuda.synchronize(s.dev)   # the carry-in may come from another shard's stream
        with torch.cuda.stream(s.stream):
            c = s.carry(c).clone()
    for s in shards:
        s.encode()
    return [s.result() for s in shards]


def _allgather_heads(head: Head, group=None):
    """All-gather every rank's head: one int64 meta all-gather, then one padded byte buffer."""
    world = dist.get_world_size(group)
    dev = head.ts.device
    meta = torch.tensor([head.n, head.h, head.keys.numel(), head.vals.numel()], dtype=torch.int64, device=dev)
    metas = [torch.zeros_like(meta) for _ in range(world)]
    dist.all_gather(metas, meta, group=group)
    metas = [m.cpu().tolist() for m in metas]
    H = max(m[1] for m in metas)
    KB = max(m[2] for m in metas)
    VB = max(m[3] for m in metas)

    def pad(t, n):
        out = torch.zeros(n, dtype=t.dtype, device=dev)
        out[:t.numel()].copy_(t)
        return out
    buf = torch.cat([pad(head.ko, H + 1).view(torch.uint8), pad(head.vo, H + 1).view(torch.uint8),
                     pad(head.ts, max(H, 1)).view(torch.uint8), pad(head.keys, max(KB, 1)),
                     pad(head.vals, max(VB, 1)), pad(head.ks, max(H, 1))])
    bufs = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(bufs, buf, group=group)
    heads = []
    o1 = 8 * (H + 1)
    o2, o3 = 2 * o1, 2 * o1 + 8 * max(H, 1)
    o4 = o3 + max(KB, 1)
    o5 = o4 + max(VB, 1)
    for (n, h, kb, vb), b in zip(metas, bufs):
        heads.append(Head(n, b[:o1].view(torch.int64)[:h + 1], b[o1:o2].view(torch.int64)[:h + 1],
                          b[o2:o3].view(torch.int64)[:h], b[o3:o3 + kb], b[o4:o4 + vb], b[o5:o5 + h]))
    return heads


def _allgather_bytes(items, cdev, group=None):
    """All-gather every rank's list of byte strings (or None), in rank order: lengths, then one
    padded byte buffer (exact keys, unlike the sampled splitter exchange)."""
    world = dist.get_world_size(group)
    lens = torch.tensor([-1 if x is None else len(x) for x in items], dtype=torch.int64, device=cdev)
    all_lens = [torch.zeros_like(lens) for _ in range(world)]
    dist.all_gather(all_lens, lens, group=group)
    all_lens = [x.cpu().tolist() for x in all_lens]
    L = max([max(0, v) for ls in all_lens for v in ls] + [1])
    buf = torch.zeros(len(items) * L, dtype=torch.uint8)
    for i, x in enumerate(items):
        if x:
            buf[i * L:i * L + len(x)] = torch.frombuffer(bytearray(x), dtype=torch.uint8)
    buf = buf.to(cdev)
    bufs = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(bufs, buf, group=group)
    out = []
    for ls, b in zip(all_lens, bufs):
        b = b.cpu()
        for i, v in enumerate(ls):
            out.append(None if v < 0 else bytes(b[i * L:i * L + v].numpy()))
    return out


def compact_dist(shard, group=None):
    """Key ranges over torch.distributed, rank order = key order: one RangeShard per rank, or a list
    of R shards per rank (the same R on every rank; rank r holds ranges r*R .. r*R + R - 1 -- a
    compaction larger than one call's 4 GiB KV arenas).  Merge, all-gather the heads, prepare,
    carry through the rank's ranges from rank - 1 to rank + 1, encode.  Returns the result (or the
    list of results)."""
    shards = shard if isinstance(shard, (list, tuple)) else [shard]
    s0 = shards[0]
    if s0.dev.type == "cuda":
        with torch.cuda.stream(s0.stream):
            res = _compact_dist(shards, group)
    else:
        res = _compact_dist(shards, group)
    return res if isinstance(shard, (list, tuple)) else res[0]


def comm_device(device, group=None):
    """Where a collective's tensors live: the GPU for RCCL, the host for gloo."""
    return torch.device("cpu") if dist.get_backend(group) == "gloo" else torch.device(device)


def _compact_dist(shards, group):
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    R = len(shards)
    cdev = comm_device(shards[0].dev, group)
    if getattr(shards[0], "two", False):  # two-level: b's last key over the whole compaction
        ends = [e for e in _allgather_bytes([s.b_end() for s in shards], cdev, group) if e is not None]
        for s in shards:
            s.set_b_end(max(ends) if ends else None)
    for s in shards:
        s.merge()
    # one all-gather per local range index: heads[r * R + i] = rank r's range i
    per = [_allgather_heads(s.head().to(cdev), group) for s in shards]
    heads = [per[i][r] for r in range(world) for i in range(R)]
    for i, s in enumerate(shards):
        halo = assemble_halo(heads, rank * R + i, s.W)
        s.set_halo(*[x.to(s.dev) for x in halo[:5]], halo[5], ks=halo[6].to(s.dev))
        s.prepare()
    cin = torch.zeros(2, dtype=torch.int64, device=cdev)
    if rank > 0:
        dist.recv(cin, src=rank - 1, group=group)
    c = cin.to(shards[0].dev)
    for s in shards:
        if s.dev.type == "cuda":
            torch.cuda.synchronize(s.dev)   # the carry-in may come from another range's stream
            with torch.cuda.stream(s.stream):  # the carry kernel and its copy on the shard's stream
                c = s.carry(c.to(s.dev)).clone()
        else:
            c = s.carry(c.to(s.dev)).clone()
    if shards[-1].dev.type == "cuda":
        shards[-1].stream.synchronize()     # the carry-out is read on the exchange's stream
    if rank + 1 < world:
        dist.send(c.to(cdev), dst=rank + 1, group=group)
    for s in shards:
        s.encode()
    return [s.result() for s in shards]
