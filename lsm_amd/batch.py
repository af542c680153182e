"""Batch (device) API: whole flush / compaction batches through the HIP kernels.

  decode_blocks  replaces SsTable::read_block -> Block::decode -> BlockIterator::next over a
                 batch of blocks (reference src/table.rs:213-233, src/table/iterator.rs:86-97)
  encode_kv      replaces SsTableBuilder::add -> BlockBuilder::add / finish_block over a batch
                 of segments (reference src/table/builder.rs:48-65,112-123)
  crc32_blocks   the per-block SST framing checksum (crc32fast::hash, reference
                 src/table/builder.rs:120-122, verified at src/table.rs:226-230)
  block_meta     the SST BlockMeta section of every segment (BlockMeta::encode_block_meta,
                 reference src/table.rs:29-63, written by SsTableBuilder::build :68-77)
  encode_sst     encode_kv + the segment -> block table + block_meta in one stream
  compact_filter compaction's keep/drop rules over a merged stream (reference
                 src/compact.rs:234-299: watermark, bottom-level tombstones, prefix filters)

Tensors live on a ROCm device (torch is only the allocator / stream provider).  The work
is done by liblsmblk.so; there is no CPU path here.
"""
import ctypes
import threading
from dataclasses import dataclass

import numpy as np
import torch

from ._lib import (CompactOptsC, KVStreamC, KeyRangeC, LSMBLK_DECODE_VERIFY_CRC, LSMBLK_E_CAPACITY,
                   LSMBLK_ENCODE_FRAMED, LSMBLK_ENCODE_SEG_SLOTS, LSMBLK_MERGE_RUNS, LSMBLK_MERGE_TWO_LEVEL, LSMBLK_SHARD_LAST, LsmBlkError, check, lib)

STATS_WORDS = 4
_ctx_lock = threading.Lock()
_ctxs = {}


class _Ctx:
    """One lsmblk_ctx per (device, stream): a context's device workspace is reused by every call
    on it, so two streams never share one (release_contexts frees them).  `lock` serialises call sequences that depend on the
    workspace between calls (encode_into -> segment_blocks_into) across host threads."""

    def __init__(self, handle):
        self.h = handle
        self.lock = threading.RLock()


def _ctx_for(device: int, stream_ptr: int) -> _Ctx:
    key = (device, stream_ptr)
    with _ctx_lock:
        c = _ctxs.get(key)
        if c is None:
            h = ctypes.c_void_p()
            check(lib().lsmblk_ctx_create(device, ctypes.byref(h)), "lsmblk_ctx_create")
            c = _ctxs[key] = _Ctx(h.value)
        return c


def release_contexts(device: int = None):
    """Destroy the cached per-(device, stream) contexts (all, or those of `device`) after their
    work is done.  Each context keeps its own decode / encode / compaction / SST workspaces, which
    reach several GiB for 4 GiB batches, so a caller cycling through many streams releases them
    here; the next call on a stream creates a fresh context."""
    with _ctx_lock:
        keys = [k for k in _ctxs if device is None or k[0] == device]
        for k in keys:
            c = _ctxs.pop(k)
            with c.lock:  # waits for a call in progress on it (batch wrappers hold the lock)
                torch.cuda.synchronize(k[0])
                lib().lsmblk_ctx_destroy(c.h)
                c.h = None  # a thread that fetched c before the pop takes a fresh context
    return len(keys)


def _ctx(device: int, stream=None):
    """Context handle for `device` and `stream` (default: the device's current stream).  For
    diagnostics calls; the batch wrappers go through _native, which holds the context's lock."""
    return _ctx_for(device, _stream_ptr(stream, device)).h


def _native(fn, device: int, stream, *args, what=None, own=None):
    """One library call on the (device, stream) context (or on `own`, an OwnCtx), with that
    context's lock held for the whole call, so release_contexts cannot destroy it meanwhile; a
    context released before the lock was taken is replaced by a fresh one."""
    if own is not None:
        return check(getattr(lib(), fn)(own.h, *args), what or fn)
    while True:
        c = _ctx_for(device, _stream_ptr(stream, device))
        with c.lock:
            if c.h is not None:
                return check(getattr(lib(), fn)(c.h, *args), what or fn)


class OwnCtx:
    """A context owned by one object (e.g. a shard.RangeShard, whose rotation state lives on its
    context between calls), independent of the stream it is used on."""

    def __init__(self, device: int):
        h = ctypes.c_void_p()
        check(lib().lsmblk_ctx_create(device, ctypes.byref(h)), "lsmblk_ctx_create")
        self.h = h.value

    def __del__(self):
        if getattr(self, "h", None):
            lib().lsmblk_ctx_destroy(self.h)
            self.h = None


def _stream_ptr(stream, device):
    s = stream if stream is not None else torch.cuda.current_stream(device)
    return s.cuda_stream


def _dev_index(t: torch.Tensor) -> int:
    if t.device.type != "cuda":
        raise ValueError("batch API needs device tensors (ROCm); got " + str(t.device))
    return t.device.index if t.device.index is not None else torch.cuda.current_device()


def _ptr(t):
    return t.data_ptr() if t is not None and t.numel() else None


def _need(t, dtype, name, dev, min_numel=0):
    """The C ABI reads raw pointers: check dtype, contiguity, device and size before a call."""
    if t is None:
        raise ValueError(f"{name}: missing tensor")
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if t.device.type != "cuda" or _dev_index(t) != dev:
        raise ValueError(f"{name}: must be on cuda:{dev}, got {t.device}")
    if t.numel() < min_numel:
        raise ValueError(f"{name}: needs >= {min_numel} elements, has {t.numel()}")
    return t


def _aligned_empty(nbytes: int, device) -> torch.Tensor:
    # torch's caching allocator returns >=512-B aligned blocks; the kernels need 16 B.
    t = torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)
    assert t.data_ptr() % 16 == 0
    return t


@dataclass
class KVStream:
    """SoA KV stream on device: keys[key_off[i]:key_off[i+1]], vals[...], ts[i].

    key_off / val_off are u32 stored in int32 tensors (n+1 entries); ts is u64 in int64.
    """
    keys: torch.Tensor
    key_off: torch.Tensor
    vals: torch.Tensor
    val_off: torch.Tensor
    ts: torch.Tensor
    n: int

    def _c(self, entry_cap=None, key_cap=None, val_cap=None):
        return KVStreamC(_ptr(self.keys), _ptr(self.key_off), _ptr(self.vals), _ptr(self.val_off),
                         _ptr(self.ts), self.n,
                         self.n if entry_cap is None else entry_cap,
                         self.keys.numel() if key_cap is None else key_cap,
                         self.vals.numel() if val_cap is None else val_cap)

    def check(self, dev, name="kv", entries=None):
        """Dtypes / contiguity / device / sizes of the five arrays for `entries` (default n)."""
        e = self.n if entries is None else entries
        _need(self.keys, torch.uint8, name + ".keys", dev)
        _need(self.vals, torch.uint8, name + ".vals", dev)
        _need(self.key_off, torch.int32, name + ".key_off", dev, e + 1)
        _need(self.val_off, torch.int32, name + ".val_off", dev, e + 1)
        _need(self.ts, torch.int64, name + ".ts", dev, e)
        return self

    @staticmethod
    def from_numpy(keys, key_off, vals, val_off, ts, device="cuda"):
        dev = torch.device(device)
        n = len(ts)
        k = _aligned_empty(len(keys), dev)
        v = _aligned_empty(len(vals), dev)
        if len(keys):
            k[:len(keys)].copy_(torch.from_numpy(np.ascontiguousarray(keys, np.uint8)))
        if len(vals):
            v[:len(vals)].copy_(torch.from_numpy(np.ascontiguousarray(vals, np.uint8)))
        ko = torch.from_numpy(np.ascontiguousarray(key_off, np.uint32).view(np.int32)).to(dev)
        vo = torch.from_numpy(np.ascontiguousarray(val_off, np.uint32).view(np.int32)).to(dev)
        t = torch.from_numpy(np.ascontiguousarray(ts, np.uint64).view(np.int64)).to(dev)
        if n == 0:
            t = torch.zeros(1, dtype=torch.int64, device=dev)
        return KVStream(k, ko, v, vo, t, n)

    @staticmethod
    def empty(n, key_bytes, val_bytes, device):
        """Output buffers for up to n entries / key_bytes / val_bytes (16-B aligned arenas)."""
        return KVStream(_aligned_empty(key_bytes + 16, device), torch.zeros(n + 1, dtype=torch.int32, device=device),
                        _aligned_empty(val_bytes + 16, device), torch.zeros(n + 1, dtype=torch.int32, device=device),
                        torch.zeros(max(n, 1), dtype=torch.int64, device=device), 0)

    def caps(self):
        """(entry_cap, key_cap, val_cap) of a stream made by empty()."""
        return self.key_off.numel() - 1, self.keys.numel(), self.vals.numel()

    def byte_sizes(self):
        """(key bytes, value bytes) of the stream (reads the sentinels: synchronizes)."""
        if self.n == 0:
            return 0, 0
        return (int(self.key_off[self.n].item()) & 0xFFFFFFFF, int(self.val_off[self.n].item()) & 0xFFFFFFFF)

    def to_numpy(self):
        """-> (keys u8, key_off u32, vals u8, val_off u32, ts u64) trimmed to the stream."""
        ko = self.key_off[:self.n + 1].cpu().numpy().view(np.uint32)
        vo = self.val_off[:self.n + 1].cpu().numpy().view(np.uint32)
        kb, vb = int(ko[-1]) if len(ko) else 0, int(vo[-1]) if len(vo) else 0
        return (self.keys[:kb].cpu().numpy(), ko, self.vals[:vb].cpu().numpy(), vo,
                self.ts[:self.n].cpu().numpy().view(np.uint64))


def _status(stats: torch.Tensor) -> int:
    return lib().lsmblk_stats_status(int(stats[3].item()) & 0xFFFFFFFFFFFFFFFF)


def _u32_table(x, dev):
    if not isinstance(x, torch.Tensor):
        x = torch.from_numpy(np.ascontiguousarray(x, np.uint32).view(np.int32))
    return x.to(dev).contiguous()


def decode_into(blocks, blk_off, nblk, out: KVStream, stats, entry_cap, key_cap, val_cap, stream=None):
    """Asynchronous decode into preallocated buffers (no host sync). stats: int64[4] device."""
    dev = _dev_index(blk_off)
    _need(blk_off, torch.int64, "blk_off", dev, nblk + 1)
    if nblk:
        _need(blocks, torch.uint8, "blocks", dev)
    _need(stats, torch.int64, "stats", dev, STATS_WORDS)
    out.check(dev, "out", 0)
    if out.key_off.numel() < entry_cap + 1 or out.ts.numel() < entry_cap or out.keys.numel() < key_cap \
            or out.vals.numel() < val_cap:
        raise ValueError("decode_into: capacities exceed the output tensors")
    c = out._c(entry_cap, key_cap, val_cap)
    _native("lsmblk_decode_batch", dev, stream, _ptr(blocks), _ptr(blk_off), nblk, ctypes.byref(c),
            stats.data_ptr(), _stream_ptr(stream, dev), what="lsmblk_decode_batch")


def decode_ex_into(blocks, blk_off, nblk, out: KVStream, stats, entry_cap, key_cap, val_cap, tail=0, verify=False,
                   blk_ent=None, stream=None):
    """Asynchronous lsmblk_decode_batch_ex: framed ranges (tail), CRC verification, block entry index."""
    dev = _dev_index(blk_off)
    _need(blk_off, torch.int64, "blk_off", dev, nblk + 1)
    if nblk:
        _need(blocks, torch.uint8, "blocks", dev)
    _need(stats, torch.int64, "stats", dev, STATS_WORDS)
    if blk_ent is not None:
        _need(blk_ent, torch.int64, "blk_ent", dev, nblk + 1)
    out.check(dev, "out", 0)
    if out.key_off.numel() < entry_cap + 1 or out.ts.numel() < entry_cap or out.keys.numel() < key_cap \
            or out.vals.numel() < val_cap:
        raise ValueError("decode_ex_into: capacities exceed the output tensors")
    c = out._c(entry_cap, key_cap, val_cap)
    _native("lsmblk_decode_batch_ex", dev, stream, _ptr(blocks), _ptr(blk_off), nblk, tail,
            LSMBLK_DECODE_VERIFY_CRC if verify else 0, ctypes.byref(c), _ptr(blk_ent),
            stats.data_ptr(), _stream_ptr(stream, dev), what="lsmblk_decode_batch_ex")


def decode_blocks(blocks: torch.Tensor, blk_off: torch.Tensor, stream=None, tail: int = 0, verify: bool = False,
                  with_blk_ent: bool = False):
    """Decode blocks[blk_off[b]:blk_off[b+1] - tail] for every b into a KVStream (synchronizes).
    tail=4 reads a framed SST data section by its BlockMeta offsets (SsTable::read_block,
    reference src/table.rs:213-233); verify=True checks every block's stored crc32fast.
    with_blk_ent: also return the first entry index of every block (int64[nblk+1])."""
    dev = torch.device("cuda", _dev_index(blk_off))
    nblk = blk_off.numel() - 1
    total = int(blocks.numel())
    entry_cap = total // 16 + 1
    key_cap, val_cap = total + 16, total + 16
    blk_ent = torch.zeros(nblk + 1, dtype=torch.int64, device=dev) if with_blk_ent else None
    for _ in range(2):
        out = KVStream(_aligned_empty(key_cap, dev), torch.empty(entry_cap + 1, dtype=torch.int32, device=dev),
                       _aligned_empty(val_cap, dev), torch.empty(entry_cap + 1, dtype=torch.int32, device=dev),
                       torch.empty(max(entry_cap, 1), dtype=torch.int64, device=dev), 0)
        stats = torch.zeros(STATS_WORDS, dtype=torch.int64, device=dev)
        if tail or verify or with_blk_ent:
            decode_ex_into(blocks, blk_off, nblk, out, stats, entry_cap, key_cap, val_cap, tail, verify, blk_ent,
                           stream)
        else:
            decode_into(blocks, blk_off, nblk, out, stats, entry_cap, key_cap, val_cap, stream)
        torch.cuda.synchronize(dev)
        st = _status(stats)
        s = stats.cpu().tolist()
        if st == LSMBLK_E_CAPACITY:
            entry_cap, key_cap, val_cap = max(s[0], 1), max(s[1], 16), max(s[2], 16)
            continue
        if st:
            raise LsmBlkError(st, "decode_blocks")
        out.n = s[0]
        return (out, blk_ent) if with_blk_ent else out
    raise LsmBlkError(LSMBLK_E_CAPACITY, "decode_blocks")


def encode_bound(kv: KVStream, key_bytes: int, val_bytes: int, framed: bool = False):
    """Exact worst-case output sizes: (bytes, blk_off entries); framed: + 4 CRC bytes per block."""
    return key_bytes + val_bytes + (22 if framed else 18) * kv.n + 16, kv.n + 2


def encode_into(kv: KVStream, seg_start: torch.Tensor, nseg: int, block_size: int, out, out_cap,
                blk_off, blk_cap, stats, stream=None, seg_out=None, framed=False):
    """Asynchronous encode into preallocated buffers (no host sync).  With seg_out (int64[2 nseg])
    the output is per-segment slots (LSMBLK_ENCODE_SEG_SLOTS, include/lsmblk.h): every segment's
    blocks at its own slot, seg_out[s] = (slot, bytes); slots_to_packed packs them.  framed: every
    block followed by its big-endian crc32 -- the SST data section (LSMBLK_ENCODE_FRAMED)."""
    dev = _dev_index(seg_start)
    kv.check(dev, "kv")
    _need(seg_start, torch.int32, "seg_start", dev, nseg + 1)
    _need(out, torch.uint8, "out", dev, out_cap)
    _need(blk_off, torch.int64, "blk_off", dev, blk_cap)
    _need(stats, torch.int64, "stats", dev, STATS_WORDS)
    c = kv._c()
    if seg_out is None and not framed:
        _native("lsmblk_encode_batch", dev, stream, ctypes.byref(c), seg_start.data_ptr(), nseg, block_size,
                _ptr(out), out_cap, blk_off.data_ptr(), blk_cap, stats.data_ptr(),
                _stream_ptr(stream, dev), what="lsmblk_encode_batch")
        return
    if seg_out is not None:
        _need(seg_out, torch.int64, "seg_out", dev, 2 * nseg)
    flags = (LSMBLK_ENCODE_SEG_SLOTS if seg_out is not None else 0) | (LSMBLK_ENCODE_FRAMED if framed else 0)
    _native("lsmblk_encode_batch_ex", dev, stream, ctypes.byref(c), seg_start.data_ptr(), nseg, block_size,
            flags, _ptr(out), out_cap, blk_off.data_ptr(), blk_cap, _ptr(seg_out),
            stats.data_ptr(), _stream_ptr(stream, dev), what="lsmblk_encode_batch_ex")


def encode_kv_framed(kv: KVStream, seg_start, block_size: int, stream=None, slots: bool = False):
    """The SST data sections of kv's segments (LSMBLK_ENCODE_FRAMED): every block followed by its
    big-endian crc32fast, as SsTableBuilder::finish_block writes them (reference
    src/table/builder.rs:112-123).  -> (out u8 tensor, blk_off int64 tensor[nblk+1]) -- packed:
    blk_off[b+1] - blk_off[b] = block b's size + 4, the layout lsmblk_decode_batch_ex(tail=4)
    reads; with slots=True also seg_out int64 tensor[nseg, 2] (every segment at its slot)."""
    dev = torch.device("cuda", _dev_index(kv.key_off))
    seg_start = _u32_table(seg_start, dev)
    nseg = seg_start.numel() - 1
    kb, vb = kv.byte_sizes()
    out_cap, blk_cap = encode_bound(kv, kb, vb, framed=True)
    out = _aligned_empty(out_cap, dev)
    blk_off = torch.zeros(blk_cap, dtype=torch.int64, device=dev)
    seg_out = torch.zeros(max(2 * nseg, 1), dtype=torch.int64, device=dev) if slots else None
    stats = torch.zeros(STATS_WORDS, dtype=torch.int64, device=dev)
    encode_into(kv, seg_start, nseg, block_size, out, out_cap, blk_off, blk_cap, stats, stream, seg_out=seg_out,
                framed=True)
    torch.cuda.synchronize(dev)
    st = _status(stats)
    if st:
        raise LsmBlkError(st, "encode_kv_framed")
    nblk, nbytes = stats[0].item(), stats[1].item()
    if slots:
        return out, blk_off[:nblk + 1], seg_out[:2 * nseg].view(-1, 2)
    return out[:nbytes], blk_off[:nblk + 1]


def encode_kv_slots(kv: KVStream, seg_start, block_size: int, stream=None):
    """Per-segment slot output (LSMBLK_ENCODE_SEG_SLOTS) -> (out u8 tensor, blk_off int64
    tensor[nblk+1], seg_out int64 tensor[nseg, 2] of (slot, bytes))."""
    dev = torch.device("cuda", _dev_index(kv.key_off))
    seg_start = _u32_table(seg_start, dev)
    nseg = seg_start.numel() - 1
    kb, vb = kv.byte_sizes()
    out_cap, blk_cap = encode_bound(kv, kb, vb)
    out = _aligned_empty(out_cap, dev)
    blk_off = torch.zeros(blk_cap, dtype=torch.int64, device=dev)
    seg_out = torch.zeros(max(2 * nseg, 1), dtype=torch.int64, device=dev)
    stats = torch.zeros(STATS_WORDS, dtype=torch.int64, device=dev)
    encode_into(kv, seg_start, nseg, block_size, out, out_cap, blk_off, blk_cap, stats, stream, seg_out=seg_out)
    torch.cuda.synchronize(dev)
    st = _status(stats)
    if st:
        raise LsmBlkError(st, "encode_kv_slots")
    nblk = stats[0].item()
    return out, blk_off[:nblk + 1], seg_out[:2 * nseg].view(-1, 2)


def slots_to_packed(out: torch.Tensor, blk_off: torch.Tensor, seg_out: torch.Tensor):
    """The slot output of encode_kv_slots / encode_into(seg_out=...) packed as lsmblk_encode_batch
    writes it: (blocks, blk_off[nblk+1]).  Test and bench helper (copies every segment)."""
    so = seg_out.view(-1, 2)
    starts, lens = so[:, 0].contiguous(), so[:, 1].contiguous()
    dense = torch.cumsum(lens, 0) - lens
    sl, ll = starts.tolist(), lens.tolist()
    parts = [out[a:a + b] for a, b in zip(sl, ll) if b]
    blocks = torch.cat(parts) if parts else out[:0]
    nblk = blk_off.numel() - 1
    b = blk_off[:nblk]
    seg = torch.searchsorted(starts, b, right=True) - 1
    packed = torch.empty(nblk + 1, dtype=torch.int64, device=out.device)
    packed[:nblk] = b - starts[seg] + dense[seg]
    packed[nblk] = int(lens.sum().item())
    return blocks, packed


def encode_kv(kv: KVStream, seg_start, block_size: int, stream=None):
    """Greedy block packing per segment -> (blocks u8 tensor, blk_off int64 tensor[nblk+1])."""
    dev = torch.device("cuda", _dev_index(kv.key_off))
    seg_start = _u32_table(seg_start, dev)
    nseg = seg_start.numel() - 1
    kb, vb = kv.byte_sizes()
    out_cap, blk_cap = encode_bound(kv, kb, vb)
    out = _aligned_empty(out_cap, dev)
    blk_off = torch.zeros(blk_cap, dtype=torch.int64, device=dev)
    stats = torch.zeros(STATS_WORDS, dtype=torch.int64, device=dev)
    encode_into(kv, seg_start, nseg, block_size, out, out_cap, blk_off, blk_cap, stats, stream)
    torch.cuda.synchronize(dev)
    st = _status(stats)
    if st:
        raise LsmBlkError(st, "encode_kv")
    nblk, nbytes = stats[0].item(), stats[1].item()
    return out[:nbytes], blk_off[:nblk + 1]


def crc32_into(blocks: torch.Tensor, blk_off: torch.Tensor, nblk: int, crc: torch.Tensor, stats, stream=None,
               tail: int = 0):
    """Asynchronous per-block CRC-32 into a preallocated int32 tensor (no host sync)."""
    dev = _dev_index(blk_off)
    _need(blk_off, torch.int64, "blk_off", dev, nblk + 1)
    _need(crc, torch.int32, "crc", dev, nblk)
    _need(stats, torch.int64, "stats", dev, STATS_WORDS)
    if nblk:
        _need(blocks, torch.uint8, "blocks", dev)
    _native("lsmblk_crc32_batch", dev, stream, _ptr(blocks), blk_off.data_ptr(), nblk, tail, _ptr(crc),
            stats.data_ptr(), _stream_ptr(stream, dev), what="lsmblk_crc32_batch")


def crc32_blocks(blocks: torch.Tensor, blk_off: torch.Tensor, stream=None, tail: int = 0) -> torch.Tensor:
    """crc32fast::hash of every block -- the SST framing checksum SsTableBuilder::finish_block
    appends (reference src/table/builder.rs:120-122) and SsTable::read_block verifies
    (src/table.rs:226-230).  Block b = blocks[blk_off[b] : blk_off[b+1] - tail] (tail=4 over a
    framed SST data section).  Returns an int32 tensor[nblk] holding the u32 CRCs."""
    dev = torch.device("cuda", _dev_index(blk_off))
    nblk = blk_off.numel() - 1
    crc = torch.zeros(max(nblk, 1), dtype=torch.int32, device=dev)
    stats = torch.zeros(STATS_WORDS, dtype=torch.int64, device=dev)
    crc32_into(blocks, blk_off, nblk, crc, stats, stream, tail)
    torch.cuda.synchronize(dev)
    st = _status(stats)
    if st:
        raise LsmBlkError(st, "crc32_blocks")
    return crc[:nblk]


def segment_blocks_into(seg_start: torch.Tensor, nseg: int, enc_stats: torch.Tensor, seg_blk: torch.Tensor,
                        stream=None):
    """After encode_into on the same device/stream: seg_blk[s] = first block of segment s."""
    dev = _dev_index(seg_start)
    _need(seg_start, torch.int32, "seg_start", dev, nseg + 1)
    _need(seg_blk, torch.int32, "seg_blk", dev, nseg + 1)
    _need(enc_stats, torch.int64, "enc_stats", dev, STATS_WORDS)
    _native("lsmblk_encode_segment_blocks", dev, stream, seg_start.data_ptr(), nseg, enc_stats.data_ptr(),
            seg_blk.data_ptr(), _stream_ptr(stream, dev), what="lsmblk_encode_segment_blocks")


def block_meta_into(blocks, blk_off, nblk, seg_blk, nseg, meta, meta_cap, meta_off, stats, stream=None, tail=0):
    """Asynchronous BlockMeta sections into preallocated buffers (no host sync)."""
    dev = _dev_index(blk_off)
    _need(blk_off, torch.int64, "blk_off", dev, nblk + 1)
    _need(seg_blk, torch.int32, "seg_blk", dev, nseg + 1)
    _need(meta, torch.uint8, "meta", dev, meta_cap)
    _need(meta_off, torch.int64, "meta_off", dev, nseg + 1)
    _need(stats, torch.int64, "stats", dev, STATS_WORDS)
    _native("lsmblk_block_meta_batch", dev, stream, _ptr(blocks), blk_off.data_ptr(), nblk, tail,
            seg_blk.data_ptr(), nseg, meta.data_ptr(), meta_cap, meta_off.data_ptr(),
            stats.data_ptr(), _stream_ptr(stream, dev), what="lsmblk_block_meta_batch")


def block_meta(blocks: torch.Tensor, blk_off: torch.Tensor, seg_blk, stream=None, tail: int = 0):
    """BlockMeta::encode_block_meta (reference src/table.rs:29-63) of every segment, as
    SsTableBuilder::build writes it after the SST data section (src/table/builder.rs:68-77).
    seg_blk[s] .. seg_blk[s+1] are segment s's blocks.  Returns (meta u8 tensor, meta_off
    int64 tensor[nseg+1]); section s = meta[meta_off[s]:meta_off[s+1]]."""
    dev = torch.device("cuda", _dev_index(blk_off))
    seg_blk = _u32_table(seg_blk, dev)
    nseg, nblk = seg_blk.numel() - 1, blk_off.numel() - 1
    meta_off = torch.zeros(nseg + 1, dtype=torch.int64, device=dev)
    stats = torch.zeros(STATS_WORDS, dtype=torch.int64, device=dev)
    cap = 16 * nseg + 56 * max(nblk, 1)
    for _ in range(2):
        meta = _aligned_empty(cap, dev)
        block_meta_into(blocks, blk_off, nblk, seg_blk, nseg, meta, cap, meta_off, stats, stream, tail)
        torch.cuda.synchronize(dev)
        st = _status(stats)
        if st == LSMBLK_E_CAPACITY:
            cap = int(stats[1].item())
            continue
        if st:
            raise LsmBlkError(st, "block_meta")
        return meta[:int(stats[1].item())], meta_off
    raise LsmBlkError(LSMBLK_E_CAPACITY, "block_meta")


def encode_sst(kv: KVStream, seg_start, block_size: int, stream=None):
    """One SsTableBuilder per segment, on the device: the packed blocks, their per-block
    CRC-32s (finish_block, src/table/builder.rs:112-123) and the BlockMeta sections (build,
    :68-77).  Returns dict(blocks, blk_off, seg_blk, crc, meta, meta_off)."""
    dev = torch.device("cuda", _dev_index(kv.key_off))
    seg_start = _u32_table(seg_start, dev)
    nseg = seg_start.numel() - 1
    kb, vb = kv.byte_sizes()
    out_cap, blk_cap = encode_bound(kv, kb, vb)
    out = _aligned_empty(out_cap, dev)
    blk_off = torch.zeros(blk_cap, dtype=torch.int64, device=dev)
    stats = torch.zeros(STATS_WORDS, dtype=torch.int64, device=dev)
    seg_blk = torch.zeros(nseg + 1, dtype=torch.int32, device=dev)
    # the segment -> block table reads the encode's workspace: no other encode on this context
    # (same device and stream) may run in between
    with _ctx_for(dev.index, _stream_ptr(stream, dev.index)).lock:
        encode_into(kv, seg_start, nseg, block_size, out, out_cap, blk_off, blk_cap, stats, stream)
        segment_blocks_into(seg_start, nseg, stats, seg_blk, stream)
    torch.cuda.synchronize(dev)
    st = _status(stats)
    if st:
        raise LsmBlkError(st, "encode_sst")
    nblk, nbytes = stats[0].item(), stats[1].item()
    blocks, blk_off = out[:nbytes], blk_off[:nblk + 1]
    crc = crc32_blocks(blocks, blk_off, stream)
    meta, meta_off = block_meta(blocks, blk_off, seg_blk, stream)
    return dict(blocks=blocks, blk_off=blk_off, seg_blk=seg_blk, crc=crc, meta=meta, meta_off=meta_off)


def _prefix_tables(prefixes, dev):
    pf = b"".join(bytes(p) for p in prefixes)
    po = np.zeros(len(prefixes) + 1, np.uint32)
    po[1:] = np.cumsum([len(p) for p in prefixes]) if prefixes else []
    pfx = torch.frombuffer(bytearray(pf or b"\0"), dtype=torch.uint8).to(dev)
    pfo = torch.from_numpy(po.view(np.int32)).to(dev)
    return pfx, pfo


def compact_filter(kv: KVStream, watermark: int, bottom_level: bool, prefixes=(), stream=None) -> KVStream:
    """compact_generate_sst's per-entry rules (reference src/compact.rs:234-299) over a merged
    stream (keys ascending, versions newest first) -> the kept entries as a new KVStream."""
    dev = torch.device("cuda", _dev_index(kv.key_off))
    kv.check(dev.index, "kv")
    pfx, pfo = _prefix_tables(prefixes, dev)
    kb, vb = kv.byte_sizes()
    n = kv.n
    out = KVStream.empty(n, kb, vb, dev)
    stats = torch.zeros(STATS_WORDS, dtype=torch.int64, device=dev)
    ci, co = kv._c(), out._c(n, kb + 16, vb + 16)
    _native("lsmblk_compact_filter_batch", dev.index, stream, ctypes.byref(ci), watermark,
            int(bool(bottom_level)), pfx.data_ptr(), pfo.data_ptr(), len(prefixes),
            ctypes.byref(co), stats.data_ptr(), _stream_ptr(stream, dev.index), what="lsmblk_compact_filter_batch")
    torch.cuda.synchronize(dev)
    st = _status(stats)
    if st:
        raise LsmBlkError(st, "compact_filter")
    out.n = int(stats[0].item())
    return out


def merge_into(kv: KVStream, run_start: torch.Tensor, nrun: int, out: KVStream, stats, stream=None,
               merge_mode=LSMBLK_MERGE_RUNS):
    """Asynchronous merge of the runs of kv into preallocated `out` (no host sync): MergeIterator
    (LSMBLK_MERGE_RUNS) or the reference's TwoMergeIterator with run nrun-1 as b
    (LSMBLK_MERGE_TWO_LEVEL)."""
    dev = _dev_index(run_start)
    kv.check(dev, "kv")
    _need(run_start, torch.int32, "run_start", dev, nrun + 1)
    out.check(dev, "out", 0)
    _need(stats, torch.int64, "stats", dev, STATS_WORDS)
    ci, co = kv._c(), out._c(*out.caps())
    _native("lsmblk_merge_batch_ex", dev, stream, ctypes.byref(ci), run_start.data_ptr(), nrun, merge_mode,
            ctypes.byref(co), stats.data_ptr(), _stream_ptr(stream, dev), what="lsmblk_merge_batch_ex")


def merge_runs(kv: KVStream, run_start, stream=None, merge_mode=LSMBLK_MERGE_RUNS) -> KVStream:
    """MergeIterator (reference src/iterators/merge_iterator.rs:59-184) over the sorted runs
    kv[run_start[r]:run_start[r+1]] (run 0 = highest priority) -> the merged KVStream.
    merge_mode=LSMBLK_MERGE_TWO_LEVEL: TwoMergeIterator(MergeIterator(runs[:-1]), runs[-1])
    (two_merge_iterator.rs:19-93 as written)."""
    dev = torch.device("cuda", _dev_index(kv.key_off))
    rs = _u32_table(run_start, dev)
    kb, vb = kv.byte_sizes()
    out = KVStream.empty(kv.n, kb, vb, dev)
    stats = torch.zeros(STATS_WORDS, dtype=torch.int64, device=dev)
    merge_into(kv, rs, rs.numel() - 1, out, stats, stream, merge_mode)
    torch.cuda.synchronize(dev)
    st = _status(stats)
    if st:
        raise LsmBlkError(st, "merge_runs")
    out.n = int(stats[0].item())
    return out


def sst_rotation(kv: KVStream, block_size: int, target_sst_size: int, stream=None):
    """SST cut points of compact_generate_sst (reference src/compact.rs:278-289) over the stream
    handed to SsTableBuilder::add -> u32 numpy array of SST first entries, then kv.n."""
    dev = torch.device("cuda", _dev_index(kv.key_off))
    kv.check(dev.index, "kv")
    cap = kv.n + 2
    starts = torch.zeros(cap, dtype=torch.int32, device=dev)
    stats = torch.zeros(STATS_WORDS, dtype=torch.int64, device=dev)
    c = kv._c()
    _native("lsmblk_sst_rotation_batch", dev.index, stream, ctypes.byref(c), block_size, target_sst_size,
            starts.data_ptr(), cap, stats.data_ptr(), _stream_ptr(stream, dev.index), what="lsmblk_sst_rotation_batch")
    torch.cuda.synchronize(dev)
    st = _status(stats)
    if st:
        raise LsmBlkError(st, "sst_rotation")
    ns = int(stats[0].item())
    return starts[:ns + 1].cpu().numpy().view(np.uint32)


class CompactBuffers:
    """Preallocated outputs of lsmblk_compact_batch for an input of n entries / K key bytes /
    V value bytes (worst case: every entry kept, every entry its own block and SST)."""

    def __init__(self, n, key_bytes, val_bytes, device, sst_cap=None, target_sst_size=None):
        self.kept = KVStream.empty(n, key_bytes, val_bytes, device)
        self.out_cap = key_bytes + val_bytes + 18 * n + 16
        self.out = _aligned_empty(self.out_cap, device)
        self.blk_cap = n + 2
        self.blk_off = torch.zeros(self.blk_cap, dtype=torch.int64, device=device)
        if sst_cap is None:
            # every SST but the last holds >= target bytes of blocks + CRCs, and the blocks take at
            # most klen + vlen + 22 bytes per entry (header, ts, offset slot, trailer, CRC)
            sst_cap = n + 2 if not target_sst_size else min(n + 2, (key_bytes + val_bytes + 22 * n) // target_sst_size + 3)
        self.sst_cap = sst_cap
        self.sst_start = torch.zeros(self.sst_cap, dtype=torch.int32, device=device)
        self.sst_blk = torch.zeros(self.sst_cap, dtype=torch.int32, device=device)
        self.stats = torch.zeros(8, dtype=torch.int64, device=device)


def compact_into(kv: KVStream, run_start: torch.Tensor, nrun: int, opts: dict, buf: CompactBuffers, stream=None,
                 _keep=None):
    """Asynchronous lsmblk_compact_batch into preallocated buffers (no host sync)."""
    dev = _dev_index(run_start)
    kv.check(dev, "kv")
    _need(run_start, torch.int32, "run_start", dev, nrun + 1)
    o = _opts_c(opts)
    ci, ck = kv._c(), buf.kept._c(*buf.kept.caps())
    _native("lsmblk_compact_batch", dev, stream, ctypes.byref(ci), run_start.data_ptr(), nrun, ctypes.byref(o),
            ctypes.byref(ck), buf.out.data_ptr(), buf.out_cap, buf.blk_off.data_ptr(),
            buf.blk_cap, buf.sst_start.data_ptr(), buf.sst_blk.data_ptr(), buf.sst_cap,
            buf.stats.data_ptr(), _stream_ptr(stream, dev), what="lsmblk_compact_batch")


def _opts_c(opts):
    pfx, pfo = opts["_pfx"]
    return CompactOptsC(opts.get("watermark", 0), int(bool(opts.get("bottom_level", False))), opts["_npfx"],
                        pfx.data_ptr(), pfo.data_ptr(), opts["block_size"], opts.get("merge_mode", LSMBLK_MERGE_RUNS),
                        opts["target_sst_size"])


def compact_opts(watermark=0, bottom_level=False, prefixes=(), block_size=4096, target_sst_size=2 << 20,
                 device="cuda", merge_mode=LSMBLK_MERGE_RUNS):
    """Options of lsmblk_compact_batch (prefix tables staged on the device once)."""
    return dict(watermark=watermark, bottom_level=bottom_level, block_size=block_size,
                target_sst_size=target_sst_size, _pfx=_prefix_tables(prefixes, torch.device(device)),
                _npfx=len(prefixes), merge_mode=merge_mode)


def compact_runs(kv: KVStream, run_start, watermark=0, bottom_level=False, prefixes=(), block_size=4096,
                 target_sst_size=2 << 20, stream=None, merge_mode=LSMBLK_MERGE_RUNS):
    """compact_generate_sst (reference src/compact.rs:223-311) on the device over the sorted runs
    of kv (run 0 = highest priority): merge (merge_mode, see include/lsmblk.h), keep/drop rules,
    SST rotation, block packing.  Returns dict(kept KVStream, blocks, blk_off, sst_start, sst_blk,
    stats)."""
    dev = torch.device("cuda", _dev_index(kv.key_off))
    rs = _u32_table(run_start, dev)
    kb, vb = kv.byte_sizes()
    buf = CompactBuffers(kv.n, kb, vb, dev, target_sst_size=target_sst_size)
    opts = compact_opts(watermark, bottom_level, prefixes, block_size, target_sst_size, dev, merge_mode)
    compact_into(kv, rs, rs.numel() - 1, opts, buf, stream)
    torch.cuda.synchronize(dev)
    st = _status(buf.stats)
    if st:
        raise LsmBlkError(st, "compact_runs")
    s = buf.stats.cpu().tolist()
    nblk, nbytes, nsst = s[0], s[1], s[2]
    buf.kept.n = s[5]
    return dict(kept=buf.kept, blocks=buf.out[:nbytes], blk_off=buf.blk_off[:nblk + 1],
                sst_start=buf.sst_start[:nsst + 1], sst_blk=buf.sst_blk[:nsst + 1], stats=s)


# ------------------------------------------------------------------ key-range sharded compaction
def key_range_c(lo, hi):
    """lsmblk_key_range over device byte tensors (None: unbounded side).  Keep the tensors alive."""
    r = KeyRangeC()
    if lo is not None:
        r.lo, r.lo_len, r.has_lo = _ptr(lo), lo.numel(), 1
    if hi is not None:
        r.hi, r.hi_len, r.has_hi = _ptr(hi), hi.numel(), 1
    return r


def compact_merge_into(kv: KVStream, run_start: torch.Tensor, nrun: int, opts: dict, key_range, kept: KVStream,
                       stats, stream=None, ctx=None, two_end=0, kept_same=None):
    """Asynchronous lsmblk_compact_merge_batch_ex: merge + rules restricted to key_range (a KeyRangeC
    or None) into preallocated `kept`.  stats: int64[5] device.  Two-level merges (opts merge_mode):
    two_end (LSMBLK_TWO_END_*) and kept_same (uint8 device tensor, the loop's same_as_last_key per
    kept entry) as include/lsmblk.h describes."""
    dev = _dev_index(run_start)
    kv.check(dev, "kv")
    _need(run_start, torch.int32, "run_start", dev, nrun + 1)
    kept.check(dev, "kept", 0)
    _need(stats, torch.int64, "stats", dev, 5)
    o = _opts_c(opts)
    ci, ck = kv._c(), kept._c(*kept.caps())
    if kept_same is not None:
        _need(kept_same, torch.uint8, "kept_same", dev, kept.caps()[0])
    _native("lsmblk_compact_merge_batch_ex", dev, stream, ctypes.byref(ci), run_start.data_ptr(), nrun,
            ctypes.byref(o), ctypes.byref(key_range) if key_range is not None else None, two_end,
            ctypes.byref(ck), _ptr(kept_same), stats.data_ptr(), _stream_ptr(stream, dev),
            what="lsmblk_compact_merge_batch_ex", own=ctx)


def shard_prepare(ext: KVStream, n_own: int, last: bool, block_size: int, target_sst_size: int, sst_cap: int,
                  stream=None, ctx=None, ext_same=None):
    """lsmblk_shard_rotation_prepare_ex; ext_same (uint8 device tensor, two-level merges): every ext
    entry's same_as_last_key."""
    dev = _dev_index(ext.key_off)
    ext.check(dev, "ext")
    if ext_same is not None:
        _need(ext_same, torch.uint8, "ext_same", dev, ext.n)
    c = ext._c()
    _native("lsmblk_shard_rotation_prepare_ex", dev, stream, ctypes.byref(c), _ptr(ext_same), n_own,
            LSMBLK_SHARD_LAST if last else 0, block_size, target_sst_size, sst_cap,
            _stream_ptr(stream, dev), what="lsmblk_shard_rotation_prepare_ex", own=ctx)


def shard_carry(carry_in: torch.Tensor, carry_out: torch.Tensor, stream=None, ctx=None):
    dev = _dev_index(carry_in)
    _need(carry_in, torch.int64, "carry_in", dev, 2)
    _need(carry_out, torch.int64, "carry_out", dev, 2)
    _native("lsmblk_shard_rotation_carry", dev, stream, carry_in.data_ptr(), carry_out.data_ptr(),
            _stream_ptr(stream, dev), what="lsmblk_shard_rotation_carry", own=ctx)


def shard_encode_into(ext: KVStream, out, out_cap, blk_off, blk_cap, seg_start, seg_blk, seg_cap, stats,
                      stream=None, ctx=None):
    dev = _dev_index(ext.key_off)
    ext.check(dev, "ext")
    _need(out, torch.uint8, "out", dev, out_cap)
    _need(blk_off, torch.int64, "blk_off", dev, blk_cap)
    _need(seg_start, torch.int32, "seg_start", dev, seg_cap)
    _need(seg_blk, torch.int32, "seg_blk", dev, seg_cap)
    _need(stats, torch.int64, "stats", dev, 8)
    c = ext._c()
    _native("lsmblk_shard_encode_batch", dev, stream, ctypes.byref(c), out.data_ptr(), out_cap,
            blk_off.data_ptr(), blk_cap, seg_start.data_ptr(), seg_blk.data_ptr(),
            seg_cap, stats.data_ptr(), _stream_ptr(stream, dev), what="lsmblk_shard_encode_batch", own=ctx)


def seek_blocks(blocks: torch.Tensor, blk_off: torch.Tensor, q_blk, qkeys, tail: int = 0, stream=None):
    """BlockIterator::create_and_seek_to_key (reference src/block/iterator.rs:73-94) for a batch of
    (block index, key) lookups -> int64 numpy array of the entry indices the iterators land on
    (a block's entry count = ended invalid)."""
    dev = torch.device("cuda", _dev_index(blk_off))
    nblk = blk_off.numel() - 1
    _need(blk_off, torch.int64, "blk_off", dev.index, nblk + 1)
    kb = b"".join(bytes(k) for k in qkeys)
    ko = np.zeros(len(qkeys) + 1, np.uint32)
    ko[1:] = np.cumsum([len(k) for k in qkeys]) if qkeys else []
    qk = torch.frombuffer(bytearray(kb or b"\0"), dtype=torch.uint8).to(dev)
    qo, qb = _u32_table(ko, dev), _u32_table(np.asarray(q_blk, np.uint32), dev)
    idx = torch.zeros(max(len(qkeys), 1), dtype=torch.int32, device=dev)
    stats = torch.zeros(STATS_WORDS, dtype=torch.int64, device=dev)
    _native("lsmblk_seek_batch", dev.index, stream, _ptr(blocks), blk_off.data_ptr(), nblk, tail,
            qk.data_ptr(), qo.data_ptr(), qb.data_ptr(), len(qkeys), idx.data_ptr(),
            stats.data_ptr(), _stream_ptr(stream, dev.index), what="lsmblk_seek_batch")
    torch.cuda.synchronize(dev)
    st = _status(stats)
    if st:
        raise LsmBlkError(st, "seek_blocks")
    return idx[:len(qkeys)].cpu().numpy().view(np.uint32).astype(np.int64)
