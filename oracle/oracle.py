"""ctypes wrapper over the C restatement (lsmblk_oracle.c) -- TEST INFRASTRUCTURE ONLY.

Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as
the checker or the timed CPU baseline.  The product package (lsm_amd) never imports it.
"""
import ctypes
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "liblsmblk_oracle.so")
_lib = None

ORC_OK, ORC_E_INVAL, ORC_E_MALFORMED, ORC_E_CAPACITY, ORC_E_OVERFLOW = 0, -1, -2, -3, -7


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        P, S, U32, U64, I = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
        L.orc_builder_new.restype = P
        L.orc_builder_new.argtypes = [S]
        L.orc_builder_free.argtypes = [P]
        L.orc_builder_add.argtypes = [P, P, S, U64, P, S]
        L.orc_builder_add.restype = I
        L.orc_builder_is_empty.argtypes = [P]
        L.orc_builder_estimated_size.argtypes = [P]
        L.orc_builder_estimated_size.restype = S
        L.orc_builder_finish.argtypes = [P, P, S, ctypes.POINTER(S)]
        L.orc_encode_segments.argtypes = [P, P, U32, S, P, U64, P, U64,
                                          ctypes.POINTER(U64), ctypes.POINTER(U64)]
        L.orc_decode_blocks.argtypes = [P, P, U64, P, U64, U64, U64,
                                        ctypes.POINTER(U64), ctypes.POINTER(U64), ctypes.POINTER(U64)]
        L.orc_segment_like_compaction.argtypes = [P, S, U64, P, U64, ctypes.POINTER(U64)]
        L.orc_block_seek_key.argtypes = [P, S, P, S]
        L.orc_block_seek_key.restype = S
        L.orc_block_entry_verbatim.argtypes = [P, S, S, ctypes.POINTER(U32), ctypes.POINTER(U32),
                                               ctypes.POINTER(S), ctypes.POINTER(S)]
        L.orc_crc32.argtypes = [P, S]
        L.orc_crc32.restype = U32
        L.orc_merge_runs.argtypes = [P, P, U32, P, U64, ctypes.POINTER(U64)]
        L.orc_compact.argtypes = [P, P, U64, U64, I, P, P, U32, S, U64, P, U64, P, U64, P, P, U64, P, U64,
                                  ctypes.POINTER(U64), ctypes.POINTER(U64), ctypes.POINTER(U64),
                                  ctypes.POINTER(U64)]
        L.orc_shard_rotation.argtypes = [P, U64, I, U64, U64, S, U64, P, U64, ctypes.POINTER(U64),
                                         ctypes.POINTER(U64), ctypes.POINTER(U64)]
        L.orc_shard_rotation_ex.argtypes = [P, P, U64, I, U64, U64, S, U64, P, U64, ctypes.POINTER(U64),
                                            ctypes.POINTER(U64), ctypes.POINTER(U64)]
        _lib = L
    return _lib


class _OrcKV(ctypes.Structure):
    _fields_ = [("keys", ctypes.c_void_p), ("key_off", ctypes.c_void_p), ("vals", ctypes.c_void_p),
                ("val_off", ctypes.c_void_p), ("ts", ctypes.c_void_p), ("n", ctypes.c_uint64)]


@dataclass
class KV:
    """SoA KV stream in host memory (numpy)."""
    keys: np.ndarray      # u8
    key_off: np.ndarray   # u32[n+1]
    vals: np.ndarray      # u8
    val_off: np.ndarray   # u32[n+1]
    ts: np.ndarray        # u64[n]

    @property
    def n(self):
        return len(self.ts)

    def entry(self, i):
        return (bytes(self.keys[self.key_off[i]:self.key_off[i + 1]]), int(self.ts[i]),
                bytes(self.vals[self.val_off[i]:self.val_off[i + 1]]))

    def entries(self):
        return [self.entry(i) for i in range(self.n)]

    @staticmethod
    def from_entries(entries):
        keys = b"".join(k for k, _, _ in entries)
        vals = b"".join(v for _, _, v in entries)
        ko = np.zeros(len(entries) + 1, np.uint32)
        vo = np.zeros(len(entries) + 1, np.uint32)
        ko[1:] = np.cumsum([len(k) for k, _, _ in entries]) if entries else []
        vo[1:] = np.cumsum([len(v) for _, _, v in entries]) if entries else []
        return KV(np.frombuffer(keys, np.uint8).copy(), ko, np.frombuffer(vals, np.uint8).copy(), vo,
                  np.array([t for _, t, _ in entries], np.uint64))

    def _c(self):
        for a in (self.keys, self.key_off, self.vals, self.val_off, self.ts):
            assert a.flags["C_CONTIGUOUS"]
        s = _OrcKV(self.keys.ctypes.data, self.key_off.ctypes.data, self.vals.ctypes.data,
                   self.val_off.ctypes.data, self.ts.ctypes.data, self.n)
        return s


def _ptr(a):
    return a.ctypes.data if a.size else None


def encode_segments(kv: KV, seg_start, block_size: int):
    """-> (rc, blocks u8, blk_off u64[nblk+1])."""
    seg = np.ascontiguousarray(seg_start, np.uint32)
    nseg = len(seg) - 1
    # upper bounds: every entry its own block, plus trailer bytes
    out_cap = int(len(kv.keys) + len(kv.vals) + 18 * kv.n + 16)
    blk_cap = kv.n + 1
    out = np.zeros(max(out_cap, 1), np.uint8)
    blk_off = np.zeros(blk_cap, np.uint64)
    nb, nbytes = ctypes.c_uint64(), ctypes.c_uint64()
    c = kv._c()
    rc = lib().orc_encode_segments(ctypes.byref(c), seg.ctypes.data, nseg, block_size,
                                   out.ctypes.data, out_cap, blk_off.ctypes.data, blk_cap,
                                   ctypes.byref(nb), ctypes.byref(nbytes))
    return rc, out[:nbytes.value], blk_off[:nb.value + 1]


def decode_blocks(blocks, blk_off):
    """-> (rc, KV)."""
    blocks = np.ascontiguousarray(blocks, np.uint8)
    blk_off = np.ascontiguousarray(blk_off, np.uint64)
    nblk = len(blk_off) - 1
    n, K, V = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    L = lib()
    # first pass with zero capacity to learn the totals
    empty = _OrcKV(None, None, None, None, None, 0)
    rc = L.orc_decode_blocks(_ptr(blocks), blk_off.ctypes.data, nblk, ctypes.byref(empty), 0, 0, 0,
                             ctypes.byref(n), ctypes.byref(K), ctypes.byref(V))
    if rc not in (ORC_OK, ORC_E_CAPACITY):
        return rc, None
    kv = KV(np.zeros(max(K.value, 1), np.uint8), np.zeros(n.value + 1, np.uint32),
            np.zeros(max(V.value, 1), np.uint8), np.zeros(n.value + 1, np.uint32),
            np.zeros(n.value, np.uint64))
    c = _OrcKV(kv.keys.ctypes.data, kv.key_off.ctypes.data, kv.vals.ctypes.data,
               kv.val_off.ctypes.data, kv.ts.ctypes.data if n.value else None, 0)
    rc = L.orc_decode_blocks(_ptr(blocks), blk_off.ctypes.data, nblk, ctypes.byref(c), n.value,
                             K.value, V.value, ctypes.byref(n), ctypes.byref(K), ctypes.byref(V))
    kv.keys = kv.keys[:K.value]
    kv.vals = kv.vals[:V.value]
    return rc, kv


def segment_like_compaction(kv: KV, block_size: int, target_sst_size: int):
    seg = np.zeros(kv.n + 2, np.uint32)
    ns = ctypes.c_uint64()
    c = kv._c()
    rc = lib().orc_segment_like_compaction(ctypes.byref(c), block_size, target_sst_size,
                                           seg.ctypes.data, len(seg), ctypes.byref(ns))
    assert rc == ORC_OK, rc
    return seg[:ns.value + 1]


def merge_runs(kv: KV, run_start):
    """MergeIterator over the sorted runs of kv -> src u32[n_merged] (input indices)."""
    rs = np.ascontiguousarray(run_start, np.uint32)
    src = np.zeros(max(kv.n, 1), np.uint32)
    n = ctypes.c_uint64()
    c = kv._c()
    rc = lib().orc_merge_runs(ctypes.byref(c), rs.ctypes.data, len(rs) - 1, src.ctypes.data, len(src),
                              ctypes.byref(n))
    assert rc == ORC_OK, rc
    return src[:n.value]


def gather(kv: KV, idx) -> KV:
    """The sub-stream kv[idx] (entries in the order of idx)."""
    idx = np.asarray(idx, np.int64)
    kl = (kv.key_off[idx + 1] - kv.key_off[idx]).astype(np.int64)
    vl = (kv.val_off[idx + 1] - kv.val_off[idx]).astype(np.int64)
    ko = np.zeros(len(idx) + 1, np.uint32)
    vo = np.zeros(len(idx) + 1, np.uint32)
    ko[1:] = np.cumsum(kl)
    vo[1:] = np.cumsum(vl)

    def cat(arena, off, ln):
        total = int(ln.sum())
        out = np.zeros(total, np.uint8)
        if len(idx) == 0 or total == 0:
            return out
        starts = off[idx].astype(np.int64)
        dst = np.concatenate([[0], np.cumsum(ln)])
        # in chunks of entries: the per-byte int64 index arrays of one chunk only (a 4 GB arena
        # gathered at once took 2 x 8 bytes of index per byte, ~50 GiB of host memory)
        step = 1 << 20
        for a in range(0, len(idx), step):
            b = min(a + step, len(idx))
            lo, hi = int(dst[a]), int(dst[b])
            if hi > lo:
                rep = np.repeat(starts[a:b] - dst[a:b], ln[a:b])
                out[lo:hi] = arena[np.arange(lo, hi, dtype=np.int64) + rep]
        return out
    return KV(cat(kv.keys, kv.key_off, kl), ko, cat(kv.vals, kv.val_off, vl), vo, kv.ts[idx].copy())


def compact(kv: KV, src, watermark, bottom, prefixes, block_size, target, kept_only=False):
    """compact_generate_sst over the merged stream kv[src] -> dict(blocks, blk_off, sst_blk,
    sst_ent, kept) (kept = merged positions added to an SST).  kept_only: only `kept` (no output
    buffers: the rules alone, for a range check that needs just the kept stream)."""
    src = np.ascontiguousarray(src, np.uint32)
    n = len(src)
    if kept_only:
        out_cap, out, blk_off, sst_blk, sst_ent = 0, np.zeros(1, np.uint8), np.zeros(1, np.uint64), \
            np.zeros(1, np.uint32), np.zeros(1, np.uint32)
        bcap = scap = 0
    else:
        kl = int((kv.key_off[src.astype(np.int64) + 1] - kv.key_off[src]).sum()) if n else 0
        vl = int((kv.val_off[src.astype(np.int64) + 1] - kv.val_off[src]).sum()) if n else 0
        out_cap = kl + vl + 18 * n + 16
        out = np.zeros(max(out_cap, 1), np.uint8)
        blk_off = np.zeros(n + 2, np.uint64)
        sst_blk = np.zeros(n + 2, np.uint32)
        sst_ent = np.zeros(n + 2, np.uint32)
        bcap = scap = n + 2
    kept = np.zeros(max(n, 1), np.uint32)
    pf = [bytes(p) for p in prefixes]
    pbufs = [ctypes.create_string_buffer(p, len(p)) for p in pf]
    parr = (ctypes.c_void_p * max(len(pf), 1))(*[ctypes.addressof(b) for b in pbufs])
    plen = (ctypes.c_size_t * max(len(pf), 1))(*[len(p) for p in pf])
    nb, nbytes, nsst, nk = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    c = kv._c()
    rc = lib().orc_compact(ctypes.byref(c), src.ctypes.data if n else None, n, watermark, int(bool(bottom)),
                           parr, plen, len(pf), block_size, target, out.ctypes.data, out_cap, blk_off.ctypes.data,
                           bcap, sst_blk.ctypes.data, sst_ent.ctypes.data, scap, kept.ctypes.data,
                           len(kept), ctypes.byref(nb), ctypes.byref(nbytes), ctypes.byref(nsst), ctypes.byref(nk))
    if kept_only:
        assert rc in (ORC_OK, ORC_E_CAPACITY) and nk.value <= len(kept), rc
        return dict(kept=kept[:nk.value])
    assert rc == ORC_OK, rc
    return dict(blocks=out[:nbytes.value], blk_off=blk_off[:nb.value + 1], sst_blk=sst_blk[:nsst.value + 1],
                sst_ent=sst_ent[:nsst.value + 1], kept=kept[:nk.value])


def shard_rotation(ext: KV, m: int, last: bool, p: int, d0: int, block_size: int, target: int, same=None):
    """compact_generate_sst's rotation resumed at a range's carry-in (orc_shard_rotation) ->
    (rc, segments u32[nseg+1], (p_out, d_out)).  same: the loop's same_as_last_key per ext entry
    (two-level compactions; None: the previous entry's key)."""
    seg = np.zeros(ext.n + 3, np.uint32)
    ns, po, do = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    c = ext._c()
    sm = None if same is None else np.ascontiguousarray(same, np.uint8)
    assert sm is None or len(sm) >= ext.n
    rc = lib().orc_shard_rotation_ex(ctypes.byref(c), None if sm is None else sm.ctypes.data, m, int(bool(last)), p,
                                     d0, block_size, target, seg.ctypes.data, len(seg), ctypes.byref(ns),
                                     ctypes.byref(po), ctypes.byref(do))
    return rc, seg[:ns.value + 1] if ns.value else seg[:0], (po.value, do.value)


def encode_span(kv: KV, seg, block_size: int):
    """Blocks of the segments seg[0..] of kv, which may start after entry 0 and end before kv.n."""
    seg = np.asarray(seg, np.int64)
    if len(seg) < 2:
        return 0, np.zeros(0, np.uint8), np.zeros(1, np.uint64)
    a, b = int(seg[0]), int(seg[-1])
    ka, va = int(kv.key_off[a]), int(kv.val_off[a])
    # entries [a, b) as views of the arenas (only the offsets are rebased, no byte copy)
    sub = KV(kv.keys[ka:int(kv.key_off[b])], (kv.key_off[a:b + 1] - ka).astype(np.uint32),
             kv.vals[va:int(kv.val_off[b])], (kv.val_off[a:b + 1] - va).astype(np.uint32), kv.ts[a:b])
    return encode_segments(sub, (seg - a).astype(np.uint32), block_size)


class Builder:
    """Per-entry BlockBuilder (src/block/builder.rs) on the C restatement."""

    def __init__(self, block_size):
        self.h = lib().orc_builder_new(block_size)

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_builder_free(self.h)

    def add(self, key: bytes, ts: int, value: bytes) -> int:
        return lib().orc_builder_add(self.h, key, len(key), ts, value, len(value))

    def is_empty(self):
        return bool(lib().orc_builder_is_empty(self.h))

    def estimated_size(self):
        return lib().orc_builder_estimated_size(self.h)

    def finish(self) -> bytes:
        cap = self.estimated_size()
        buf = ctypes.create_string_buffer(cap)
        ln = ctypes.c_size_t()
        rc = lib().orc_builder_finish(self.h, buf, cap, ctypes.byref(ln))
        assert rc == ORC_OK, rc
        return buf.raw[:ln.value]


def seek_key(block: bytes, key: bytes) -> int:
    return lib().orc_block_seek_key(block, len(block), key, len(key))


def entry_verbatim(block: bytes, idx: int):
    p, s = ctypes.c_uint32(), ctypes.c_uint32()
    vb, ve = ctypes.c_size_t(), ctypes.c_size_t()
    rc = lib().orc_block_entry_verbatim(block, len(block), idx, ctypes.byref(p), ctypes.byref(s),
                                        ctypes.byref(vb), ctypes.byref(ve))
    assert rc == ORC_OK
    return p.value, s.value, vb.value, ve.value


def crc32(data: bytes) -> int:
    return lib().orc_crc32(data, len(data))
