"""SST container (SURVEY.md §8 f, rows 3 and 4): whole SST files and the memtable flush source.

  MemTable          reference src/mem_table.rs:55-158 (host; the flush source of the encoder)
  sst_files         SsTableBuilder::build (src/table/builder.rs:68-98) for every SST of an encode
                    or compaction, on the device: framed data section, BlockMeta section,
                    meta_offset, bloom filter over farmhash::fingerprint32, bloom_offset
  flush_memtable    force_flush_next_imm_memtable's SST (src/lsm_storage.rs:692-744): memtable ->
                    KV batch -> device encode -> one SST file
  SsTable           SsTable::open / read_block / find_block_idx (src/table.rs:162-257) over a file
                    held in memory; blocks are decoded on the device from the framed data section
                    with the read_block CRC check (lsmblk_decode_batch_ex)

Device work goes through liblsmblk.so; the footer / section parsing here is host logic that mirrors
the reference's own (the CRC-32 of those small sections is zlib's, which is crc32fast's).
"""
import ctypes
import zlib

import numpy as np
import torch

from . import batch
from ._lib import LSMBLK_E_CAPACITY, LsmBlkError, check, lib


class MemTable:
    """MemTable (src/mem_table.rs:55-158): key order ignores the ts, so a put of a present key
    replaces the entry; flush() yields the entries in key order."""

    def __init__(self):
        self.h = lib().lsmblk_memtable_new()
        if not self.h:
            raise MemoryError("lsmblk_memtable_new")

    def __del__(self):
        if getattr(self, "h", None):
            lib().lsmblk_memtable_free(self.h)
            self.h = None

    def put(self, key: bytes, ts: int, value: bytes):
        check(lib().lsmblk_memtable_put(self.h, key, len(key), ts, value, len(value)), "memtable put")

    def get(self, key: bytes):
        """(value, ts) or None; the value is copied under the memtable's lock."""
        n, t = ctypes.c_size_t(), ctypes.c_uint64()
        buf = ctypes.create_string_buffer(256)
        for _ in range(8):  # a concurrent put may grow the value between the size probe and the copy
            found = lib().lsmblk_memtable_get_copy(self.h, key, len(key), buf, len(buf), ctypes.byref(n),
                                                   ctypes.byref(t))
            if found != LSMBLK_E_CAPACITY:
                break
            buf = ctypes.create_string_buffer(max(n.value, 1))
        if found < 0:
            raise LsmBlkError(found, "memtable get")
        return (buf.raw[:n.value], t.value) if found else None

    def __len__(self):
        return lib().lsmblk_memtable_len(self.h)

    def approximate_size(self):
        return lib().lsmblk_memtable_approximate_size(self.h)

    def flush_arrays(self):
        """MemTable::flush (:131-136) -> (keys u8, key_off u32, vals u8, val_off u32, ts u64)."""
        n, K, V = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        lib().lsmblk_memtable_flush(self.h, None, None, None, None, None, 0, 0, 0, ctypes.byref(n), ctypes.byref(K),
                                    ctypes.byref(V))
        keys = np.zeros(max(K.value, 1), np.uint8)
        vals = np.zeros(max(V.value, 1), np.uint8)
        ko = np.zeros(n.value + 1, np.uint32)
        vo = np.zeros(n.value + 1, np.uint32)
        ts = np.zeros(max(n.value, 1), np.uint64)
        check(lib().lsmblk_memtable_flush(self.h, keys.ctypes.data, ko.ctypes.data, vals.ctypes.data, vo.ctypes.data,
                                          ts.ctypes.data, n.value, K.value, V.value, ctypes.byref(n), ctypes.byref(K),
                                          ctypes.byref(V)), "memtable flush")
        return keys[:K.value], ko, vals[:V.value], vo, ts[:n.value]


def fingerprint32(key: bytes) -> int:
    """farmhash::fingerprint32 (src/table/builder.rs:53), the library's restatement."""
    return lib().lsmblk_fingerprint32(key, len(key))


def sst_files(blocks, blk_off, sst_blk, sst_ent, kv: batch.KVStream, stream=None):
    """Whole SST files for every SST (sst_blk / sst_ent: u32 tables of nsst+1) -> (files u8 tensor,
    file_off int64 tensor[nsst+1]); file s = files[file_off[s]:file_off[s+1]]."""
    dev = torch.device("cuda", batch._dev_index(blk_off))
    sst_blk, sst_ent = batch._u32_table(sst_blk, dev), batch._u32_table(sst_ent, dev)
    nsst, nblk = sst_blk.numel() - 1, blk_off.numel() - 1
    batch._need(blk_off, torch.int64, "blk_off", dev.index, nblk + 1)
    kv.check(dev.index, "kv")
    file_off = torch.zeros(nsst + 1, dtype=torch.int64, device=dev)
    stats = torch.zeros(batch.STATS_WORDS, dtype=torch.int64, device=dev)
    kb, _ = kv.byte_sizes()
    cap = int(blocks.numel()) + 8 * nblk + 2 * kb + 64 * nsst + 2 * kv.n + 1024
    for _ in range(2):
        files = batch._aligned_empty(cap, dev)
        c = kv._c()
        batch._native("lsmblk_sst_files_batch", dev.index, stream, batch._ptr(blocks), blk_off.data_ptr(), nblk,
                      sst_blk.data_ptr(), sst_ent.data_ptr(), nsst, ctypes.byref(c),
                      files.data_ptr(), cap, file_off.data_ptr(), stats.data_ptr(),
                      batch._stream_ptr(stream, dev.index))
        torch.cuda.synchronize(dev)
        st = batch._status(stats)
        if st == -3:
            cap = int(stats[1].item())
            continue
        if st:
            raise LsmBlkError(st, "sst_files")
        return files[:int(stats[1].item())], file_off
    raise LsmBlkError(-3, "sst_files")


def flush_memtable(mt: MemTable, block_size: int = 4096, device="cuda", stream=None) -> bytes:
    """force_flush_next_imm_memtable's SST (src/lsm_storage.rs:692-744): MemTable::flush into one
    SsTableBuilder (one segment), encoded and framed on the device -> the SST file bytes."""
    keys, ko, vals, vo, ts = mt.flush_arrays()
    if len(ts) == 0:
        raise ValueError("flushing an empty memtable builds an empty SST (the reference panics)")
    d = batch.KVStream.from_numpy(keys, ko, vals, vo, ts, device=device)
    r = batch.encode_sst(d, np.array([0, d.n], np.uint32), block_size, stream)
    files, off = sst_files(r["blocks"], r["blk_off"], r["seg_blk"], np.array([0, d.n], np.uint32), d, stream)
    return files.cpu().numpy().tobytes()


class BlockMeta:
    __slots__ = ("offset", "first_key", "last_key")

    def __init__(self, offset, first_key, last_key):
        self.offset, self.first_key, self.last_key = offset, first_key, last_key


def _decode_block_meta(buf: bytes):
    """BlockMeta::decode_block_meta (src/table.rs:65-93)."""
    num = int.from_bytes(buf[0:4], "big")
    if int.from_bytes(buf[-4:], "big") != zlib.crc32(buf[4:-4]):
        raise ValueError("meta checksum mismatched")
    pos, metas = 4, []
    for _ in range(num):
        off = int.from_bytes(buf[pos:pos + 4], "big")
        fl = int.from_bytes(buf[pos + 4:pos + 6], "big")
        fk = bytes(buf[pos + 6:pos + 6 + fl])
        pos += 6 + fl + 8
        ll = int.from_bytes(buf[pos:pos + 2], "big")
        lk = bytes(buf[pos + 2:pos + 2 + ll])
        pos += 2 + ll + 8
        metas.append(BlockMeta(off, fk, lk))
    return metas, int.from_bytes(buf[pos:pos + 8], "big")


class SsTable:
    """SsTable (src/table.rs:136-283) over a whole file in memory (the reference preads it)."""

    def __init__(self, buf: bytes, device="cuda"):
        n = len(buf)
        bloom_offset = int.from_bytes(buf[n - 4:], "big")  # open, :164-168
        raw = buf[bloom_offset:n - 4]
        if int.from_bytes(raw[-4:], "big") != zlib.crc32(raw[:-4]):
            raise ValueError("checksum mismatched for bloom filters")  # bloom.rs:49-54
        self.bloom_filter, self.bloom_k = bytes(raw[:-5]), raw[-5]
        self.block_meta_offset = int.from_bytes(buf[bloom_offset - 4:bloom_offset], "big")  # :170-172
        self.block_meta, self.max_ts = _decode_block_meta(buf[self.block_meta_offset:bloom_offset - 4])
        self.first_key = self.block_meta[0].first_key
        self.last_key = self.block_meta[-1].last_key
        self.buf, self.device = buf, device

    def num_of_blocks(self):
        return len(self.block_meta)

    def find_block_idx(self, key: bytes) -> int:  # :253-257 (partition_point, ts-agnostic)
        lo, hi = 0, len(self.block_meta)
        while lo < hi:
            mid = (lo + hi) // 2
            if self.block_meta[mid].first_key <= key:
                lo = mid + 1
            else:
                hi = mid
        return max(lo - 1, 0)

    def may_contain(self, key: bytes) -> bool:  # bloom.may_contain(fingerprint32(key)), lsm_storage.rs:389-391
        f = self.bloom_filter
        return bool(lib().lsmblk_bloom_may_contain(f, len(f), self.bloom_k, fingerprint32(key)))

    def block_offsets(self):
        """Framed block ranges: BlockMeta offsets, then the meta section (read_block, :215-220)."""
        return np.array([m.offset for m in self.block_meta] + [self.block_meta_offset], np.uint64)

    def decode_blocks(self, lo=0, hi=None, verify=True):
        """read_block for blocks [lo, hi) at once (:213-233): the framed ranges decoded on the
        device with the CRC check -> KVStream."""
        off = self.block_offsets()
        hi = len(self.block_meta) if hi is None else hi
        a, b = int(off[lo]), int(off[hi])
        data = torch.frombuffer(bytearray(self.buf[a:b]), dtype=torch.uint8).to(self.device)
        rel = torch.from_numpy((off[lo:hi + 1] - off[lo]).view(np.int64)).to(self.device)
        return batch.decode_blocks(data, rel, tail=4, verify=verify)
