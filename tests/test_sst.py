"""SST container (SURVEY.md §8 f rows 3-4): whole SST files, the bloom filter, the memtable flush
source.

CPU: the oracle's Bloom against the reference's own test (src/table/bloom.rs:123-157: raw key
hashes 123/456/789, bits_per_key 10), the library's host pieces (fingerprint32, may_contain,
memtable) against the oracle, and the product's SST parser over oracle-built files.
GPU: lsmblk_sst_files_batch bytes == oracle/pyref.sst_file (SsTableBuilder::build restated) for
flushed and compacted SSTs, LDS and global bloom paths; framed read_block round trip and CRC check.

farmhash::fingerprint32 (crate farmhash 1.1.5) has no vector in the reference: the library's and
the oracle's restatements of its published algorithm (farmhashmk Hash32) are checked against each
other only -- parity unpinned for the hash itself.
"""
import numpy as np
import pytest
import torch

from lsm_amd import batch, synth
from lsm_amd import sst as S
from lsm_amd._lib import LsmBlkError
from oracle import oracle as O
from oracle import pyref


def rand_keys(rng, n, lo=1, hi=24):
    return [bytes(rng.integers(0, 256, int(rng.integers(lo, hi)), dtype=np.uint8)) for _ in range(n)]


# ---------------------------------------------------------------- CPU
def test_bloom_reference_unit_test():  # bloom.rs:129-157
    b = pyref.Bloom.build_from_key_hashes([123, 456, 789], 10)
    d = pyref.Bloom.decode(b.encode())
    assert d.filter == b.filter and d.k == b.k == 6
    assert d.may_contain(123)
    assert pyref.Bloom.bloom_bits_per_key(3, 0.01) == 10
    assert len(d.filter) == 8  # nbits = max(3 * 10, 64) (:86-88)


def test_bloom_bits_per_key_is_10_at_every_size():
    for n in (1, 2, 7, 100, 26214, 10**6):
        assert pyref.Bloom.bloom_bits_per_key(n, 0.01) == 10


def test_library_may_contain_equals_oracle():
    rng = np.random.default_rng(1)
    for n in (1, 5, 300):
        hs = [int(h) for h in rng.integers(0, 1 << 32, n, dtype=np.uint64)]
        b = pyref.Bloom.build_from_key_hashes(hs, 10)
        assert all(S.lib().lsmblk_bloom_may_contain(b.filter, len(b.filter), b.k, h) for h in hs)
        probes = [int(h) for h in rng.integers(0, 1 << 32, 500, dtype=np.uint64)]
        got = [bool(S.lib().lsmblk_bloom_may_contain(b.filter, len(b.filter), b.k, h)) for h in probes]
        assert got == [b.may_contain(h) for h in probes]
    assert S.lib().lsmblk_bloom_may_contain(b"\x00" * 8, 8, 31, 5) == 1  # k > 30 -> true (:105-107)


def test_fingerprint32_library_equals_oracle():
    rng = np.random.default_rng(2)
    keys = [b"", b"a", b"hello"] + [bytes(rng.integers(0, 256, L, dtype=np.uint8)) for L in range(0, 70)]
    keys += rand_keys(rng, 200, 1, 300)
    assert [S.fingerprint32(k) for k in keys] == [pyref.fingerprint32(k) for k in keys]


def test_memtable_semantics_equal_oracle():
    rng = np.random.default_rng(3)
    space = rand_keys(rng, 200, 1, 6)
    puts = [(space[int(rng.integers(0, len(space)))], int(rng.integers(0, 1 << 40)),
             b"" if rng.random() < 0.1 else bytes(rng.integers(0, 256, int(rng.integers(1, 30)), dtype=np.uint8)))
            for _ in range(2000)]
    mt = S.MemTable()
    for k, t, v in puts:
        mt.put(k, t, v)
    want = pyref.memtable_flush(puts)
    keys, ko, vals, vo, ts = mt.flush_arrays()
    got = [(bytes(keys[ko[i]:ko[i + 1]]), int(ts[i]), bytes(vals[vo[i]:vo[i + 1]])) for i in range(len(ts))]
    assert got == want and len(mt) == len(want)
    assert mt.approximate_size() == sum(len(k) + 8 + len(v) for k, _, v in puts)  # mem_table.rs:119-125
    k, t, v = want[len(want) // 2]
    assert mt.get(k) == (v, t)
    assert mt.get(b"\xff" * 9) is None


def test_sst_parser_over_oracle_files():
    """The product's SsTable footer/bloom/meta parser (host logic) over pyref.sst_file bytes."""
    rng = np.random.default_rng(4)
    keys = sorted(set(rand_keys(rng, 3000, 2, 12)))
    ents = [(k, 0, bytes(rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8))) for k in keys]
    buf = pyref.sst_file(ents, 256)
    t = S.SsTable(buf, device="cpu")
    metas, max_ts, bloom, meta_off = pyref.sst_open(buf)
    assert [(m.offset, m.first_key, m.last_key) for m in t.block_meta] == metas
    assert t.block_meta_offset == meta_off and t.max_ts == max_ts == 0
    assert (t.bloom_filter, t.bloom_k) == (bloom.filter, bloom.k)
    assert t.first_key == keys[0] and t.last_key == keys[-1]
    assert all(t.may_contain(k) for k in keys)
    for k in keys[::97]:
        i = t.find_block_idx(k)
        assert metas[i][1] <= k and (i + 1 == len(metas) or metas[i + 1][1] > k)
    bad = bytearray(buf)
    bad[meta_off + 6] ^= 1
    with pytest.raises(ValueError, match="meta checksum"):
        S.SsTable(bytes(bad), device="cpu")
    bad = bytearray(buf)
    bad[-10] ^= 1
    with pytest.raises(ValueError, match="bloom"):
        S.SsTable(bytes(bad), device="cpu")


# ---------------------------------------------------------------- GPU
def _gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")


@pytest.mark.gpu
@pytest.mark.parametrize("n,bs", [(1, 4096), (37, 64), (2000, 256), (30000, 4096)])
def test_gpu_flush_memtable_file_equals_oracle(n, bs):
    """MemTable -> flush -> SsTableBuilder::build on the device == the restatement, byte for byte.
    n=30000 > 26214 keys puts the bitmap over 32 KiB: the global-atomics bloom path."""
    _gpu()
    rng = np.random.default_rng(n)
    puts = [(k, int(rng.integers(0, 1 << 50)), bytes(rng.integers(0, 256, int(rng.integers(0, 60)), dtype=np.uint8)))
            for k in rand_keys(rng, n + n // 4, 1, 20)]
    mt = S.MemTable()
    for k, t, v in puts:
        mt.put(k, t, v)
    want = pyref.sst_file(pyref.memtable_flush(puts), bs)
    got = S.flush_memtable(mt, bs)
    assert got == want


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(3))
def test_gpu_compaction_sst_files_equal_oracle(seed):
    """Every SST of a device compaction, framed into a whole file on the device == pyref.sst_file
    over the SST's entries (each SST is a fresh SsTableBuilder, compact.rs:276-300)."""
    _gpu()
    keys, ko, vals, vo, ts, rs = synth.gen_runs(6000, nrun=4, seed=20 + seed, versions=1 + seed)
    kv = batch.KVStream.from_numpy(keys, ko, vals, vo, ts)
    r = batch.compact_runs(kv, rs, watermark=int(ts.max()) // 2, bottom_level=bool(seed % 2), block_size=1024,
                           target_sst_size=64 << 10)
    kept = r["kept"]
    files, off = S.sst_files(r["blocks"], r["blk_off"], r["sst_blk"], r["sst_start"], kept)
    files, off = files.cpu().numpy().tobytes(), off.cpu().tolist()
    k2, ko2, v2, vo2, ts2 = kept.to_numpy()
    ents = [(bytes(k2[ko2[i]:ko2[i + 1]]), int(ts2[i]), bytes(v2[vo2[i]:vo2[i + 1]])) for i in range(kept.n)]
    ss = r["sst_start"].cpu().numpy().view(np.uint32)
    assert len(off) - 1 == len(ss) - 1 > 2
    for s in range(len(ss) - 1):
        assert files[off[s]:off[s + 1]] == pyref.sst_file(ents[ss[s]:ss[s + 1]], 1024), s


@pytest.mark.gpu
def test_gpu_sst_read_blocks_round_trip_and_crc():
    """SsTable::read_block for every block at once (framed decode with the CRC check) gives back
    the flushed entries; a flipped data byte raises CHECKSUM."""
    _gpu()
    rng = np.random.default_rng(9)
    ents = sorted({k: (k, 7, k[::-1] * 3) for k in rand_keys(rng, 5000, 1, 16)}.values())
    mt = S.MemTable()
    for k, t, v in ents:
        mt.put(k, t, v)
    buf = S.flush_memtable(mt, 512)
    t = S.SsTable(buf)
    d = t.decode_blocks()
    keys, ko, vals, vo, ts = d.to_numpy()
    got = [(bytes(keys[ko[i]:ko[i + 1]]), int(ts[i]), bytes(vals[vo[i]:vo[i + 1]])) for i in range(d.n)]
    assert got == ents
    mid = t.num_of_blocks() // 2
    part = t.decode_blocks(mid, mid + 2)
    assert part.n == len(pyref.block_entries(buf[t.block_meta[mid].offset:t.block_meta[mid + 1].offset - 4])) + \
        len(pyref.block_entries(buf[t.block_meta[mid + 1].offset:t.block_meta[mid + 2].offset - 4]))
    bad = bytearray(buf)
    bad[t.block_meta[mid].offset + 3] ^= 0x40
    with pytest.raises(LsmBlkError):
        S.SsTable(bytes(bad)).decode_blocks()


def test_memtable_get_copies_under_the_lock():
    """get() copies the value under the memtable's lock (lsmblk_memtable_get_copy): values larger
    than the first buffer, replaced values, absent keys, and the capacity error of the raw call."""
    import ctypes
    from lsm_amd._lib import LSMBLK_E_CAPACITY, lib
    mt = S.MemTable()
    mt.put(b"k", 1, b"x" * 5000)
    assert mt.get(b"k") == (b"x" * 5000, 1)
    mt.put(b"k", 2, b"short")
    assert mt.get(b"k") == (b"short", 2) and mt.get(b"nope") is None
    mt.put(b"e", 3, b"")
    assert mt.get(b"e") == (b"", 3)
    n, t, buf = ctypes.c_size_t(), ctypes.c_uint64(), ctypes.create_string_buffer(2)
    assert lib().lsmblk_memtable_get_copy(mt.h, b"k", 1, buf, 2, ctypes.byref(n), ctypes.byref(t)) == LSMBLK_E_CAPACITY
    assert n.value == 5 and t.value == 2
