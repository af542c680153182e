"""GPU parity: the HIP batch path (through the C ABI) against the CPU oracle.

Bar: bit-exact -- encoded blocks byte for byte, decoded KV streams array for array.
The oracle (oracle/lsmblk_oracle.c) is only the checker here.
"""
import zlib

import numpy as np
import pytest
import torch

from lsm_amd import batch, synth
from lsm_amd._lib import LSMBLK_E_CAPACITY, LSMBLK_E_MALFORMED, LsmBlkError
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")


def to_dev(kv: O.KV):
    return batch.KVStream.from_numpy(kv.keys, kv.key_off, kv.vals, kv.val_off, kv.ts)


def dev_blocks(blocks, blk_off, shift=0):
    buf = torch.zeros(len(blocks) + shift + 16, dtype=torch.uint8, device="cuda")
    if len(blocks):
        buf[shift:shift + len(blocks)] = torch.from_numpy(np.ascontiguousarray(blocks))
    off = torch.from_numpy(np.ascontiguousarray(blk_off, np.uint64).view(np.int64)).cuda()
    return buf[shift:shift + len(blocks)], off


def assert_kv_equal(dkv: batch.KVStream, ref: O.KV):
    keys, ko, vals, vo, ts = dkv.to_numpy()
    assert dkv.n == ref.n
    np.testing.assert_array_equal(ko, ref.key_off)
    np.testing.assert_array_equal(vo, ref.val_off)
    np.testing.assert_array_equal(ts, ref.ts)
    np.testing.assert_array_equal(keys, ref.keys[:ref.key_off[-1]])
    np.testing.assert_array_equal(vals, ref.vals[:ref.val_off[-1]])


def seg_slots(kv: O.KV, seg):
    """slot(s) of LSMBLK_ENCODE_SEG_SLOTS (include/lsmblk.h), in numpy."""
    s = np.asarray(seg, dtype=np.int64)
    ko, vo = kv.key_off.astype(np.int64), kv.val_off.astype(np.int64)
    return (ko[s[:-1]] - ko[s[0]]) + (vo[s[:-1]] - vo[s[0]]) + 18 * (s[:-1] - s[0])


def slot_check(kv: O.KV, seg, block_size, ref_blocks, ref_off):
    """LSMBLK_ENCODE_SEG_SLOTS through plan_walk + emit and through the fused walk + emit launch
    (LSMBLK_DEBUG_ENCODE_FUSED): every segment at its slot, the segments packed == the oracle's
    blocks and offsets."""
    from lsm_amd._lib import LSMBLK_DEBUG_ENCODE_FUSED, lib
    ctx = batch._ctx(0)
    for fused in (0, 1):
        assert lib().lsmblk_debug_set(ctx, LSMBLK_DEBUG_ENCODE_FUSED, fused) == 0
        try:
            out, off, so = batch.encode_kv_slots(to_dev(kv), seg, block_size)
        finally:
            lib().lsmblk_debug_set(ctx, LSMBLK_DEBUG_ENCODE_FUSED, 0)
        np.testing.assert_array_equal(so[:, 0].cpu().numpy(), seg_slots(kv, seg))
        blocks, poff = batch.slots_to_packed(out, off, so)
        np.testing.assert_array_equal(poff.cpu().numpy().view(np.uint64), ref_off)
        got = blocks.cpu().numpy()
        assert len(got) == len(ref_blocks)
        mism = np.flatnonzero(got != ref_blocks)
        assert mism.size == 0, f"slots (fused={fused}): first mismatching byte {mism[:8]} of {len(got)}"


def framed_want(ref_blocks, ref_off):
    """The SST data section of packed blocks: every block followed by its crc32fast, big-endian
    (SsTableBuilder::finish_block, src/table/builder.rs:112-123) -> (bytes, offsets u64[nblk+1])."""
    parts, offs, o = [], [0], 0
    for b in range(len(ref_off) - 1):
        blk = bytes(ref_blocks[int(ref_off[b]):int(ref_off[b + 1])])
        parts.append(blk + zlib.crc32(blk).to_bytes(4, "big"))
        o += len(blk) + 4
        offs.append(o)
    return b"".join(parts), np.asarray(offs, np.uint64)


def framed_check(kv: O.KV, seg, block_size, ref_blocks, ref_off):
    """LSMBLK_ENCODE_FRAMED, packed and with per-segment slots: the output is the blocks each
    followed by its BE crc32, the verifying framed decode (tail 4) reads it back."""
    want, want_off = framed_want(ref_blocks, ref_off)
    d = to_dev(kv)
    out, off = batch.encode_kv_framed(d, seg, block_size)
    np.testing.assert_array_equal(off.cpu().numpy().view(np.uint64), want_off)
    assert out.cpu().numpy().tobytes() == want
    if len(ref_off) > 1:
        dkv = batch.decode_blocks(out, off, tail=4, verify=True)
        assert dkv.n == kv.n
        k, ko, v, vo, ts = dkv.to_numpy()
        np.testing.assert_array_equal(ko, kv.key_off)
        np.testing.assert_array_equal(ts, kv.ts[:kv.n])
    sout, soff, so = batch.encode_kv_framed(d, seg, block_size, slots=True)
    so = so.cpu().numpy()
    s = np.asarray(seg, dtype=np.int64)
    ko, vo = kv.key_off.astype(np.int64), kv.val_off.astype(np.int64)
    np.testing.assert_array_equal(so[:, 0], (ko[s[:-1]] - ko[s[0]]) + (vo[s[:-1]] - vo[s[0]]) + 22 * (s[:-1] - s[0]))
    host = sout.cpu().numpy()
    assert b"".join(host[a:a + n].tobytes() for a, n in so) == want


def roundtrip_check(kv: O.KV, seg, block_size, shift=0):
    """GPU encode == oracle encode (packed, and per-segment slots); GPU decode(oracle blocks) ==
    oracle decode."""
    rc, ref_blocks, ref_off = O.encode_segments(kv, seg, block_size)
    assert rc == 0
    blocks, blk_off = batch.encode_kv(to_dev(kv), seg, block_size)
    got_off = blk_off.cpu().numpy().view(np.uint64)
    np.testing.assert_array_equal(got_off, ref_off)
    got = blocks.cpu().numpy()
    assert len(got) == len(ref_blocks)
    mism = np.flatnonzero(got != ref_blocks)
    assert mism.size == 0, f"first mismatching byte {mism[:8]} of {len(got)}"
    slot_check(kv, seg, block_size, ref_blocks, ref_off)
    framed_check(kv, seg, block_size, ref_blocks, ref_off)
    rc, ref_kv = O.decode_blocks(ref_blocks, ref_off)
    assert rc == 0
    db, do = dev_blocks(ref_blocks, ref_off, shift)
    dkv = batch.decode_blocks(db, do)
    assert_kv_equal(dkv, ref_kv)
    return ref_blocks, ref_off


def week1_day3_kv():
    # src/tests/week1_day3.rs:45-65
    return O.KV.from_entries([(b"key_%03d" % (i * 5), 0, b"value_%010d" % i) for i in range(100)])


def test_kat_week1_day3_block():
    kv = week1_day3_kv()
    blocks, off = roundtrip_check(kv, [0, 100], 10000)
    assert len(off) == 2 and len(blocks) == 3486


def test_week1_day4_day7_block_size_128():
    kv = week1_day3_kv()
    _, off = roundtrip_check(kv, [0, 100], 128)
    assert len(off) - 1 == 34  # week1_day7.rs:83-87 expects <= 34 with ts


def test_week3_day1_multi_version():
    # src/tests/week3_day1.rs:31-40
    ents = [(b"key%05d" % (i // 5), 5 - (i % 5), b"value%05d" % i) for i in range(100)]
    kv = O.KV.from_entries(ents)
    roundtrip_check(kv, [0, 100], 128)


def test_block_size_16_every_entry_own_block():
    ents = [(k, 0, v) for k, v in [(b"11", b"11"), (b"22", b"22"), (b"33", b"11"), (b"44", b"22"),
                                   (b"55", b"11"), (b"66", b"22")]]
    kv = O.KV.from_entries(ents)
    _, off = roundtrip_check(kv, [0, 6], 16)
    assert len(off) - 1 == 6


@pytest.mark.parametrize("cfg,n", [("U", 10000), ("Z", 20000), ("M", 3000)])
def test_configs_small(cfg, n):
    kv = O.KV(*synth.GENERATORS[cfg](n, seed=7))
    seg = synth.segments_by_bytes(kv.key_off, kv.val_off, 256 << 10)
    roundtrip_check(kv, seg, synth.BLOCK_SIZE[cfg])


def test_cpu_plumbing_config_323_blocks():
    kv = O.KV(*synth.gen_uniform(10000, seed=0))
    _, off = roundtrip_check(kv, [0, kv.n], 4096)
    assert len(off) - 1 == 323


def test_unaligned_block_stream():
    kv = O.KV(*synth.gen_uniform(3000, seed=3))
    roundtrip_check(kv, [0, kv.n], 4096, shift=3)


def test_block_offsets_beyond_2gib_and_4gib():
    """blk_off values past 2**31 and 2**32: byte offsets are u64 end to end (a readlane of
    the low half into a u64 once sign-extended bit 31 in an experimental decode)."""
    kv = O.KV(*synth.gen_uniform(20000, seed=5))
    seg = synth.segments_by_bytes(kv.key_off, kv.val_off, 256 << 10)
    rc, ref_blocks, ref_off = O.encode_segments(kv, seg, 4096)
    assert rc == 0
    rc, ref_kv = O.decode_blocks(ref_blocks, ref_off)
    assert rc == 0
    for base in ((1 << 31) - 5000, (1 << 32) + 3):
        buf = torch.zeros(base + len(ref_blocks) + 16, dtype=torch.uint8, device="cuda")
        buf[base:base + len(ref_blocks)] = torch.from_numpy(ref_blocks).cuda()
        off = torch.from_numpy((ref_off.astype(np.uint64) + np.uint64(base)).view(np.int64)).cuda()
        assert_kv_equal(batch.decode_blocks(buf, off), ref_kv)
        del buf, off
        torch.cuda.empty_cache()


def test_unaligned_key_and_value_arenas():
    kv = O.KV(*synth.gen_zipf(5000, seed=5))
    rc, ref_blocks, ref_off = O.encode_segments(kv, [0, kv.n], 4096)
    d = to_dev(kv)
    # re-home the arenas at odd addresses
    kbuf = torch.zeros(d.keys.numel() + 32, dtype=torch.uint8, device="cuda")
    vbuf = torch.zeros(d.vals.numel() + 32, dtype=torch.uint8, device="cuda")
    kbuf[5:5 + d.keys.numel()] = d.keys
    vbuf[11:11 + d.vals.numel()] = d.vals
    d.keys, d.vals = kbuf[5:5 + d.keys.numel()], vbuf[11:11 + d.vals.numel()]
    blocks, blk_off = batch.encode_kv(d, [0, kv.n], 4096)
    np.testing.assert_array_equal(blocks.cpu().numpy(), ref_blocks)


def test_many_tiny_entries_per_block():
    # 1-byte keys cannot be unique for long; use 2..4-byte keys and empty values (tombstones)
    rng = np.random.default_rng(1)
    keys = sorted({bytes(rng.integers(0, 256, rng.integers(1, 5), dtype=np.uint8)) for _ in range(6000)})
    ents = [(k, int(rng.integers(0, 1 << 40)), b"" if i % 3 else b"v") for i, k in enumerate(keys)]
    kv = O.KV.from_entries(ents)
    _, off = roundtrip_check(kv, [0, kv.n], 4096)
    assert (np.diff(off) > 0).all()


@pytest.mark.parametrize("value_len,shift", [(8, 0), (8, 5), (12, 3)])
def test_fast_path_blocks_with_64_to_128_entries(value_len, shift):
    # 16-B keys + small values: ~100 entries per 4 KiB block, i.e. more entries than lanes
    # in a wave but still on the LDS-table (fast) paths of encode and decode
    kv = O.KV(*synth.gen_uniform(20000, seed=12 + value_len, value_len=value_len))
    _, off = roundtrip_check(kv, [0, kv.n], 4096, shift=shift)
    per_block = kv.n / (len(off) - 1)
    assert 64 < per_block <= 128


def test_small_random_values_mixed_entry_counts():
    rng = np.random.default_rng(13)
    kv0 = O.KV(*synth.gen_uniform(15000, seed=13))
    keys = [bytes(kv0.keys[16 * i:16 * i + 16]) for i in range(kv0.n)]
    ents = [(k, int(kv0.ts[i]), bytes(rng.integers(0, 256, int(rng.integers(0, 24)), dtype=np.uint8)))
            for i, k in enumerate(keys)]
    kv = O.KV.from_entries(ents)
    roundtrip_check(kv, [0, kv.n], 4096, shift=7)


def test_long_keys_and_shared_prefixes():
    rng = np.random.default_rng(2)
    base = bytes(rng.integers(0, 256, 90, dtype=np.uint8))
    keys = sorted({base[:int(rng.integers(20, 90))] + bytes(rng.integers(0, 256, 8, dtype=np.uint8))
                   for _ in range(2000)})
    ents = [(k, i, bytes(rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8)))
            for i, k in enumerate(keys)]
    kv = O.KV.from_entries(ents)
    roundtrip_check(kv, [0, kv.n], 4096)
    roundtrip_check(kv, [0, 700, 700, 1500, kv.n], 1024)  # includes an empty segment


def test_oversize_entries_and_u16_wrap():
    # a 70000-byte value: always accepted as a block's first entry; value_len `as u16` wraps
    ents = [(b"a", 1, b"x" * 10), (b"b", 2, bytes(range(256)) * 273 + b"yz"), (b"c", 3, b"z" * 5000),
            (b"d", 4, b"w")]
    kv = O.KV.from_entries(ents)
    rc, ref_blocks, ref_off = O.encode_segments(kv, [0, kv.n], 4096)
    blocks, blk_off = batch.encode_kv(to_dev(kv), [0, kv.n], 4096)
    np.testing.assert_array_equal(blk_off.cpu().numpy().view(np.uint64), ref_off)
    np.testing.assert_array_equal(blocks.cpu().numpy(), ref_blocks)


def _encode_and_decode_like_oracle(kv, seg, bs):
    rc, ref_blocks, ref_off = O.encode_segments(kv, seg, bs)
    assert rc == 0
    blocks, blk_off = batch.encode_kv(to_dev(kv), seg, bs)
    np.testing.assert_array_equal(blk_off.cpu().numpy().view(np.uint64), ref_off)
    got = blocks.cpu().numpy()
    assert len(got) == len(ref_blocks) and np.flatnonzero(got != ref_blocks).size == 0
    # the wrapped blocks do not decode to the input; the GPU must decode (or reject) them exactly
    # as the oracle's Block::decode + iterator restatement does
    rc, ref_kv = O.decode_blocks(ref_blocks, ref_off)
    db, do = dev_blocks(ref_blocks, ref_off)
    if rc == 0:
        assert_kv_equal(batch.decode_blocks(db, do), ref_kv)
    else:
        with pytest.raises(LsmBlkError) as e:
            batch.decode_blocks(db, do)
        assert e.value.status == rc
    return ref_blocks, ref_off, rc


def test_u16_wrap_long_keys_prefix_and_suffix_len():
    """builder.rs:63-64: `prefix as u16` and `(key_len - prefix) as u16` for keys of 64 KiB and
    more (block_size 1 MiB, so several such keys share a block)."""
    rng = np.random.default_rng(17)
    base = bytes(rng.integers(0, 256, 70000, dtype=np.uint8))
    ents = [(base + b"%03d" % i, 10 + i, b"val%d" % i) for i in range(12)]
    ents += [(b"\xff" * 66000 + b"%02d" % i, 99, b"") for i in range(3)]  # suffix_len wraps too
    kv = O.KV.from_entries(ents)
    blocks, off, rc = _encode_and_decode_like_oracle(kv, [0, kv.n], 1 << 20)
    assert len(off) == 2
    e1 = 4 + len(ents[0][0]) + 10 + len(ents[0][2])  # entry 1's offset
    lcp = next(i for i, (x, y) in enumerate(zip(ents[0][0], ents[1][0])) if x != y)
    assert int.from_bytes(bytes(blocks[e1:e1 + 2]), "big") == lcp & 0xFFFF and lcp > 65535


def test_u16_wrap_offsets_and_entry_count_big_block_size():
    """builder.rs:61 (`offset as u16`) and block.rs:20 (`offsets.len() as u16`): block_size
    2 MiB > 65538, 70000 entries in one block: offsets past 64 KiB and the count wrap."""
    n = 70000
    ents = [(int(i).to_bytes(3, "big"), i, b"") for i in range(1, n + 1)]
    kv = O.KV.from_entries(ents)
    blocks, off, rc = _encode_and_decode_like_oracle(kv, [0, kv.n], 2 << 20)
    assert len(off) == 2
    assert int.from_bytes(bytes(blocks[-2:]), "big") == n & 0xFFFF
    # and a batch mixing wrapped and ordinary blocks: segments of 20000 entries each
    _encode_and_decode_like_oracle(kv, [0, 5, 20005, 40005, n], 1 << 20)


def test_one_entry_segments():
    kv = O.KV(*synth.gen_uniform(500, seed=9))
    roundtrip_check(kv, np.arange(kv.n + 1, dtype=np.uint32), 4096)


def test_malformed_block_reported():
    kv = week1_day3_kv()
    rc, blocks, off = O.encode_segments(kv, [0, 100], 4096)
    bad = blocks.copy()
    bad[int(off[1]) - 2:int(off[1])] = 0xFF  # entry count 65535: offsets would start before the block
    db, do = dev_blocks(bad, off)
    with pytest.raises(LsmBlkError) as e:
        batch.decode_blocks(db, do)
    assert e.value.status == LSMBLK_E_MALFORMED


def test_decode_capacity_reports_required_sizes():
    kv = O.KV(*synth.gen_uniform(2000, seed=4))
    rc, blocks, off = O.encode_segments(kv, [0, kv.n], 4096)
    db, do = dev_blocks(blocks, off)
    out = batch.KVStream(torch.zeros(1024, dtype=torch.uint8, device="cuda"),
                         torch.zeros(101, dtype=torch.int32, device="cuda"),
                         torch.zeros(1024, dtype=torch.uint8, device="cuda"),
                         torch.zeros(101, dtype=torch.int32, device="cuda"),
                         torch.zeros(100, dtype=torch.int64, device="cuda"), 0)
    stats = torch.zeros(4, dtype=torch.int64, device="cuda")
    batch.decode_into(db, do, len(off) - 1, out, stats, 100, 1024, 1024)
    torch.cuda.synchronize()
    s = stats.cpu().tolist()
    assert s[:3] == [kv.n, len(kv.keys), len(kv.vals)]
    assert batch._status(stats) == LSMBLK_E_CAPACITY


def test_repeated_calls_are_stable():
    kv = O.KV(*synth.gen_zipf(8000, seed=11))
    seg = synth.segments_by_bytes(kv.key_off, kv.val_off, 128 << 10)
    rc, ref_blocks, ref_off = O.encode_segments(kv, seg, 4096)
    d = to_dev(kv)
    db, do = dev_blocks(ref_blocks, ref_off)
    for _ in range(5):
        blocks, blk_off = batch.encode_kv(d, seg, 4096)
        np.testing.assert_array_equal(blocks.cpu().numpy(), ref_blocks)
        dkv = batch.decode_blocks(db, do)
        assert dkv.n == kv.n


@pytest.mark.parametrize("cfg,n,target", [("U", 400_000, 2 << 20), ("Z", 400_000, 2 << 20), ("M", 40_000, 8 << 20)])
def test_roundtrip_properties_large(cfg, n, target):
    """At sizes beyond quick oracle checks: decode(encode(kv)) == kv and
    encode(decode(blocks)) == blocks, plus an oracle check of a sampled segment."""
    kv = O.KV(*synth.GENERATORS[cfg](n, seed=21))
    seg = synth.segments_by_bytes(kv.key_off, kv.val_off, target)
    d = to_dev(kv)
    blocks, blk_off = batch.encode_kv(d, seg, synth.BLOCK_SIZE[cfg])
    dkv = batch.decode_blocks(blocks, blk_off)
    keys, ko, vals, vo, ts = dkv.to_numpy()
    np.testing.assert_array_equal(ko, kv.key_off)
    np.testing.assert_array_equal(vo, kv.val_off)
    np.testing.assert_array_equal(ts, kv.ts)
    assert torch.equal(dkv.keys[:len(kv.keys)].cpu(), torch.from_numpy(kv.keys))
    assert torch.equal(dkv.vals[:len(kv.vals)].cpu(), torch.from_numpy(kv.vals))
    blocks2, blk_off2 = batch.encode_kv(dkv, seg, synth.BLOCK_SIZE[cfg])
    assert torch.equal(blocks2, blocks) and torch.equal(blk_off2, blk_off)
    # full oracle check (the C restatement handles these sizes in about a second)
    rc, rb, ro = O.encode_segments(kv, seg, synth.BLOCK_SIZE[cfg])
    assert rc == 0
    np.testing.assert_array_equal(blk_off.cpu().numpy().view(np.uint64), ro)
    np.testing.assert_array_equal(blocks.cpu().numpy(), rb)


@pytest.mark.parametrize("order", ["shuffled", "one_inversion", "descending", "dup_runs"])
def test_key_order_adjacent_lcp_and_direct_fallback(order):
    # The plan walk derives LCP(first key, key) as the running min of adjacent-pair LCPs,
    # valid only for non-decreasing keys; windows holding an out-of-order pair must fall back
    # to the direct first-key compare (builder.rs:19-33 compares against the first key only).
    rng = np.random.default_rng(21)
    n = 6000
    pre = [bytes(rng.integers(0, 256, int(rng.integers(0, 6)), dtype=np.uint8)) for _ in range(8)]
    keys = sorted({pre[int(rng.integers(0, 8))] + bytes(rng.integers(0, 256, int(rng.integers(1, 20)), dtype=np.uint8))
                   for _ in range(n)})
    if order == "shuffled":
        keys = [keys[i] for i in rng.permutation(len(keys))]
    elif order == "one_inversion":
        i = len(keys) // 2
        keys[i], keys[i + 1] = keys[i + 1], keys[i]
    elif order == "descending":
        keys = keys[::-1]
    else:  # long runs of one key (multi-version), lcp == full length
        keys = [k for k in keys[:600] for _ in range(int(rng.integers(1, 12)))]
    ents = [(k, i, bytes(rng.integers(0, 256, int(rng.integers(0, 160)), dtype=np.uint8)))
            for i, k in enumerate(keys)]
    kv = O.KV.from_entries(ents)
    roundtrip_check(kv, [0, kv.n], 4096)
    roundtrip_check(kv, [0, kv.n // 3, kv.n], 512)


def test_crc32_blocks_match_crc32fast():
    """Per-block CRC-32 of SST framing (src/table/builder.rs:120-122, src/table.rs:226-230)
    against the oracle's CRC-32 (pinned to crc32fast by the reference's MANIFEST records) and
    zlib: empty and 1-3-byte blocks, 64-B and 4-KiB boundaries, multi-chunk blocks, ragged
    random lengths, unaligned block starts, and enough blocks for the persistent stride."""
    rng = np.random.default_rng(31)
    lens = [0, 1, 2, 3, 4, 5, 63, 64, 65, 127, 128, 4095, 4096, 4097, 8191, 8192, 8193, 65536, 70001, 0, 17]
    lens += [int(x) for x in rng.integers(0, 9000, 300)] + [int(x) for x in rng.integers(0, 200, 5000)]
    data = rng.integers(0, 256, sum(lens), dtype=np.uint8)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    want = np.array([O.crc32(data[int(off[i]):int(off[i + 1])].tobytes()) for i in range(len(lens))], np.uint32)
    assert all(int(want[i]) == zlib.crc32(data[int(off[i]):int(off[i + 1])].tobytes()) for i in range(40))
    for shift in (0, 5, 11):
        db, do = dev_blocks(data, off, shift)
        got = batch.crc32_blocks(db, do).cpu().numpy().view(np.uint32)
        np.testing.assert_array_equal(got, want)


def test_crc32_of_encoded_blocks():
    """CRC of GPU-encoded U blocks == crc32fast of the oracle's blocks (the SST data section's
    checksums), including a batch of one block."""
    kv = O.KV(*synth.gen_uniform(30000, seed=17))
    seg = synth.segments_by_bytes(kv.key_off, kv.val_off, 256 << 10)
    rc, ref_blocks, ref_off = O.encode_segments(kv, seg, 4096)
    assert rc == 0
    blocks, blk_off = batch.encode_kv(to_dev(kv), seg, 4096)
    got = batch.crc32_blocks(blocks, blk_off).cpu().numpy().view(np.uint32)
    want = [O.crc32(ref_blocks[int(ref_off[i]):int(ref_off[i + 1])].tobytes()) for i in range(len(ref_off) - 1)]
    np.testing.assert_array_equal(got, np.array(want, np.uint32))
    one = batch.crc32_blocks(blocks, blk_off[:2]).cpu().numpy().view(np.uint32)
    assert int(one[0]) == want[0]
    # a framed SST data section (block || u32 BE crc per block, finish_block) read back with the
    # BlockMeta offsets and tail=4 (read_block: block_len = offset_end - offset - 4)
    parts, meta = [], [0]
    for i in range(len(ref_off) - 1):
        blk = ref_blocks[int(ref_off[i]):int(ref_off[i + 1])].tobytes()
        parts.append(blk + int(want[i]).to_bytes(4, "big"))
        meta.append(meta[-1] + len(parts[-1]))
    framed = np.frombuffer(b"".join(parts), np.uint8).copy()
    db, do = dev_blocks(framed, np.array(meta, np.uint64), 3)
    got = batch.crc32_blocks(db, do, tail=4).cpu().numpy().view(np.uint32)
    stored = np.array([int.from_bytes(framed[m - 4:m].tobytes(), "big") for m in meta[1:]], np.uint32)
    np.testing.assert_array_equal(got, stored)


@pytest.mark.parametrize("shift", [0, 9])
def test_large_blocks_decode_paths(shift):
    """Blocks over the LDS image: <= 128 entries take the HBM->HBM copy path, more take the
    byte path.  Long shared prefixes, 1-5-byte key tails, values of 0-17 B next to 1-5 KB ones
    (short runs at block ends), unaligned block stream."""
    rng = np.random.default_rng(23)
    base = bytes(rng.integers(0, 256, 60, dtype=np.uint8))
    keys = sorted({base[:int(rng.integers(0, 60))] + bytes(rng.integers(0, 256, int(rng.integers(1, 6)), dtype=np.uint8))
                   for _ in range(3000)})
    sizes = [0, 1, 3, 7, 15, 16, 17, 100, 1000, 5000]
    ents = [(k, i, bytes(rng.integers(0, 256, int(rng.choice(sizes)), dtype=np.uint8))) for i, k in enumerate(keys)]
    kv = O.KV.from_entries(ents)
    for bs in (65536, 16384):
        _, off = roundtrip_check(kv, [0, kv.n], bs, shift=shift)
        assert (np.diff(off) > 4400).mean() > 0.9  # mostly beyond the LDS image


def _meta_want(kv: O.KV, seg, block_size):
    from oracle import pyref
    ents = kv.entries()
    return [pyref.encode_block_meta(pyref.sst_block_metas(ents[seg[g]:seg[g + 1]], block_size))
            for g in range(len(seg) - 1)]


def _meta_check(kv: O.KV, seg, block_size):
    r = batch.encode_sst(to_dev(kv), seg, block_size)
    rc, ref_blocks, ref_off = O.encode_segments(kv, seg, block_size)
    assert rc == 0
    np.testing.assert_array_equal(r["blocks"].cpu().numpy(), ref_blocks)
    want = _meta_want(kv, seg, block_size)
    meta = r["meta"].cpu().numpy().tobytes()
    mo = r["meta_off"].cpu().numpy()
    assert len(mo) == len(want) + 1 and mo[-1] == len(meta)
    for g, w in enumerate(want):
        got = meta[mo[g]:mo[g + 1]]
        assert got == w, f"segment {g}: {len(got)} B vs {len(w)} B"
    return r, ref_blocks, ref_off


@pytest.mark.parametrize("cfg", ["U", "Z", "M"])
def test_block_meta_sections_match_sst_builder(cfg):
    """lsmblk_block_meta_batch == BlockMeta::encode_block_meta of one SsTableBuilder per segment
    (src/table.rs:29-63, src/table/builder.rs:48-77), byte for byte, incl. the section CRC."""
    gen = {"U": synth.gen_uniform, "Z": synth.gen_zipf, "M": synth.gen_mixed}[cfg]
    n = 4000 if cfg == "M" else 20000
    kv = O.KV(*gen(n, seed=21))
    bs = 65536 if cfg == "M" else 4096
    seg = synth.segments_by_bytes(kv.key_off, kv.val_off, (1 << 20) if cfg == "M" else (128 << 10))
    r, _, _ = _meta_check(kv, seg, bs)
    seg_blk = r["seg_blk"].cpu().numpy().view(np.uint32)
    assert seg_blk[0] == 0 and seg_blk[-1] == r["blk_off"].numel() - 1


def test_block_meta_empty_and_one_entry_segments_long_keys():
    rng = np.random.default_rng(5)
    base = bytes(rng.integers(0, 256, 90, dtype=np.uint8))
    keys = sorted({base[:int(rng.integers(20, 90))] + bytes(rng.integers(0, 256, 8, dtype=np.uint8))
                   for _ in range(1500)})
    ents = [(k, i, bytes(rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8)))
            for i, k in enumerate(keys)]
    kv = O.KV.from_entries(ents)
    n = kv.n
    _meta_check(kv, [0, 0, 1, 2, 700, 700, 1400, n, n], 1024)  # empty segments first, inside, last
    kv1 = O.KV(*synth.gen_uniform(300, seed=8))
    _meta_check(kv1, np.arange(kv1.n + 1, dtype=np.uint32), 4096)  # one-entry SSTs


def test_block_meta_over_framed_data_section_and_errors():
    """tail = 4: the section computed from a framed data section (block || BE u32 CRC) with the
    BlockMeta offsets, as a reader holding the SST file would; a block without entries and a
    bad segment table report errors."""
    kv = O.KV(*synth.gen_uniform(6000, seed=4))
    seg = [0, 2500, kv.n]
    rc, ref_blocks, ref_off = O.encode_segments(kv, seg, 4096)
    want = _meta_want(kv, seg, 4096)
    r = batch.encode_sst(to_dev(kv), seg, 4096)
    seg_blk = r["seg_blk"]
    parts, off = [], [0]
    for i in range(len(ref_off) - 1):
        blk = ref_blocks[int(ref_off[i]):int(ref_off[i + 1])].tobytes()
        parts.append(blk + zlib.crc32(blk).to_bytes(4, "big"))
        off.append(off[-1] + len(parts[-1]))
    framed = np.frombuffer(b"".join(parts), np.uint8).copy()
    db, do = dev_blocks(framed, np.array(off, np.uint64), 5)
    meta, mo = batch.block_meta(db, do, seg_blk, tail=4)
    meta, mo = meta.cpu().numpy().tobytes(), mo.cpu().numpy()
    assert [meta[mo[g]:mo[g + 1]] for g in range(len(seg) - 1)] == want
    # an entry-less block (u16 count 0) is malformed; a segment table not ending at nblk too
    bad = np.concatenate([ref_blocks, np.zeros(2, np.uint8)])
    boff = np.concatenate([ref_off, [ref_off[-1] + 2]]).astype(np.uint64)
    db, do = dev_blocks(bad, boff)
    nb = len(boff) - 1
    with pytest.raises(LsmBlkError) as e:
        batch.block_meta(db, do, np.array([0, nb], np.uint32))
    assert e.value.status == LSMBLK_E_MALFORMED
    db, do = dev_blocks(ref_blocks, ref_off)
    with pytest.raises(LsmBlkError):
        batch.block_meta(db, do, np.array([0, 1], np.uint32))


@pytest.mark.parametrize("seed", range(3))
def test_compact_filter_matches_reference_loop(seed):
    """lsmblk_compact_filter_batch == compact_generate_sst's keep/drop loop (src/compact.rs:234-299,
    restated in oracle/pyref.py) on merged streams: watermarks, bottom-level tombstones, prefix
    filters, long and empty values, unaligned arenas."""
    from oracle import pyref
    rng = np.random.default_rng(100 + seed)
    ents = []
    for k in range(3000):
        key = (b"ab" if rng.random() < 0.2 else b"key-") + b"%08d" % k + (b"x" * int(rng.integers(0, 40)))
        for t in sorted(rng.choice(1000, size=int(rng.integers(1, 7)), replace=False), reverse=True):
            v = b"" if rng.random() < 0.25 else bytes(rng.integers(0, 256, int(rng.integers(1, 300)), dtype=np.uint8))
            ents.append((key, int(t), v))
    kv = to_dev(O.KV.from_entries(ents))
    for wm, bottom, pf in ((0, False, ()), (500, True, ()), (500, False, (b"ab",)), (10**6, True, (b"ab", b"key-0000"))):
        got = batch.compact_filter(kv, wm, bottom, pf)
        want = O.KV.from_entries(pyref.compact_filter_loop(ents, wm, bottom, pf))
        assert_kv_equal(got, want)
    empty = batch.compact_filter(to_dev(O.KV.from_entries([])), 5, True)
    assert empty.n == 0


def test_compact_filter_many_tiles_against_loop():
    """~450 K entries (hundreds of 1024-entry tiles, many runs per wave): the GPU filter vs the
    restated loop, watermark mid-range, bottom level, one prefix filter."""
    from oracle import pyref
    rng = np.random.default_rng(77)
    base = O.KV(*synth.gen_uniform(200000, seed=31))
    reps = rng.integers(1, 4, base.n)
    ents = []
    for i in range(base.n):
        k = bytes(base.keys[16 * i:16 * i + 16])
        for t in sorted(rng.choice(1 << 20, size=int(reps[i]), replace=False), reverse=True):
            ents.append((k, int(t), b"" if rng.random() < 0.2 else bytes(8 + (t % 90))))
    pf = (ents[5][0][:1],)
    got = batch.compact_filter(to_dev(O.KV.from_entries(ents)), 1 << 19, True, pf)
    assert_kv_equal(got, O.KV.from_entries(pyref.compact_filter_loop(ents, 1 << 19, True, pf)))


def test_golden_fixtures_through_hip():
    """Every committed block fixture (tests/golden/*.npz) replayed through the HIP path: GPU encode
    of the fixture's KV stream == its blocks, GPU decode of its blocks == the oracle's decode."""
    import json
    import os
    g = os.path.join(os.path.dirname(__file__), "golden")
    meta = json.load(open(os.path.join(g, "golden.json")))
    for name, m in meta.items():
        z = np.load(os.path.join(g, name + ".npz"))
        kv = O.KV(z["keys"], z["key_off"], z["vals"], z["val_off"], z["ts"])
        blocks, blk_off = batch.encode_kv(to_dev(kv), z["seg_start"], m["block_size"])
        np.testing.assert_array_equal(blk_off.cpu().numpy().view(np.uint64), z["blk_off"], err_msg=name)
        np.testing.assert_array_equal(blocks.cpu().numpy(), z["blocks"], err_msg=name)
        # decode is compared with the oracle's decode of the blocks: an `as u16`-wrapped value
        # length (u16_wrap_oversize) reads back shorter than it was written, as in the reference
        rc, ref_kv = O.decode_blocks(z["blocks"], z["blk_off"])
        assert rc == 0
        db, do = dev_blocks(z["blocks"], z["blk_off"], 1)
        assert_kv_equal(batch.decode_blocks(db, do), ref_kv)


def test_decode_framed_section_verify_crc_and_block_entries():
    """lsmblk_decode_batch_ex over a framed SST data section (block || BE u32 crc32fast, the
    BlockMeta offsets): tail = 4, the read_block checksum test, and the per-block entry index."""
    from lsm_amd._lib import LSMBLK_E_CHECKSUM
    kv = O.KV(*synth.gen_uniform(30000, seed=19))
    seg = synth.segments_by_bytes(kv.key_off, kv.val_off, 256 << 10)
    rc, ref_blocks, ref_off = O.encode_segments(kv, seg, 4096)
    parts, off = [], [0]
    for i in range(len(ref_off) - 1):
        blk = ref_blocks[int(ref_off[i]):int(ref_off[i + 1])].tobytes()
        parts.append(blk + zlib.crc32(blk).to_bytes(4, "big"))
        off.append(off[-1] + len(parts[-1]))
    framed = np.frombuffer(b"".join(parts), np.uint8).copy()
    db, do = dev_blocks(framed, np.array(off, np.uint64), 7)
    got, ent = batch.decode_blocks(db, do, tail=4, verify=True, with_blk_ent=True)
    assert_kv_equal(got, kv)
    counts = [int.from_bytes(ref_blocks[int(ref_off[i + 1]) - 2:int(ref_off[i + 1])].tobytes(), "big")
              for i in range(len(ref_off) - 1)]
    np.testing.assert_array_equal(ent.cpu().numpy(), np.concatenate([[0], np.cumsum(counts)]))
    bad = framed.copy()
    bad[off[17] - 1] ^= 0x40  # one stored checksum byte
    db, do = dev_blocks(bad, np.array(off, np.uint64))
    with pytest.raises(LsmBlkError) as e:
        batch.decode_blocks(db, do, tail=4, verify=True)
    assert e.value.status == LSMBLK_E_CHECKSUM


def _framed(ref_blocks, ref_off, corrupt=None):
    """Framed data section (block || BE crc32fast); corrupt(i, bytearray) may edit block i first
    (its CRC is computed after the edit, so only the decode rules can catch it)."""
    parts, off = [], [0]
    for i in range(len(ref_off) - 1):
        blk = bytearray(ref_blocks[int(ref_off[i]):int(ref_off[i + 1])].tobytes())
        if corrupt:
            corrupt(i, blk)
        parts.append(bytes(blk) + zlib.crc32(blk).to_bytes(4, "big"))
        off.append(off[-1] + len(parts[-1]))
    return np.frombuffer(b"".join(parts), np.uint8).copy(), np.array(off, np.uint64)


@pytest.mark.parametrize("gen,n,bs", [("mixed", 6000, 65536), ("uniform", 20000, 256), ("mixed", 3000, 4096)])
def test_verifying_decode_counts_in_the_crc_pass(gen, n, bs):
    """verify=True replaces dec_count_kernel by the CRC pass's fused count (blocks over one 4-KiB
    CRC chunk count from global memory): same KV stream, block entry index, and MALFORMED for a
    block that breaks the decode rules under a correct checksum."""
    from lsm_amd._lib import LSMBLK_E_MALFORMED
    g = {"mixed": synth.gen_mixed, "uniform": synth.gen_uniform}[gen]
    kv = O.KV(*g(n, seed=23))
    seg = synth.segments_by_bytes(kv.key_off, kv.val_off, 1 << 20)
    rc, ref_blocks, ref_off = O.encode_segments(kv, seg, bs)
    assert rc == 0
    framed, off = _framed(ref_blocks, ref_off)
    db, do = dev_blocks(framed, off, 3)
    got, ent = batch.decode_blocks(db, do, tail=4, verify=True, with_blk_ent=True)
    assert_kv_equal(got, kv)
    counts = [int.from_bytes(ref_blocks[int(ref_off[i + 1]) - 2:int(ref_off[i + 1])].tobytes(), "big")
              for i in range(len(ref_off) - 1)]
    np.testing.assert_array_equal(ent.cpu().numpy(), np.concatenate([[0], np.cumsum(counts)]))
    nb = len(ref_off) - 1
    for victim in {0, nb // 2, nb - 1}:
        def corrupt(i, blk, victim=victim):
            if i == victim:
                blk[-2:] = b"\xff\xff"  # entry count beyond the block
        bad, boff = _framed(ref_blocks, ref_off, corrupt)
        db, do = dev_blocks(bad, boff)
        with pytest.raises(LsmBlkError) as e:
            batch.decode_blocks(db, do, tail=4, verify=True)
        assert e.value.status == LSMBLK_E_MALFORMED


@pytest.mark.parametrize("cfg,n", [("U", 30000), ("Z", 30000), ("M", 4000)])
@pytest.mark.parametrize("mode", ["two_pass", "lag128", "lag_beyond_batch", "lag_bytes"])
def test_decode_modes(cfg, n, mode):
    """The A/B decode paths give the oracle's stream and block entry index: count + scan + decode
    (LSMBLK_DEBUG_TWO_PASS_DECODE), and the lagged decode at its smallest lag (128: each tile's
    finisher, lag / 2 + 63 workgroups after the tile's first count, just ahead of the tile's first
    decoder), at a lag beyond the batch (every count before any decode), and at a lag scaled from
    bytes below the largest lag (the decode's range loaded a second time: U/Z ~300 blocks, M's
    large blocks clamped to 128)."""
    from lsm_amd._lib import lib
    kv = O.KV(*synth.GENERATORS[cfg](n, seed=21))
    seg = synth.segments_by_bytes(kv.key_off, kv.val_off, 128 << 10)
    rc, ref_blocks, ref_off = O.encode_segments(kv, seg, synth.BLOCK_SIZE[cfg])
    rc, ref_kv = O.decode_blocks(ref_blocks, ref_off)
    assert rc == 0
    ctx = batch._ctx(0)
    if mode == "two_pass":
        assert lib().lsmblk_debug_set(ctx, 3, 1) == 0
    elif mode == "lag_bytes":
        assert lib().lsmblk_debug_set(ctx, 6, 300 * 4096) == 0
    else:
        assert lib().lsmblk_debug_set(ctx, 4, 128 if mode == "lag128" else 1 << 20) == 0
    try:
        for shift in (0, 5):
            db, do = dev_blocks(ref_blocks, ref_off, shift)
            assert_kv_equal(batch.decode_blocks(db, do), ref_kv)
        out, ent = batch.decode_blocks(*dev_blocks(ref_blocks, ref_off), with_blk_ent=True)
        counts = [int.from_bytes(ref_blocks[int(ref_off[i + 1]) - 2:int(ref_off[i + 1])].tobytes(), "big")
                  for i in range(len(ref_off) - 1)]
        np.testing.assert_array_equal(ent.cpu().numpy().view(np.uint64), np.concatenate([[0], np.cumsum(counts)]))
    finally:
        lib().lsmblk_debug_set(ctx, 3, 0)
        lib().lsmblk_debug_set(ctx, 4, 0)


def test_decode_lag_setting_bounds():
    """Lags below two tiles or above 2^24 blocks are refused."""
    from lsm_amd._lib import lib
    ctx = batch._ctx(0)
    assert lib().lsmblk_debug_set(ctx, 4, 127) != 0
    assert lib().lsmblk_debug_set(ctx, 4, (1 << 24) + 1) != 0
    assert lib().lsmblk_debug_set(ctx, 4, 10240) == 0
    assert lib().lsmblk_debug_set(ctx, 4, 0) == 0  # the default (scaled by the block size)


@pytest.mark.parametrize("cfg,n,seg_bytes", [("U", 400_000, 2 << 20), ("Z", 400_000, 2 << 20), ("U", 200_000, 64 << 10),
                                             ("M", 30_000, 8 << 20)])
def test_slot_encode_large_matches_packed_and_writes_only_its_segments(cfg, n, seg_bytes):
    """LSMBLK_ENCODE_SEG_SLOTS at sizes where the fused launch has many walkers, several segments
    per walker and every emitter busy (and M's big blocks through emit_big_kernel): the packed
    segments equal lsmblk_encode_batch's output, nothing between the segments is written, the
    stats and blk_off[nblk] follow the header, and a second call (next epoch) gives the same."""
    kv = O.KV(*synth.GENERATORS[cfg](n, seed=33))
    seg = synth.segments_by_bytes(kv.key_off, kv.val_off, seg_bytes)
    bs = synth.BLOCK_SIZE[cfg]
    d = to_dev(kv)
    blocks, blk_off = batch.encode_kv(d, seg, bs)
    kb, vb = d.byte_sizes()
    out_cap, blk_cap = batch.encode_bound(d, kb, vb)
    nseg = len(seg) - 1
    seg_t = torch.from_numpy(np.asarray(seg, np.uint32).view(np.int32)).cuda()
    from lsm_amd._lib import LSMBLK_DEBUG_ENCODE_FUSED, lib
    ctx = batch._ctx(0)
    for rep in range(4):  # (plan walk + emit twice, then the fused launch twice: epochs advance)
        assert lib().lsmblk_debug_set(ctx, LSMBLK_DEBUG_ENCODE_FUSED, rep // 2) == 0
        out = batch._aligned_empty(out_cap, "cuda")
        out.fill_(0xA5)
        off = torch.zeros(blk_cap, dtype=torch.int64, device="cuda")
        so = torch.full((2 * nseg,), -1, dtype=torch.int64, device="cuda")
        st = torch.zeros(4, dtype=torch.int64, device="cuda")
        batch.encode_into(d, seg_t, nseg, bs, out, out_cap, off, blk_cap, st, seg_out=so)
        torch.cuda.synchronize()
        nblk, nbytes, _, err = st.cpu().tolist()
        assert err == 0 and nblk == blk_off.numel() - 1 and nbytes == blocks.numel()
        so2 = so.view(-1, 2)
        np.testing.assert_array_equal(so2[:, 0].cpu().numpy(), seg_slots(kv, seg))
        assert int(off[nblk].item()) == int(so2[-1, 0].item() + so2[-1, 1].item())
        pb, po = batch.slots_to_packed(out, off[:nblk + 1], so)
        assert torch.equal(po, blk_off) and torch.equal(pb, blocks), f"rep {rep}"
        untouched = torch.ones(out_cap, dtype=torch.bool, device="cuda")
        for a, b in so2.cpu().tolist():
            untouched[a:a + b] = False
        assert bool((out[untouched] == 0xA5).all())
    lib().lsmblk_debug_set(ctx, LSMBLK_DEBUG_ENCODE_FUSED, 0)


def test_slot_encode_refuses_missing_seg_out_and_bad_flags():
    from lsm_amd._lib import lib
    import ctypes
    kv = O.KV(*synth.gen_uniform(1000, seed=1))
    d = to_dev(kv)
    c = d._c()
    seg_t = torch.tensor([0, kv.n], dtype=torch.int32, device="cuda")
    out = batch._aligned_empty(1 << 20, "cuda")
    off = torch.zeros(kv.n + 2, dtype=torch.int64, device="cuda")
    st = torch.zeros(4, dtype=torch.int64, device="cuda")
    ctx = batch._ctx(0)
    f = lib().lsmblk_encode_batch_ex
    assert f(ctx, ctypes.byref(c), seg_t.data_ptr(), 1, 4096, 1, out.data_ptr(), 1 << 20, off.data_ptr(), kv.n + 2,
             None, st.data_ptr(), None) != 0
    so = torch.zeros(2, dtype=torch.int64, device="cuda")
    assert f(ctx, ctypes.byref(c), seg_t.data_ptr(), 1, 4096, 4, out.data_ptr(), 1 << 20, off.data_ptr(), kv.n + 2,
             so.data_ptr(), st.data_ptr(), None) != 0  # (flag 4: unknown; 2 is LSMBLK_ENCODE_FRAMED)


def _slot_encode_raw(kv_dev, seg, bs, out_cap=None, fused=0):
    """One lsmblk_encode_batch_ex(SEG_SLOTS) call -> (status, stats, out, blk_off, seg_out)."""
    from lsm_amd._lib import LSMBLK_DEBUG_ENCODE_FUSED, lib
    ctx = batch._ctx(0)
    nseg = len(seg) - 1
    kb, vb = kv_dev.byte_sizes()
    cap, blk_cap = batch.encode_bound(kv_dev, kb, vb)
    out_cap = cap if out_cap is None else out_cap
    out = batch._aligned_empty(max(out_cap, 16), "cuda")
    off = torch.zeros(blk_cap, dtype=torch.int64, device="cuda")
    so = torch.full((max(2 * nseg, 1),), -1, dtype=torch.int64, device="cuda")
    st = torch.zeros(4, dtype=torch.int64, device="cuda")
    seg_t = torch.from_numpy(np.asarray(seg, np.int64).astype(np.uint32).view(np.int32)).cuda()
    assert lib().lsmblk_debug_set(ctx, LSMBLK_DEBUG_ENCODE_FUSED, fused) == 0
    try:
        batch.encode_into(kv_dev, seg_t, nseg, bs, out, out_cap, off, blk_cap, st, seg_out=so)
        torch.cuda.synchronize()
    finally:
        lib().lsmblk_debug_set(ctx, LSMBLK_DEBUG_ENCODE_FUSED, 0)
    return batch._status(st), st.cpu().tolist(), out, off, so


@pytest.mark.parametrize("fused", [0, 1])
def test_slot_encode_empty_stream_and_empty_segments(fused):
    """No entries: every segment empty, slot 0, zero blocks, blk_off[0] = 0 -- as the packed
    encode with the same segment table."""
    kv = O.KV.from_entries([])
    d = to_dev(kv)
    for seg in ([0, 0], [0, 0, 0, 0]):
        status, st, out, off, so = _slot_encode_raw(d, seg, 4096, fused=fused)
        assert status == 0 and st[0] == 0 and st[1] == 0
        assert so.cpu().tolist()[:2 * (len(seg) - 1)] == [0, 0] * (len(seg) - 1)
        assert int(off[0].item()) == 0


@pytest.mark.parametrize("fused", [0, 1])
def test_slot_encode_refuses_bad_segment_tables(fused):
    """A segment table that does not start at 0, decreases, or ends past / before n fails with
    LSMBLK_E_INVAL (the walkers' SEGMENTS flag) -- no fault, no hang: emit writes nothing over
    tables the plan refused (a decreasing table once gave a block whose end entry preceded its
    start, which emit_big walked as ~2^32 entries) -- and the context then encodes a good table
    correctly.  The packed encode is held to the same."""
    from lsm_amd._lib import LSMBLK_E_INVAL
    kv = O.KV(*synth.gen_uniform(3000, seed=12))
    d = to_dev(kv)
    n = kv.n
    # (the last two: an interior / first entry far past n, which the slot of a segment must never
    # use as an index -- ADVICE round 5)
    for seg in ([5, n], [0, 2000, 1000, n], [0, 1000, n - 1], [0, 1000, n + 7], [0, 0xFFFFFFFF, n],
                [0xFFFFFFF0, n]):
        status, *_ = _slot_encode_raw(d, seg, 4096, fused=fused)
        assert status == LSMBLK_E_INVAL, seg
        if not fused:  # the packed encode
            kb, vb = d.byte_sizes()
            cap, blk_cap = batch.encode_bound(d, kb, vb)
            out = batch._aligned_empty(cap, "cuda")
            off = torch.zeros(blk_cap, dtype=torch.int64, device="cuda")
            st = torch.zeros(4, dtype=torch.int64, device="cuda")
            seg_t = torch.from_numpy(np.asarray(seg, np.int64).astype(np.uint32).view(np.int32)).cuda()
            batch.encode_into(d, seg_t, len(seg) - 1, 4096, out, cap, off, blk_cap, st)
            torch.cuda.synchronize()
            assert batch._status(st) == LSMBLK_E_INVAL, seg
    seg = [0, 1000, 2000, n]
    rc, ref_blocks, ref_off = O.encode_segments(kv, seg, 4096)
    status, st, out, off, so = _slot_encode_raw(d, seg, 4096, fused=fused)
    assert status == 0
    pb, po = batch.slots_to_packed(out, off[:st[0] + 1], so)
    assert np.array_equal(pb.cpu().numpy(), ref_blocks)


@pytest.mark.parametrize("fused", [0, 1])
def test_slot_encode_capacity_below_the_bound_reported(fused):
    """out_cap below the segments' slots: LSMBLK_E_CAPACITY, nothing written past out_cap."""
    from lsm_amd._lib import LSMBLK_E_CAPACITY
    kv = O.KV(*synth.gen_uniform(4000, seed=13))
    d = to_dev(kv)
    seg = [0, 1500, 3000, kv.n]
    kb, vb = d.byte_sizes()
    cap, _ = batch.encode_bound(d, kb, vb)
    small = cap // 2 & ~15
    status, st, out, off, so = _slot_encode_raw(d, seg, 4096, out_cap=small, fused=fused)
    assert status == LSMBLK_E_CAPACITY


@pytest.mark.parametrize("mode", ["packed", "slots", "fused"])
def test_encode_refuses_an_empty_key(mode):
    """An empty key (BlockBuilder::add asserts `!key.is_empty()`, src/block/builder.rs:55) fails
    the call with LSMBLK_E_INVAL -- the walkers' EMPTY_KEY flag -- and emit writes nothing: the
    output buffer keeps its fill bytes."""
    from lsm_amd._lib import LSMBLK_E_INVAL
    ents = [(b"k%05d" % i, i, b"v" * 40) for i in range(600)]
    ents[300] = (b"", 300, b"v" * 40)
    d = to_dev(O.KV.from_entries(ents))
    seg = [0, 250, 600]
    if mode == "packed":
        kb, vb = d.byte_sizes()
        cap, blk_cap = batch.encode_bound(d, kb, vb)
        out = batch._aligned_empty(cap, "cuda")
        out.fill_(0xA5)
        off = torch.zeros(blk_cap, dtype=torch.int64, device="cuda")
        st = torch.zeros(4, dtype=torch.int64, device="cuda")
        seg_t = torch.tensor(seg, dtype=torch.int32, device="cuda")
        batch.encode_into(d, seg_t, len(seg) - 1, 4096, out, cap, off, blk_cap, st)
        torch.cuda.synchronize()
        status = batch._status(st)
    else:
        status, st, out, off, so = _slot_encode_raw(d, seg, 4096, fused=int(mode == "fused"))
    assert status == LSMBLK_E_INVAL
    if mode == "packed":
        assert bool((out == 0xA5).all())


@pytest.mark.parametrize("mode", ["packed", "slots", "fused"])
@pytest.mark.parametrize("which", ["key_off", "val_off"])
def test_encode_refuses_decreasing_offsets(mode, which):
    """A KV stream whose key or value offsets decrease (a corrupt stream: an entry of wrapped,
    ~4 GiB length) fails the call with LSMBLK_E_MALFORMED -- the plan helpers' flag, one of the
    plan's fatal flags -- and nothing is written (the packed output keeps its fill bytes); the walk
    never runs over the wrapped lengths."""
    ents = [(b"k%05d" % i, i, b"v" * 40) for i in range(600)]
    d = to_dev(O.KV.from_entries(ents))
    arr = getattr(d, which)
    arr[301] = arr[299]  # entry 300 ends before it starts
    seg = [0, 250, 600]
    if mode == "packed":
        cap, blk_cap = batch.encode_bound(d, 600 * 6, 600 * 40)
        out = batch._aligned_empty(cap, "cuda")
        out.fill_(0xA5)
        off = torch.zeros(blk_cap, dtype=torch.int64, device="cuda")
        st = torch.zeros(4, dtype=torch.int64, device="cuda")
        seg_t = torch.tensor(seg, dtype=torch.int32, device="cuda")
        batch.encode_into(d, seg_t, len(seg) - 1, 4096, out, cap, off, blk_cap, st)
        torch.cuda.synchronize()
        status = batch._status(st)
    else:
        status, st, out, off, so = _slot_encode_raw(d, seg, 4096, fused=int(mode == "fused"))
    if mode == "fused":  # (emits while it walks: another block's size self-check may fail first)
        from lsm_amd._lib import LSMBLK_E_INTERNAL
        assert status in (LSMBLK_E_MALFORMED, LSMBLK_E_INTERNAL)
    else:
        assert status == LSMBLK_E_MALFORMED
    if mode == "packed":
        assert bool((out == 0xA5).all())


def test_framed_encode_is_the_sst_builders_data_section():
    """LSMBLK_ENCODE_FRAMED of one segment == the data section of the SST file that
    oracle/pyref.py's line-by-line SsTableBuilder restatement writes (its bytes before
    meta_offset, src/table/builder.rs:68-98 + 112-123), for the week1_day3 KAT entries at two
    block sizes and a U sample; and the BlockMeta offsets of that file are the framed blk_off."""
    from oracle import pyref
    cases = [(week1_day3_kv(), 128), (week1_day3_kv(), 4096), (O.KV(*synth.gen_uniform(3000, seed=31)), 4096)]
    for kv, bs in cases:
        ents = kv.entries()
        f = pyref.sst_file(ents, bs)
        out, off = batch.encode_kv_framed(to_dev(kv), [0, kv.n], bs)
        data = out.cpu().numpy().tobytes()
        assert f[:len(data)] == data
        metas = pyref.sst_block_metas(ents, bs)
        assert [m[0] for m in metas] == off.cpu().numpy()[:-1].tolist()


def test_framed_encode_u_large_equals_blocks_and_crcs():
    """At 400 K entries: the framed encode == the packed encode with lsmblk_crc32_batch's CRCs
    interleaved (and a sample of them == zlib), the verifying framed decode reads it back."""
    kv = O.KV(*synth.gen_uniform(400_000, seed=33))
    seg = synth.segments_by_bytes(kv.key_off, kv.val_off, 2 << 20)
    d = to_dev(kv)
    blocks, boff = batch.encode_kv(d, seg, 4096)
    crc = batch.crc32_blocks(blocks, boff).cpu().numpy().view(np.uint32)
    out, off = batch.encode_kv_framed(d, seg, 4096)
    b, o = blocks.cpu().numpy(), boff.cpu().numpy()
    fo = off.cpu().numpy()
    nblk = len(o) - 1
    assert len(fo) == nblk + 1 and fo[-1] == o[-1] + 4 * nblk
    np.testing.assert_array_equal(fo[:-1], o[:-1] + 4 * np.arange(nblk))
    f = out.cpu().numpy()
    ends = fo[1:] - 4
    got_crc = (f[ends[:, None] + np.arange(4)].astype(np.uint32) << np.array([24, 16, 8, 0], np.uint32)).sum(1)
    np.testing.assert_array_equal(got_crc.astype(np.uint32), crc)
    for i in range(0, nblk, max(1, nblk // 50)):
        assert zlib.crc32(b[o[i]:o[i + 1]].tobytes()) == int(crc[i])
    dkv = batch.decode_blocks(out, off, tail=4, verify=True)
    assert dkv.n == kv.n
