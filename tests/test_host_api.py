"""CPU tests: the C ABI library loads, exports every symbol include/lsmblk.h declares, and the
per-entry half (BlockBuilder / Block / BlockIterator, host-synchronous by design) matches
the oracle byte for byte.  No GPU needed: nothing here calls a batch (device) function.
"""
import ctypes
import os
import re

import numpy as np
import pytest

from lsm_amd import Block, BlockBuilder, BlockIterator, KeySlice, LsmBlkError, _build, lib
from lsm_amd._lib import SIGNATURES
from oracle import oracle as O
from oracle import pyref

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "lsmblk.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(lsmblk_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    L = ctypes.CDLL(_build.SO)
    missing = [f for f in header_functions() if not hasattr(L, f)]
    assert not missing, missing
    assert len(header_functions()) >= 30


def test_integration_doc_binds_every_header_symbol():
    """INTEGRATION.md's Rust extern block (tools/gen_rust_ffi.py) names every header function."""
    doc = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "INTEGRATION.md")).read()
    missing = [f for f in header_functions() if f"pub fn {f}(" not in doc]
    assert not missing, missing


def test_python_binding_covers_header():
    bound = {n for n, _, _ in SIGNATURES}
    assert set(header_functions()) <= bound


def test_abi_version_and_errors():
    assert lib().lsmblk_abi_version() == 1
    assert lib().lsmblk_strerror(-2) == b"malformed block"
    assert lib().lsmblk_stats_status(1) == -2
    assert lib().lsmblk_stats_status(2) == -3
    assert lib().lsmblk_stats_status(0) == 0


def key_of(i):
    return b"key_%03d" % (i * 5)


def value_of(i):
    return b"value_%010d" % i


def generate_block():
    b = BlockBuilder(10000)
    for i in range(100):
        assert b.add(KeySlice.for_testing_from_slice_no_ts(key_of(i)), value_of(i))
    return b.build()


# ---- src/tests/week1_day3.rs, through the product's per-entry API ----
def test_block_build_single_key():
    b = BlockBuilder(16)
    assert b.add(KeySlice.for_testing_from_slice_no_ts(b"233"), b"233333")
    b.build()


def test_block_build_full():
    b = BlockBuilder(16)
    assert b.add(KeySlice.for_testing_from_slice_no_ts(b"11"), b"11")
    assert not b.add(KeySlice.for_testing_from_slice_no_ts(b"22"), b"22")
    b.build()


def test_block_build_large():
    b = BlockBuilder(16)
    assert b.add(KeySlice.for_testing_from_slice_no_ts(b"11"), b"1" * 100)
    b = BlockBuilder(16)
    assert b.add(KeySlice.for_testing_from_slice_no_ts(b"11"), b"1")
    assert not b.add(KeySlice.for_testing_from_slice_no_ts(b"11"), b"1" * 100)


def test_block_encode_decode():
    blk = generate_block()
    enc = blk.encode()
    dec = Block.decode(enc)
    assert dec.offsets == blk.offsets and dec.data == blk.data
    ob = O.Builder(10000)
    for i in range(100):
        ob.add(key_of(i), 0, value_of(i))
    assert enc == ob.finish()


def test_block_iterator():
    it = BlockIterator.create_and_seek_to_first(generate_block())
    for _ in range(5):
        for i in range(100):
            assert it.key().for_testing_key_ref() == key_of(i)
            assert it.value() == value_of(i)
            it.next()
        assert not it.is_valid()
        it.seek_to_first()


def test_block_seek_key():
    blk = generate_block()
    it = BlockIterator.create_and_seek_to_key(blk, KeySlice.for_testing_from_slice_no_ts(key_of(0)))
    for off in range(1, 6):
        for i in range(100):
            assert it.key().for_testing_key_ref() == key_of(i)
            assert it.value() == value_of(i)
            it.seek_to_key(KeySlice.for_testing_from_slice_no_ts(b"key_%03d" % (i * 5 + off)))
        it.seek_to_key(KeySlice.for_testing_from_slice_no_ts(b"k"))


def test_iterator_returns_ts():
    b = BlockBuilder(4096)
    assert b.add(KeySlice.for_testing_from_slice_with_ts(b"233", 233), b"233333")
    assert b.add(KeySlice.for_testing_from_slice_with_ts(b"233", 0), b"2333333")
    it = BlockIterator.create_and_seek_to_first(b.build())
    assert (it.key().key_ref(), it.key().ts(), it.value()) == (b"233", 233, b"233333")
    it.next()
    assert (it.key().key_ref(), it.key().ts(), it.value()) == (b"233", 0, b"2333333")


def test_key_ordering_ignores_ts():  # src/key.rs:63-81
    assert KeySlice(b"a", 1) == KeySlice(b"a", 99)
    assert KeySlice(b"a", 5) < KeySlice(b"b", 0)


def test_errors_instead_of_panics():
    with pytest.raises(AssertionError):
        BlockBuilder(16).add(KeySlice(b""), b"v")
    with pytest.raises(AssertionError):
        BlockBuilder(16).build()
    with pytest.raises(LsmBlkError):
        Block.decode(b"\x01")
    with pytest.raises(LsmBlkError):
        Block.decode(b"\xff\xff")


@pytest.mark.parametrize("seed", range(4))
def test_per_entry_builder_matches_oracle(seed):
    rng = np.random.default_rng(100 + seed)
    keys = sorted({bytes(rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8)) for _ in range(300)})
    ents = [(k, int(rng.integers(0, 1 << 63)), bytes(rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8)))
            for k in keys]
    bs = int(rng.choice([64, 256, 4096]))
    ours, ref = [], pyref.encode_segments(ents, [0, len(ents)], bs)
    b = BlockBuilder(bs)
    for k, ts, v in ents:  # SsTableBuilder::add (src/table/builder.rs:48-65)
        if not b.add(KeySlice(k, ts), v):
            ours.append(b.build_encoded())
            assert b.add(KeySlice(k, ts), v)
    ours.append(b.build_encoded())
    assert ours == ref
    for enc in ours:
        it = BlockIterator.create_and_seek_to_first(Block.decode(enc))
        got = []
        while it.is_valid():
            got.append((it.key().key_ref(), it.key().ts(), it.value()))
            it.next()
        assert got == pyref.block_entries(enc)
