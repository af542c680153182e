"""Batched device seek_to_key (SURVEY.md §8 a row 13, src/block/iterator.rs:80-94) against the
oracle's restatement (oracle/lsmblk_oracle.c orc_block_seek_key): the exact binary search, so with
several versions of a user key in a block the landing index is the first probe that compares equal,
not necessarily the first version."""
import numpy as np
import pytest
import torch

from lsm_amd import batch, synth
from lsm_amd._lib import LsmBlkError
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")


def blocks_of(seed, versions, bs=4096, nkeys=3000):
    keys, ko, vals, vo, ts, rs = synth.gen_runs(nkeys, nrun=1, seed=seed, versions=versions, overwrite=0.0)
    kv = O.KV(keys, ko, vals, vo, ts)
    seg = synth.segments_by_bytes(ko, vo, 64 << 10)
    rc, blocks, off = O.encode_segments(kv, seg, bs)
    assert rc == 0
    return kv, blocks, off


def queries(kv, blocks, off, rng, nq=4000):
    nb = len(off) - 1
    allk = [kv.entry(i)[0] for i in range(kv.n)]
    qb, qk = [], []
    for _ in range(nq):
        b = int(rng.integers(0, nb))
        r = rng.random()
        if r < 0.5:
            k = allk[int(rng.integers(0, len(allk)))]                     # a present key (maybe other block)
        elif r < 0.8:
            k = allk[int(rng.integers(0, len(allk)))][:int(rng.integers(1, 16))]   # a prefix: absent
        else:
            k = bytes(rng.integers(0, 256, int(rng.integers(1, 20)), dtype=np.uint8))
        qb.append(b)
        qk.append(k)
    return qb, qk


@pytest.mark.parametrize("seed,versions,bs", [(1, 1, 4096), (2, 3, 4096), (3, 2, 256), (4, 5, 1024)])
def test_seek_batch_equals_oracle(seed, versions, bs):
    rng = np.random.default_rng(seed)
    kv, blocks, off = blocks_of(50 + seed, versions, bs)
    qb, qk = queries(kv, blocks, off, rng)
    # every first key and every block's own keys too
    d_blocks = torch.from_numpy(blocks).cuda()
    d_off = torch.from_numpy(off.view(np.int64)).cuda()
    got = batch.seek_blocks(d_blocks, d_off, qb, qk)
    hb = blocks.tobytes()
    want = [O.seek_key(hb[off[b]:off[b + 1]], k) for b, k in zip(qb, qk)]
    assert got.tolist() == want


def test_seek_batch_framed_section_and_errors():
    rng = np.random.default_rng(7)
    kv, blocks, off = blocks_of(77, 2, 512)
    hb = blocks.tobytes()
    framed = b"".join(hb[off[b]:off[b + 1]] + O.crc32(hb[off[b]:off[b + 1]]).to_bytes(4, "big")
                      for b in range(len(off) - 1))
    foff = np.array([0] + list(np.cumsum([off[b + 1] - off[b] + 4 for b in range(len(off) - 1)])), np.uint64)
    qb, qk = queries(kv, blocks, off, rng, 500)
    got = batch.seek_blocks(torch.frombuffer(bytearray(framed), dtype=torch.uint8).cuda(),
                            torch.from_numpy(foff.view(np.int64)).cuda(), qb, qk, tail=4)
    assert got.tolist() == [O.seek_key(hb[off[b]:off[b + 1]], k) for b, k in zip(qb, qk)]
    with pytest.raises(LsmBlkError):   # block index out of range
        batch.seek_blocks(torch.from_numpy(blocks).cuda(), torch.from_numpy(off.view(np.int64)).cuda(),
                          [len(off) - 1], [b"x"])
    bad = bytearray(hb[off[0]:off[1]])
    bad[-1] = 0xFF                      # entry count far beyond the block
    with pytest.raises(LsmBlkError):
        batch.seek_blocks(torch.frombuffer(bad, dtype=torch.uint8).cuda(),
                          torch.tensor([0, len(bad)], dtype=torch.int64).cuda(), [0], [b"k"])
