"""Key-range sharded compaction, oracle side (CPU): compact_generate_sst resumed at a range's
carry-in (orc_shard_rotation) composes, range after range, to the single-stream compaction.

For random splits of the kept stream at key changes (empty and tiny ranges included, so a block can
cross several ranges), chaining carry = {p, D} through the ranges gives exactly orc_compact's blocks
and SST boundaries over the whole stream (src/compact.rs:223-311).  This is the decomposition the
device path (lsmblk_shard_*) evaluates; tests/test_gpu_shard.py checks the device against both.
"""
import numpy as np
import pytest

from lsm_amd import synth
from oracle import oracle as O


def kept_stream(seed, versions, nkeys=2500, nrun=4, tomb=0.05):
    keys, ko, vals, vo, ts, rs = synth.gen_runs(nkeys, nrun=nrun, seed=seed, versions=versions, tombstone=tomb)
    kv = O.KV(keys, ko, vals, vo, ts)
    src = O.merge_runs(kv, rs)
    return kv, src


def key_change_cuts(kept: O.KV, rng, nranges):
    """nranges - 1 cut positions at key changes (ascending, repeats allowed = empty ranges)."""
    n = kept.n
    change = [i for i in range(1, n) if kept.entry(i)[0] != kept.entry(i - 1)[0]]
    cuts = sorted(rng.choice(change, size=nranges - 1, replace=True).tolist()) if change else [n] * (nranges - 1)
    return [0] + cuts + [n]


def run_chain(kept: O.KV, bounds, bs, target):
    """Every range resumed from the carry of the one before; returns (blocks, sst starts, carries)."""
    W = bs // 16 + 2
    n = kept.n
    carry = (0, 0)
    blocks, starts, carries = [], [], []
    for r in range(len(bounds) - 1):
        a, b = bounds[r], bounds[r + 1]
        e = min(b + W, n)
        ext = O.gather(kept, np.arange(a, e))
        rc, seg, cout = O.shard_rotation(ext, b - a, e == n, carry[0], carry[1], bs, target)
        assert rc == 0, (r, rc)
        carries.append((carry, cout))
        if len(seg):
            rc, blk, off = O.encode_span(ext, seg, bs)
            assert rc == 0
            blocks.append(blk.tobytes())
            first = 0 if carry[1] == 0 else 1    # a continued SST does not start here
            starts += [a + int(x) for x in seg[first:-1]]
        carry = cout
    return b"".join(blocks), starts, carries


@pytest.mark.parametrize("seed", range(8))
def test_range_chain_equals_whole_stream_compaction(seed):
    rng = np.random.default_rng(seed)
    kv, src = kept_stream(300 + seed, versions=1 + seed % 3)
    bs = [256, 1024, 4096][seed % 3]
    target = [2000, 9000, 30000][seed % 3]
    wm = int(kv.ts.max()) // 2
    want = O.compact(kv, src, wm, True, (), bs, target)
    kept = O.gather(kv, src[want["kept"]])
    assert len(want["sst_blk"]) > 3
    for nranges in (1, 2, 5, 17):
        bounds = key_change_cuts(kept, rng, nranges)
        blocks, starts, _ = run_chain(kept, bounds, bs, target)
        assert blocks == want["blocks"].tobytes(), nranges
        assert starts == want["sst_ent"][:-1].tolist(), nranges


def test_tiny_ranges_swallowed_by_a_crossing_block():
    """Ranges of one or two keys inside one block: their carry passes through unchanged."""
    kv, src = kept_stream(77, versions=1, nkeys=400)
    want = O.compact(kv, src, 0, False, (), 4096, 1 << 20)
    kept = O.gather(kv, src[want["kept"]])
    bounds = [0, 10, 11, 12, 14, kept.n]
    blocks, starts, carries = run_chain(kept, bounds, 4096, 1 << 20)
    assert blocks == want["blocks"].tobytes()
    assert starts == [0]
    (cin, cout) = carries[2]            # range [11, 12): inside the block that starts before 10
    assert cin[0] >= 1 and cout == (cin[0] - 1, cin[1])
