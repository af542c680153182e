"""Key-range sharded compaction on the device (SURVEY.md §8 e, compaction-shaped): several ranges
driven through lsmblk_compact_merge_batch / lsmblk_shard_* on one GPU with the in-process exchange
(shard.compact_local -- the same phases and messages as the RCCL driver).  Bar: the concatenated
blocks and the SST boundaries equal the single-stream compaction (lsmblk_compact_batch and the C
oracle's compact_generate_sst), and every range's segments and carry equal the oracle's
compact_generate_sst resumed at that range's carry-in (orc_shard_rotation)."""
import numpy as np
import pytest
import torch

from lsm_amd import batch, shard, synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")


def case(seed, versions=1, nkeys=6000, nrun=5, tomb=0.05):
    keys, ko, vals, vo, ts, rs = synth.gen_runs(nkeys, nrun=nrun, seed=seed, versions=versions, tombstone=tomb)
    return O.KV(keys, ko, vals, vo, ts), rs


def to_dev(kv: O.KV):
    return batch.KVStream.from_numpy(kv.keys, kv.key_off, kv.vals, kv.val_off, kv.ts)


def pick_splitters(kv: O.KV, rng, k, tiny=False):
    """k sorted distinct splitters: existing keys, and byte strings between keys."""
    allk = sorted({kv.entry(i)[0] for i in range(kv.n)})
    out = set()
    while len(out) < k:
        i = int(rng.integers(1, len(allk)))
        out.add(allk[i] if rng.random() < 0.6 else allk[i][:int(rng.integers(1, 16))] + b"\x00")
        if tiny and len(out) < k:       # a range holding one key
            out.add(allk[min(i + 1, len(allk) - 1)])
    return sorted(out)[:k]


def run_ranges(kv_dev, rs, opts, splitters, inputs=None):
    shards = []
    for r in range(len(splitters) + 1):
        lo, hi = shard.range_of(r, splitters)
        kv_r, rs_r = inputs[r] if inputs else (kv_dev, rs)
        shards.append(shard.RangeShard(kv_r, rs_r, opts, lo, hi))
    return shard.compact_local(shards), shards


def check_against_single_stream(kv, rs, res, wm, bottom, bs, target):
    src = O.merge_runs(kv, rs)
    want = O.compact(kv, src, wm, bottom, (), bs, target)
    blocks = b"".join(r["blocks"].cpu().numpy().tobytes() for r in res)
    assert blocks == want["blocks"].tobytes()
    bases = np.concatenate([[0], np.cumsum([r["m"] for r in res])]).tolist()
    assert bases[-1] == len(want["kept"])
    assert shard.sst_starts(res, bases) == want["sst_ent"][:-1].tolist()
    for a, b in zip(res, res[1:]):
        assert a["carry_out"] == b["carry_in"]
    return want, O.gather(kv, src[want["kept"]]), bases


def check_each_range_against_resumed_oracle(kept, res, bases, bs, target):
    W = shard.halo_entries(bs)
    for r, base in zip(res, bases):
        e = min(base + r["m"] + W, kept.n)
        ext = O.gather(kept, np.arange(base, e))
        rc, seg, cout = O.shard_rotation(ext, r["m"], e == kept.n, *r["carry_in"], bs, target)
        assert rc == 0
        assert cout == r["carry_out"]
        assert r["seg_start"].tolist() == seg.tolist()


@pytest.mark.parametrize("seed", range(4))
def test_sharded_compaction_equals_single_stream(seed):
    rng = np.random.default_rng(seed)
    kv, rs = case(600 + seed, versions=1 + seed % 3)
    bs, target = [(4096, 32 << 10), (1024, 8 << 10), (256, 3000), (4096, 1 << 20)][seed]
    wm, bottom = int(kv.ts.max()) // 2, bool(seed % 2)
    d = to_dev(kv)
    opts = batch.compact_opts(wm, bottom, block_size=bs, target_sst_size=target)
    single = batch.compact_runs(d, rs, wm, bottom, block_size=bs, target_sst_size=target)
    for k in (1, 3, 7):
        res, _ = run_ranges(d, rs, opts, pick_splitters(kv, rng, k))
        want, kept, bases = check_against_single_stream(kv, rs, res, wm, bottom, bs, target)
        assert b"".join(r["blocks"].cpu().numpy().tobytes() for r in res) == \
            single["blocks"].cpu().numpy().tobytes()
        check_each_range_against_resumed_oracle(kept, res, bases, bs, target)


def test_tiny_and_empty_ranges():
    """Ranges of one key (swallowed by a crossing block) and ranges with no keys at all."""
    rng = np.random.default_rng(11)
    kv, rs = case(41, versions=2, nkeys=1500)
    d = to_dev(kv)
    opts = batch.compact_opts(0, False, block_size=4096, target_sst_size=16 << 10)
    sp = pick_splitters(kv, rng, 6, tiny=True) + [b"\xff\xff\xff\xff\xff\xff\xff\xff\xff\xff\xff\xff\xff\xff\xff\xff\xff"]
    sp = [b"\x00"] + sorted(set(sp))             # range 0 empty, the last range empty
    res, _ = run_ranges(d, rs, opts, sp)
    assert res[0]["m"] == 0 and res[-1]["m"] == 0
    want, kept, bases = check_against_single_stream(kv, rs, res, 0, False, 4096, 16 << 10)
    check_each_range_against_resumed_oracle(kept, res, bases, 4096, 16 << 10)


def range_inputs(kv, rs, splitters, bs):
    """Every run encoded as SST blocks; per key range, the KV input decoded from only the blocks of
    each run that overlap the range (BlockMeta first / last keys; straddling blocks go to both
    neighbours) and its run starts."""
    runs = []
    for r in range(len(rs) - 1):
        sub = O.gather(kv, np.arange(rs[r], rs[r + 1]))
        if sub.n == 0:
            runs.append(None)
            continue
        seg = synth.segments_by_bytes(sub.key_off, sub.val_off, 64 << 10)
        blocks, off = batch.encode_kv(to_dev(sub), seg, bs)
        dec = batch.decode_blocks(blocks, off)
        keys, ko, _, _, _ = dec.to_numpy()
        runs.append((blocks, off.cpu().numpy().view(np.uint64), keys, ko))
    inputs = []
    for g in range(len(splitters) + 1):
        lo, hi = shard.range_of(g, splitters)
        parts, rstarts = [], [0]
        for run in runs:
            if run is None:
                rstarts.append(rstarts[-1])
                continue
            blocks, off, keys, ko = run
            # block first / last keys from the decoded run (BlockMeta's first_key / last_key)
            dec = batch.decode_blocks(blocks, torch.from_numpy(off.view(np.int64)).cuda(), with_blk_ent=True)[1]
            ent = dec.cpu().numpy().view(np.uint64)
            fk = [bytes(keys[ko[ent[b]]:ko[ent[b] + 1]]) for b in range(len(off) - 1)]
            lk = [bytes(keys[ko[ent[b + 1] - 1]:ko[ent[b + 1]]]) for b in range(len(off) - 1)]
            sel = [b for b in range(len(off) - 1) if (lo is None or lk[b] >= lo) and (hi is None or fk[b] < hi)]
            if sel:
                a, z = sel[0], sel[-1] + 1
                seg_blocks = blocks[int(off[a]):int(off[z])]
                seg_off = torch.from_numpy((off[a:z + 1] - off[a]).view(np.int64)).cuda()
                parts.append(batch.decode_blocks(seg_blocks.contiguous(), seg_off))
            rstarts.append(rstarts[-1] + (parts[-1].n if sel else 0))
        cat = [p.to_numpy() for p in parts]
        k_all = np.concatenate([c[0] for c in cat]) if cat else np.zeros(0, np.uint8)
        v_all = np.concatenate([c[2] for c in cat]) if cat else np.zeros(0, np.uint8)
        ko_all = np.concatenate([[0]] + [c[1][1:].astype(np.int64) + sum(len(x[0]) for x in cat[:i])
                                         for i, c in enumerate(cat)]).astype(np.uint32)
        vo_all = np.concatenate([[0]] + [c[3][1:].astype(np.int64) + sum(len(x[2]) for x in cat[:i])
                                         for i, c in enumerate(cat)]).astype(np.uint32)
        ts_all = np.concatenate([c[4] for c in cat]) if cat else np.zeros(0, np.uint64)
        inputs.append((batch.KVStream.from_numpy(k_all, ko_all, v_all, vo_all, ts_all),
                       np.array(rstarts, np.uint32)))
    return inputs


def test_ranges_read_only_their_blocks_decode_merge_encode():
    """The §8 e pipeline from SST blocks: each range decodes only the blocks of every run that
    overlap it (straddling blocks read by both neighbours), merges its own keys, and the ranges
    together give the single-stream compaction."""
    rng = np.random.default_rng(5)
    kv, rs = case(900, versions=2, nkeys=8000, nrun=4)
    bs, target = 4096, 48 << 10
    splitters = pick_splitters(kv, rng, 3)
    inputs = range_inputs(kv, rs, splitters, bs)
    wm = int(kv.ts.max()) // 3
    opts = batch.compact_opts(wm, True, block_size=bs, target_sst_size=target)
    res, _ = run_ranges(None, None, opts, splitters, inputs)
    want, kept, bases = check_against_single_stream(kv, rs, res, wm, True, bs, target)
    check_each_range_against_resumed_oracle(kept, res, bases, bs, target)


def _shards_on_own_streams(d, rs, opts, splitters):
    out = []
    for r in range(len(splitters) + 1):
        lo, hi = shard.range_of(r, splitters)
        out.append(shard.RangeShard(d, rs, opts, lo, hi, stream=torch.cuda.Stream()))
    return out


def test_ranges_on_distinct_streams_local():
    """compact_local with every RangeShard on its own HIP stream: the carry chain crosses streams."""
    rng = np.random.default_rng(21)
    kv, rs = case(77, versions=2, nkeys=8000)
    d = to_dev(kv)
    bs, target, wm = 1024, 8 << 10, int(kv.ts.max()) // 2
    opts = batch.compact_opts(wm, True, block_size=bs, target_sst_size=target)
    res = shard.compact_local(_shards_on_own_streams(d, rs, opts, pick_splitters(kv, rng, 5)))
    check_against_single_stream(kv, rs, res, wm, True, bs, target)


def test_ranges_on_distinct_streams_compact_dist_single_rank():
    """compact_dist's driver (gloo, world 1, R = 4 ranges on distinct streams): the ranges' carry
    chain and the carry-out read after it, each on the right stream."""
    import os
    import socket
    import torch.distributed as dist
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        rng = np.random.default_rng(22)
        kv, rs = case(78, versions=3, nkeys=6000)
        d = to_dev(kv)
        bs, target = 4096, 24 << 10
        opts = batch.compact_opts(0, False, block_size=bs, target_sst_size=target)
        res = shard.compact_dist(_shards_on_own_streams(d, rs, opts, pick_splitters(kv, rng, 3)))
        check_against_single_stream(kv, rs, res, 0, False, bs, target)
    finally:
        dist.destroy_process_group()


def test_fresh_contexts_on_distinct_streams_repeatedly():
    """The round-4 hang, found: a context's first call grew its workspace and
    zeroed it with hipMemset on the null stream, which does not order with the caller's
    non-blocking stream -- the fill could land after the rotation had written its levels there,
    leaving links that never advance (round 4: rot_f_kernel spun forever; round 5, with the
    lifting bounded: LSMBLK_E_INTERNAL on ~70 % of these runs).  Fresh ranges (fresh contexts) on
    fresh streams, eight times over, every time equal to the single-stream compaction."""
    import os
    import socket
    import torch.distributed as dist
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        rng = np.random.default_rng(22)
        kv, rs = case(78, versions=3, nkeys=6000)
        d = to_dev(kv)
        bs, target = 4096, 24 << 10
        opts = batch.compact_opts(0, False, block_size=bs, target_sst_size=target)
        splitters = pick_splitters(kv, rng, 3)
        for _ in range(8):
            res = shard.compact_dist(_shards_on_own_streams(d, rs, opts, splitters))
            check_against_single_stream(kv, rs, res, 0, False, bs, target)
    finally:
        dist.destroy_process_group()


# ---------------------------------------------------------------- two-level merge (TwoMergeIterator) by key range
from lsm_amd._lib import LSMBLK_MERGE_TWO_LEVEL as TWO  # noqa: E402


def two_level_input(seed, nkeys, b_frac, versions=3):
    """Multi-version upper runs and a lower level b (the last run) that ends b_frac of the way
    through the key space (0: b empty): upper keys beyond b's last key are lost by the reference's
    TwoMergeIterator, and ranges above that key get nothing of a."""
    keys, ko, vals, vo, ts, rs = synth.gen_runs(nkeys, nrun=4, seed=seed, versions=versions, tombstone=0.1)
    kv = O.KV(keys, ko, vals, vo, ts)
    ents = kv.entries()
    runs = [ents[rs[r]:rs[r + 1]] for r in range(4)]
    runs[-1] = runs[-1][:int(len(runs[-1]) * b_frac)]
    flat = [e for r in runs for e in r]
    rs2 = np.concatenate([[0], np.cumsum([len(r) for r in runs])]).astype(np.uint32)
    return O.KV.from_entries(flat), rs2


@pytest.mark.parametrize("seed,b_frac,bottom", [(0, 0.6, True), (1, 1.0, False), (2, 0.25, True), (3, 0.0, False)])
def test_two_level_sharded_compaction_equals_single_stream(seed, b_frac, bottom):
    """LSMBLK_MERGE_TWO_LEVEL by key range (lsmblk_compact_merge_batch_ex + the kept entries'
    same_as_last_key carried through the halo into lsmblk_shard_rotation_prepare_ex): the ranges'
    blocks and SST starts equal the single-stream two-level compaction (lsmblk_compact_batch, which
    tests/test_gpu_compact.py pins to the line-by-line iterator) -- splitters below, at and above b's
    last key, ranges wholly past it, and an empty b."""
    rng = np.random.default_rng(70 + seed)
    kv, rs = two_level_input(500 + seed, 5000, b_frac)
    d = to_dev(kv)
    bs, target = [(4096, 24 << 10), (1024, 6 << 10), (512, 3000), (4096, 1 << 20)][seed]
    wm = int(kv.ts.max()) // 2
    single = batch.compact_runs(d, rs, wm, bottom, block_size=bs, target_sst_size=target, merge_mode=TWO)
    want_blocks = single["blocks"].cpu().numpy().tobytes()
    want_starts = single["sst_start"].cpu().numpy().view(np.uint32).astype(np.int64)[:-1].tolist()
    opts = batch.compact_opts(wm, bottom, block_size=bs, target_sst_size=target, merge_mode=TWO)
    b_last = kv.entry(int(rs[-1]) - 1)[0] if rs[-1] > rs[-2] else None
    for k in (1, 4, 9):
        sp = pick_splitters(kv, rng, k)
        if b_last is not None:
            sp = sorted(set(sp) | {b_last})  # a range starting exactly at b's last key
        res, _ = run_ranges(d, rs, opts, sp)
        assert b"".join(r["blocks"].cpu().numpy().tobytes() for r in res) == want_blocks
        bases = np.concatenate([[0], np.cumsum([r["m"] for r in res])]).tolist()
        assert bases[-1] == single["stats"][5]
        assert shard.sst_starts(res, bases) == want_starts
        for a, b in zip(res, res[1:]):
            assert a["carry_out"] == b["carry_in"]
    if b_frac == 0.0:
        assert want_blocks == b""


def test_two_level_sharded_small_vs_iterator():
    """A small two-level case through the ranges against compact_generate_sst over the reference's
    TwoMergeIterator restated line by line (oracle/pyref.py): b's second, fourth, ... versions of a
    shared key, upper keys past b's end dropped, a tombstone at the bottom level."""
    from oracle import pyref
    a = [(b"a", 9, b"A9"), (b"c", 8, b"C8"), (b"k", 9, b"K9"), (b"m", 7, b""), (b"x", 6, b"X6"), (b"z", 5, b"Z5")]
    b = [(b"c", 5, b"c5"), (b"c", 4, b"c4"), (b"c", 3, b"c3"), (b"k", 2, b"k2"), (b"m", 1, b"m1"), (b"q", 1, b"q1")]
    runs = [a, b]
    want = pyref.compact_generate_sst(pyref.two_merge_iter(runs), 0, True, (), 64, 100)
    kv = O.KV.from_entries(a + b)
    rs = np.array([0, len(a), len(a) + len(b)], np.uint32)
    opts = batch.compact_opts(0, True, block_size=64, target_sst_size=100, merge_mode=TWO)
    for sp in ([b"d"], [b"k", b"q"], [b"m\x00", b"r"], [b"q"]):
        res, _ = run_ranges(to_dev(kv), rs, opts, sp)
        assert b"".join(r["blocks"].cpu().numpy().tobytes() for r in res) == b"".join(blk for sst, _ in want for blk in sst)


@pytest.mark.parametrize("seed,b_frac", [(0, 0.6), (1, 1.0), (2, 0.3)])
def test_two_level_ranges_read_only_their_blocks(seed, b_frac):
    """The two-level merge with every range decoding only the blocks of each run that overlap it
    (ADVICE round 4): no range holds all of b, so b's last key -- where TwoMergeIterator's stream
    ends -- reaches the ranges through compact_local's b-end exchange (the same message as
    compact_dist's all-gather), and the ranges give the single-stream two-level compaction."""
    rng = np.random.default_rng(930 + seed)
    kv, rs = two_level_input(940 + seed, 6000, b_frac)
    bs, target = 4096, 32 << 10
    wm = int(kv.ts.max()) // 2
    single = batch.compact_runs(to_dev(kv), rs, wm, True, block_size=bs, target_sst_size=target, merge_mode=TWO)
    want_blocks = single["blocks"].cpu().numpy().tobytes()
    want_starts = single["sst_start"].cpu().numpy().view(np.uint32).astype(np.int64)[:-1].tolist()
    sp = pick_splitters(kv, rng, 4)
    if rs[-1] > rs[-2]:
        sp = sorted(set(sp) | {kv.entry(int(rs[-1]) - 1)[0]})  # a range starting exactly at b's last key
    opts = batch.compact_opts(wm, True, block_size=bs, target_sst_size=target, merge_mode=TWO)
    res, _ = run_ranges(None, None, opts, sp, range_inputs(kv, rs, sp, bs))
    assert b"".join(r["blocks"].cpu().numpy().tobytes() for r in res) == want_blocks
    bases = np.concatenate([[0], np.cumsum([r["m"] for r in res])]).tolist()
    assert bases[-1] == single["stats"][5]
    assert shard.sst_starts(res, bases) == want_starts
    for a, b in zip(res, res[1:]):
        assert a["carry_out"] == b["carry_in"]
