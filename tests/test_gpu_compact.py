"""GPU parity of the compaction path (merge, rules, SST rotation, fused pipeline) through the C
ABI against the oracle: MergeIterator / compact_generate_sst restated line by line
(oracle/pyref.py) and their C forms (oracle/lsmblk_oracle.c).  Bit-exact bar."""
import numpy as np
import pytest
import torch

from lsm_amd import batch, synth
from lsm_amd._lib import LSMBLK_E_INVAL, LSMBLK_E_MALFORMED, LSMBLK_MERGE_RUNS, LSMBLK_MERGE_TWO_LEVEL, LsmBlkError
from oracle import oracle as O
from oracle import pyref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")


def kv_runs(runs):
    ents = [e for r in runs for e in r]
    rs = np.zeros(len(runs) + 1, np.uint32)
    rs[1:] = np.cumsum([len(r) for r in runs])
    return O.KV.from_entries(ents), rs


def to_dev(kv: O.KV):
    return batch.KVStream.from_numpy(kv.keys, kv.key_off, kv.vals, kv.val_off, kv.ts)


def dev_entries(d: batch.KVStream):
    keys, ko, vals, vo, ts = d.to_numpy()
    return [(bytes(keys[ko[i]:ko[i + 1]]), int(ts[i]), bytes(vals[vo[i]:vo[i + 1]])) for i in range(d.n)]


def assert_kv_equal(d: batch.KVStream, ref: O.KV):
    keys, ko, vals, vo, ts = d.to_numpy()
    assert d.n == ref.n
    np.testing.assert_array_equal(ko, ref.key_off)
    np.testing.assert_array_equal(vo, ref.val_off)
    np.testing.assert_array_equal(ts, ref.ts)
    np.testing.assert_array_equal(keys, ref.keys[:ref.key_off[-1]])
    np.testing.assert_array_equal(vals, ref.vals[:ref.val_off[-1]])


def gpu_merge(runs):
    kv, rs = kv_runs(runs)
    return dev_entries(batch.merge_runs(to_dev(kv), rs))


def kvs(pairs):
    return [(k.encode(), 0, v.encode()) for k, v in pairs]


def random_runs(rng, nrun, nkeys, max_versions=3, maxlen=6):
    space = sorted({bytes(rng.integers(97, 100, int(rng.integers(1, maxlen)), dtype=np.uint8)) for _ in range(nkeys)})
    runs = []
    for r in range(nrun):
        take = sorted(rng.choice(len(space), size=int(rng.integers(0, len(space) + 1)), replace=False))
        run = []
        for i in take:
            for t in sorted(rng.choice(1000, size=int(rng.integers(1, max_versions + 1)), replace=False), reverse=True):
                run.append((space[i], int(t), b"" if rng.random() < 0.2 else b"r%d-%d" % (r, t)))
        runs.append(run)
    return runs


# ---------------------------------------------------------------- merge
def test_merge_week1_day2_fixtures():
    i1 = kvs([("a", "1.1"), ("b", "2.1"), ("c", "3.1"), ("e", "")])
    i2 = kvs([("a", "1.2"), ("b", "2.2"), ("c", "3.2"), ("d", "4.2")])
    i3 = kvs([("b", "2.3"), ("c", "3.3"), ("d", "4.3")])
    assert gpu_merge([i1, i2, i3]) == kvs([("a", "1.1"), ("b", "2.1"), ("c", "3.1"), ("d", "4.2"), ("e", "")])
    assert gpu_merge([i3, i1, i2]) == kvs([("a", "1.1"), ("b", "2.3"), ("c", "3.3"), ("d", "4.3"), ("e", "")])
    j1 = kvs([("a", "1.1"), ("b", "2.1"), ("c", "3.1")])
    j2 = kvs([("d", "1.2"), ("e", "2.2"), ("f", "3.2"), ("g", "4.2")])
    j3 = kvs([("h", "1.3"), ("i", "2.3"), ("j", "3.3"), ("k", "4.3")])
    assert gpu_merge([j2, [], j3, j1]) == j1 + j2 + j3
    assert gpu_merge([j1, []]) == j1
    assert gpu_merge([[], []]) == []


@pytest.mark.parametrize("seed", range(8))
def test_merge_random_runs_vs_heap_restatement(seed):
    rng = np.random.default_rng(seed)
    runs = random_runs(rng, int(rng.integers(1, 12)), int(rng.integers(1, 400)), maxlen=8)
    assert gpu_merge(runs) == pyref.merge_runs(runs)


@pytest.mark.parametrize("nrun,versions", [(8, 1), (5, 3), (64, 1), (1, 2)])
def test_merge_synthetic_runs_vs_c_oracle(nrun, versions):
    keys, ko, vals, vo, ts, rs = synth.gen_runs(60000 // versions, nrun=nrun, seed=nrun, versions=versions)
    kv = O.KV(keys, ko, vals, vo, ts)
    src = O.merge_runs(kv, rs)
    assert_kv_equal(batch.merge_runs(to_dev(kv), rs), O.gather(kv, src))


def test_merge_big_tiles_global_path():
    """Tiles beyond the LDS tables: one key with thousands of versions in several runs, long
    keys (> the LDS key image), many short runs."""
    rng = np.random.default_rng(3)
    hot = b"hot-key"
    runs = []
    for r in range(6):
        run = [(b"a%05d" % i, 5, b"v") for i in sorted(rng.choice(3000, 200, replace=False))]
        run += [(hot, int(t), b"h%d" % r) for t in range(3000 - r, 0, -1)]
        run += [(b"z" * 300 + b"%04d" % i, 1, b"w") for i in sorted(rng.choice(2000, 150, replace=False))]
        runs.append(run)
    assert gpu_merge(runs) == pyref.merge_runs_rule(runs)


def test_merge_errors():
    kv, rs = kv_runs([kvs([("a", "1")]), kvs([("b", "2")])])
    d = to_dev(kv)
    with pytest.raises(LsmBlkError) as e:
        batch.merge_runs(d, np.array([0, 2, 1], np.uint32))  # decreasing run table
    assert e.value.status == LSMBLK_E_INVAL
    bad, rs = kv_runs([kvs([("b", "1"), ("a", "2")]), kvs([("c", "3")])])  # an unsorted run
    with pytest.raises(LsmBlkError) as e:
        batch.merge_runs(to_dev(bad), rs)
    assert e.value.status == LSMBLK_E_MALFORMED


def test_merge_rejects_keys_over_64k():
    """A key over 65 535 bytes is refused with LSMBLK_E_INVAL (the merge tiles keep
    u16 key lengths, so 65 537 and 1 bytes would compare as one length); 65 535 bytes still merge."""
    a, b = b"k" * 65536 + b"a", b"k"
    kv, rs = kv_runs([[(a, 2, b"x")], [(b, 1, b"y")]])
    with pytest.raises(LsmBlkError) as e:
        batch.merge_runs(to_dev(kv), rs)
    assert e.value.status == LSMBLK_E_INVAL
    with pytest.raises(LsmBlkError) as e:
        batch.compact_runs(to_dev(kv), rs, 0, False, (), 4096, 1 << 20)
    assert e.value.status == LSMBLK_E_INVAL
    a2 = b"k" * 65534 + b"a"
    kv, rs = kv_runs([[(a2, 2, b"x")], [(b, 1, b"y"), (a2, 1, b"z")]])
    assert dev_entries(batch.merge_runs(to_dev(kv), rs)) == [(b, 1, b"y"), (a2, 2, b"x")]


# ---------------------------------------------------------------- two-level (TwoMergeIterator) input
from test_merge_oracle import DIFF_CLASSES, WEEK1_DAY5  # noqa: E402  (fixture tables, CPU-side data)

TWO = LSMBLK_MERGE_TWO_LEVEL


def gpu_merge_mode(runs, mode):
    kv, rs = kv_runs(runs)
    return dev_entries(batch.merge_runs(to_dev(kv), rs, merge_mode=mode))


def ref_compact(it, wm, bottom, pf, bs, target):
    try:
        return pyref.compact_generate_sst(it, wm, bottom, pf, bs, target)
    except AssertionError:  # the reference panics building an empty SST
        return None


def check_compact_mode(runs, mode, wm, bottom, pf, bs, target):
    """lsmblk_compact_batch in `mode` == compact_generate_sst over MergeIterator(runs) (RUNS) or over
    TwoMergeIterator(MergeIterator(runs[:-1]), runs[-1]) (TWO_LEVEL), line by line."""
    it = pyref.two_merge_iter(runs) if mode == TWO else pyref.MergeIterator([pyref.ListIter(r) for r in runs])
    want = ref_compact(it, wm, bottom, pf, bs, target)
    kv, rs = kv_runs(runs)
    got = batch.compact_runs(to_dev(kv), rs, wm, bottom, pf, bs, target, merge_mode=mode)
    if want is None:
        assert got["stats"][2] == 0 and got["stats"][5] == 0
        return got
    assert dev_entries(got["kept"]) == [e for _, es in want for e in es]
    assert got["blocks"].cpu().numpy().tobytes() == b"".join(b for sst, _ in want for b in sst)
    np.testing.assert_array_equal(np.diff(got["sst_blk"].cpu().numpy().view(np.uint32).astype(np.int64)),
                                  [len(s) for s, _ in want])
    np.testing.assert_array_equal(np.diff(got["sst_start"].cpu().numpy().view(np.uint32).astype(np.int64)),
                                  [len(e) for _, e in want])
    return got


@pytest.mark.parametrize("case", sorted(WEEK1_DAY5))
def test_week1_day5_fixtures_through_hip(case):
    """src/tests/week1_day5.rs:15-129 through lsmblk_merge_batch_ex and lsmblk_compact_batch with b
    (the lower level) as the last run: LSMBLK_MERGE_RUNS meets every expectation; TWO_LEVEL gives
    what two_merge_iterator.rs as written gives (merge_2, merge_3, merge_4a differ)."""
    a, b, want = WEEK1_DAY5[case]
    assert gpu_merge_mode([a, b], LSMBLK_MERGE_RUNS) == want
    assert gpu_merge_mode([a, b], TWO) == pyref.two_merge_runs([a, b])
    for mode in (LSMBLK_MERGE_RUNS, TWO):
        check_compact_mode([a, b], mode, 0, False, (), 4096, 1 << 20)
        check_compact_mode([a, b], mode, 0, False, (), 16, 40)  # one entry per block, several SSTs


@pytest.mark.parametrize("case", sorted(DIFF_CLASSES))
def test_two_merge_difference_classes_through_hip(case):
    runs, runs_merge, two_merge = DIFF_CLASSES[case]
    assert gpu_merge_mode(runs, LSMBLK_MERGE_RUNS) == runs_merge
    assert gpu_merge_mode(runs, TWO) == two_merge


@pytest.mark.parametrize("seed", range(10))
def test_two_level_random_runs_vs_iterator(seed):
    """Multi-version b, empty runs, upper keys past b's last key; the compaction rules over the
    two-level order (b's older versions before a's newer ones) run as the reference's loop."""
    rng = np.random.default_rng(300 + seed)
    runs = random_runs(rng, int(rng.integers(1, 6)), int(rng.integers(1, 150)), max_versions=5, maxlen=7)
    assert gpu_merge_mode(runs, TWO) == pyref.two_merge_runs(runs)
    for wm, bottom, pf, bs, target in ((0, False, (), 64, 200), (500, True, (), 128, 300),
                                       (500, False, (b"a",), 96, 1), (10**6, True, (b"ab",), 4096, 1 << 20),
                                       (300, True, (b"b",), 48, 100)):
        check_compact_mode(runs, TWO, wm, bottom, pf, bs, target)


def test_two_level_synthetic_and_big_tiles():
    """Tile-sized inputs (LDS tiles) and one hot key with thousands of versions in a and b (the
    one-wave global path), against the closed form restated in oracle/pyref.py."""
    keys, ko, vals, vo, ts, rs = synth.gen_runs(30000, nrun=5, seed=11, versions=3, tombstone=0.1)
    kv = O.KV(keys, ko, vals, vo, ts)
    ents = kv.entries()
    runs = [ents[rs[r]:rs[r + 1]] for r in range(5)]
    runs[-1] = runs[-1][:len(runs[-1]) * 3 // 4]  # b ends before the upper runs do
    assert gpu_merge_mode(runs, TWO) == pyref.two_merge_rule(runs)
    hot, rng = b"hot-key", np.random.default_rng(5)
    big = []
    for r in range(4):
        run = [(b"a%05d" % i, 5, b"v%d" % r) for i in sorted(rng.choice(3000, 200, replace=False))]
        run += [(hot, int(t), b"h%d" % r) for t in range(3000 - r, 0, -1)]
        run += [(b"z" * 300 + b"%04d" % i, 1, b"w") for i in sorted(rng.choice(2000, 150, replace=False))]
        big.append(run)
    assert gpu_merge_mode(big, TWO) == pyref.two_merge_rule(big)
    assert gpu_merge_mode(big, LSMBLK_MERGE_RUNS) == pyref.merge_runs_rule(big)


@pytest.mark.parametrize("versions", [(130, 150, 200, 170), (400, 380, 300, 420), (520, 1, 0, 600)])
def test_merge_tiles_over_the_small_lds_limit(versions):
    """Tiles of 512 < n <= 2048 entries go to merge_big_kernel's LDS tables (and past 2048 to the
    global path): hot keys with hundreds of versions per run, next to ordinary keys."""
    rng = np.random.default_rng(sum(versions))
    runs = []
    for r, nv in enumerate(versions):
        run = [(b"k%05d" % i, 7, b"v%d" % r) for i in sorted(rng.choice(4000, 300, replace=False))]
        run += [(b"k02000x", int(t), b"h%d" % r) for t in range(nv + 1000 * (4 - r), 1000 * (4 - r), -1)]
        run += [(b"k03000y", int(t), b"y%d" % r) for t in range(nv // 2 + 1000 * (4 - r), 1000 * (4 - r), -1)]
        runs.append(sorted(run, key=lambda e: e[0]))  # stable: versions stay newest first
    assert gpu_merge_mode(runs, TWO) == pyref.two_merge_rule(runs)
    assert gpu_merge_mode(runs, LSMBLK_MERGE_RUNS) == pyref.merge_runs_rule(runs)


def test_merge_many_runs_natural_big_tiles():
    """Twelve overlapping runs: candidate gaps leave a few percent of the tiles over 512 entries
    (merge_big_kernel) among the ordinary ones."""
    keys, ko, vals, vo, ts, rs = synth.gen_runs(60000, nrun=12, seed=17, versions=2)
    ents = O.KV(keys, ko, vals, vo, ts).entries()
    runs = [ents[rs[r]:rs[r + 1]] for r in range(12)]
    assert gpu_merge_mode(runs, LSMBLK_MERGE_RUNS) == pyref.merge_runs_rule(runs)
    assert gpu_merge_mode(runs, TWO) == pyref.two_merge_rule(runs)


def test_two_level_key_range_argument_errors():
    """Key ranges take the two-level merge through lsmblk_compact_merge_batch_ex only, with the
    kept entries' same_as_last_key output and a valid b-end mode (tests/test_gpu_shard.py runs it)."""
    from lsm_amd._lib import lib
    kv, rs = kv_runs([kvs([("a", "1")]), kvs([("b", "2")])])
    d = to_dev(kv)
    opts = batch.compact_opts(0, False, (), 4096, 1 << 20, merge_mode=TWO)
    kept = batch.KVStream.empty(d.n, 16, 16, torch.device("cuda"))
    stats = torch.zeros(5, dtype=torch.int64, device="cuda")
    rs_t = batch._u32_table(rs, "cuda")
    with pytest.raises(LsmBlkError) as e:  # no kept_same
        batch.compact_merge_into(d, rs_t, 2, opts, None, kept, stats)
    assert e.value.status == LSMBLK_E_INVAL
    ks = torch.zeros(d.n + 1, dtype=torch.uint8, device="cuda")
    with pytest.raises(LsmBlkError) as e:  # no such b-end mode
        batch.compact_merge_into(d, rs_t, 2, opts, None, kept, stats, two_end=3, kept_same=ks)
    assert e.value.status == LSMBLK_E_INVAL
    import ctypes
    ci, ck, o = d._c(), kept._c(*kept.caps()), batch._opts_c(opts)
    assert lib().lsmblk_compact_merge_batch(batch._ctx(0), ctypes.byref(ci), rs_t.data_ptr(), 2, ctypes.byref(o),
                                            None, ctypes.byref(ck), stats.data_ptr(), None) == LSMBLK_E_INVAL
    torch.cuda.synchronize()


# ---------------------------------------------------------------- SST rotation
@pytest.mark.parametrize("bs,target", [(4096, 64 << 10), (4096, 1), (128, 700), (65536, 1 << 40), (512, 5000)])
def test_sst_rotation_vs_restated_loop(bs, target):
    """lsmblk_sst_rotation_batch == orc_segment_like_compaction (the rotation of compact.rs:278-289
    over the entries handed to SsTableBuilder::add), multi-version keys.  The capacity is n + 2
    (2^15 slots): the SST chain's walk + fill run with K = 6 doubling levels, and target 1 (an SST
    at every key change, ~6 700 of them) walks ~105 anchors, 2 loads each; the bench's C sizes use K = 3."""
    keys, ko, vals, vo, ts, rs = synth.gen_runs(20000, nrun=4, seed=7, versions=3, tombstone=0.05)
    kv = O.KV(keys, ko, vals, vo, ts)
    src = O.merge_runs(kv, rs)
    kept = O.gather(kv, src)
    want = O.segment_like_compaction(kept, bs, target)
    got = batch.sst_rotation(to_dev(kept), bs, target)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("versions", [1, 3])
def test_sst_rotation_large_capacity_long_chain(versions):
    """A capacity far above 2^17 (n + 2 ~ 2^18, so every doubling level runs and no walk / fill
    does) with a long chain (64-B blocks and target 1: one entry per block and an SST at every key
    change, 10^4 - 10^5 of them): bit-exact, and no serial chain walk that grows with the capacity
    (K = lc - 9 made each fill thread follow ~sst_cap / 512 elements) -- checked on
    the launches themselves (the context's kernel log), not on wall-clock time."""
    from lsm_amd._lib import check, kernel_log, lib
    keys, ko, vals, vo, ts, rs = synth.gen_runs(200000 // versions, nrun=2, seed=17, versions=versions)
    kv = O.KV(keys, ko, vals, vo, ts)
    kept = O.gather(kv, O.merge_runs(kv, rs))
    want = O.segment_like_compaction(kept, 64, 1)
    d = to_dev(kept)
    ctx = batch._ctx(torch.cuda.current_device())
    torch.cuda.synchronize()
    check(lib().lsmblk_debug_set(ctx, 2, 1))
    try:
        kernel_log(ctx)  # empties the log
        got = batch.sst_rotation(d, 64, 1)
        log = kernel_log(ctx)
    finally:
        check(lib().lsmblk_debug_set(ctx, 2, 0))
    np.testing.assert_array_equal(got, want)
    cap = kept.n + 2
    levels = int(np.ceil(np.log2(cap)))
    assert cap > (1 << 17) and len(want) > 20000, (kept.n, len(want))
    assert "rot_walk_kernel" not in log and "rot_fill_kernel" not in log, log
    assert log["rot_chain_kernel"][0] <= levels, (log["rot_chain_kernel"], levels)


def test_sst_rotation_unsorted_and_long_keys():
    rng = np.random.default_rng(9)
    base = bytes(rng.integers(0, 256, 80, dtype=np.uint8))
    keys = sorted({base[:int(rng.integers(0, 80))] + bytes(rng.integers(0, 256, 4, dtype=np.uint8))
                   for _ in range(3000)})
    keys = [k for k in keys for _ in range(int(rng.integers(1, 4)))]
    for order in ("sorted", "shuffled"):
        ks = keys if order == "sorted" else [keys[i] for i in rng.permutation(len(keys))]
        ents = [(k, i, bytes(rng.integers(0, 256, int(rng.integers(0, 200)), dtype=np.uint8))) for i, k in enumerate(ks)]
        kv = O.KV.from_entries(ents)
        for bs, target in ((1024, 20000), (4096, 3000)):
            np.testing.assert_array_equal(batch.sst_rotation(to_dev(kv), bs, target),
                                          O.segment_like_compaction(kv, bs, target))


# ---------------------------------------------------------------- fused compaction
def check_compact(kv: O.KV, rs, wm, bottom, pf, bs, target):
    src = O.merge_runs(kv, rs)
    want = O.compact(kv, src, wm, bottom, pf, bs, target)
    got = batch.compact_runs(to_dev(kv), rs, wm, bottom, pf, bs, target)
    assert got["stats"][4] == len(src)
    assert_kv_equal(got["kept"], O.gather(kv, src[want["kept"]]))
    np.testing.assert_array_equal(got["blk_off"].cpu().numpy().view(np.uint64), want["blk_off"])
    g = got["blocks"].cpu().numpy()
    assert len(g) == len(want["blocks"])
    mism = np.flatnonzero(g != want["blocks"])
    assert mism.size == 0, f"first mismatching byte {mism[:8]}"
    np.testing.assert_array_equal(got["sst_start"].cpu().numpy().view(np.uint32), want["sst_ent"])
    np.testing.assert_array_equal(got["sst_blk"].cpu().numpy().view(np.uint32), want["sst_blk"])
    return got, want


@pytest.mark.parametrize("versions,wm_frac,bottom,pf,bs,target", [
    (1, 0.0, False, (), 4096, 256 << 10),
    (2, 0.5, True, (), 4096, 128 << 10),
    (3, 0.7, True, (b"\x00", b"\x7f\xff"), 1024, 50000),
    (1, 1.0, True, (), 65536, 1 << 20),
])
def test_compact_pipeline_vs_c_oracle(versions, wm_frac, bottom, pf, bs, target):
    """decode-side runs -> merge -> rules -> rotation -> blocks, byte-identical to compact_generate_sst
    (restated in C, itself checked line by line against oracle/pyref.py on CPU)."""
    keys, ko, vals, vo, ts, rs = synth.gen_runs(60000 // versions, nrun=6, seed=versions, versions=versions,
                                                tombstone=0.1)
    kv = O.KV(keys, ko, vals, vo, ts)
    wm = int(int(ts.max()) * wm_frac)
    got, want = check_compact(kv, rs, wm, bottom, pf, bs, target)
    assert len(want["sst_blk"]) > 2


@pytest.mark.parametrize("seed", range(6))
def test_compact_small_random_vs_line_by_line(seed):
    rng = np.random.default_rng(200 + seed)
    runs = random_runs(rng, int(rng.integers(1, 6)), 120, max_versions=4, maxlen=7)
    kv, rs = kv_runs(runs)
    for wm, bottom, pf, bs, target in ((0, False, (), 64, 200), (500, True, (), 128, 300), (500, False, (b"a",), 96, 1)):
        try:
            want = pyref.compact_generate_sst(pyref.MergeIterator([pyref.ListIter(r) for r in runs]), wm, bottom,
                                              pf, bs, target)
        except AssertionError:  # the reference panics building an empty SST
            want = []
        got, _ = check_compact(kv, rs, wm, bottom, pf, bs, target)
        assert b"".join(b for sst, _ in want for b in sst) == got["blocks"].cpu().numpy().tobytes()
        assert got["stats"][2] == len(want)


def test_compact_nothing_kept_and_capacity():
    ents = [(b"k%03d" % i, 1, b"") for i in range(300)]  # tombstones only, bottom level
    kv, rs = kv_runs([ents[:150], ents[150:]])
    got = batch.compact_runs(to_dev(kv), rs, 10, True, (), 4096, 1 << 20)
    assert got["stats"][2] == 0 and got["stats"][5] == 0 and got["blocks"].numel() == 0
    keys, ko, vals, vo, ts, rs = synth.gen_runs(5000, nrun=3, seed=1)
    d = to_dev(O.KV(keys, ko, vals, vo, ts))
    buf = batch.CompactBuffers(d.n, len(keys), len(vals), torch.device("cuda"), sst_cap=3)
    batch.compact_into(d, batch._u32_table(rs, "cuda"), 3, batch.compact_opts(0, False, (), 4096, 4096), buf)
    torch.cuda.synchronize()
    assert batch._status(buf.stats) == -3  # LSMBLK_E_CAPACITY: more SSTs than sst_cap - 1


def test_compaction_golden_fixtures_through_hip():
    """tests/golden/compact_runs_*.npz (the line-by-line restatement's SSTs) through
    lsmblk_compact_batch."""
    import json
    import os
    g = os.path.join(os.path.dirname(__file__), "golden")
    meta = json.load(open(os.path.join(g, "golden_compaction.json")))
    for name, m in meta.items():
        z = np.load(os.path.join(g, name + ".npz"))
        kv = O.KV(z["keys"], z["key_off"], z["vals"], z["val_off"], z["ts"])
        got = batch.compact_runs(to_dev(kv), z["run_start"], m["watermark"], m["bottom_level"],
                                 [p.encode() for p in m["prefixes"]], m["block_size"], m["target_sst_size"])
        np.testing.assert_array_equal(got["blocks"].cpu().numpy(), z["blocks"], err_msg=name)
        np.testing.assert_array_equal(got["blk_off"].cpu().numpy().view(np.uint64), z["blk_off"])
        np.testing.assert_array_equal(got["sst_blk"].cpu().numpy().view(np.uint32), z["sst_blk"])
        np.testing.assert_array_equal(got["sst_start"].cpu().numpy().view(np.uint32), z["sst_ent"])


def test_decode_runs_then_merge_with_block_entry_index():
    """The compaction read path: every run's SSTs decoded in ONE call, run boundaries from the
    decode's per-block entry index, then the merge (== C oracle)."""
    keys, ko, vals, vo, ts, rs = synth.gen_runs(40000, nrun=5, seed=4, versions=2)
    kv = O.KV(keys, ko, vals, vo, ts)
    parts, offs, run_blk, base = [], [], [0], 0
    for r in range(5):
        sub = O.gather(kv, np.arange(rs[r], rs[r + 1]))
        rc, b, o = O.encode_segments(sub, synth.segments_by_bytes(sub.key_off, sub.val_off, 64 << 10), 4096)
        parts.append(b)
        offs.append(o[:-1] + base)
        base += len(b)
        run_blk.append(run_blk[-1] + len(o) - 1)
    blocks = np.concatenate(parts)
    blk_off = np.concatenate(offs + [np.array([base], np.uint64)])
    db, do = torch.from_numpy(blocks).cuda(), torch.from_numpy(blk_off.view(np.int64)).cuda()
    d, ent = batch.decode_blocks(db, do, with_blk_ent=True)
    run_start = ent[torch.tensor(run_blk, device="cuda")].to(torch.int32)
    np.testing.assert_array_equal(run_start.cpu().numpy(), rs.astype(np.int32))
    assert_kv_equal(batch.merge_runs(d, run_start), O.gather(kv, O.merge_runs(kv, rs)))
