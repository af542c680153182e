"""The merge / compaction oracle (CPU only): MergeIterator, TwoMergeIterator and
compact_generate_sst restated line by line, pinned on the reference's own fixtures and checked
against the closed forms the GPU evaluates.

  src/tests/week1_day2.rs  test_task2_merge_1 / _2 / _empty: MergeIterator expectations
  src/iterators/merge_iterator.rs:59-184, two_merge_iterator.rs:5-98, src/compact.rs:223-311
"""
import numpy as np
import pytest

from lsm_amd import synth
from oracle import oracle as O
from oracle import pyref


def kv_runs(runs):
    ents = [e for r in runs for e in r]
    rs = np.zeros(len(runs) + 1, np.uint32)
    rs[1:] = np.cumsum([len(r) for r in runs])
    return O.KV.from_entries(ents), rs


def c_merge(runs):
    kv, rs = kv_runs(runs)
    src = O.merge_runs(kv, rs)
    ents = kv.entries()
    return [ents[i] for i in src]


def kvs(pairs):
    return [(k.encode(), 0, v.encode()) for k, v in pairs]


# ---------------------------------------------------------------- week1_day2 fixtures
I1 = kvs([("a", "1.1"), ("b", "2.1"), ("c", "3.1"), ("e", "")])
I2 = kvs([("a", "1.2"), ("b", "2.2"), ("c", "3.2"), ("d", "4.2")])
I3 = kvs([("b", "2.3"), ("c", "3.3"), ("d", "4.3")])


@pytest.mark.parametrize("merge", [pyref.merge_runs, pyref.merge_runs_rule, c_merge])
def test_week1_day2_merge_1(merge):  # week1_day2.rs:86-135
    assert merge([I1, I2, I3]) == kvs([("a", "1.1"), ("b", "2.1"), ("c", "3.1"), ("d", "4.2"), ("e", "")])
    assert merge([I3, I1, I2]) == kvs([("a", "1.1"), ("b", "2.3"), ("c", "3.3"), ("d", "4.3"), ("e", "")])


@pytest.mark.parametrize("merge", [pyref.merge_runs, pyref.merge_runs_rule, c_merge])
def test_week1_day2_merge_2(merge):  # :137-190
    j1 = kvs([("a", "1.1"), ("b", "2.1"), ("c", "3.1")])
    j2 = kvs([("d", "1.2"), ("e", "2.2"), ("f", "3.2"), ("g", "4.2")])
    j3 = kvs([("h", "1.3"), ("i", "2.3"), ("j", "3.3"), ("k", "4.3")])
    want = j1 + j2 + j3
    assert merge([j1, j2, j3, []]) == want
    assert merge([j2, [], j3, j1]) == want
    assert merge([[], j3, j2, j1]) == want


@pytest.mark.parametrize("merge", [pyref.merge_runs, pyref.merge_runs_rule, c_merge])
def test_week1_day2_merge_empty(merge):  # :192-212
    assert merge([]) == []
    j1 = kvs([("a", "1.1"), ("b", "2.1"), ("c", "3.1")])
    assert merge([j1, []]) == j1
    assert merge([[], []]) == []


# ---------------------------------------------------------------- random runs
def random_runs(rng, nrun, nkeys, max_versions=3, key_space=None):
    """Sorted runs over a shared key space with multi-version keys (newest first), empty values,
    variable-length keys with shared prefixes (so key order != length order)."""
    space = key_space or sorted({bytes(rng.integers(97, 100, int(rng.integers(1, 6)), dtype=np.uint8))
                                 for _ in range(nkeys)})
    runs = []
    for r in range(nrun):
        take = sorted(rng.choice(len(space), size=int(rng.integers(0, len(space) + 1)), replace=False))
        run = []
        for i in take:
            nv = int(rng.integers(1, max_versions + 1))
            for t in sorted(rng.choice(1000, size=nv, replace=False), reverse=True):
                v = b"" if rng.random() < 0.2 else b"r%d-%d" % (r, t)
                run.append((space[i], int(t), v))
        runs.append(run)
    return runs


@pytest.mark.parametrize("seed", range(12))
def test_merge_heap_restatement_equals_rule_and_c(seed):
    """Literal BinaryHeap simulation == per-key lowest-run rule == the C heap merge."""
    rng = np.random.default_rng(seed)
    runs = random_runs(rng, int(rng.integers(1, 9)), int(rng.integers(1, 60)))
    want = pyref.merge_runs(runs)
    assert pyref.merge_runs_rule(runs) == want
    assert c_merge(runs) == want


def test_two_merge_iterator_quirks_and_intended_regime():
    """TwoMergeIterator (two_merge_iterator.rs) equals the lowest-priority-run model only while b
    holds one version per key and outlives a; its quirks are documented here."""
    a = kvs([("a", "A"), ("c", "C")])
    b = kvs([("a", "x"), ("b", "y"), ("d", "z")])
    got = pyref.drain(pyref.TwoMergeIterator(pyref.ListIter(a), pyref.ListIter(b)))
    assert got == pyref.merge_runs([a, b])
    # quirk 1: b exhausted -> the merged stream ends, a's tail is lost (choose_a :36-38)
    assert pyref.drain(pyref.TwoMergeIterator(pyref.ListIter(a), pyref.ListIter([]))) == []
    b2 = kvs([("a", "x")])
    assert pyref.drain(pyref.TwoMergeIterator(pyref.ListIter(a), pyref.ListIter(b2))) == []
    # quirk 2: skip_b skips ONE equal version of b, the next one is chosen before a (:45-50)
    b3 = [(b"a", 5, b"b5"), (b"a", 4, b"b4"), (b"z", 1, b"z")]
    got = pyref.drain(pyref.TwoMergeIterator(pyref.ListIter([(b"a", 9, b"a9")]), pyref.ListIter(b3)))
    assert got == [(b"a", 4, b"b4"), (b"a", 9, b"a9"), (b"z", 1, b"z")]


# ---------------------------------------------------------------- week1_day5: TwoMergeIterator
# src/tests/week1_day5.rs:15-129 (MockIterator pairs, ts 0): (a, b, expected), b = the lower level.
W5_1 = kvs([("a", "1.1"), ("b", "2.1"), ("c", "3.1")])
W5_2 = kvs([("a", "1.2"), ("b", "2.2"), ("c", "3.2"), ("d", "4.2")])
W5_3 = kvs([("b", "2.2"), ("c", "3.2"), ("d", "4.2")])
WEEK1_DAY5 = {
    "merge_1": (W5_1, W5_2, kvs([("a", "1.1"), ("b", "2.1"), ("c", "3.1"), ("d", "4.2")])),      # :16-38
    "merge_2": (W5_2, W5_1, kvs([("a", "1.2"), ("b", "2.2"), ("c", "3.2"), ("d", "4.2")])),      # :41-63
    "merge_3": (W5_3, W5_1, kvs([("a", "1.1"), ("b", "2.2"), ("c", "3.2"), ("d", "4.2")])),      # :66-87
    "merge_4a": (W5_3, [], W5_3),                                                                # :90-105
    "merge_4b": ([], W5_3, W5_3),                                                                # :106-120
    "merge_5": ([], [], []),                                                                     # :124-129
}
# what two_merge_iterator.rs as written yields where it differs from week1_day5's expectation
TWO_MERGE_AS_WRITTEN = {
    "merge_2": kvs([("a", "1.2"), ("b", "2.2")]),  # a holds b's last key "c": a's c and d are lost
    "merge_3": kvs([("a", "1.1"), ("b", "2.2")]),  # b ends after "c": a's c and d are lost
    "merge_4a": [],                                # empty b: nothing at all
}


@pytest.mark.parametrize("case", sorted(WEEK1_DAY5))
def test_week1_day5_fixtures(case):
    """The run-priority merge (LSMBLK_MERGE_RUNS: a's runs first, b last) gives every expectation of
    week1_day5.rs; the reference's TwoMergeIterator as written fails merge_2, merge_3 and merge_4a."""
    a, b, want = WEEK1_DAY5[case]
    for merge in (pyref.merge_runs, pyref.merge_runs_rule, c_merge):
        assert merge([a, b]) == want
    got = pyref.two_merge_runs([a, b])
    assert got == TWO_MERGE_AS_WRITTEN.get(case, want)
    assert pyref.two_merge_rule([a, b]) == got


# Input classes on which the reference binary's compaction input (TwoMergeIterator) differs from
# the run-priority merge; DESIGN.md section 3 reproduces this table.  (a runs..., b): both outputs.
DIFF_CLASSES = {
    "b exhausted before a": (
        [kvs([("a", "A"), ("x", "X"), ("y", "Y")]), kvs([("a", "b"), ("m", "M")])],
        kvs([("a", "A"), ("m", "M"), ("x", "X"), ("y", "Y")]),
        kvs([("a", "A"), ("m", "M")])),
    "empty b": (
        [kvs([("a", "A"), ("c", "C")]), []],
        kvs([("a", "A"), ("c", "C")]),
        []),
    "a holds b's last key": (
        [kvs([("a", "A"), ("m", "M2")]), kvs([("a", "b"), ("m", "M1")])],
        kvs([("a", "A"), ("m", "M2")]),
        kvs([("a", "A")])),
    ">= 2 b versions of a key a holds": (
        [[(b"k", 9, b"a9")], [(b"k", 5, b"b5"), (b"k", 4, b"b4"), (b"k", 3, b"b3"), (b"k", 2, b"b2"), (b"z", 1, b"z")]],
        [(b"k", 9, b"a9"), (b"z", 1, b"z")],
        [(b"k", 4, b"b4"), (b"k", 2, b"b2"), (b"k", 9, b"a9"), (b"z", 1, b"z")]),
}


@pytest.mark.parametrize("case", sorted(DIFF_CLASSES))
def test_two_merge_difference_classes(case):
    runs, runs_merge, two_merge = DIFF_CLASSES[case]
    assert pyref.merge_runs(runs) == runs_merge == pyref.merge_runs_rule(runs)
    assert pyref.two_merge_runs(runs) == two_merge == pyref.two_merge_rule(runs)
    assert runs_merge != two_merge


def test_two_merge_agrees_in_the_intended_regime():
    """One version per key in b and b's last key above every upper key: the two modes agree."""
    rng = np.random.default_rng(7)
    for _ in range(30):
        runs = random_runs(rng, int(rng.integers(2, 6)), 40, max_versions=3)
        b = sorted({e[0] for r in runs[:-1] for e in r} | {e[0] for e in runs[-1]})
        runs[-1] = [(k, 0, b"lower") for k in b] + [(b"\xff", 0, b"end")]
        assert pyref.two_merge_runs(runs) == pyref.merge_runs(runs)


@pytest.mark.parametrize("seed", range(40))
def test_two_merge_rule_equals_iterator(seed):
    """The closed form the GPU evaluates == two_merge_iterator.rs line by line, on random runs with
    multi-version keys in b, empty runs, upper keys beyond b's last key."""
    rng = np.random.default_rng(1000 + seed)
    runs = random_runs(rng, int(rng.integers(1, 6)), int(rng.integers(1, 50)), max_versions=5)
    assert pyref.two_merge_rule(runs) == pyref.two_merge_runs(runs)


def compact_two_ref(runs, wm, bottom, pf, bs, target):
    """compact_generate_sst over the reference's TwoMergeIterator input, line by line."""
    return pyref.compact_generate_sst(pyref.two_merge_iter(runs), wm, bottom, pf, bs, target)


def compact_ref(runs, wm, bottom, pf, bs, target):
    """compact_generate_sst over MergeIterator (restated line by line): [(blocks, entries)]."""
    return pyref.compact_generate_sst(pyref.MergeIterator([pyref.ListIter(r) for r in runs]),
                                      wm, bottom, pf, bs, target)


def check_c_compact(runs, wm, bottom, pf, bs, target):
    kv, rs = kv_runs(runs)
    src = O.merge_runs(kv, rs)
    got = O.compact(kv, src, wm, bottom, pf, bs, target)
    try:
        want = compact_ref(runs, wm, bottom, pf, bs, target)
    except AssertionError:  # the reference panics building an empty SST
        assert len(got["sst_blk"]) == 1 and len(got["kept"]) == 0
        return got
    blocks = [b for sst, _ in want for b in sst]
    assert len(got["sst_blk"]) - 1 == len(want)
    assert b"".join(blocks) == got["blocks"].tobytes()
    np.testing.assert_array_equal(np.diff(got["blk_off"].astype(np.int64)), [len(b) for b in blocks])
    np.testing.assert_array_equal(np.diff(got["sst_blk"].astype(np.int64)), [len(s) for s, _ in want])
    np.testing.assert_array_equal(np.diff(got["sst_ent"].astype(np.int64)), [len(e) for _, e in want])
    ents = kv.entries()
    assert [ents[src[j]] for j in got["kept"]] == [e for _, es in want for e in es]
    return got


@pytest.mark.parametrize("seed", range(10))
def test_c_compact_equals_line_by_line_restatement(seed):
    rng = np.random.default_rng(50 + seed)
    runs = random_runs(rng, int(rng.integers(1, 6)), 80, max_versions=4)
    for wm, bottom, pf, bs, target in ((0, False, (), 64, 200), (500, True, (), 128, 300),
                                       (500, False, (b"a",), 96, 1), (10**6, True, (b"ab", b"c"), 4096, 1 << 20)):
        check_c_compact(runs, wm, bottom, pf, bs, target)


def test_c_compact_rotation_on_synthetic_runs():
    """Multi-SST output: SST boundaries only at key changes, once the data section reaches the
    target (every SST of unique keys ends with a one-entry block); against the restatement."""
    keys, ko, vals, vo, ts, rs = synth.gen_runs(3000, nrun=4, seed=3, versions=2)
    kv = O.KV(keys, ko, vals, vo, ts)
    runs = [kv.entries()[rs[r]:rs[r + 1]] for r in range(4)]
    got = check_c_compact(runs, int(ts.max()) // 2, True, (), 4096, 64 << 10)
    assert len(got["sst_blk"]) > 5


def test_rotation_closed_form_on_kept_stream():
    """The GPU cuts SSTs on the KEPT stream: a boundary at kept entry e iff the open SST's data
    section (blocks + 4-B CRCs) >= target and key(e) != key(e-1).  orc_segment_like_compaction
    states that form; it must give compact_generate_sst's boundaries."""
    for seed in range(6):
        keys, ko, vals, vo, ts, rs = synth.gen_runs(2000, nrun=5, seed=10 + seed, versions=1 + seed % 3,
                                                    tombstone=0.1)
        kv = O.KV(keys, ko, vals, vo, ts)
        src = O.merge_runs(kv, rs)
        for wm, bottom, target in ((0, False, 16 << 10), (int(ts.max()) // 2, True, 8 << 10), (1 << 62, True, 3000)):
            got = O.compact(kv, src, wm, bottom, (), 4096, target)
            kept = O.gather(kv, src[got["kept"]])
            seg = O.segment_like_compaction(kept, 4096, target)
            np.testing.assert_array_equal(seg, got["sst_ent"])


def test_compaction_golden_fixtures_c_oracle():
    """tests/golden/compact_runs_*.npz (made by oracle/gen_golden.py from the line-by-line
    restatement) replayed through the C oracle."""
    import json
    import os
    g = os.path.join(os.path.dirname(__file__), "golden")
    meta = json.load(open(os.path.join(g, "golden_compaction.json")))
    for name, m in meta.items():
        z = np.load(os.path.join(g, name + ".npz"))
        kv = O.KV(z["keys"], z["key_off"], z["vals"], z["val_off"], z["ts"])
        src = O.merge_runs(kv, z["run_start"])
        got = O.compact(kv, src, m["watermark"], m["bottom_level"], [p.encode() for p in m["prefixes"]],
                        m["block_size"], m["target_sst_size"])
        np.testing.assert_array_equal(got["blocks"], z["blocks"])
        np.testing.assert_array_equal(got["blk_off"], z["blk_off"])
        np.testing.assert_array_equal(got["sst_blk"], z["sst_blk"])
        np.testing.assert_array_equal(got["sst_ent"], z["sst_ent"])
        assert len(got["sst_blk"]) - 1 == m["ssts"]
