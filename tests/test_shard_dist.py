"""Key-range sharded compaction over torch.distributed (gloo, CPU, world 2 and 3): the product's
exchange driver shard.compact_dist -- splitter all-gather, head all-gather + halo assembly, carry
send/recv -- run with a CPU stand-in for the device stages (OracleShard: the C oracle's merge /
compact_generate_sst rules / resumed rotation / encode, test infrastructure only).  Bar: the ranks'
outputs concatenate to the single-stream compaction, SST boundaries included."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from lsm_amd import shard, synth

BS, TARGET = 1024, 12 << 10


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def global_input(seed=7):
    from oracle import oracle as O
    keys, ko, vals, vo, ts, rs = synth.gen_runs(3000, nrun=4, seed=seed, versions=2, tombstone=0.05)
    return O.KV(keys, ko, vals, vo, ts), rs


class OracleShard:
    """CPU stand-in for shard.RangeShard (same phase methods) over the C oracle."""

    def __init__(self, kv, rs, wm, bottom, lo, hi):
        from oracle import oracle as O
        self.O, self.dev, self.W = O, torch.device("cpu"), BS // 16 + 2
        src = O.merge_runs(kv, rs)
        kept = O.gather(kv, src[O.compact(kv, src, wm, bottom, (), BS, 1 << 62)["kept"]])
        keep = [i for i in range(kept.n) if (lo is None or kept.entry(i)[0] >= lo) and
                (hi is None or kept.entry(i)[0] < hi)]
        self.kept = O.gather(kept, np.array(keep, np.int64))

    def merge(self):
        self.m = self.kept.n
        return self.m

    def head(self):
        h = min(self.W, self.m)
        k = self.kept
        t = (lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).astype(dt)))
        return shard.Head(self.m, t(k.key_off[:h + 1], np.int64), t(k.val_off[:h + 1], np.int64),
                          t(k.ts[:h].view(np.int64), np.int64), t(k.keys[:k.key_off[h]], np.uint8),
                          t(k.vals[:k.val_off[h]], np.uint8))

    def set_halo(self, keys, ko, vals, vo, ts, last, ks=None):
        O, k = self.O, self.kept
        self.ext = O.KV(np.concatenate([k.keys[:k.key_off[-1]], keys.numpy()]),
                        np.concatenate([k.key_off, ko.numpy()[1:] + k.key_off[-1]]).astype(np.uint32),
                        np.concatenate([k.vals[:k.val_off[-1]], vals.numpy()]),
                        np.concatenate([k.val_off, vo.numpy()[1:] + k.val_off[-1]]).astype(np.uint32),
                        np.concatenate([k.ts, ts.numpy().view(np.uint64)]))
        self.last = last

    def prepare(self):
        pass

    def carry(self, cin):
        self.cin = tuple(int(x) for x in cin.tolist())
        rc, self.seg, cout = self.O.shard_rotation(self.ext, self.m, self.last, *self.cin, BS, TARGET)
        assert rc == 0
        self.cout = cout
        return torch.tensor(cout, dtype=torch.int64)

    def encode(self):
        rc, self.blocks, _ = self.O.encode_span(self.ext, self.seg, BS)
        assert rc == 0

    def result(self):
        nseg = max(len(self.seg) - 1, 0)
        return dict(blocks=self.blocks.tobytes(), seg_start=self.seg, nseg=nseg, m=self.m,
                    first_continues=nseg > 0 and self.cin[1] > 0, carry_in=self.cin, carry_out=self.cout)


class OracleShard2(OracleShard):
    """OracleShard for a two-level (TwoMergeIterator) compaction: the range's slices of the runs,
    merged by pyref.two_merge_rule with the WHOLE compaction's b last key (which compact_dist
    all-gathers: a range's own slice of b ends earlier), the rules trace with the loop's own
    same_as_last_key, which travels with the head entries into the next rank's halo and drives the
    resumed rotation (orc_shard_rotation_ex)."""
    two = True

    def __init__(self, runs, wm, bottom, lo, hi):
        from oracle import oracle as O
        self.O, self.dev, self.W = O, torch.device("cpu"), BS // 16 + 2
        inr = (lambda k: (lo is None or k >= lo) and (hi is None or k < hi))
        self.runs = [[e for e in r if inr(e[0])] for r in runs]
        self.wm, self.bottom, self.kb = wm, bottom, Ellipsis

    def b_end(self):
        b = self.runs[-1]
        return b[-1][0] if b else None

    def set_b_end(self, kb):
        self.kb = kb

    def merge(self):
        from oracle import pyref
        assert self.kb is not Ellipsis, "compact_dist must set b's last key before the merge"
        tr = pyref.compact_rules_trace(pyref.two_merge_rule(self.runs, kb=self.kb), self.wm, self.bottom)
        self.kept = self.O.KV.from_entries([e for e, _ in tr])
        self.same = np.array([s for _, s in tr], np.uint8)
        self.m = len(tr)
        return self.m

    def head(self):
        hd = super().head()
        return shard.Head(hd.n, hd.ko, hd.vo, hd.ts, hd.keys, hd.vals, torch.from_numpy(self.same[:hd.h].copy()))

    def set_halo(self, keys, ko, vals, vo, ts, last, ks=None):
        super().set_halo(keys, ko, vals, vo, ts, last)
        self.ext_same = np.concatenate([self.same, ks.numpy().astype(np.uint8)])

    def carry(self, cin):
        self.cin = tuple(int(x) for x in cin.tolist())
        rc, self.seg, cout = self.O.shard_rotation(self.ext, self.m, self.last, *self.cin, BS, TARGET,
                                                   same=self.ext_same)
        assert rc == 0
        self.cout = cout
        return torch.tensor(cout, dtype=torch.int64)


def two_level_runs(seed=11):
    """Four runs, three versions per key, 15 % tombstones, b (the last run) cut 60 % of the way
    through the key space: upper keys past b's end are lost (TwoMergeIterator as written)."""
    from oracle import oracle as O
    keys, ko, vals, vo, ts, rs = synth.gen_runs(1200, nrun=4, seed=seed, versions=3, tombstone=0.15)
    ents = O.KV(keys, ko, vals, vo, ts).entries()
    runs = [ents[rs[r]:rs[r + 1]] for r in range(4)]
    runs[-1] = runs[-1][:int(len(runs[-1]) * 0.6)]
    return runs


def _worker2(rank, world, port, q, R):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        runs = two_level_runs()
        allk = sorted({e[0] for r in runs for e in r})
        b_last = runs[-1][-1][0]
        # splitters: the key after b's last (the last range lies wholly past b's end), b's last key
        # itself when there is room, the others spread below
        succ = allk[allk.index(b_last) + 1]
        fixed = {succ} | ({b_last} if world * R >= 3 else set())
        spread = [k for k in allk[:allk.index(b_last)][::max(1, len(allk) // (world * R))] if k not in fixed]
        splitters = sorted(fixed | set(spread[1:1 + world * R - 1 - len(fixed)]))
        assert len(splitters) == world * R - 1
        wm = max(e[1] for r in runs for e in r) // 2
        shards = [OracleShard2(runs, wm, True, *shard.range_of(rank * R + i, splitters)) for i in range(R)]
        outs = shard.compact_dist(shards if R > 1 else shards[0])
        outs = outs if R > 1 else [outs]
        for i, (s, res) in enumerate(zip(shards, outs)):
            assert s.kb == b_last  # the all-gathered b end, not the range's own slice's
            q.put((rank * R + i, res["blocks"], res["seg_start"].tolist(), res["nseg"], res["m"],
                   res["first_continues"], res["carry_in"], res["carry_out"], splitters))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(240)
@pytest.mark.parametrize("world,R", [(2, 1), (3, 1), (2, 2)])
def test_gloo_two_level_sharded_compaction_equals_single_stream(world, R):
    """LSMBLK_MERGE_TWO_LEVEL through compact_dist over gloo: b's last key
    all-gathered (_allgather_bytes), the heads' same_as_last_key bytes in the halo all-gather, the
    carry from rank to rank -- the ranks' blocks and SST starts equal compact_generate_sst over the
    reference's TwoMergeIterator restated line by line (oracle/pyref.py), bottom-level tombstones
    included."""
    from oracle import pyref
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker2, args=(r, world, port, q, R)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=200) for _ in range(world * R)), key=lambda x: x[0])
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    runs = two_level_runs()
    wm = max(e[1] for r in runs for e in r) // 2
    want = pyref.compact_generate_sst(pyref.two_merge_iter(runs), wm, True, (), BS, TARGET)
    assert b"".join(r[1] for r in res) == b"".join(blk for blocks, _ in want for blk in blocks)
    results = [dict(seg_start=np.array(r[2], np.uint32), nseg=r[3], first_continues=r[5]) for r in res]
    bases = np.concatenate([[0], np.cumsum([r[4] for r in res])]).tolist()
    assert shard.sst_starts(results, bases) == np.cumsum([0] + [len(e) for _, e in want])[:-1].tolist()
    for a, b in zip(res, res[1:]):
        assert a[7] == b[6]
    assert sum(r[4] == 0 for r in res) >= 1  # a range wholly past b's last key keeps nothing


def test_rules_trace_same_flags_drive_the_rotation():
    """pyref.compact_rules_trace + orc_shard_rotation_ex over the whole stream (one range) give
    compact_generate_sst's SST starts, and its same flags differ from plain key equality where a
    dropped bottom-level tombstone moved last_key (the reason two-level shards carry them)."""
    from oracle import oracle as O, pyref
    runs = two_level_runs()
    wm = max(e[1] for r in runs for e in r) // 2
    ents = pyref.drain(pyref.two_merge_iter(runs))
    tr = pyref.compact_rules_trace(ents, wm, True)
    kept = O.KV.from_entries([e for e, _ in tr])
    same = np.array([s for _, s in tr], np.uint8)
    rc, seg, cout = O.shard_rotation(kept, kept.n, True, 0, 0, BS, TARGET, same=same)
    assert rc == 0 and cout == (0, 0)
    want = pyref.compact_generate_sst(pyref.two_merge_iter(runs), wm, True, (), BS, TARGET)
    assert seg.tolist() == np.cumsum([0] + [len(e) for _, e in want]).tolist()
    adj = np.array([i > 0 and tr[i][0][0] == tr[i - 1][0][0] for i in range(len(tr))], np.uint8)
    assert (adj != same).any()


def _worker(rank, world, port, q, R=1):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        kv, rs = global_input()
        # every rank "holds" a slice of every run: sample the first keys of its slice's 32-entry blocks
        n = kv.n
        mine = [kv.entry(i)[0] for i in range(rank * n // world, (rank + 1) * n // world, 32)]
        splitters = shard.exchange_splitters(sorted(mine), samples=16, ranges=world * R)
        wm = int(kv.ts.max()) // 2
        if R == 1:
            lo, hi = shard.range_of(rank, splitters)
            outs = [shard.compact_dist(OracleShard(kv, rs, wm, True, lo, hi))]
        else:  # R ranges per rank: one list through compact_dist
            shards = [OracleShard(kv, rs, wm, True, *shard.range_of(rank * R + i, splitters)) for i in range(R)]
            outs = shard.compact_dist(shards)
        for i, res in enumerate(outs):
            q.put((rank * R + i, res["blocks"], res["seg_start"].tolist(), res["nseg"], res["m"],
                   res["first_continues"], res["carry_in"], res["carry_out"], splitters))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(240)
@pytest.mark.parametrize("world,R", [(2, 1), (3, 1), (2, 3)])
def test_gloo_sharded_compaction_equals_single_stream(world, R):
    from oracle import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, R)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=200) for _ in range(world * R)), key=lambda x: x[0])
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert all(r[8] == res[0][8] and len(r[8]) == world * R - 1 for r in res)
    kv, rs = global_input()
    src = O.merge_runs(kv, rs)
    want = O.compact(kv, src, int(kv.ts.max()) // 2, True, (), BS, TARGET)
    assert b"".join(r[1] for r in res) == want["blocks"].tobytes()
    results = [dict(seg_start=np.array(r[2], np.uint32), nseg=r[3], first_continues=r[5]) for r in res]
    bases = np.concatenate([[0], np.cumsum([r[4] for r in res])]).tolist()
    assert shard.sst_starts(results, bases) == want["sst_ent"][:-1].tolist()
    for a, b in zip(res, res[1:]):
        assert a[7] == b[6]
    assert any(r[5] for r in res)  # some SST crosses a rank boundary


def test_assemble_halo_spans_short_ranges():
    """A range shorter than the halo contributes all its entries and the next range continues;
    the entries' same_as_last_key bytes (two-level merges) travel with them."""
    def head(n, h, base):
        return shard.Head(n, torch.arange(h + 1, dtype=torch.int64) * 2, torch.arange(h + 1, dtype=torch.int64),
                          torch.arange(base, base + h, dtype=torch.int64),
                          torch.arange(2 * h, dtype=torch.uint8), torch.arange(h, dtype=torch.uint8),
                          (torch.arange(h, dtype=torch.uint8) + base // 100) % 2)
    heads = [head(100, 5, 0), head(2, 2, 100), head(0, 0, 200), head(50, 5, 300)]
    keys, ko, vals, vo, ts, last, ks = shard.assemble_halo(heads, 0, 5)
    assert ts.tolist() == [100, 101, 300, 301, 302] and not last
    assert ko.tolist() == [0, 2, 4, 6, 8, 10] and keys.numel() == 10 and vals.numel() == 5
    assert ks.tolist() == [1, 0, 1, 0, 1]
    keys, ko, vals, vo, ts, last, ks = shard.assemble_halo(heads, 1, 5)
    assert ts.tolist() == [300, 301, 302, 303, 304] and not last
    assert shard.assemble_halo(heads, 3, 5)[5] is True           # the last range
    heads[3] = head(3, 3, 300)
    assert shard.assemble_halo(heads, 0, 9)[4].tolist() == [100, 101, 300, 301, 302]
    assert shard.assemble_halo(heads, 0, 9)[5] is True           # the halo reached the stream's end


def test_two_end_mode():
    """Where b's last key lies relative to a range (two-level merges, include/lsmblk.h)."""
    from lsm_amd._lib import LSMBLK_TWO_END_ABOVE as A, LSMBLK_TWO_END_BELOW as B, LSMBLK_TWO_END_IN_RANGE as I
    assert shard.two_end_mode(None, None, None) == B                 # b empty everywhere
    assert shard.two_end_mode(b"m", None, None) == I
    assert shard.two_end_mode(b"m", b"a", b"m") == A                 # hi exclusive: kb above the range
    assert shard.two_end_mode(b"m", b"m", b"z") == I
    assert shard.two_end_mode(b"m", b"m\x00", None) == B
    assert shard.two_end_mode(b"m", None, b"c") == A
