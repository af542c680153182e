"""The key-range sharded compaction with its real device stages AND its real exchange, more than one
rank (Missing #3 / What's weak #9): two processes, both on cuda:0, gloo as the
comm backend, real shard.RangeShard ranges (lsmblk_compact_merge_batch, lsmblk_shard_rotation_*,
lsmblk_shard_encode_batch) driven by shard.compact_dist -- splitter all-gather, b-end all-gather
(two-level), head all-gather + halo, the carry from rank to rank -- in both merge modes, one and two
ranges per rank.  That is the code the driver's multi-GPU compaction extra runs (bench.py --gpus N,
with RCCL instead of gloo).  Bar: the ranks' blocks concatenate to the single-stream compaction
(RUNS: the C oracle's merge + compact_generate_sst; TWO_LEVEL: compact_generate_sst over the
reference's TwoMergeIterator restated line by line, oracle/pyref.py), the SST cuts included, and
every rank's carry-out is the next rank's carry-in.

The ranks are child processes started with subprocess (fork + exec of a fresh interpreter); the
test process itself needs no GPU call for this test."""
import json
import os
import socket
import subprocess
import sys
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BS, TARGET = 1024, 12 << 10

RANK = r"""
import json, os, sys
import numpy as np
import torch
import torch.distributed as dist
sys.path.insert(0, %(root)r)
from lsm_amd import batch, shard
from lsm_amd._lib import LSMBLK_MERGE_RUNS, LSMBLK_MERGE_TWO_LEVEL
sys.path.insert(0, os.path.join(%(root)r, "tests"))
import test_gpu_shard_dist as T

rank, world, mode, R, outdir = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], int(sys.argv[4]), sys.argv[5]
dist.init_process_group("gloo", rank=rank, world_size=world)
try:
    kv, rs, runs, wm, bottom = T.workload(mode)
    d = batch.KVStream.from_numpy(kv.keys, kv.key_off, kv.vals, kv.val_off, kv.ts)
    # every rank samples the first keys of its own slice of the input (as from its SSTs' BlockMeta)
    n = kv.n
    mine = sorted(kv.entry(i)[0] for i in range(rank * n // world, (rank + 1) * n // world, 24))
    splitters = shard.exchange_splitters(mine, samples=16, ranges=world * R)
    mm = LSMBLK_MERGE_TWO_LEVEL if mode == "two" else LSMBLK_MERGE_RUNS
    opts = batch.compact_opts(wm, bottom, block_size=T.BS, target_sst_size=T.TARGET, merge_mode=mm)
    shards = [shard.RangeShard(d, rs, opts, *shard.range_of(rank * R + i, splitters)) for i in range(R)]
    outs = shard.compact_dist(shards)
    torch.cuda.synchronize()
    res = []
    for i, r in enumerate(outs):
        blocks = r["blocks"].cpu().numpy()
        np.save(os.path.join(outdir, "blocks_%%d.npy" %% (rank * R + i)), blocks)
        res.append(dict(g=rank * R + i, seg_start=[int(x) for x in r["seg_start"].tolist()], nseg=int(r["nseg"]),
                        m=int(r["m"]), first_continues=bool(r["first_continues"]),
                        carry_in=[int(x) for x in r["carry_in"]], carry_out=[int(x) for x in r["carry_out"]],
                        splitters=[s.hex() for s in splitters]))
    with open(os.path.join(outdir, "rank_%%d.json" %% rank), "w") as f:
        json.dump(res, f)
finally:
    dist.destroy_process_group()
"""


def workload(mode):
    """(KV of the concatenated runs, run_start, runs as entry lists, watermark, bottom level).
    Three versions per key and 10 % tombstones; in the two-level mode b (the last run) is cut 60 %
    of the way through the key space, so TwoMergeIterator's loss of upper keys past b's end is in
    the output as the reference binary writes it."""
    from lsm_amd import synth
    from oracle import oracle as O
    keys, ko, vals, vo, ts, rs = synth.gen_runs(4000, nrun=4, seed=41 if mode == "two" else 43, versions=3,
                                                tombstone=0.10)
    kv = O.KV(keys, ko, vals, vo, ts)
    ents = kv.entries()
    runs = [ents[rs[r]:rs[r + 1]] for r in range(len(rs) - 1)]
    if mode == "two":
        runs[-1] = runs[-1][:int(len(runs[-1]) * 0.6)]
        kv = O.KV.from_entries([e for r in runs for e in r])
        rs = np.cumsum([0] + [len(r) for r in runs]).astype(np.uint32)
    wm = int(max(e[1] for r in runs for e in r)) // 2
    return kv, np.asarray(rs, np.uint32), runs, wm, True


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_ranks(world, mode, R, outdir):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), PYTHONPATH=ROOT)
    script = RANK % {"root": ROOT}
    procs = [subprocess.Popen([sys.executable, "-c", script, str(r), str(world), mode, str(R), outdir], env=env,
                              cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for r in range(world)]
    logs = []
    try:
        for p in procs:
            out, err = p.communicate(timeout=150)
            logs.append((p.returncode, out[-2000:], err[-4000:]))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for rc, out, err in logs:
        assert rc == 0, out + err
    res = []
    for r in range(world):
        with open(os.path.join(outdir, "rank_%d.json" % r)) as f:
            res += json.load(f)
    res.sort(key=lambda x: x["g"])
    for x in res:
        x["blocks"] = np.load(os.path.join(outdir, "blocks_%d.npy" % x["g"])).tobytes()
    return res


@pytest.mark.timeout(240)
@pytest.mark.parametrize("mode,R", [("runs", 1), ("runs", 2), ("two", 1), ("two", 2)])
def test_two_ranks_on_one_gpu_equal_single_stream(mode, R):
    from lsm_amd import shard
    from oracle import oracle as O, pyref
    world = 2
    with tempfile.TemporaryDirectory() as outdir:
        res = _run_ranks(world, mode, R, outdir)
    assert len(res) == world * R
    assert all(r["splitters"] == res[0]["splitters"] and len(r["splitters"]) == world * R - 1 for r in res)
    kv, rs, runs, wm, bottom = workload(mode)
    if mode == "two":
        want = pyref.compact_generate_sst(pyref.two_merge_iter(runs), wm, bottom, (), BS, TARGET)
        want_blocks = b"".join(blk for blocks, _ in want for blk in blocks)
        want_starts = np.cumsum([0] + [len(e) for _, e in want])[:-1].tolist()
        want_n = sum(len(e) for _, e in want)
    else:
        src = O.merge_runs(kv, rs)
        w = O.compact(kv, src, wm, bottom, (), BS, TARGET)
        want_blocks = w["blocks"].tobytes()
        want_starts = w["sst_ent"][:-1].tolist()
        want_n = len(w["kept"])
    assert b"".join(r["blocks"] for r in res) == want_blocks
    bases = np.concatenate([[0], np.cumsum([r["m"] for r in res])]).tolist()
    assert bases[-1] == want_n
    results = [dict(seg_start=np.array(r["seg_start"], np.uint32), nseg=r["nseg"],
                    first_continues=r["first_continues"]) for r in res]
    assert shard.sst_starts(results, bases) == want_starts
    for a, b in zip(res, res[1:]):
        assert a["carry_out"] == b["carry_in"]
    assert res[0]["carry_in"] == [0, 0]
    assert any(r["first_continues"] for r in res)  # an SST crosses a range boundary
