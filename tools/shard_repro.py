"""GPU box, diagnostics: repeat the key-range compaction over ranges on distinct streams (the
scenario of tests/test_gpu_shard.py::test_ranges_on_distinct_streams_compact_dist_single_rank)
and report every iteration whose status is not OK, with each range's stats, carry and segment
table.  usage: python tools/shard_repro.py [iterations] [--concurrency-first] [--local]"""
import json
import os
import socket
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from lsm_amd import batch, shard  # noqa: E402
from lsm_amd._lib import LsmBlkError  # noqa: E402
import test_gpu_shard as T  # noqa: E402


def one(kv, rs, d, splitters, bs, target, local):
    opts = batch.compact_opts(0, False, block_size=bs, target_sst_size=target)
    shards = T._shards_on_own_streams(d, rs, opts, splitters)
    try:
        res = shard.compact_local(shards) if local else shard.compact_dist(shards)
    except LsmBlkError as e:
        info = []
        for s in shards:
            torch.cuda.synchronize()
            info.append(dict(m=s.m, h=s.h, est=s.estats.cpu().tolist(), cin=s.carry_in.cpu().tolist(),
                             cout=s.cout.cpu().tolist(), seg=s.seg[:8].cpu().tolist(),
                             mstats=s.mstats.cpu().tolist()))
        s = shards[0]
        torch.cuda.synchronize()
        again = {}
        with torch.cuda.stream(s.stream):
            z = torch.zeros(2, dtype=torch.int64, device="cuda")
            again["carry_same_state"] = s.carry(z).clone().cpu().tolist()
            s.prepare()
            again["carry_after_prepare"] = s.carry(z).clone().cpu().tolist()
        torch.cuda.synchronize()
        again.update(n=s.ext.n, m=s.m, h=s.h, last=s.last, sst_cap=s.sst_cap,
                     ko_tail=s.ext.key_off[s.m - 2:s.m + 3].cpu().tolist())
        return dict(ok=False, err=str(e), shards=info[:1], again=again)
    try:
        T.check_against_single_stream(kv, rs, res, 0, False, bs, target)
    except AssertionError as e:
        return dict(ok=False, err="mismatch " + str(e)[:300])
    return dict(ok=True)


def probe(kv, rs, d, splitters, bs, target):
    """The dist driver's phases by hand, with shard 0's carry taken right after its own prepare and
    again after every range's prepare: a difference means its rotation state changed in between."""
    opts = batch.compact_opts(0, False, block_size=bs, target_sst_size=target)
    shards = T._shards_on_own_streams(d, rs, opts, splitters)
    for s in shards:
        s.merge()
    heads = [s.head() for s in shards]
    out = {}
    z = torch.zeros(2, dtype=torch.int64, device="cuda")
    for g, s in enumerate(shards):
        h = shard.assemble_halo(heads, g, s.W)
        s.set_halo(*h[:6], ks=h[6])
        s.prepare()
        torch.cuda.synchronize()
        with torch.cuda.stream(shards[0].stream):
            out.setdefault("c0", []).append(shards[0].carry(z).clone().cpu().tolist())
        torch.cuda.synchronize()
    return out


def patch(mode):
    """Bisect the hazard: a device sync before or after every prepare()."""
    orig = shard.RangeShard.prepare

    def prep(self):
        if mode == "before":
            torch.cuda.synchronize()
        orig(self)
        if mode == "after":
            torch.cuda.synchronize()
    shard.RangeShard.prepare = prep


def main():
    it = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 20
    local = "--local" in sys.argv
    for m in ("before", "after"):
        if "--sync-" + m in sys.argv:
            patch(m)
    if "--concurrency-first" in sys.argv:
        import test_gpu_concurrency as TC
        TC.test_threads_on_their_own_streams_match_the_oracle()
        TC.test_threads_sharing_one_stream_share_its_context()
        print("concurrency tests done", flush=True)
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=0, world_size=1)
    fails = 0
    try:
        rng = np.random.default_rng(22)
        kv, rs = T.case(78, versions=3, nkeys=6000)
        d = T.to_dev(kv)
        splitters = T.pick_splitters(kv, rng, 3)
        if "--probe" in sys.argv:
            for i in range(it):
                print(i, json.dumps(probe(kv, rs, d, splitters, 4096, 24 << 10)), flush=True)
            return
        for i in range(it):
            r = one(kv, rs, d, splitters, 4096, 24 << 10, local)
            if not r["ok"]:
                fails += 1
                print(i, json.dumps(r), flush=True)
            elif i % 5 == 0:
                print(i, "ok", flush=True)
    finally:
        dist.destroy_process_group()
    print(json.dumps(dict(iterations=it, fails=fails, local=local, argv=sys.argv[1:])), flush=True)


if __name__ == "__main__":
    main()
