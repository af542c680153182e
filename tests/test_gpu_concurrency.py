"""The concurrency contract of include/lsmblk.h (Missing #4): a context's calls
are serialised by its lock and its device work is ordered on the stream each call is given; work
that runs concurrently takes one context each -- the Python wrappers keep one per (device,
stream).  Here several host threads, each on its own HIP stream and so its own context, run
decode -> re-encode round trips (packed and per-segment slots), block CRCs and a compaction at
the same time, and threads sharing one stream share one context through its lock.  Every result
must equal the oracle's, computed on the host before the threads start.

Bar: bit-exact, as tests/test_gpu_parity.py."""
import threading
import zlib

import numpy as np
import pytest
import torch

from lsm_amd import batch, synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu

ROUNDS = 3


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")


def _case(name):
    """(kv, seg, block_size) of one round-trip workload, and the oracle's blocks / offsets / CRCs."""
    if name == "U":
        kv, bs, tgt = O.KV(*synth.gen_uniform(60000, seed=21)), 4096, 256 << 10
    elif name == "Z":
        kv, bs, tgt = O.KV(*synth.gen_zipf(60000, seed=22)), 4096, 256 << 10
    elif name == "M":
        kv, bs, tgt = O.KV(*synth.gen_mixed(8000, seed=23)), 65536, 2 << 20
    else:  # small blocks: many blocks per segment
        kv, bs, tgt = O.KV(*synth.gen_uniform(30000, seed=24, value_len=20)), 1024, 64 << 10
    seg = synth.segments_by_bytes(kv.key_off, kv.val_off, tgt)
    rc, blocks, off = O.encode_segments(kv, seg, bs)
    assert rc == 0
    crc = np.array([zlib.crc32(blocks[int(off[i]):int(off[i + 1])].tobytes()) for i in range(len(off) - 1)],
                   np.uint32)
    return dict(kv=kv, seg=np.asarray(seg, np.int64), bs=bs, blocks=blocks, off=off, crc=crc)


def _round_trips(c, stream, errors, tag):
    """ROUNDS x (decode the oracle's blocks, re-encode packed and as slots, CRC the packed blocks)
    on `stream`, all asynchronous; checks after each round's stream synchronize."""
    try:
        dev = torch.device("cuda", 0)
        kv = c["kv"]
        with torch.cuda.stream(stream):
            db = torch.from_numpy(np.ascontiguousarray(c["blocks"])).to(dev)
            do = torch.from_numpy(c["off"].view(np.int64).copy()).to(dev)
            nblk = len(c["off"]) - 1
            n, K, V = kv.n, int(kv.key_off[-1]), int(kv.val_off[-1])
            out_kv = batch.KVStream.empty(n, K, V, dev)
            seg_t = torch.from_numpy(c["seg"].astype(np.uint32).view(np.int32)).to(dev)
            nseg = len(c["seg"]) - 1
            cap, blk_cap = K + V + 18 * n + 16, n + 2
            out = batch._aligned_empty(cap, dev)
            off = torch.zeros(blk_cap, dtype=torch.int64, device=dev)
            sout = batch._aligned_empty(cap, dev)
            soff = torch.zeros(blk_cap, dtype=torch.int64, device=dev)
            so = torch.zeros(2 * nseg, dtype=torch.int64, device=dev)
            crc = torch.zeros(max(nblk, 1), dtype=torch.int32, device=dev)
            st = [torch.zeros(batch.STATS_WORDS, dtype=torch.int64, device=dev) for _ in range(4)]
        stream.synchronize()
        for r in range(ROUNDS):
            with torch.cuda.stream(stream):
                for s in st:
                    s.zero_()
                out.fill_(r)
                batch.decode_into(db, do, nblk, out_kv, st[0], n, K + 16, V + 16, stream=stream)
                out_kv.n = n
                batch.encode_into(out_kv, seg_t, nseg, c["bs"], out, cap, off, blk_cap, st[1], stream=stream)
                batch.encode_into(out_kv, seg_t, nseg, c["bs"], sout, cap, soff, blk_cap, st[2], stream=stream,
                                  seg_out=so)
                batch.crc32_into(out, off, nblk, crc, st[3], stream=stream)
            stream.synchronize()
            assert [batch._status(s) for s in st] == [0, 0, 0, 0], (tag, r)
            E = int(c["off"][-1])
            assert int(st[1][0].item()) == nblk and int(st[1][1].item()) == E, (tag, r)
            assert np.array_equal(off[:nblk + 1].cpu().numpy().view(np.uint64), c["off"]), (tag, r)
            assert np.array_equal(out[:E].cpu().numpy(), c["blocks"]), (tag, r)
            pb, po = batch.slots_to_packed(sout, soff[:nblk + 1], so)
            assert np.array_equal(pb.cpu().numpy(), c["blocks"]), (tag, r)
            assert np.array_equal(crc[:nblk].cpu().numpy().view(np.uint32), c["crc"]), (tag, r)
    except BaseException as e:  # reported by the main thread
        errors.append((tag, repr(e)))


def _compaction(stream, errors, tag):
    try:
        keys, ko, vals, vo, ts, rs = synth.gen_runs(40000, nrun=4, seed=25, versions=2, tombstone=0.03)
        kv = O.KV(keys, ko, vals, vo, ts)
        src = O.merge_runs(kv, rs)
        want = O.compact(kv, src, 0, False, (), 4096, 128 << 10)
        for r in range(ROUNDS):
            d = batch.KVStream.from_numpy(kv.keys, kv.key_off, kv.vals, kv.val_off, kv.ts)
            got = batch.compact_runs(d, rs, 0, False, (), 4096, 128 << 10, stream=stream)
            assert np.array_equal(got["blk_off"].cpu().numpy().view(np.uint64), want["blk_off"]), (tag, r)
            assert np.array_equal(got["blocks"].cpu().numpy(), want["blocks"]), (tag, r)
            assert np.array_equal(got["sst_start"].cpu().numpy().view(np.uint32), want["sst_ent"]), (tag, r)
    except BaseException as e:
        errors.append((tag, repr(e)))


def _run_threads(targets):
    errors = []
    start = threading.Barrier(len(targets))

    def wrap(fn, *args):
        def go():
            start.wait()
            fn(*args, errors)
        return go

    threads = [threading.Thread(target=wrap(fn, *args)) for fn, *args in targets]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=110)
    assert not any(t.is_alive() for t in threads), "a thread did not finish"
    assert not errors, errors


def test_threads_on_their_own_streams_match_the_oracle():
    """Four round-trip workloads (U, Z, M, 1 KiB blocks) and a compaction, five host threads,
    five streams, five contexts, all at once."""
    cases = {k: _case(k) for k in ("U", "Z", "M", "S")}
    streams = [torch.cuda.Stream() for _ in range(5)]
    targets = [(_round_trips, cases[k], streams[i], k) for i, k in enumerate(cases)]
    targets.append((_compaction, streams[4], "C"))
    _run_threads(targets)
    torch.cuda.synchronize()


def test_threads_sharing_one_stream_share_its_context():
    """Three host threads on ONE stream: one context, its lock serialising the calls, its
    workspace reused call after call on the same stream -- every result still the oracle's."""
    cases = [_case(k) for k in ("U", "S", "M")]
    s = torch.cuda.Stream()
    _run_threads([(_round_trips, c, s, f"shared{i}") for i, c in enumerate(cases)])
    torch.cuda.synchronize()
