"""Generate tests/golden/ fixtures from the restatement (test infrastructure only).

No reference-produced vectors exist (the Rust reference cannot be built here); these pin
our restatement against regressions and give the GPU tests fixed inputs.  Also copies the
reference's lsm.db/MANIFEST (a data file its tests hold) for the CRC-32 pin.
Run:  python oracle/gen_golden.py
"""
import json
import os
import shutil
import sys
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:] = [p for p in sys.path if os.path.abspath(p or ".") != os.path.dirname(os.path.abspath(__file__))]
sys.path.insert(0, ROOT)
from lsm_amd import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


def cases():
    kat = [(b"key_%03d" % (i * 5), 0, b"value_%010d" % i) for i in range(100)]
    yield "kat_week1_day3", O.KV.from_entries(kat), [0, 100], 10000
    yield "kat_week1_day7_bs128", O.KV.from_entries(kat), [0, 100], 128
    mv = [(b"key%05d" % (i // 5), 5 - (i % 5), b"value%05d" % i) for i in range(100)]
    yield "week3_day1_bs128", O.KV.from_entries(mv), [0, 100], 128
    kv = O.KV(*synth.gen_uniform(10000, seed=0))
    yield "plumbing_U_10k", kv, [0, kv.n], 4096
    kv = O.KV(*synth.gen_zipf(3000, seed=1))
    yield "zipf_3k", kv, synth.segments_by_bytes(kv.key_off, kv.val_off, 64 << 10), 4096
    kv = O.KV(*synth.gen_mixed(600, seed=2))
    yield "mixed_600_bs64k", kv, [0, kv.n], 65536
    rng = np.random.default_rng(3)
    keys = sorted({bytes(rng.integers(0, 256, int(rng.integers(1, 5)), dtype=np.uint8)) for _ in range(3000)})
    ents = [(k, int(rng.integers(0, 1 << 40)), b"" if i % 3 else b"v") for i, k in enumerate(keys)]
    yield "tiny_entries_tombstones", O.KV.from_entries(ents), [0, len(ents)], 4096
    ents = [(b"a", 1, b"x" * 10), (b"b", 2, bytes(range(256)) * 273 + b"yz"), (b"c", 3, b"z" * 5000), (b"d", 4, b"w")]
    yield "u16_wrap_oversize", O.KV.from_entries(ents), [0, 4], 4096


def compaction_cases():
    """Merge + compaction vectors from the line-by-line restatement (oracle/pyref.py:
    MergeIterator, compact_generate_sst): runs, options, and every SST's blocks."""
    from oracle import pyref
    rng = np.random.default_rng(11)
    space = sorted({b"k%04d" % int(rng.integers(0, 900)) + bytes(rng.integers(97, 100, int(rng.integers(0, 3)),
                                                                              dtype=np.uint8))
                    for _ in range(700)})
    runs = []
    for r in range(5):
        take = sorted(rng.choice(len(space), size=int(rng.integers(100, len(space))), replace=False))
        run = []
        for i in take:
            for t in sorted(rng.choice(1000, size=int(rng.integers(1, 4)), replace=False), reverse=True):
                run.append((space[i], int(t) + 1000 * (5 - r), b"" if rng.random() < 0.15 else b"r%d-%d" % (r, t)))
        runs.append(run)
    for name, wm, bottom, pf, bs, target in (("compact_runs_bottom", 3500, True, (b"k00",), 256, 3000),
                                              ("compact_runs_upper", 2500, False, (), 512, 6000)):
        ssts = pyref.compact_generate_sst(pyref.MergeIterator([pyref.ListIter(x) for x in runs]), wm, bottom, pf,
                                          bs, target)
        yield name, runs, dict(watermark=wm, bottom_level=bottom, prefixes=[p.decode() for p in pf],
                               block_size=bs, target_sst_size=target), ssts


def main():
    os.makedirs(OUT, exist_ok=True)
    meta = {}
    for name, kv, seg, bs in cases():
        seg = np.asarray(seg, np.uint32)
        rc, blocks, off = O.encode_segments(kv, seg, bs)
        assert rc == 0, (name, rc)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), keys=kv.keys, key_off=kv.key_off, vals=kv.vals,
                            val_off=kv.val_off, ts=kv.ts, seg_start=seg, blocks=blocks, blk_off=off)
        meta[name] = {"block_size": bs, "entries": int(kv.n), "blocks": int(len(off) - 1),
                      "bytes": int(len(blocks)), "crc32": zlib.crc32(blocks.tobytes())}
    with open(os.path.join(OUT, "golden.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    cmeta = {}
    for name, runs, opts, ssts in compaction_cases():
        kv = O.KV.from_entries([e for r in runs for e in r])
        rs = np.concatenate([[0], np.cumsum([len(r) for r in runs])]).astype(np.uint32)
        blocks = [b for sst, _ in ssts for b in sst]
        blk_off = np.concatenate([[0], np.cumsum([len(b) for b in blocks])]).astype(np.uint64)
        sst_blk = np.concatenate([[0], np.cumsum([len(s) for s, _ in ssts])]).astype(np.uint32)
        sst_ent = np.concatenate([[0], np.cumsum([len(e) for _, e in ssts])]).astype(np.uint32)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), keys=kv.keys, key_off=kv.key_off, vals=kv.vals,
                            val_off=kv.val_off, ts=kv.ts, run_start=rs,
                            blocks=np.frombuffer(b"".join(blocks), np.uint8), blk_off=blk_off, sst_blk=sst_blk,
                            sst_ent=sst_ent)
        cmeta[name] = dict(opts, ssts=len(ssts), blocks=len(blocks), entries=int(kv.n))
    with open(os.path.join(OUT, "golden_compaction.json"), "w") as f:
        json.dump(cmeta, f, indent=1, sort_keys=True)
    src = "/root/reference/lsm.db/MANIFEST"
    if os.path.exists(src):
        shutil.copyfile(src, os.path.join(OUT, "lsm_db_MANIFEST.bin"))
    print(json.dumps(meta, indent=1))


if __name__ == "__main__":
    main()
