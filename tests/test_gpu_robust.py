"""Failure containment on the device (the GPU-suite hang): every data-dependent
loop of the SST rotation is bounded by its own progress, so corrupt or stale block-chain levels end
the call with LSMBLK_E_INTERNAL instead of a kernel that never finishes.  The levels are corrupted
by the diagnostics library's fault injection (LSMBLK_DEBUG_ROT_POISON: links J(s) = s, S(s) = 0
over a third of the stream -- before the bound, rot_f_kernel's top-level loop spun on them
forever), in a child process so that the suite itself keeps the product library.  Then the same
context, poison off, gives the oracle's answer again."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys
import numpy as np
import torch
sys.path.insert(0, %(root)r)
from lsm_amd import batch, shard, synth
from lsm_amd._lib import lib, LsmBlkError
from oracle import oracle as O

POISON = 7  # LSMBLK_DEBUG_ROT_POISON
out = {}
keys, ko, vals, vo, ts, rs = synth.gen_runs(30000, nrun=3, seed=5, versions=2, tombstone=0.05)
kv = O.KV(keys, ko, vals, vo, ts)
kept = O.gather(kv, O.merge_runs(kv, rs))
d = batch.KVStream.from_numpy(kept.keys, kept.key_off, kept.vals, kept.val_off, kept.ts)
bs, target = 1024, 16 << 10
want = O.segment_like_compaction(kept, bs, target)

def status(fn):
    try:
        fn()
        return 0
    except LsmBlkError as e:
        return e.status

h = batch._ctx(0)
assert lib().lsmblk_debug_set(h, POISON, 1) == 0
out["rotation"] = status(lambda: batch.sst_rotation(d, bs, target))
dkv = batch.KVStream.from_numpy(kv.keys, kv.key_off, kv.vals, kv.val_off, kv.ts)
out["compact"] = status(lambda: batch.compact_runs(dkv, rs, 0, False, (), bs, target))
assert lib().lsmblk_debug_set(h, POISON, 0) == 0
out["rotation_after"] = bool(np.array_equal(batch.sst_rotation(d, bs, target), want))

# the key-range sharded path: one range over the whole stream, its own context poisoned
opts = batch.compact_opts(0, False, block_size=bs, target_sst_size=target)
s = shard.RangeShard(dkv, rs, opts)
assert lib().lsmblk_debug_set(s.ctx.h, POISON, 1) == 0
out["shard"] = status(lambda: shard.compact_local([s]))
torch.cuda.synchronize()
print(json.dumps(out))
"""


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")


def test_corrupt_rotation_levels_report_internal_not_hang():
    from lsm_amd import _build
    from lsm_amd._lib import LSMBLK_E_INTERNAL
    _build.build(diag=True)
    env = dict(os.environ, LSMBLK_SO_OVERRIDE=_build.DIAG_SO)
    r = subprocess.run([sys.executable, "-c", CHILD % {"root": ROOT}], env=env, cwd=ROOT, capture_output=True,
                       text=True, timeout=100)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["rotation"] == LSMBLK_E_INTERNAL, res
    assert res["compact"] == LSMBLK_E_INTERNAL, res
    assert res["shard"] == LSMBLK_E_INTERNAL, res
    assert res["rotation_after"], res


EMIT_CHILD = r"""
import json, sys
import numpy as np
import torch
sys.path.insert(0, %(root)r)
from lsm_amd import batch, synth
from lsm_amd._lib import lib, LsmBlkError
from oracle import oracle as O

POISON = 10  # LSMBLK_DEBUG_EMIT_POISON
out = {}
kv = O.KV(*synth.gen_uniform(60000, seed=21))
seg = [0, 20000, 40000, kv.n]
rc, ref_blocks, ref_off = O.encode_segments(kv, seg, 4096)
assert rc == 0
d = batch.KVStream.from_numpy(kv.keys, kv.key_off, kv.vals, kv.val_off, kv.ts)

def status(fn):
    try:
        fn()
        return 0
    except LsmBlkError as e:
        return e.status

h = batch._ctx(0)
assert lib().lsmblk_debug_set(h, POISON, 1) == 0
out["packed"] = status(lambda: batch.encode_kv(d, seg, 4096))
out["slots"] = status(lambda: batch.encode_kv_slots(d, seg, 4096))
assert lib().lsmblk_debug_set(h, POISON, 0) == 0
blocks, off = batch.encode_kv(d, seg, 4096)
out["packed_after"] = bool(np.array_equal(blocks.cpu().numpy(), ref_blocks) and
                           np.array_equal(off.cpu().numpy(), np.asarray(ref_off, np.int64)))
ob, oo, so = batch.encode_kv_slots(d, seg, 4096)
pb, po = batch.slots_to_packed(ob, oo, so)
out["slots_after"] = bool(np.array_equal(pb.cpu().numpy(), ref_blocks))
torch.cuda.synchronize()
print(json.dumps(out))
"""


def test_corrupt_block_table_refused_by_emit():
    """a block table whose end entry precedes its start (or lies past n) --
    what a raced or stale plan table looks like, and what sent the round-5 single-block emit
    experiment's emit_big walk into ~2^32 entries of unchecked loads -- is refused by emit_kernel
    and emit_big_kernel with LSMBLK_E_INTERNAL, none of its entries read.  The table is corrupted by
    the diagnostics library's LSMBLK_DEBUG_EMIT_POISON after the plan walk; then the same context
    encodes the oracle's bytes again, packed and with per-segment slots."""
    from lsm_amd import _build
    from lsm_amd._lib import LSMBLK_E_INTERNAL
    _build.build(diag=True)
    env = dict(os.environ, LSMBLK_SO_OVERRIDE=_build.DIAG_SO)
    r = subprocess.run([sys.executable, "-c", EMIT_CHILD % {"root": ROOT}], env=env, cwd=ROOT, capture_output=True,
                       text=True, timeout=100)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["packed"] == LSMBLK_E_INTERNAL, res
    assert res["slots"] == LSMBLK_E_INTERNAL, res
    assert res["packed_after"] and res["slots_after"], res
