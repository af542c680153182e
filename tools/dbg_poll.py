import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from lsm_amd import batch, synth
mode = os.environ.get("LSMBLK_POLL_MODE")
for n in (400_000, 2_000_000):
    kv = synth.gen_uniform(n, seed=21)
    seg = synth.segments_by_bytes(kv[1], kv[3], 2 << 20)
    d = batch.KVStream.from_numpy(*kv)
    try:
        t = time.time(); blocks, blk_off = batch.encode_kv(d, seg, 4096); te = time.time() - t
        t = time.time(); dkv = batch.decode_blocks(blocks, blk_off); td = time.time() - t
        b2, o2 = batch.encode_kv(dkv, seg, 4096)
        ok = torch.equal(b2, blocks) and torch.equal(o2, blk_off) and dkv.n == n
        print(f"mode={mode} n={n} blocks={blk_off.numel()-1} enc={te:.3f}s dec={td:.3f}s roundtrip_ok={ok}", flush=True)
    except Exception as e:
        print(f"mode={mode} n={n} ERR {e}", flush=True)
