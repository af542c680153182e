import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch, time
from lsm_amd import batch, synth
from oracle import oracle as O
for n in (20000, 100000, 400000):
    kv = O.KV(*synth.gen_uniform(n, seed=21))
    seg = synth.segments_by_bytes(kv.key_off, kv.val_off, 2 << 20)
    d = batch.KVStream.from_numpy(kv.keys, kv.key_off, kv.vals, kv.val_off, kv.ts)
    blocks, blk_off = batch.encode_kv(d, seg, 4096)
    print("n", n, "blocks", blk_off.numel() - 1, flush=True)
    t = time.time()
    try:
        dkv = batch.decode_blocks(blocks, blk_off)
        print("ok", dkv.n, time.time() - t, flush=True)
    except Exception as e:
        print("ERR", e, time.time() - t, flush=True)
