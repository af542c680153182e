import sys, numpy as np, torch
sys.path.insert(0, '.')
from lsm_amd import batch
from oracle import oracle as O
kv = O.KV.from_entries([(b"key_%03d" % (i * 5), 0, b"value_%010d" % i) for i in range(100)])
rc, ref_blocks, ref_off = O.encode_segments(kv, [0, kv.n], 4096)
print("ref", ref_off)
d = batch.KVStream.from_numpy(kv.keys, kv.key_off, kv.vals, kv.val_off, kv.ts)
seg = torch.tensor([0, kv.n], dtype=torch.int32, device="cuda")
out_cap, blk_cap = batch.encode_bound(d, int(kv.key_off[-1]), int(kv.val_off[-1]))
out = batch._aligned_empty(out_cap, torch.device("cuda"))
blk_off = torch.zeros(blk_cap, dtype=torch.int64, device="cuda")
stats = torch.zeros(batch.STATS_WORDS, dtype=torch.int64, device="cuda")
batch.encode_into(d, seg, 1, 4096, out, out_cap, blk_off, blk_cap, stats)
torch.cuda.synchronize()
print("stats", stats.cpu().tolist(), "blk_off", blk_off[:4].cpu().tolist())
