import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from lsm_amd import batch
from lsm_amd._lib import lib
from oracle import oracle as O
kv = O.KV.from_entries([(b"key_%03d" % (i * 5), 0, b"value_%010d" % i) for i in range(100)])
rc, blocks, off = O.encode_segments(kv, [0, 100], 10000)
db = torch.from_numpy(blocks).cuda(); do = torch.from_numpy(off.view(np.int64)).cuda()
print("blocks", db.shape, db.data_ptr() % 16, do.cpu().tolist())
cap = 1000
out = batch.KVStream(torch.zeros(4096, dtype=torch.uint8, device="cuda"), torch.full((cap+1,), -1, dtype=torch.int32, device="cuda"),
                     torch.zeros(4096, dtype=torch.uint8, device="cuda"), torch.full((cap+1,), -1, dtype=torch.int32, device="cuda"),
                     torch.zeros(cap, dtype=torch.int64, device="cuda"), 0)
stats = torch.full((4,), -7, dtype=torch.int64, device="cuda")
batch.decode_into(db, do, 1, out, stats, cap, 4096, 4096)
torch.cuda.synchronize()
print("stats", stats.cpu().tolist())
print("key_off", out.key_off[:8].cpu().tolist(), "ts", out.ts[:4].cpu().tolist())
print("keys", bytes(out.keys[:40].cpu().numpy()))
