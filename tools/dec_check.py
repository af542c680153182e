"""GPU box: decode (and encode) a small batch of each config with the library named by
LSMBLK_SO_OVERRIDE (or the in-tree one) and compare with the oracle; prints the first mismatch.
usage: python3 tools/dec_check.py [n_entries]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from lsm_amd import batch, synth  # noqa: E402
from oracle import oracle as O  # noqa: E402


def first_bad(name, g, w):
    if len(g) != len(w):
        return f"{name}: len {len(g)} != {len(w)}"
    bad = np.flatnonzero(g != w)
    return f"{name}: {bad.size} bad, first {bad[:6].tolist()}" if bad.size else None


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 60000
    for cfg in ("U", "Z", "M"):
        kv = O.KV(*synth.GENERATORS[cfg](n if cfg != "M" else n // 8, seed=3))
        seg = synth.segments_by_bytes(kv.key_off, kv.val_off, 256 << 10)
        rc, ref_blocks, ref_off = O.encode_segments(kv, seg, synth.BLOCK_SIZE[cfg])
        rc2, ref_kv = O.decode_blocks(ref_blocks, ref_off)
        assert rc == 0 and rc2 == 0
        buf = torch.from_numpy(ref_blocks).cuda()
        off = torch.from_numpy(np.ascontiguousarray(ref_off, np.uint64).view(np.int64)).cuda()
        d = batch.decode_blocks(buf, off)
        torch.cuda.synchronize()
        keys, ko, vals, vo, ts = d.to_numpy()
        errs = [e for e in (first_bad("key_off", ko, ref_kv.key_off), first_bad("val_off", vo, ref_kv.val_off),
                            first_bad("ts", ts, ref_kv.ts), first_bad("keys", keys, ref_kv.keys[:ref_kv.key_off[-1]]),
                            first_bad("vals", vals, ref_kv.vals[:ref_kv.val_off[-1]])) if e]
        print(cfg, "decode", "ok" if not errs else errs, flush=True)
        blocks, blk_off = batch.encode_kv(batch.KVStream.from_numpy(kv.keys, kv.key_off, kv.vals, kv.val_off, kv.ts), seg, synth.BLOCK_SIZE[cfg])
        torch.cuda.synchronize()
        e = first_bad("blk_off", blk_off.cpu().numpy().view(np.uint64), ref_off) or \
            first_bad("blocks", blocks.cpu().numpy(), ref_blocks)
        print(cfg, "encode", "ok" if not e else e, flush=True)


if __name__ == "__main__":
    main()
