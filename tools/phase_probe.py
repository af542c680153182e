"""GPU-box probe for per-phase PMC counts: runs encode (or decode) of the U workload a few
times with one ablation mask (lsmblk_debug_set key 1) so that a rocprofv3 --pmc pass sees
dispatches of a single configuration.

usage: python3 tools/phase_probe.py {encode|decode} MASK [entries]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# the ablation masks exist only in the diagnostics build
os.environ.setdefault("LSMBLK_SO_OVERRIDE", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                         "lsm_amd", "liblsmblk_diag.so"))

import torch  # noqa: E402

from lsm_amd import batch, synth  # noqa: E402
from lsm_amd._lib import check, lib  # noqa: E402


def main():
    which, mask = sys.argv[1], int(sys.argv[2])
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 8 << 20
    keys, key_off, vals, val_off, ts = synth.gen_uniform(n)
    kv = batch.KVStream.from_numpy(keys, key_off, vals, val_off, ts, device="cuda")
    seg = synth.segments_by_bytes(key_off, val_off)
    blocks, blk_off = batch.encode_kv(kv, seg, synth.BLOCK_SIZE["U"])
    ctx = batch._ctx(0)
    check(lib().lsmblk_debug_set(ctx, 1, mask))
    check(lib().lsmblk_debug_set(ctx, 3, int(os.environ.get("PROBE_TWO_PASS", "0"))))  # two-pass decode (A/B)
    if os.environ.get("PROBE_LAG"):
        check(lib().lsmblk_debug_set(ctx, 4, int(os.environ["PROBE_LAG"])))
    for _ in range(3):
        if which == "encode":
            batch.encode_kv(kv, seg, synth.BLOCK_SIZE["U"])
        else:
            batch.decode_blocks(blocks, blk_off)
    torch.cuda.synchronize()
    check(lib().lsmblk_debug_set(ctx, 1, 0))
    print(which, mask, "blocks", blk_off.numel() - 1)


if __name__ == "__main__":
    main()
