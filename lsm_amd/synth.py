"""Synthetic KV streams for the bench / tests (BASELINE.json configs).

All keys are sorted and unique (as a memtable flush or compaction feeds SsTableBuilder),
ts are 40-bit random, values random bytes, seeds fixed.

  U  uniform     16-B keys, 100-B values                       (block_size 4096)
  Z  zipf        16-B key = one of 1024 random 12-B prefixes (Zipf s=1.1) || 4-B BE counter
  M  mixed       16-B keys, values log-uniform in [8, 4096]    (block_size 65536)
"""
import numpy as np


def _offsets(lengths):
    off = np.zeros(len(lengths) + 1, np.uint64)
    np.cumsum(lengths, out=off[1:])
    if off[-1] >= 2 ** 32:
        raise ValueError("arena exceeds the u32 offsets of one batch")
    return off.astype(np.uint32)


def _random_bytes(rng, n):
    return np.frombuffer(rng.bytes(int(n)), np.uint8).copy() if n else np.zeros(0, np.uint8)


def _sorted_keys16(rng, n, key_slice=(0, 1)):
    """n sorted unique 16-B keys spread uniformly over the 128-bit space, or over slice s of w
    equal slices of it (key_slice = (s, w): a storage shard of a key-range-partitioned dataset),
    or over `span` consecutive slices from s (key_slice = (s, w, span))."""
    s, w = key_slice[:2]
    span = key_slice[2] if len(key_slice) > 2 else 1
    width = (2 ** 64 - 1) // w
    step = np.uint64(width * span // max(n, 1))
    hi = np.uint64(s * width) + np.arange(n, dtype=np.uint64) * step + rng.integers(0, int(step), n, dtype=np.uint64)
    lo = rng.integers(0, 2 ** 63, n, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, n, dtype=np.uint64)
    k = np.empty((n, 16), np.uint8)
    k[:, :8] = hi.astype(">u8").view(np.uint8).reshape(n, 8)
    k[:, 8:] = lo.astype(">u8").view(np.uint8).reshape(n, 8)
    return k.reshape(-1)


def _ts(rng, n):
    return rng.integers(0, 2 ** 40, n, dtype=np.uint64)


def gen_uniform(n, seed=42, key_len=16, value_len=100):
    rng = np.random.default_rng(seed)
    assert key_len == 16
    keys = _sorted_keys16(rng, n)
    vals = _random_bytes(rng, n * value_len)
    return (keys, _offsets(np.full(n, key_len, np.uint64)), vals,
            _offsets(np.full(n, value_len, np.uint64)), _ts(rng, n))


def gen_zipf(n, seed=43, nprefix=1024, s=1.1, value_len=100):
    rng = np.random.default_rng(seed)
    prefixes = np.frombuffer(rng.bytes(12 * nprefix), np.uint8).reshape(nprefix, 12)
    order = np.lexsort(prefixes.T[::-1])          # sort prefixes bytewise
    prefixes = prefixes[order]
    w = 1.0 / np.arange(1, nprefix + 1) ** s
    popularity = rng.permutation(nprefix)          # which sorted prefix gets which Zipf rank
    p = w[popularity]
    p /= p.sum()
    counts = rng.multinomial(n, p)
    if counts.max() >= 2 ** 32:
        raise ValueError("counter overflow")
    pidx = np.repeat(np.arange(nprefix), counts)
    starts = np.repeat(np.cumsum(counts) - counts, counts)
    ctr = (np.arange(n) - starts).astype(np.uint32)
    keys = np.empty((n, 16), np.uint8)
    keys[:, :12] = prefixes[pidx]
    keys[:, 12:] = ctr.astype(">u4").view(np.uint8).reshape(n, 4)
    vals = _random_bytes(rng, n * value_len)
    return (keys.reshape(-1), _offsets(np.full(n, 16, np.uint64)), vals,
            _offsets(np.full(n, value_len, np.uint64)), _ts(rng, n))


def gen_mixed(n, seed=44, vmin=8, vmax=4096):
    rng = np.random.default_rng(seed)
    keys = _sorted_keys16(rng, n)
    vl = np.exp(rng.uniform(np.log(vmin), np.log(vmax + 1), n)).astype(np.uint64)
    vl = np.clip(vl, vmin, vmax)
    vals = _random_bytes(rng, int(vl.sum()))
    return keys, _offsets(np.full(n, 16, np.uint64)), vals, _offsets(vl), _ts(rng, n)


def gen_runs(n_keys, nrun=8, overwrite=0.10, tombstone=0.02, seed=45, value_len=100, versions=1, key_slice=(0, 1)):
    """Compaction-shaped input (SURVEY.md section 8(d) config 5 at one-GPU scale): `nrun` sorted
    runs (L0 SSTs, run 0 the newest) over one key space with overlapping ranges.  Every key has
    a home run; a fraction `overwrite` also appears in a second run.  A run holds `versions`
    versions per key it contains (newest first, as SsTableBuilder receives them); ts are larger
    in newer runs; `tombstone` of the values are empty (deletes).  Returns (keys, key_off, vals,
    val_off, ts, run_start) with the runs concatenated in priority order.  key_slice: keys from
    one slice of the key space only (see _sorted_keys16)."""
    rng = np.random.default_rng(seed)
    base = _sorted_keys16(rng, n_keys, key_slice).reshape(n_keys, 16)
    home = rng.integers(0, nrun, n_keys)
    extra = rng.random(n_keys) < overwrite
    second = (home + rng.integers(1, max(nrun, 2), n_keys)) % max(nrun, 1)
    idx, run = [np.arange(n_keys)], [home]
    if nrun > 1 and extra.any():
        idx.append(np.flatnonzero(extra))
        run.append(second[extra])
    idx, run = np.concatenate(idx), np.concatenate(run)
    order = np.lexsort((idx, run))            # by run, then key
    idx, run = idx[order], run[order]
    # ts: run r's versions lie in band (nrun - r); inside a key, versions newest first
    ts = ((np.uint64(nrun) - run.astype(np.uint64)) << np.uint64(32)) + \
        (rng.integers(0, 1 << 24, len(idx), dtype=np.uint64) << np.uint64(4))
    if versions > 1:
        idx, run, ts = np.repeat(idx, versions), np.repeat(run, versions), np.repeat(ts, versions)
        ts += np.tile(np.arange(versions, dtype=np.uint64)[::-1], len(ts) // versions)
    n = len(idx)
    keys = base[idx].reshape(-1)
    vlen = np.where(rng.random(n) < tombstone, 0, value_len).astype(np.uint64)
    vals = _random_bytes(rng, int(vlen.sum()))
    run_start = np.searchsorted(run, np.arange(nrun + 1)).astype(np.uint32)
    return keys, _offsets(np.full(n, 16, np.uint64)), vals, _offsets(vlen), ts, run_start


GENERATORS = {"U": gen_uniform, "Z": gen_zipf, "M": gen_mixed}
BLOCK_SIZE = {"U": 4096, "Z": 4096, "M": 65536}


def segments_by_bytes(key_off, val_off, target=2 << 20):
    """Segment (SST) starts: a new segment each time the running encoded-size estimate
    (klen + vlen + 16 per entry) crosses a multiple of `target` bytes."""
    n = len(key_off) - 1
    if n == 0:
        return np.zeros(1, np.uint32)
    sz = (np.diff(key_off.astype(np.int64)) + np.diff(val_off.astype(np.int64)) + 16)
    seg_id = (np.cumsum(sz) - sz) // target
    starts = np.flatnonzero(np.diff(seg_id)) + 1
    return np.concatenate([[0], starts, [n]]).astype(np.uint32)
