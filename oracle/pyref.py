"""Pure-Python restatement of the reference block codec -- TEST INFRASTRUCTURE ONLY.

An independent second restatement (written separately from lsmblk_oracle.c) used to
cross-check the C oracle on small inputs.  Only tests/ may import it.

Follows /root/reference:
  BlockBuilder           src/block/builder.rs:19-89
  Block.encode / decode  src/block.rs:14-34
  BlockIterator          src/block/iterator.rs:23-139 (seek_to_offset corrected: the 8-byte
                         ts after the key suffix is skipped and becomes the key's ts)
  SsTableBuilder.add     src/table/builder.rs:48-65 (finish_block on rejection)
"""
import struct

U16 = struct.Struct(">H")
U64 = struct.Struct(">Q")


def common_prefix(first_key: bytes, key: bytes) -> int:
    """builder.rs:19-33 -- LCP against the block's first key (ts ignored)."""
    i = 0
    while i < len(first_key) and i < len(key) and first_key[i] == key[i]:
        i += 1
    return i


class BlockBuilder:
    """builder.rs:8-89."""

    def __init__(self, block_size: int):
        self.data = bytearray()
        self.offsets = []
        self.first_key = b""
        self.block_size = block_size

    def estimated_size(self) -> int:  # builder.rs:48-50
        return len(self.data) + 2 * len(self.offsets) + 2

    def is_empty(self) -> bool:  # builder.rs:76-78
        return not self.offsets

    def add(self, key: bytes, ts: int, value: bytes) -> bool:  # builder.rs:54-73
        assert len(key) > 0, "key must not be empty"
        add_on = len(key) + 8 + len(value) + 6
        if self.estimated_size() + add_on > self.block_size and not self.is_empty():
            return False
        self.offsets.append(len(self.data) & 0xFFFF)
        p = common_prefix(self.first_key, key)
        self.data += U16.pack(p & 0xFFFF)
        self.data += U16.pack((len(key) - p) & 0xFFFF)
        self.data += key[p:]
        self.data += U64.pack(ts)
        self.data += U16.pack(len(value) & 0xFFFF)
        self.data += value
        if not self.first_key:
            self.first_key = bytes(key)
        return True

    def build_encoded(self) -> bytes:  # build (:81-89) + Block::encode (block.rs:14-22)
        assert not self.is_empty(), "block should not be empty!"
        out = bytes(self.data)
        out += b"".join(U16.pack(o) for o in self.offsets)
        out += U16.pack(len(self.offsets) & 0xFFFF)
        return out


def block_decode(buf: bytes):
    """Block::decode, block.rs:24-34 -> (data, offsets)."""
    n = U16.unpack_from(buf, len(buf) - 2)[0]
    data_end = len(buf) - 2 - 2 * n
    offsets = [U16.unpack_from(buf, data_end + 2 * i)[0] for i in range(n)]
    return bytes(buf[:data_end]), offsets


def block_entries(buf: bytes):
    """Corrected BlockIterator walk: list of (key, ts, value)."""
    data, offsets = block_decode(buf)
    if not offsets:
        return []
    fk_len = U16.unpack_from(data, 2)[0]  # get_first_key, iterator.rs:23-34
    first_key = data[4:4 + fk_len]
    out = []
    for off in offsets:  # seek_to_offset, iterator.rs:125-139 (corrected)
        p, s = U16.unpack_from(data, off)[0], U16.unpack_from(data, off + 2)[0]
        key = first_key[:p] + data[off + 4:off + 4 + s]
        ts = U64.unpack_from(data, off + 4 + s)[0]
        vlen = U16.unpack_from(data, off + 12 + s)[0]
        out.append((key, ts, data[off + 14 + s:off + 14 + s + vlen]))
    return out


def encode_segments(entries, seg_start, block_size):
    """SsTableBuilder-style greedy packing of each segment -> list of encoded blocks."""
    blocks = []
    for g in range(len(seg_start) - 1):
        b = BlockBuilder(block_size)
        for key, ts, value in entries[seg_start[g]:seg_start[g + 1]]:
            if not b.add(key, ts, value):  # table/builder.rs:55-62
                blocks.append(b.build_encoded())
                b = BlockBuilder(block_size)
                assert b.add(key, ts, value)
        if not b.is_empty():
            blocks.append(b.build_encoded())
    return blocks


def sst_block_metas(entries, block_size):
    """SsTableBuilder::add / finish_block (table/builder.rs:48-65, 112-123) for ONE SST ->
    [(offset, first_key, last_key)] per block.  offset = data.len() before the block, where the
    data section holds every block followed by its u32 CRC (:118-122).  first_key / last_key are
    set with KeyVec::set_from_slice (key.rs:166-169), which copies the key bytes only: the
    BlockMeta keys keep ts 0."""
    metas, data_len = [], 0
    b, first, last = BlockBuilder(block_size), b"", b""
    for key, ts, value in entries:
        if not first:  # :49-51
            first = key
        if b.add(key, ts, value):  # :55-58
            last = key
            continue
        blk = b.build_encoded()  # finish_block, :112-123
        metas.append((data_len, first, last))
        data_len += len(blk) + 4
        b = BlockBuilder(block_size)
        assert b.add(key, ts, value)  # :62-64
        first = last = key
    if not b.is_empty():  # build() -> finish_block (:73)
        metas.append((data_len, first, last))
    return metas


def encode_block_meta(metas, max_ts=0) -> bytes:
    """BlockMeta::encode_block_meta (table.rs:29-63): u32 num | {u32 offset | u16 len | first
    key | u64 ts | u16 len | last key | u64 ts}* | u64 max_ts | u32 crc32 of everything after
    num (`buf[original_len + 4..]`).  Key ts are 0 (see sst_block_metas); SsTableBuilder never
    raises max_ts from 0 (table/builder.rs:41, 77)."""
    import zlib
    body = bytearray()
    for off, fk, lk in metas:
        body += struct.pack(">I", off & 0xFFFFFFFF)
        body += U16.pack(len(fk) & 0xFFFF) + fk + U64.pack(0)
        body += U16.pack(len(lk) & 0xFFFF) + lk + U64.pack(0)
    body += U64.pack(max_ts)
    return struct.pack(">I", len(metas) & 0xFFFFFFFF) + bytes(body) + struct.pack(">I", zlib.crc32(body))


def decode_block_meta(buf: bytes):
    """BlockMeta::decode_block_meta (table.rs:65-93) -> ([(offset, first_key, last_key)], max_ts);
    raises ValueError on the reference's "meta checksum mismatched"."""
    import zlib
    num = struct.unpack_from(">I", buf, 0)[0]
    checksum = zlib.crc32(buf[4:len(buf) - 4])
    pos, metas = 4, []
    for _ in range(num):
        off = struct.unpack_from(">I", buf, pos)[0]
        fl = U16.unpack_from(buf, pos + 4)[0]
        fk = bytes(buf[pos + 6:pos + 6 + fl])
        pos += 6 + fl + 8
        ll = U16.unpack_from(buf, pos)[0]
        lk = bytes(buf[pos + 2:pos + 2 + ll])
        pos += 2 + ll + 8
        metas.append((off, fk, lk))
    max_ts = U64.unpack_from(buf, pos)[0]
    if struct.unpack_from(">I", buf, pos + 8)[0] != checksum:
        raise ValueError("meta checksum mismatched")
    return metas, max_ts


def compact_filter_loop(entries, watermark, bottom_level, prefixes=()):
    """compact_generate_sst (src/compact.rs:223-311), the per-entry loop restated line by line
    over a merged stream [(key, ts, value)] (keys ascending, versions newest first); returns
    the entries handed to SsTableBuilder::add (:292).  SST rotation (:278-289) is left out:
    it does not change which entries are kept."""
    out, last_key, first_key_below_watermark = [], b"", False
    have_last = False
    for key, ts, value in entries:
        same_as_last_key = have_last and key == last_key  # :239
        if not same_as_last_key:
            first_key_below_watermark = True  # :240-242
        if bottom_level and not same_as_last_key and ts <= watermark and len(value) == 0:  # :244-254
            last_key, have_last = key, True
            first_key_below_watermark = False
            continue
        if ts <= watermark:  # :256-276
            if same_as_last_key and not first_key_below_watermark:
                continue
            first_key_below_watermark = False
            if any(key.startswith(p) for p in prefixes):
                continue
        out.append((key, ts, value))  # :292
        if not same_as_last_key:
            last_key, have_last = key, True
    return out


class ListIter:
    """StorageIterator over a list of (key, ts, value) -- the role SsTableIterator / MockIterator
    play for MergeIterator (src/iterators.rs:5-23, src/tests/harness.rs:18-84).  key() returns the
    user key only: Key's Eq / Ord ignore the ts (src/key.rs:63-81)."""

    def __init__(self, entries):
        self.e, self.i = list(entries), 0

    def is_valid(self):
        return self.i < len(self.e)

    def key(self):
        return self.e[self.i][0]

    def entry(self):
        return self.e[self.i]

    def next(self):
        self.i += 1


class MergeIterator:
    """src/iterators/merge_iterator.rs:59-184, line by line.  The BinaryHeap of HeapWrapper(idx,
    iter) is a max-heap under the REVERSED (key, idx) order (:21-33), i.e. a min-heap on
    (user key, idx): heapq with (key, idx) tuples pops the same element (idx are distinct)."""

    def __init__(self, iters):
        import heapq
        self._hq = heapq
        self.iters = {}
        self.heap = []
        self.current = None
        if not iters:  # :73-78
            return
        if all(not it.is_valid() for it in iters):  # :84-90
            self.current = (0, iters[-1])
            return
        for idx, it in enumerate(iters):  # :93-97
            if it.is_valid():
                self.iters[idx] = it
                heapq.heappush(self.heap, (it.key(), idx))
        _, idx = heapq.heappop(self.heap)  # :100
        self.current = (idx, self.iters.pop(idx))

    def is_valid(self):  # :123-128
        return self.current is not None and self.current[1].is_valid()

    def entry(self):
        return self.current[1].entry()

    def next(self):  # :130-169
        hq = self._hq
        cidx, cur = self.current
        while self.heap:  # peek_mut
            key, idx = self.heap[0]
            if key == cur.key():  # :139, ts-agnostic Eq
                it = self.iters[idx]
                it.next()
                hq.heappop(self.heap)
                if it.is_valid():  # PeekMut drop re-sifts the advanced iterator
                    hq.heappush(self.heap, (it.key(), idx))
                else:  # :146-148
                    del self.iters[idx]
            else:
                break
        cur.next()  # :154
        if not cur.is_valid():  # :156-161
            if self.heap:
                _, idx = hq.heappop(self.heap)
                self.current = (idx, self.iters.pop(idx))
            return
        if self.heap:  # :163-167: swap when current's (key, idx) is greater than the top's
            key, idx = self.heap[0]
            if (cur.key(), cidx) > (key, idx):
                hq.heappop(self.heap)
                top = self.iters.pop(idx)
                self.iters[cidx] = cur
                hq.heappush(self.heap, (cur.key(), cidx))
                self.current = (idx, top)


class TwoMergeIterator:
    """src/iterators/two_merge_iterator.rs:5-98, line by line, quirks included: skip_b advances b
    ONCE per equal key (:45-50), choose_a is false as soon as b is invalid (:32-42), so the
    merged stream ends with b."""

    def __init__(self, a, b):
        self.a, self.b = a, b
        self._skip_b()
        self.choose_a = self._choose_a()

    def _choose_a(self):
        if not self.a.is_valid() or not self.b.is_valid():
            return False
        return self.a.entry()[0] < self.b.entry()[0]

    def _skip_b(self):
        if self.a.is_valid() and self.b.is_valid() and self.b.entry()[0] == self.a.entry()[0]:
            self.b.next()

    def is_valid(self):
        return self.a.is_valid() if self.choose_a else self.b.is_valid()

    def entry(self):
        return self.a.entry() if self.choose_a else self.b.entry()

    def next(self):
        (self.a if self.choose_a else self.b).next()
        self._skip_b()
        self.choose_a = self._choose_a()


def drain(it):
    out = []
    while it.is_valid():
        out.append(it.entry())
        it.next()
    return out


def merge_runs(runs):
    """MergeIterator over sorted runs (run 0 = highest priority, e.g. the newest L0 SST)."""
    return drain(MergeIterator([ListIter(r) for r in runs]))


def two_merge_iter(runs):
    """The iterator compact() hands to compact_generate_sst (src/compact.rs:170-173, 206-215):
    TwoMergeIterator(MergeIterator(runs[:-1]), runs[-1] as the lower level's SstConcatIterator)."""
    return TwoMergeIterator(MergeIterator([ListIter(r) for r in runs[:-1]]), ListIter(runs[-1]))


def two_merge_runs(runs):
    return drain(two_merge_iter(runs))


def two_merge_rule(runs, kb=Ellipsis):
    """The closed form the GPU evaluates for LSMBLK_MERGE_TWO_LEVEL (lsmblk_compact.hip), b =
    runs[-1]: nothing past b's last key kb (and nothing at all for an empty b); a key of the upper
    runs only: its lowest-index upper run's versions (below kb); a key of b only: all of b's
    versions; a key of both: b's 2nd, 4th, ... versions, then (below kb) the upper run's.
    kb given (a key range of a sharded compaction, whose runs are the range's slices): the whole
    compaction's b last key, None for an empty b."""
    upper, b = runs[:-1], runs[-1]
    if kb is Ellipsis:
        kb = b[-1][0] if b else None
    if kb is None:
        return []
    owner, av, bv = {}, {}, {}
    for r, run in enumerate(upper):
        for e in run:
            if owner.setdefault(e[0], r) == r:
                av.setdefault(e[0], []).append(e)
    for e in b:
        bv.setdefault(e[0], []).append(e)
    out = []
    for k in sorted(set(av) | set(bv)):
        if k > kb:
            break
        if k in av:
            out += bv.get(k, [])[1::2]
            if k < kb:
                out += av[k]
        else:
            out += bv[k]
    return out


def merge_runs_rule(runs):
    """The closed form the GPU merge evaluates: for every user key, all the versions held by the
    lowest-index run containing that key, in that run's order; keys ascending."""
    owner = {}
    for r, run in enumerate(runs):
        for k, _, _ in run:
            owner.setdefault(k, r)
    out = []
    for k in sorted(owner):
        out += [e for e in runs[owner[k]] if e[0] == k]
    return out


class SsTableBuilderRef:
    """SsTableBuilder (src/table/builder.rs:16-123) for one SST: blocks, the data section
    length estimate_size() (blocks + 4-B CRC each, :105-107, 112-123) and the entries added."""

    def __init__(self, block_size):
        self.block_size = block_size
        self.builder = BlockBuilder(block_size)
        self.blocks, self.data_len, self.entries = [], 0, []

    def add(self, key, ts, value):  # :48-65
        self.entries.append((key, ts, value))
        if self.builder.add(key, ts, value):
            return
        self.finish_block()
        assert self.builder.add(key, ts, value)

    def finish_block(self):  # :112-123
        blk = self.builder.build_encoded()
        self.builder = BlockBuilder(self.block_size)
        self.blocks.append(blk)
        self.data_len += len(blk) + 4

    def estimate_size(self):
        return self.data_len

    def build(self):  # :68-74 (the file layout after the data section is not modelled here)
        self.finish_block()
        return self.blocks, self.entries


def compact_generate_sst(it, watermark, bottom_level, prefixes, block_size, target_sst_size):
    """compact_generate_sst (src/compact.rs:223-311) line by line over a StorageIterator:
    the compaction rules AND the SST rotation (:278-289).  Returns [(blocks, entries)] per SST."""
    builder, new_sst = None, []
    last_key, first_key_below_watermark = b"", False
    while it.is_valid():  # :234
        if builder is None:  # :235-237
            builder = SsTableBuilderRef(block_size)
        key, ts, value = it.entry()
        same_as_last_key = key == last_key  # :239
        if not same_as_last_key:
            first_key_below_watermark = True
        if bottom_level and not same_as_last_key and ts <= watermark and len(value) == 0:  # :244-254
            last_key = key
            it.next()
            first_key_below_watermark = False
            continue
        if ts <= watermark:  # :256-276
            if same_as_last_key and not first_key_below_watermark:
                it.next()
                continue
            first_key_below_watermark = False
            if any(key.startswith(p) for p in prefixes):
                it.next()
                continue
        if builder.estimate_size() >= target_sst_size and not same_as_last_key:  # :278-289
            new_sst.append(builder.build())
            builder = SsTableBuilderRef(block_size)
        builder.add(key, ts, value)  # :291-292
        if not same_as_last_key:  # :294-297
            last_key = key
        it.next()
    if builder is not None:  # :301-309
        new_sst.append(builder.build())
    return new_sst


def compact_rules_trace(entries, watermark, bottom_level, prefixes=()):
    """The rules half of compact_generate_sst (src/compact.rs:239-297) over a merged entry list:
    [(entry, same_as_last_key)] for every entry handed to SsTableBuilder::add, with the loop's
    own same_as_last_key (a dropped bottom-level tombstone moves last_key, :244-254; a prefix-filter
    drop does not).  The rotation (:278-289) reads only those flags, so the rules and the rotation
    separate."""
    out, last_key, first_below = [], b"", False
    for key, ts, value in entries:
        same = key == last_key
        if not same:
            first_below = True
        if bottom_level and not same and ts <= watermark and len(value) == 0:
            last_key, first_below = key, False
            continue
        if ts <= watermark:
            if same and not first_below:
                continue
            first_below = False
            if any(key.startswith(p) for p in prefixes):
                continue
        out.append(((key, ts, value), same))
        if not same:
            last_key = key
    return out


def compact_filter_rule(entries, watermark, bottom_level, prefixes=()):
    """The closed form the GPU evaluates per entry (lsmblk_gpu.hip, filt_keep): an entry needs
    only itself and its predecessor."""
    out = []
    for i, (key, ts, value) in enumerate(entries):
        if ts > watermark:
            out.append((key, ts, value))
            continue
        start = i == 0 or entries[i - 1][0] != key
        if not start and entries[i - 1][1] <= watermark:
            continue
        if bottom_level and start and len(value) == 0:
            continue
        if any(key.startswith(p) for p in prefixes):
            continue
        out.append((key, ts, value))
    return out


# ---------------------------------------------------------------- SST container (row 3)
# farmhash 1.1.5 `fingerprint32` (the hash SsTableBuilder::add records, src/table/builder.rs:53)
# = farmhashmk::Hash32 of Google's published FarmHash, restated here.  farmhash is not
# importable in this image and the reference cannot run, so this function is PARITY UNPINNED
# beyond its own self-consistency; the bloom arithmetic around it is pinned by the reference's
# raw-integer unit test (src/table/bloom.rs:123-160).
_C1, _C2, _M32 = 0xCC9E2D51, 0x1B873593, 0xFFFFFFFF


def _rot32(v, s):  # Rotate32: a right rotation
    return ((v >> s) | (v << (32 - s))) & _M32 if s else v


def _fmix(h):
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & _M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & _M32
    h ^= h >> 16
    return h


def _mur(a, h):
    a = (a * _C1) & _M32
    a = _rot32(a, 17)
    a = (a * _C2) & _M32
    h ^= a
    h = _rot32(h, 19)
    return (h * 5 + 0xE6546B64) & _M32


def _f32(s, i):
    return int.from_bytes(s[i:i + 4], "little")


def fingerprint32(s: bytes) -> int:
    n = len(s)
    if n <= 4:
        b, c = 0, 9
        for x in s:
            v = x - 256 if x >= 128 else x  # signed char
            b = (b * _C1 + v) & _M32
            c ^= b
        return _fmix(_mur(b, _mur(n, c)))
    if n <= 12:
        a, b, c = n, n * 5, 9
        d = b
        a = (a + _f32(s, 0)) & _M32
        b = (b + _f32(s, n - 4)) & _M32
        c = (c + _f32(s, (n >> 1) & 4)) & _M32
        return _fmix(_mur(c, _mur(b, _mur(a, d))))
    if n <= 24:
        a = _f32(s, (n >> 1) - 4)
        b = _f32(s, 4)
        c = _f32(s, n - 8)
        d = _f32(s, n >> 1)
        e = _f32(s, 0)
        f = _f32(s, n - 4)
        h = (d * _C1 + n) & _M32
        a = (_rot32(a, 12) + f) & _M32
        h = (_mur(c, h) + a) & _M32
        a = (_rot32(a, 3) + c) & _M32
        h = (_mur(e, h) + a) & _M32
        a = (_rot32((a + f) & _M32, 12) + d) & _M32
        h = (_mur(b, h) + a) & _M32
        return _fmix(h)
    h, g = n & _M32, (_C1 * n) & _M32
    f = g

    def a_(off):
        return (_rot32((_f32(s, off) * _C1) & _M32, 17) * _C2) & _M32
    a0, a1, a2, a3, a4 = a_(n - 4), a_(n - 8), a_(n - 16), a_(n - 12), a_(n - 20)
    h ^= a0
    h = (_rot32(h, 19) * 5 + 0xE6546B64) & _M32
    h ^= a2
    h = (_rot32(h, 19) * 5 + 0xE6546B64) & _M32
    g ^= a1
    g = (_rot32(g, 19) * 5 + 0xE6546B64) & _M32
    g ^= a3
    g = (_rot32(g, 19) * 5 + 0xE6546B64) & _M32
    f = (f + a4) & _M32
    f = (_rot32(f, 19) + 113) & _M32
    iters, p = (n - 1) // 20, 0
    while True:
        a, b, c, d, e = (_f32(s, p + 4 * i) for i in range(5))
        h = (h + a) & _M32
        g = (g + b) & _M32
        f = (f + c) & _M32
        h = (_mur(d, h) + e) & _M32
        g = (_mur(c, g) + a) & _M32
        f = (_mur((b + e * _C1) & _M32, f) + d) & _M32
        f = (f + g) & _M32
        g = (g + f) & _M32
        p += 20
        iters -= 1
        if iters == 0:
            break
    g = (_rot32(g, 11) * _C1) & _M32
    g = (_rot32(g, 17) * _C1) & _M32
    f = (_rot32(f, 11) * _C1) & _M32
    f = (_rot32(f, 17) * _C1) & _M32
    h = _rot32((h + g) & _M32, 19)
    h = (h * 5 + 0xE6546B64) & _M32
    h = (_rot32(h, 17) * _C1) & _M32
    h = _rot32((h + f) & _M32, 19)
    h = (h * 5 + 0xE6546B64) & _M32
    h = (_rot32(h, 17) * _C1) & _M32
    return h


class Bloom:
    """src/table/bloom.rs:7-120, line by line."""

    def __init__(self, filt: bytes, k: int):
        self.filter, self.k = bytes(filt), k

    @staticmethod
    def bloom_bits_per_key(entries, false_positive_rate):  # :72-77 (f64 arithmetic)
        import math
        size = -1.0 * entries * math.log(false_positive_rate) / (math.log(2) * math.log(2))
        locs = math.ceil(size / entries) if entries else 0  # NaN `as usize` = 0
        return int(locs)

    @staticmethod
    def build_from_key_hashes(keys, bits_per_key):  # :80-101
        k = min(max(int(bits_per_key * 0.69), 1), 30)
        nbits = max(len(keys) * bits_per_key, 64)
        nbytes = (nbits + 7) // 8
        nbits = nbytes * 8
        filt = bytearray(nbytes)
        for h in keys:
            delta = ((h >> 17) | (h << 15)) & _M32
            for _ in range(k):
                bit = h % nbits
                filt[bit // 8] |= 1 << (bit % 8)
                h = (h + delta) & _M32
        return Bloom(filt, k)

    def encode(self) -> bytes:  # :63-69
        import zlib
        body = self.filter + bytes([self.k])
        return body + zlib.crc32(body).to_bytes(4, "big")

    @staticmethod
    def decode(buf: bytes):  # :49-60
        import zlib
        if int.from_bytes(buf[-4:], "big") != zlib.crc32(buf[:-4]):
            raise ValueError("checksum mismatched for bloom filters")
        return Bloom(buf[:-5], buf[-5])

    def may_contain(self, h: int) -> bool:  # :104-120
        if self.k > 30:
            return True
        nbits = len(self.filter) * 8
        delta = ((h >> 17) | (h << 15)) & _M32
        for _ in range(self.k):
            bit = h % nbits
            if not (self.filter[bit // 8] >> (bit % 8)) & 1:
                return False
            h = (h + delta) & _M32
        return True


def sst_file(entries, block_size) -> bytes:
    """SsTableBuilder::add* + build (src/table/builder.rs:48-98): the whole SST file --
    blocks each followed by its BE u32 crc32fast | BlockMeta section | u32 meta_offset |
    bloom (filter | k | crc) | u32 bloom_offset."""
    import zlib
    blocks = encode_segments(entries, [0, len(entries)], block_size)
    data = b"".join(b + zlib.crc32(b).to_bytes(4, "big") for b in blocks)
    meta = encode_block_meta(sst_block_metas(entries, block_size))
    buf = data + meta + len(data).to_bytes(4, "big")
    hashes = [fingerprint32(k) for k, _, _ in entries]
    bloom = Bloom.build_from_key_hashes(hashes, Bloom.bloom_bits_per_key(len(hashes), 0.01))
    return buf + bloom.encode() + len(buf).to_bytes(4, "big")


def sst_open(buf: bytes):
    """SsTable::open (src/table.rs:162-186): footer offsets, bloom (CRC checked), BlockMeta
    (CRC checked) -> (metas, max_ts, bloom, meta_offset)."""
    n = len(buf)
    bloom_offset = int.from_bytes(buf[n - 4:], "big")
    bloom = Bloom.decode(buf[bloom_offset:n - 4])
    meta_offset = int.from_bytes(buf[bloom_offset - 4:bloom_offset], "big")
    metas, max_ts = decode_block_meta(buf[meta_offset:bloom_offset - 4])
    return metas, max_ts, bloom, meta_offset


def memtable_flush(puts):
    """MemTable::put + flush (src/mem_table.rs:113-136): a crossbeam SkipMap keyed by KeyBytes
    whose Ord ignores the ts (src/key.rs:63-81), so a later put of a key replaces the entry (key
    ts and value); flush yields the map in key order."""
    m = {}
    for key, ts, value in puts:
        m[bytes(key)] = (bytes(key), ts, bytes(value))
    return [m[k] for k in sorted(m)]
