"""Reference-shaped block API over liblsmblk.so's per-entry half.

Mirrors CrystalAnalyst/Lsm (paths relative to the reference repository):
  KeySlice / KeyVec   src/key.rs:15-213      (ordering and equality ignore the ts, :63-81)
  BlockBuilder        src/block/builder.rs:8-89
  Block               src/block.rs:7-34
  BlockIterator       src/block/iterator.rs:11-139 (seek_to_offset corrected: the ts after
                      the key suffix is skipped and becomes the key's ts)

Where the reference panics (empty key, empty build, malformed decode) these raise
LsmBlkError / AssertionError instead.
"""
import ctypes
import functools

from ._lib import LSMBLK_E_INVAL, LsmBlkError, check, lib


@functools.total_ordering
class KeySlice:
    """Key<T>(bytes, ts): src/key.rs:15. Eq/Ord compare the bytes only (key.rs:63-81)."""

    __slots__ = ("_key", "_ts")

    def __init__(self, key: bytes, ts: int = 0):
        self._key = bytes(key)
        self._ts = int(ts)

    @classmethod
    def for_testing_from_slice_no_ts(cls, key: bytes):  # key.rs:95-97
        return cls(key, 0)

    @classmethod
    def for_testing_from_slice_with_ts(cls, key: bytes, ts: int):  # key.rs:91-93
        return cls(key, ts)

    def key_ref(self) -> bytes:
        return self._key

    for_testing_key_ref = key_ref

    def ts(self) -> int:
        return self._ts

    def key_len(self) -> int:  # key.rs:24-26
        return len(self._key)

    def raw_len(self) -> int:  # key.rs:29-31
        return len(self._key) + 8

    def is_empty(self) -> bool:
        return not self._key

    def __eq__(self, other):
        return self._key == other._key

    def __lt__(self, other):
        return self._key < other._key

    def __hash__(self):
        return hash(self._key)

    def __repr__(self):
        return f"KeySlice({self._key!r}, ts={self._ts})"


KeyVec = KeySlice


class Block:
    """Block { data, offsets } (src/block.rs:7-10); reference counted like Arc<Block>."""

    def __init__(self, handle):
        self._h = handle

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib().lsmblk_block_free(h)
            self._h = None

    @classmethod
    def decode(cls, data: bytes) -> "Block":  # block.rs:24-34
        h = ctypes.c_void_p()
        check(lib().lsmblk_block_decode(data, len(data), ctypes.byref(h)), "Block::decode")
        return cls(h.value)

    def encode(self) -> bytes:  # block.rs:14-22
        n = lib().lsmblk_block_encoded_len(self._h)
        buf = ctypes.create_string_buffer(n)
        ln = ctypes.c_size_t()
        check(lib().lsmblk_block_encode(self._h, buf, n, ctypes.byref(ln)), "Block::encode")
        return buf.raw[:ln.value]

    @property
    def data(self) -> bytes:
        p, n = ctypes.c_void_p(), ctypes.c_size_t()
        check(lib().lsmblk_block_data(self._h, ctypes.byref(p), ctypes.byref(n)))
        return ctypes.string_at(p.value, n.value) if n.value else b""

    @property
    def offsets(self):
        p, n = ctypes.c_void_p(), ctypes.c_size_t()
        check(lib().lsmblk_block_offsets(self._h, ctypes.byref(p), ctypes.byref(n)))
        if not n.value:
            return []
        return list((ctypes.c_uint16 * n.value).from_address(p.value))


class BlockBuilder:
    """src/block/builder.rs:8-89."""

    def __init__(self, block_size: int):  # :37-44
        self._h = lib().lsmblk_builder_new(block_size)
        if not self._h:
            raise MemoryError("lsmblk_builder_new")

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib().lsmblk_builder_free(h)
            self._h = None

    def add(self, key: KeySlice, value: bytes) -> bool:  # :54-73
        acc = ctypes.c_int()
        st = lib().lsmblk_builder_add(self._h, key.key_ref(), key.key_len(), key.ts(), bytes(value),
                                      len(value), ctypes.byref(acc))
        if st == LSMBLK_E_INVAL:
            raise AssertionError("key must not be empty")
        check(st, "BlockBuilder::add")
        return bool(acc.value)

    def is_empty(self) -> bool:  # :76-78
        return bool(lib().lsmblk_builder_is_empty(self._h))

    def estimated_size(self) -> int:  # :48-50
        return lib().lsmblk_builder_estimated_size(self._h)

    def build(self) -> Block:  # :81-89
        if self.is_empty():
            raise AssertionError("block should not be empty!")
        h = ctypes.c_void_p()
        check(lib().lsmblk_builder_build(self._h, ctypes.byref(h)), "BlockBuilder::build")
        return Block(h.value)

    def build_encoded(self) -> bytes:
        """build().encode() in one call (what SsTableBuilder::finish_block does)."""
        n = self.estimated_size()
        buf = ctypes.create_string_buffer(n)
        ln = ctypes.c_size_t()
        st = lib().lsmblk_builder_finish(self._h, buf, n, ctypes.byref(ln))
        if st == LSMBLK_E_INVAL:
            raise AssertionError("block should not be empty!")
        check(st)
        return buf.raw[:ln.value]


class BlockIterator:
    """src/block/iterator.rs:11-139 (corrected seek_to_offset)."""

    def __init__(self, handle, block):
        self._h = handle
        self._block = block  # keep the Python wrapper alive too

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib().lsmblk_iter_free(h)
            self._h = None

    @classmethod
    def create_and_seek_to_first(cls, block: Block) -> "BlockIterator":  # :66-70
        h = ctypes.c_void_p()
        check(lib().lsmblk_iter_create_and_seek_to_first(block._h, ctypes.byref(h)))
        return cls(h.value, block)

    @classmethod
    def create_and_seek_to_key(cls, block: Block, key: KeySlice) -> "BlockIterator":  # :73-77
        h = ctypes.c_void_p()
        check(lib().lsmblk_iter_create_and_seek_to_key(block._h, key.key_ref(), key.key_len(),
                                                        ctypes.byref(h)))
        return cls(h.value, block)

    def seek_to_first(self):  # :99-101
        check(lib().lsmblk_iter_seek_to_first(self._h))

    def seek_to_key(self, key: KeySlice):  # :80-94
        check(lib().lsmblk_iter_seek_to_key(self._h, key.key_ref(), key.key_len()))

    def next(self):  # :104-107
        check(lib().lsmblk_iter_next(self._h))

    def is_valid(self) -> bool:  # :59-61
        return bool(lib().lsmblk_iter_is_valid(self._h))

    def key(self) -> KeySlice:  # :51-53
        p, n, ts = ctypes.c_void_p(), ctypes.c_size_t(), ctypes.c_uint64()
        check(lib().lsmblk_iter_key(self._h, ctypes.byref(p), ctypes.byref(n), ctypes.byref(ts)))
        return KeySlice(ctypes.string_at(p.value, n.value) if n.value else b"", ts.value)

    def value(self) -> bytes:  # :55-57
        p, n = ctypes.c_void_p(), ctypes.c_size_t()
        check(lib().lsmblk_iter_value(self._h, ctypes.byref(p), ctypes.byref(n)))
        return ctypes.string_at(p.value, n.value) if n.value else b""


__all__ = ["KeySlice", "KeyVec", "Block", "BlockBuilder", "BlockIterator", "LsmBlkError"]
