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
