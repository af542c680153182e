"""lsm_amd -- MI355X-native SSTable block encode/decode for the CrystalAnalyst/Lsm format.

  lsm_amd.block  reference-shaped per-entry API (BlockBuilder, Block, BlockIterator, KeySlice)
  lsm_amd.batch  device batch API (decode_blocks, encode_kv) over the HIP kernels
  lsm_amd.synth  synthetic KV streams (U / Z / M configs)

Everything executes in liblsmblk.so (built by __graft_entry__.build()).
"""
from ._lib import LsmBlkError, lib  # noqa: F401
from .block import Block, BlockBuilder, BlockIterator, KeySlice, KeyVec  # noqa: F401

__all__ = ["Block", "BlockBuilder", "BlockIterator", "KeySlice", "KeyVec", "LsmBlkError", "lib"]
