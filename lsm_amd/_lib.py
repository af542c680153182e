"""ctypes binding of liblsmblk.so (include/lsmblk.h).

The library is built in-tree by lsm_amd/_build.py (``__graft_entry__.build()``).  There is
no fallback: if the library is missing or fails to load, every call raises.
"""
import ctypes
import os

from . import _build

_lib = None

P, S, U32, U64, I = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
PP = ctypes.POINTER(ctypes.c_void_p)

LSMBLK_OK = 0
LSMBLK_E_INVAL = -1
LSMBLK_E_MALFORMED = -2
LSMBLK_E_CAPACITY = -3
LSMBLK_E_NOMEM = -4
LSMBLK_E_HIP = -5
LSMBLK_E_TIMEOUT = -6
LSMBLK_E_OVERFLOW = -7
LSMBLK_E_INTERNAL = -8
LSMBLK_E_CHECKSUM = -9
LSMBLK_DECODE_VERIFY_CRC = 1
LSMBLK_ENCODE_SEG_SLOTS = 1
LSMBLK_ENCODE_FRAMED = 2
LSMBLK_DEBUG_ENCODE_FUSED = 8
LSMBLK_SHARD_LAST = 1
LSMBLK_MERGE_RUNS = 0
LSMBLK_MERGE_TWO_LEVEL = 1
LSMBLK_TWO_END_IN_RANGE = 0
LSMBLK_TWO_END_ABOVE = 1
LSMBLK_TWO_END_BELOW = 2


class LsmBlkError(RuntimeError):
    def __init__(self, status, what=""):
        self.status = status
        msg = lib().lsmblk_strerror(status).decode() if _lib is not None else str(status)
        super().__init__(f"{what}: {msg} ({status})" if what else f"{msg} ({status})")


class KVStreamC(ctypes.Structure):
    _fields_ = [("keys", P), ("key_off", P), ("vals", P), ("val_off", P), ("ts", P),
                ("n", U64), ("entry_cap", U64), ("key_cap", U64), ("val_cap", U64)]


class CompactOptsC(ctypes.Structure):
    _fields_ = [("watermark", U64), ("bottom_level", ctypes.c_int32), ("nprefix", U32), ("prefixes", P),
                ("prefix_off", P), ("block_size", U32), ("merge_mode", U32), ("target_sst_size", U64)]


class KernelStatC(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 56), ("launches", U32), ("ms", ctypes.c_float)]


class KeyRangeC(ctypes.Structure):
    _fields_ = [("lo", P), ("hi", P), ("lo_len", U32), ("hi_len", U32), ("has_lo", U32), ("has_hi", U32)]


# (name, restype, argtypes) for every symbol of include/lsmblk.h
SIGNATURES = [
    ("lsmblk_abi_version", I, []),
    ("lsmblk_strerror", ctypes.c_char_p, [I]),
    ("lsmblk_stats_status", I, [U64]),
    ("lsmblk_builder_new", P, [S]),
    ("lsmblk_builder_free", None, [P]),
    ("lsmblk_builder_add", I, [P, P, S, U64, P, S, ctypes.POINTER(I)]),
    ("lsmblk_builder_is_empty", I, [P]),
    ("lsmblk_builder_estimated_size", S, [P]),
    ("lsmblk_builder_finish", I, [P, P, S, ctypes.POINTER(S)]),
    ("lsmblk_builder_build", I, [P, PP]),
    ("lsmblk_block_decode", I, [P, S, PP]),
    ("lsmblk_block_encode", I, [P, P, S, ctypes.POINTER(S)]),
    ("lsmblk_block_encoded_len", S, [P]),
    ("lsmblk_block_data", I, [P, PP, ctypes.POINTER(S)]),
    ("lsmblk_block_offsets", I, [P, PP, ctypes.POINTER(S)]),
    ("lsmblk_block_free", None, [P]),
    ("lsmblk_iter_create_and_seek_to_first", I, [P, PP]),
    ("lsmblk_iter_create_and_seek_to_key", I, [P, P, S, PP]),
    ("lsmblk_iter_seek_to_first", I, [P]),
    ("lsmblk_iter_seek_to_key", I, [P, P, S]),
    ("lsmblk_iter_next", I, [P]),
    ("lsmblk_iter_is_valid", I, [P]),
    ("lsmblk_iter_key", I, [P, PP, ctypes.POINTER(S), ctypes.POINTER(U64)]),
    ("lsmblk_iter_value", I, [P, PP, ctypes.POINTER(S)]),
    ("lsmblk_iter_free", None, [P]),
    ("lsmblk_ctx_create", I, [I, PP]),
    ("lsmblk_ctx_destroy", None, [P]),
    ("lsmblk_ctx_reserve", I, [P, U64, U64, U64]),
    ("lsmblk_debug_set", I, [P, I, U32]),
    ("lsmblk_ctx_kernel_times", I, [P, ctypes.POINTER(ctypes.c_float)]),
    ("lsmblk_ctx_kernel_log", I, [P, ctypes.POINTER(KernelStatC), U32, ctypes.POINTER(U32)]),
    ("lsmblk_debug_counters", I, [P, ctypes.POINTER(ctypes.c_uint64), U32]),
    ("lsmblk_decode_batch", I, [P, P, P, U64, ctypes.POINTER(KVStreamC), P, P]),
    ("lsmblk_decode_batch_ex", I, [P, P, P, U64, U32, U32, ctypes.POINTER(KVStreamC), P, P, P]),
    ("lsmblk_encode_batch", I, [P, ctypes.POINTER(KVStreamC), P, U32, U32, P, U64, P, U64, P, P]),
    ("lsmblk_encode_batch_ex", I, [P, ctypes.POINTER(KVStreamC), P, U32, U32, U32, P, U64, P, U64, P, P, P]),
    ("lsmblk_crc32_batch", I, [P, P, P, U64, U32, P, P, P]),
    ("lsmblk_encode_segment_blocks", I, [P, P, U32, P, P, P]),
    ("lsmblk_block_meta_batch", I, [P, P, P, U64, U32, P, U32, P, U64, P, P, P]),
    ("lsmblk_compact_filter_batch", I, [P, ctypes.POINTER(KVStreamC), U64, I, P, P, U32,
                                        ctypes.POINTER(KVStreamC), P, P]),
    ("lsmblk_merge_batch", I, [P, ctypes.POINTER(KVStreamC), P, U32, ctypes.POINTER(KVStreamC), P, P]),
    ("lsmblk_merge_batch_ex", I, [P, ctypes.POINTER(KVStreamC), P, U32, U32, ctypes.POINTER(KVStreamC), P, P]),
    ("lsmblk_sst_rotation_batch", I, [P, ctypes.POINTER(KVStreamC), U32, U64, P, U32, P, P]),
    ("lsmblk_compact_batch", I, [P, ctypes.POINTER(KVStreamC), P, U32, ctypes.POINTER(CompactOptsC),
                                 ctypes.POINTER(KVStreamC), P, U64, P, U64, P, P, U32, P, P]),
    ("lsmblk_shard_halo_entries", U64, [U32]),
    ("lsmblk_compact_merge_batch", I, [P, ctypes.POINTER(KVStreamC), P, U32, ctypes.POINTER(CompactOptsC),
                                       ctypes.POINTER(KeyRangeC), ctypes.POINTER(KVStreamC), P, P]),
    ("lsmblk_compact_merge_batch_ex", I, [P, ctypes.POINTER(KVStreamC), P, U32, ctypes.POINTER(CompactOptsC),
                                          ctypes.POINTER(KeyRangeC), U32, ctypes.POINTER(KVStreamC), P, P, P]),
    ("lsmblk_shard_rotation_prepare", I, [P, ctypes.POINTER(KVStreamC), U64, U32, U32, U64, U32, P]),
    ("lsmblk_shard_rotation_prepare_ex", I, [P, ctypes.POINTER(KVStreamC), P, U64, U32, U32, U64, U32, P]),
    ("lsmblk_shard_rotation_carry", I, [P, P, P, P]),
    ("lsmblk_shard_encode_batch", I, [P, ctypes.POINTER(KVStreamC), P, U64, P, U64, P, P, U32, P, P]),
    ("lsmblk_memtable_new", P, []),
    ("lsmblk_memtable_free", None, [P]),
    ("lsmblk_memtable_put", I, [P, P, S, U64, P, S]),
    ("lsmblk_memtable_get", I, [P, P, S, PP, ctypes.POINTER(S), ctypes.POINTER(U64)]),
    ("lsmblk_memtable_get_copy", I, [P, P, S, P, S, ctypes.POINTER(S), ctypes.POINTER(U64)]),
    ("lsmblk_memtable_len", S, [P]),
    ("lsmblk_memtable_approximate_size", S, [P]),
    ("lsmblk_memtable_flush", I, [P, P, P, P, P, P, U64, U64, U64, ctypes.POINTER(U64), ctypes.POINTER(U64),
                                  ctypes.POINTER(U64)]),
    ("lsmblk_sst_files_batch", I, [P, P, P, U64, P, P, U32, ctypes.POINTER(KVStreamC), P, U64, P, P, P]),
    ("lsmblk_seek_batch", I, [P, P, P, U64, U32, P, P, P, U64, P, P, P]),
    ("lsmblk_fingerprint32", U32, [P, S]),
    ("lsmblk_bloom_may_contain", I, [P, S, U32, U32]),
]


def lib():
    global _lib
    if _lib is None:
        so = os.environ.get("LSMBLK_SO_OVERRIDE", _build.SO)  # debug builds only
        if not os.path.exists(so):
            raise RuntimeError(f"liblsmblk.so not built ({so}); run __graft_entry__.build()")
        L = ctypes.CDLL(so)
        for name, res, args in SIGNATURES:
            if so != _build.SO and not hasattr(L, name):
                continue  # (an A/B build from an earlier revision: its missing symbols stay unbound)
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.lsmblk_abi_version() != 1:
            raise RuntimeError("liblsmblk.so ABI version mismatch")
        _lib = L
    return _lib


def kernel_log(ctx):
    """{kernel name: (launches, ms)} of every launch on ctx since the previous read (kernel timing on)."""
    buf = (KernelStatC * 256)()
    n = U32(0)
    check(lib().lsmblk_ctx_kernel_log(ctx, buf, 256, ctypes.byref(n)), "lsmblk_ctx_kernel_log")
    return {buf[i].name.decode(): (int(buf[i].launches), float(buf[i].ms)) for i in range(n.value)}


def check(status, what=""):
    if status != LSMBLK_OK:
        raise LsmBlkError(status, what)
    return status
