/*
 * lsmblk_oracle.h -- CPU restatement of the CrystalAnalyst/Lsm SSTable block codec.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in lsm_amd/ links, loads or calls this code.
 * It may be used only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg, and there only as the checker / the timed CPU baseline -- never as the product.
 *
 * Parity pinning: see the header of lsmblk_oracle.c.
 */
#ifndef LSMBLK_ORACLE_H
#define LSMBLK_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  ORC_OK = 0,
  ORC_E_INVAL = -1,     /* bad argument (empty key, empty build, bad segment table) */
  ORC_E_MALFORMED = -2, /* block bytes do not parse (where the reference would panic) */
  ORC_E_CAPACITY = -3,  /* caller buffer too small; required sizes reported */
  ORC_E_OVERFLOW = -7,  /* a batch total does not fit the u32 KV-stream offsets */
};

/* ---- per-entry builder: src/block/builder.rs:8-89 ---- */
typedef struct orc_builder orc_builder;
orc_builder* orc_builder_new(size_t block_size);
void orc_builder_free(orc_builder* b);
/* returns 1 accepted, 0 rejected ("block full"), ORC_E_INVAL for an empty key */
int orc_builder_add(orc_builder* b, const uint8_t* key, size_t klen, uint64_t ts,
                    const uint8_t* val, size_t vlen);
int orc_builder_is_empty(const orc_builder* b);
size_t orc_builder_estimated_size(const orc_builder* b);
/* build()+encode(): writes the encoded block, resets the builder. */
int orc_builder_finish(orc_builder* b, uint8_t* out, size_t cap, size_t* len);

/* ---- Block::decode (src/block.rs:24-34) ---- */
int orc_block_decode(const uint8_t* blk, size_t len, size_t* data_len, uint16_t* offsets,
                     size_t offsets_cap, size_t* n);

/* ---- corrected BlockIterator semantics (src/block/iterator.rs) over an encoded block ---- */
typedef struct {
  const uint8_t* key_suffix; /* pointer into the block */
  uint32_t prefix, suffix;   /* key = first_key[0..prefix) ++ key_suffix[0..suffix) */
  uint64_t ts;
  const uint8_t* value;
  uint32_t vlen;
} orc_entry;
/* parse entry idx the way the corrected seek_to_offset does (ts skipped, ts set). */
int orc_block_entry(const uint8_t* blk, size_t len, size_t idx, orc_entry* e,
                    const uint8_t** first_key, uint32_t* first_klen);
/* the reference's seek_to_offset VERBATIM (src/block/iterator.rs:125-139), bug included:
 * value_len is read at the ts position and the ts bytes are never skipped. */
int orc_block_entry_verbatim(const uint8_t* blk, size_t len, size_t idx, uint32_t* prefix,
                             uint32_t* suffix, size_t* value_begin, size_t* value_end);
/* seek_to_key (src/block/iterator.rs:80-94): first idx with key >= target (ts-agnostic). */
size_t orc_block_seek_key(const uint8_t* blk, size_t len, const uint8_t* key, size_t klen);

/* ---- batch restatement over the SoA KV stream ----
 * KV stream: keys arena + key_off[n+1] (u32), vals arena + val_off[n+1] (u32), ts[n].   */
typedef struct {
  uint8_t* keys;
  uint32_t* key_off;
  uint8_t* vals;
  uint32_t* val_off;
  uint64_t* ts;
  uint64_t n;
} orc_kv;

/* Greedy packing of each segment [seg_start[g], seg_start[g+1]) with BlockBuilder, the way
 * SsTableBuilder::add drives it (src/table/builder.rs:48-65, 112-123), blocks tightly packed
 * (no CRC). blk_off has nblk+1 entries. */
int orc_encode_segments(const orc_kv* kv, const uint32_t* seg_start, uint32_t nseg,
                        size_t block_size, uint8_t* out, uint64_t out_cap, uint64_t* blk_off,
                        uint64_t blk_cap, uint64_t* nblk, uint64_t* nbytes);
/* Decode every block into the SoA stream (corrected iterator order). Caps are element /
 * byte capacities; on ORC_E_CAPACITY the required totals are still reported. */
int orc_decode_blocks(const uint8_t* blocks, const uint64_t* blk_off, uint64_t nblk,
                      orc_kv* out, uint64_t entry_cap, uint64_t key_cap, uint64_t val_cap,
                      uint64_t* n, uint64_t* kbytes, uint64_t* vbytes);

/* SST rotation of compact_generate_sst (src/compact.rs:278-289): a new segment starts at
 * entry i when the open SST's estimate_size() (finished blocks + 4-B CRC each,
 * src/table/builder.rs:105-107,112-123) >= target and key i differs from key i-1.
 * Writes seg_start[0..nseg] (nseg+1 values). */
int orc_segment_like_compaction(const orc_kv* kv, size_t block_size, uint64_t target_sst_size,
                                uint32_t* seg_start, uint64_t seg_cap, uint64_t* nseg);

/* MergeIterator (src/iterators/merge_iterator.rs:59-184) over the sorted runs
 * [run_start[r], run_start[r+1]) of `in` (run 0 = highest priority): src[j] = the input index
 * of the j-th merged entry. */
int orc_merge_runs(const orc_kv* in, const uint32_t* run_start, uint32_t nrun, uint32_t* src,
                   uint64_t src_cap, uint64_t* n_out);

/* compact_generate_sst (src/compact.rs:223-311) over the merged stream src[0..n): compaction
 * rules, SST rotation at target_sst_size, one SsTableBuilder per SST.  Blocks packed (no CRC)
 * with blk_off[nblk+1]; per SST its first block sst_blk[] and first kept entry sst_ent[]
 * (nsst+1 values); kept[] = merged positions handed to SsTableBuilder::add. */
int orc_compact(const orc_kv* in, const uint32_t* src, uint64_t n, uint64_t watermark, int bottom,
                const uint8_t* const* prefixes, const size_t* prefix_len, uint32_t nprefix,
                size_t block_size, uint64_t target, uint8_t* out, uint64_t out_cap, uint64_t* blk_off,
                uint64_t blk_cap, uint32_t* sst_blk, uint32_t* sst_ent, uint64_t sst_cap, uint32_t* kept,
                uint64_t kept_cap, uint64_t* nblk_out, uint64_t* nbytes_out, uint64_t* nsst_out,
                uint64_t* nkept_out);

/* compact_generate_sst's SST rotation (src/compact.rs:278-289 with SsTableBuilder::add,
 * table/builder.rs:48-65,105-123) resumed mid-stream, for one range of a key-range split: the
 * stream `ext` holds the range's m kept entries, then the next entries of the whole stream (the
 * halo; `last`: ext ends where the whole stream ends).  The loop's state when it reaches the
 * range's entry p -- a new block starts at p, the open SST's data section holds d0 bytes (d0 = 0:
 * an SST starts at p) -- is the carry-in.  The loop runs from there until its first event at or
 * after entry m: an SST starting there (carry-out {e - m, 0}) or a block starting there (carry-out
 * {e - m, data section}).  seg_start[0..nseg] = p, the SSTs starting in [p, m), the end entry. */
int orc_shard_rotation(const orc_kv* ext, uint64_t m, int last, uint64_t p, uint64_t d0, size_t block_size,
                       uint64_t target, uint32_t* seg_start, uint64_t seg_cap, uint64_t* nseg, uint64_t* p_out,
                       uint64_t* d_out);
/* orc_shard_rotation with the loop's same_as_last_key per ext entry (two-level compactions);
 * same == NULL: the previous ext entry's key. */
int orc_shard_rotation_ex(const orc_kv* ext, const uint8_t* same, uint64_t m, int last, uint64_t p, uint64_t d0,
                          size_t block_size, uint64_t target, uint32_t* seg_start, uint64_t seg_cap, uint64_t* nseg,
                          uint64_t* p_out, uint64_t* d_out);

/* CRC-32/ISO-HDLC (crc32fast 1.4.0 == zlib crc32), used by SST framing. */
uint32_t orc_crc32(const uint8_t* p, size_t n);

#ifdef __cplusplus
}
#endif
#endif
