/*
 * lsmblk.h -- C ABI of the MI355X-native SSTable block codec (liblsmblk.so).
 *
 * Drop-in boundary for the CrystalAnalyst/Lsm block path (paths relative to the reference
 * repository root).  Two halves:
 *
 *  1. Per-entry API, host-synchronous, mirroring the reference's Rust API one-to-one so that
 *     SsTableBuilder / SsTable / SsTableIterator keep their call shape:
 *       lsmblk_builder_*  <-  BlockBuilder          src/block/builder.rs:37-89
 *       lsmblk_block_*    <-  Block::encode/decode  src/block.rs:14-34
 *       lsmblk_iter_*     <-  BlockIterator         src/block/iterator.rs:37-139
 *     (the reference calls these at src/table/builder.rs:34,55,62,113-114, src/table.rs:232,
 *      src/table/iterator.rs:35,59,64,75-92).  `add` must answer "accepted?" synchronously,
 *     so this half runs on the host CPU inside liblsmblk.so; it is product code, not a
 *     fallback for the batch half.
 *
 *  2. Batch / device API (the HIP kernels, gfx950): whole flush / compaction batches.
 *       lsmblk_decode_batch  replaces the per-block loop  SsTable::read_block -> Block::decode
 *                            -> BlockIterator::next        (src/table.rs:213-233,
 *                                                           src/table/iterator.rs:86-97)
 *       lsmblk_encode_batch  replaces the per-entry loop  SsTableBuilder::add ->
 *                            BlockBuilder::add / finish_block  (src/table/builder.rs:48-65,
 *                                                           112-123), one segment per SST
 *       lsmblk_crc32_batch   the per-block framing checksum  (src/table/builder.rs:120-122,
 *                                                           src/table.rs:226-230)
 *       lsmblk_block_meta_batch  the SST BlockMeta section per segment  (src/table.rs:29-63,
 *                                                           src/table/builder.rs:68-77)
 *       lsmblk_compact_filter_batch  compaction's per-entry keep/drop rules  (src/compact.rs:234-299)
 *     All pointers are DEVICE pointers; calls are asynchronous on `stream` (a hipStream_t
 *     passed as void*; NULL = the default stream).  Concurrency: a context's calls are
 *     serialised by its lock (any host thread) and its device work is ordered on the stream each
 *     call is given; a context's workspace is reused by its next call, so work that must run
 *     concurrently (several streams, several host threads at once) takes one context each.
 *     Every device-side wait is bounded (LSMBLK_E_TIMEOUT) and every data-dependent walk is
 *     bounded by its progress (LSMBLK_E_INTERNAL), so no call can leave a kernel running forever.
 *
 * Errors: every function returns 0 (LSMBLK_OK) or a negative LSMBLK_E_* code.  Where the
 * reference panics (empty key builder.rs:55, empty build :82-83, malformed decode
 * block.rs:25-27) the ABI returns an error code instead.
 *
 * Block format (bit-exact with the reference builder):
 *   entry  = u16 prefix | u16 suffix_len | key[prefix..] | u64 ts | u16 value_len | value
 *   block  = entry* | u16 offset* | u16 num_entries          (all integers big-endian)
 *   prefix = LCP(key, first key of the block); fields use the reference's `as u16` wrap.
 */
#ifndef LSMBLK_H
#define LSMBLK_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LSMBLK_ABI_VERSION 1

enum {
  LSMBLK_OK = 0,
  LSMBLK_E_INVAL = -1,     /* bad argument: empty key, empty build, bad segment table, misaligned output */
  LSMBLK_E_MALFORMED = -2, /* a block does not parse (the reference would panic); an encode input's offsets decrease */
  LSMBLK_E_CAPACITY = -3,  /* an output buffer is too small; the stats hold the required sizes */
  LSMBLK_E_NOMEM = -4,     /* host or device allocation failed */
  LSMBLK_E_HIP = -5,       /* a HIP runtime call failed */
  LSMBLK_E_TIMEOUT = -6,   /* a device-side look-back wait exceeded its bound (must not happen) */
  LSMBLK_E_OVERFLOW = -7,  /* a batch total does not fit the u32 KV-stream offsets */
  LSMBLK_E_INTERNAL = -8,  /* device self-check failed */
  LSMBLK_E_CHECKSUM = -9,  /* a block's framing CRC does not match (read_block, src/table.rs:228-230) */
};

int lsmblk_abi_version(void);
const char* lsmblk_strerror(int status);

/* ------------------------------------------------------------------ per-entry (host) */
typedef struct lsmblk_builder lsmblk_builder;
typedef struct lsmblk_block lsmblk_block;
typedef struct lsmblk_iter lsmblk_iter;

/* BlockBuilder::new (builder.rs:37-44). NULL on allocation failure. */
lsmblk_builder* lsmblk_builder_new(size_t block_size);
void lsmblk_builder_free(lsmblk_builder* b);
/* BlockBuilder::add (builder.rs:54-73). *accepted = 0 means "block full" (the reference's
 * `false`); LSMBLK_E_INVAL for an empty key (the reference's assert!). */
int lsmblk_builder_add(lsmblk_builder* b, const uint8_t* key, size_t klen, uint64_t ts,
                       const uint8_t* val, size_t vlen, int* accepted);
/* BlockBuilder::is_empty (builder.rs:76-78). */
int lsmblk_builder_is_empty(const lsmblk_builder* b);
/* estimated_size (builder.rs:48-50) == the encoded length finish() will produce. */
size_t lsmblk_builder_estimated_size(const lsmblk_builder* b);
/* build() + Block::encode() (builder.rs:81-89 + block.rs:14-22); the builder is reset to
 * empty as SsTableBuilder::finish_block does (src/table/builder.rs:113). */
int lsmblk_builder_finish(lsmblk_builder* b, uint8_t* out, size_t cap, size_t* len);
/* build() without encode: hands the Block to the caller (refcount 1). */
int lsmblk_builder_build(lsmblk_builder* b, lsmblk_block** out);

/* Block::decode (block.rs:24-34). The returned block is reference counted (the reference
 * shares it as Arc<Block>); iterators hold a reference. */
int lsmblk_block_decode(const uint8_t* buf, size_t len, lsmblk_block** out);
/* Block::encode (block.rs:14-22). */
int lsmblk_block_encode(const lsmblk_block* blk, uint8_t* out, size_t cap, size_t* len);
size_t lsmblk_block_encoded_len(const lsmblk_block* blk);
/* Block { data, offsets } fields (block.rs:7-10). */
int lsmblk_block_data(const lsmblk_block* blk, const uint8_t** data, size_t* len);
int lsmblk_block_offsets(const lsmblk_block* blk, const uint16_t** offsets, size_t* n);
void lsmblk_block_free(lsmblk_block* blk); /* drops one reference */

/* BlockIterator (iterator.rs). seek_to_offset is the CORRECTED inverse of the builder: the
 * 8-byte ts after the key suffix is skipped and returned as the key's ts (the reference
 * reads value_len from the ts bytes, iterator.rs:133-134). */
int lsmblk_iter_create_and_seek_to_first(lsmblk_block* blk, lsmblk_iter** out); /* :66-70 */
int lsmblk_iter_create_and_seek_to_key(lsmblk_block* blk, const uint8_t* key, size_t klen,
                                       lsmblk_iter** out);                         /* :73-77 */
int lsmblk_iter_seek_to_first(lsmblk_iter* it);                                     /* :99-101 */
int lsmblk_iter_seek_to_key(lsmblk_iter* it, const uint8_t* key, size_t klen);      /* :80-94 */
int lsmblk_iter_next(lsmblk_iter* it);                                              /* :104-107 */
int lsmblk_iter_is_valid(const lsmblk_iter* it);                                    /* :59-61 */
/* key() (:51-53): pointer valid until the next seek/next; ts is the entry's timestamp. */
int lsmblk_iter_key(const lsmblk_iter* it, const uint8_t** key, size_t* klen, uint64_t* ts);
int lsmblk_iter_value(const lsmblk_iter* it, const uint8_t** val, size_t* vlen);    /* :55-57 */
void lsmblk_iter_free(lsmblk_iter* it);

/* ------------------------------------------------------------------ batch (device) */
/* SoA KV stream in device memory (the decoded form of a batch of blocks):
 *   keys[key_off[i] .. key_off[i+1]), vals[val_off[i] .. val_off[i+1]), ts[i],  i < n.
 * key_off / val_off hold n+1 entries; arenas are limited to 4 GiB each per batch. */
typedef struct {
  uint8_t* keys;
  uint32_t* key_off;
  uint8_t* vals;
  uint32_t* val_off;
  uint64_t* ts;
  uint64_t n;          /* encode input: number of entries. decode output: ignored */
  uint64_t entry_cap;  /* decode output capacities: entries (key_off/val_off hold cap+1) */
  uint64_t key_cap;    /*   bytes */
  uint64_t val_cap;    /*   bytes */
} lsmblk_kv_stream;

/* Device-side result words (u64[LSMBLK_STATS_WORDS], device memory, written by the call):
 *   decode: [0] entries  [1] key bytes  [2] value bytes  [3] error flags
 *   encode: [0] blocks   [1] out bytes  [2] 0            [3] error flags             */
#define LSMBLK_STATS_WORDS 4
#define LSMBLK_ERR_MALFORMED 1u
#define LSMBLK_ERR_CAPACITY 2u
#define LSMBLK_ERR_OVERFLOW 4u
#define LSMBLK_ERR_TIMEOUT 8u
#define LSMBLK_ERR_SEGMENTS 16u
#define LSMBLK_ERR_INTERNAL 32u
#define LSMBLK_ERR_EMPTY_KEY 64u
#define LSMBLK_ERR_CHECKSUM 128u
/* Map a stats[3] error-flag word (copied to the host) to an LSMBLK_E_* status. */
int lsmblk_stats_status(uint64_t error_flags);

typedef struct lsmblk_ctx lsmblk_ctx;
/* One context per (device, stream user). Holds the look-back / plan workspace. */
int lsmblk_ctx_create(int device, lsmblk_ctx** out);
void lsmblk_ctx_destroy(lsmblk_ctx* ctx);
/* Pre-size the workspace (optional; calls grow it on demand, which synchronizes). */
int lsmblk_ctx_reserve(lsmblk_ctx* ctx, uint64_t max_blocks, uint64_t max_entries,
                       uint64_t max_segments);

/* Diagnostics (timing experiments only; results are WRONG while a skip mask is set):
 *   LSMBLK_DEBUG_POLL_MODE    look-back poll protocol: 0 sc1 loads, 1 + agent acquire,
 *                             2 sc1 first then agent atomic-RMW re-polls (default)
 *   LSMBLK_DEBUG_DECODE_SKIP  decode ablation mask: 1 look-back, 2 keys, 4 values, 8 metadata */
#define LSMBLK_DEBUG_POLL_MODE 0
#define LSMBLK_DEBUG_DECODE_SKIP 1
#define LSMBLK_DEBUG_KERNEL_TIMING 2 /* 1: dispatch start/stop events on every kernel launch */
#define LSMBLK_DEBUG_TWO_PASS_DECODE 3 /* 1: count + tile scan + decode (three launches) instead of the lagged decode (A/B) */
#define LSMBLK_DEBUG_DECODE_LAG 4 /* blocks the lagged decode counts ahead of its decodes (>= 128; default: 40 MiB of
                                     blocks at the batch's mean block size, at most 10240); setting it fixes the lag, 0 restores the default */
#define LSMBLK_DEBUG_DECODE_LAG_BYTES 6 /* the lagged decode's lag in bytes of blocks (default 40 MiB; 0: the lag set by key 4) */
#define LSMBLK_DEBUG_COUNTERS 5 /* 1: the lagged decode records a realtime trace per tile (lsmblk_debug_counters) */
#define LSMBLK_DEBUG_ROT_POISON 7 /* diagnostics builds only (fault injection): 1 = the SST rotation's block-chain levels
                                     get links that do not advance (J(s) = s, S(s) = 0) over a third of the
                                     stream; the rotation must report LSMBLK_E_INTERNAL, never loop */
#define LSMBLK_DEBUG_ENCODE_FUSED 8 /* 1: LSMBLK_ENCODE_SEG_SLOTS with block_size <= 4096 through one launch
                                       that walks and emits at once (encode_fused_kernel; measured slower
                                       than the plan walk + emit launches) */
#define LSMBLK_DEBUG_PLAN_PIPE 9 /* 0: the plan walk's helper waits for each chunk's offsets, then its keys
                                    (two round trips per chunk, the default); 1: pipelined over batches */
#define LSMBLK_DEBUG_EMIT_POISON 10 /* diagnostics builds only (fault injection): 1 = after the plan walk,
                                       every fifth block's first entry is set past its end entry (a
                                       block table with e < s, and e > n at the end); emit must report
                                       LSMBLK_E_INTERNAL and read none of those entries */
int lsmblk_debug_set(lsmblk_ctx* ctx, int key, uint32_t value);
/* The trace of the last lagged decode with LSMBLK_DEBUG_COUNTERS on (n <= 16 + 8 * 32768 words;
 * synchronizes).  Words 16 + 8 t + k, 100 MHz s_memrealtime stamps of 64-block tile t: k = 0 tile
 * finish starts, 1 the tile's bases are published, 2 / 3 its first decoder's base wait begins /
 * ends, 4 its first count starts, 5 its first decoder starts. */
int lsmblk_debug_counters(lsmblk_ctx* ctx, uint64_t* out, uint32_t n);
/* Durations (ms) of the kernels of the last timed decode / encode call on this context:
 * [0] dec_count [1] dec_scan [2] decode [3] plan [4] emit; -1 if not recorded.  Waits for
 * the recorded events. */
#define LSMBLK_KERNELS 5
int lsmblk_ctx_kernel_times(lsmblk_ctx* ctx, float* ms);
/* Every kernel launched on this context since the previous call (or since LSMBLK_DEBUG_KERNEL_TIMING
 * was switched on), summed by kernel name: out[0 .. *n).  The log holds the last 16384 launches;
 * LSMBLK_E_CAPACITY if more were made (or more than cap distinct kernels).  Waits for the events.
 * Diagnostics (bench.py's per-kernel roofline of every config); the log is cleared by the call. */
typedef struct {
  char name[56];
  uint32_t launches;
  float ms;
} lsmblk_kernel_stat;
int lsmblk_ctx_kernel_log(lsmblk_ctx* ctx, lsmblk_kernel_stat* out, uint32_t cap, uint32_t* n);

/* Decode nblk blocks (block b = blocks[blk_off[b] .. blk_off[b+1]), blk_off u64[nblk+1])
 * into the SoA stream `out` (outputs must be 16-byte aligned).  Asynchronous: completion
 * and error flags are in `stats` once the stream reaches this point. */
int lsmblk_decode_batch(lsmblk_ctx* ctx, const uint8_t* blocks, const uint64_t* blk_off,
                        uint64_t nblk, const lsmblk_kv_stream* out, uint64_t* stats,
                        void* stream);

/* Decode of an SST data section as SsTable::read_block reads it (src/table.rs:213-233): block b =
 * blocks[blk_off[b] .. blk_off[b+1] - tail) -- tail = 4 over a framed data section addressed by its
 * BlockMeta offsets (block_len = offset_end - offset - 4), 0 for packed blocks.  With
 * LSMBLK_DECODE_VERIFY_CRC (tail must be 4) the u32 BE after every block is checked against its
 * crc32fast; a mismatch sets LSMBLK_ERR_CHECKSUM ("block checksum mismatched").  blk_ent (device
 * u64[nblk+1], optional) receives every block's first entry index in `out` and then the total, e.g.
 * the run boundaries for lsmblk_merge_batch.  Otherwise as lsmblk_decode_batch. */
#define LSMBLK_DECODE_VERIFY_CRC 1u
int lsmblk_decode_batch_ex(lsmblk_ctx* ctx, const uint8_t* blocks, const uint64_t* blk_off, uint64_t nblk,
                           uint32_t tail, uint32_t flags, const lsmblk_kv_stream* out, uint64_t* blk_ent,
                           uint64_t* stats, void* stream);

/* Encode the SoA stream `in` greedily into blocks of `block_size`, restarting the block
 * packing at every segment start (seg_start u32[nseg+1], seg_start[0] = 0, seg_start[nseg]
 * = in->n, non-decreasing), exactly as one SsTableBuilder per segment would.  Blocks are
 * written tightly packed to `out` (16-byte aligned, out_cap bytes); blk_off (u64, room for
 * blk_cap values) receives nblk+1 offsets.  key_off / val_off must be non-decreasing: an entry whose
 * offsets decrease fails the call with LSMBLK_ERR_MALFORMED and nothing is written. */
int lsmblk_encode_batch(lsmblk_ctx* ctx, const lsmblk_kv_stream* in, const uint32_t* seg_start,
                        uint32_t nseg, uint32_t block_size, uint8_t* out, uint64_t out_cap,
                        uint64_t* blk_off, uint64_t blk_cap, uint64_t* stats, void* stream);

/* lsmblk_encode_batch with flags.  LSMBLK_ENCODE_SEG_SLOTS writes every segment -- one SST's data
 * section, as its SsTableBuilder accumulates it (src/table/builder.rs:112-123, without the CRCs) --
 * back to back at its own slot instead of packing all segments together:
 *   slot(s) = (key_off[seg_start[s]] - key_off[seg_start[0]]) + (val_off[seg_start[s]] -
 *             val_off[seg_start[0]]) + 18 * (seg_start[s] - seg_start[0]),
 * an upper bound of the encoded size of the segments before s, so out_cap >= key bytes + value
 * bytes + 18 * n always suffices, and every SST's place is known before the encode runs.  The
 * block bytes are the same as lsmblk_encode_batch's.  seg_out (u64[2 * nseg], required): [2 s] = slot(s),
 * [2 s + 1] = segment s's encoded bytes.  blk_off[b] = where block b starts; a block ends where the
 * next starts unless it is its segment's last (then at seg_out[2 s] + seg_out[2 s + 1]);
 * blk_off[nblk] = the end of the last segment.  stats[1] = the encoded bytes (their sum). */
#define LSMBLK_ENCODE_SEG_SLOTS 1u
/* LSMBLK_ENCODE_FRAMED writes every block followed by its crc32fast as a big-endian u32 -- the SST
 * data section exactly as SsTableBuilder::finish_block builds it (src/table/builder.rs:112-123:
 * the encoded block, then put_u32(crc32(block))).  blk_off[b] = where block b starts; its CRC sits
 * at the block's end, and (without SEG_SLOTS) blk_off[b + 1] = blk_off[b] + block size + 4, so
 * lsmblk_decode_batch_ex(tail = 4, LSMBLK_DECODE_VERIFY_CRC) reads the output as read_block reads
 * the file.  stats[1] counts the CRC bytes too.  With SEG_SLOTS the slot bound is 22 bytes per
 * entry instead of 18 (4 more per block, at most one block per entry) and seg_out[2 s + 1] includes
 * the segment's CRCs.  The CRCs are a pass over the encoded blocks (the streaming CRC kernel of
 * lsmblk_crc32_batch) after emit. */
#define LSMBLK_ENCODE_FRAMED 2u
int lsmblk_encode_batch_ex(lsmblk_ctx* ctx, const lsmblk_kv_stream* in, const uint32_t* seg_start,
                           uint32_t nseg, uint32_t block_size, uint32_t flags, uint8_t* out,
                           uint64_t out_cap, uint64_t* blk_off, uint64_t blk_cap, uint64_t* seg_out,
                           uint64_t* stats, void* stream);

/* SST block framing (SURVEY.md §8 f, row 1): crc[b] = crc32fast::hash(block b) for block
 * b = blocks[blk_off[b] .. blk_off[b+1] - tail) -- the checksum SsTableBuilder::finish_block
 * appends after every encoded block as a big-endian u32 (src/table/builder.rs:120-122) and
 * SsTable::read_block verifies before Block::decode (src/table.rs:219-230).  tail = 0 for
 * tightly packed blocks (lsmblk_encode_batch output); tail = 4 over a framed SST data section
 * with blk_off = the BlockMeta offsets plus the meta-section offset (read_block's
 * block_len = offset_end - offset - 4).  CRC-32/ISO-HDLC (reflected 0xEDB88320, init and
 * xorout 0xFFFFFFFF); an empty block's CRC is 0.  stats: [0] blocks [1] bytes spanned
 * [3] error flags (LSMBLK_ERR_MALFORMED: a range is shorter than tail, decreasing, or over
 * 2 GiB; its crc is then 0).  Asynchronous like the calls above. */
int lsmblk_crc32_batch(lsmblk_ctx* ctx, const uint8_t* blocks, const uint64_t* blk_off,
                       uint64_t nblk, uint32_t tail, uint32_t* crc, uint64_t* stats, void* stream);

/* Segment -> block table after an encode: seg_blk[s] (u32[nseg+1]) = index of segment s's
 * first block in the lsmblk_encode_batch output (seg_blk[nseg] = nblk).  Must be called on the
 * same context and stream as that encode, before the next encode on the context; seg_start and
 * enc_stats are the encode's own arguments (device pointers).  After a failed encode every
 * entry is 0.  Asynchronous. */
int lsmblk_encode_segment_blocks(lsmblk_ctx* ctx, const uint32_t* seg_start, uint32_t nseg,
                                 const uint64_t* enc_stats, uint32_t* seg_blk, void* stream);

/* SST BlockMeta sections (SURVEY.md §8 f, row 1): for every segment s (an SST, blocks
 * seg_blk[s] .. seg_blk[s+1]) the bytes BlockMeta::encode_block_meta writes after the SST data
 * section (src/table.rs:29-63, called at src/table/builder.rs:77), as SsTableBuilder produces
 * them: offset = the block's position in the framed data section (every block followed by its
 * u32 CRC, builder.rs:118-122), first/last key = the block's first/last key with ts 0
 * (key.rs:166-169), max_ts = 0, CRC-32 of the section after its u32 count.  The keys are parsed
 * from the blocks themselves.  Block b = blocks[blk_off[b] .. blk_off[b+1] - tail): tail = 0 for
 * packed blocks (encode output), 4 over a framed data section.  Section s is written to
 * meta[meta_off[s] .. meta_off[s+1]) (meta_off u64[nseg+1]; meta_cap >= 16).  stats: [0] nseg
 * [1] bytes required [3] error flags (MALFORMED: a block without entries or whose first/last
 * entry does not parse; CAPACITY: meta_cap too small, stats[1] = required; SEGMENTS: bad
 * seg_blk).  A segment without blocks gets the 16-byte section of an empty meta list (the
 * reference would panic building an empty SST).  Asynchronous. */
int lsmblk_block_meta_batch(lsmblk_ctx* ctx, const uint8_t* blocks, const uint64_t* blk_off,
                            uint64_t nblk, uint32_t tail, const uint32_t* seg_blk, uint32_t nseg,
                            uint8_t* meta, uint64_t meta_cap, uint64_t* meta_off, uint64_t* stats,
                            void* stream);

/* Compaction filter (SURVEY.md §8 f, row 2 -- the per-entry rules of compact_generate_sst,
 * src/compact.rs:234-299) over a MERGED stream `in` (user keys ascending, versions newest
 * first, as MergeIterator yields them).  Keeps every version newer than `watermark` and, of
 * each key's versions at or below it, only the newest -- unless bottom_level and that version
 * is a tombstone (empty value) with no newer version (:244-254), or the key starts with one of
 * the nprefix prefixes (prefixes[prefix_off[f] .. prefix_off[f+1]), device memory;
 * CompactionFilter::Prefix, :264-275).  The kept entries are written in order to `out` (any
 * alignment).  stats: [0] kept entries [1] key bytes [2] value bytes [3] error flags
 * (CAPACITY: out's entry_cap / key_cap / val_cap too small, stats hold the required sizes,
 * nothing written).  SST rotation (:278-289) stays with the encode's segment table.
 * Asynchronous. */
int lsmblk_compact_filter_batch(lsmblk_ctx* ctx, const lsmblk_kv_stream* in, uint64_t watermark,
                                int bottom_level, const uint8_t* prefixes, const uint32_t* prefix_off,
                                uint32_t nprefix, const lsmblk_kv_stream* out, uint64_t* stats,
                                void* stream);

/* Merge modes (lsmblk_merge_batch_ex, lsmblk_compact_opts.merge_mode).  The reference's compact()
 * never merges its inputs with one MergeIterator: every task reads them through
 * TwoMergeIterator(a, b) with a = MergeIterator(L0 SSTs) or SstConcatIterator(upper level) and b =
 * SstConcatIterator(lower level) (src/compact.rs:170-173, 188-196, 206-215).
 *   LSMBLK_MERGE_RUNS       run-priority merge of all runs, the lower level as the LAST run: for every
 *                           user key, all versions of the lowest-index run holding it.  This is what
 *                           the reference's own TwoMergeIterator tests expect (src/tests/week1_day5.rs:
 *                           15-129: test_task1_merge_1..5) and what MergeIterator does
 *                           (merge_iterator.rs:59-184).  Default.
 *   LSMBLK_MERGE_TWO_LEVEL  two_merge_iterator.rs:19-93 exactly as written, with a = MergeIterator over
 *                           runs 0..nrun-2 and b = run nrun-1; it fails week1_day5's merge_3 / merge_4:
 *                           the stream ends with b (an empty b yields nothing; a's keys >= b's last key
 *                           are dropped), and for a key in both, skip_b drops b's 1st, 3rd, ... version
 *                           and the 2nd, 4th, ... come BEFORE a's versions.  Byte-identical to what the
 *                           reference binary's compaction writes for the same inputs.
 * DESIGN.md §3 tabulates the input classes on which the two differ. */
#define LSMBLK_MERGE_RUNS 0u
#define LSMBLK_MERGE_TWO_LEVEL 1u

/* k-way merge of sorted runs (SURVEY.md §8 f, row 2) with MergeIterator's semantics
 * (src/iterators/merge_iterator.rs:59-184) = LSMBLK_MERGE_RUNS: run r = entries [run_start[r], run_start[r+1]) of `in`
 * (run_start: device u32[nrun+1], [0] = 0, [nrun] = in->n; 1 <= nrun <= 64), run 0 the highest
 * priority (MergeIterator::create's index 0, e.g. the newest L0 SST).  Heads compare by user key
 * only (src/key.rs:63-81) with the run index breaking ties, and every step advances the other
 * runs' heads equal to the current key (:134-152): for every user key the output holds all the
 * versions of the lowest-index run containing it, in that run's order.  Each run must be sorted
 * by key (the reference's debug_assert :135-138); a merged order that is not reports
 * LSMBLK_ERR_MALFORMED.  The merged stream is written to `out` (any alignment; capacities as
 * for decode).  stats: [0] entries [1] key bytes [2] value bytes [3] error flags (CAPACITY with
 * the required sizes in [0..2]; SEGMENTS: bad run_start, or a key over 65 535 bytes -- the merge
 * tiles hold u16 key lengths, as the block format does).  Asynchronous. */
int lsmblk_merge_batch(lsmblk_ctx* ctx, const lsmblk_kv_stream* in, const uint32_t* run_start, uint32_t nrun,
                       const lsmblk_kv_stream* out, uint64_t* stats, void* stream);
/* lsmblk_merge_batch in merge_mode LSMBLK_MERGE_RUNS or LSMBLK_MERGE_TWO_LEVEL (run nrun-1 = b). */
int lsmblk_merge_batch_ex(lsmblk_ctx* ctx, const lsmblk_kv_stream* in, const uint32_t* run_start, uint32_t nrun,
                          uint32_t merge_mode, const lsmblk_kv_stream* out, uint64_t* stats, void* stream);

/* SST rotation of compact_generate_sst (src/compact.rs:278-289) over `in`, the stream of entries
 * handed to SsTableBuilder::add (one key's versions newest first): a new SST starts before entry e
 * when the open SST's estimate_size() -- its finished blocks plus a 4-byte CRC each
 * (src/table/builder.rs:105-123) -- is >= target_sst_size and key(e) differs from key(e-1).  The
 * blocks are BlockBuilder's greedy packing of block_size restarted at every SST start, so this
 * is exactly the segment table under which lsmblk_encode_batch reproduces the compaction's SSTs.
 * sst_start (device u32[sst_cap]) receives the nsst SST first entries and then in->n.  stats: [0]
 * nsst [3] error flags (CAPACITY: sst_cap < nsst + 1).  Asynchronous. */
int lsmblk_sst_rotation_batch(lsmblk_ctx* ctx, const lsmblk_kv_stream* in, uint32_t block_size,
                              uint64_t target_sst_size, uint32_t* sst_start, uint32_t sst_cap, uint64_t* stats,
                              void* stream);

/* Options of lsmblk_compact_batch: the compaction rules (src/compact.rs:239-276) and the SST
 * layout (LsmStorageOptions::block_size / target_sst_size, src/lsm_storage.rs:68-94). */
typedef struct {
  uint64_t watermark;          /* LsmMvccInner::watermark() */
  int32_t bottom_level;        /* compact_to_bottom_level: drop tombstones at or below the watermark */
  uint32_t nprefix;            /* CompactionFilter::Prefix filters (device memory) */
  const uint8_t* prefixes;
  const uint32_t* prefix_off;  /* u32[nprefix+1] */
  uint32_t block_size;
  uint32_t merge_mode;         /* LSMBLK_MERGE_RUNS (0) or LSMBLK_MERGE_TWO_LEVEL (run nrun-1 = the lower level) */
  uint64_t target_sst_size;
} lsmblk_compact_opts;

#define LSMBLK_COMPACT_STATS_WORDS 8
/* compact_generate_sst (src/compact.rs:223-311) on the device for sorted runs already decoded
 * into `in` (run_start as for lsmblk_merge_batch): merge (opts->merge_mode: the run-priority merge,
 * or the reference's TwoMergeIterator with the lower level as the last run) -> keep/drop rules ->
 * SST rotation -> SsTableBuilder block packing.  `kept` receives the entries handed to
 * SsTableBuilder::add (capacities as for decode); the blocks of every SST are written packed to
 * `out` (16-byte aligned) with blk_off (u64[blk_cap], nblk+1 values), as lsmblk_encode_batch writes
 * them; sst_start / sst_blk (u32[sst_cap], sst_cap >= 2) receive each SST's first kept entry / first
 * block, then kept count / nblk.  Per-block CRCs and BlockMeta sections follow from
 * lsmblk_crc32_batch / lsmblk_block_meta_batch with seg_blk = sst_blk.  When nothing is kept the
 * result is zero SSTs (the reference panics building an empty SST).  stats (u64[8]): [0] blocks
 * [1] bytes [2] SSTs [3] error flags [4] merged entries [5] kept entries [6] kept key bytes
 * [7] kept value bytes.  Asynchronous; allocates workspace on the context (~45 B per input entry
 * plus 8 B per entry per rotation level). */
int lsmblk_compact_batch(lsmblk_ctx* ctx, const lsmblk_kv_stream* in, const uint32_t* run_start, uint32_t nrun,
                         const lsmblk_compact_opts* opts, const lsmblk_kv_stream* kept, uint8_t* out,
                         uint64_t out_cap, uint64_t* blk_off, uint64_t blk_cap, uint32_t* sst_start,
                         uint32_t* sst_blk, uint32_t sst_cap, uint64_t* stats, void* stream);

/* ------------------------------------------------------------------ key-range sharded compaction (§8 e) */
/* One GPU's share of a compaction split by user-key range over W ranks (SURVEY.md §8 e): the
 * concatenation of every rank's output is byte-identical to the single-stream compact_generate_sst
 * (src/compact.rs:223-311) over all the input, SST boundaries included.  Per rank:
 *   1. lsmblk_compact_merge_batch: merge + rules over the decoded input blocks, keeping only the
 *      keys in [lo, hi) (blocks straddling a splitter are read by both neighbours);
 *   2. the caller appends the halo -- the first lsmblk_shard_halo_entries(block_size) kept entries
 *      of the ranks after this one -- to the kept stream (one small all-gather);
 *   3. lsmblk_shard_rotation_prepare: everything of the SST rotation that does not depend on the
 *      state entering the range (block chains, SST-end function, its powers);
 *   4. lsmblk_shard_rotation_carry: the boundary carry, rank after rank (send/recv of 16 bytes):
 *      carry = {p, D}: the open SST's next block starts at entry p of the receiving rank's range and
 *      the SST's data section (blocks + CRCs) holds D bytes there (D = 0: an SST starts at p);
 *      rank 0 receives {0, 0};
 *   5. lsmblk_shard_encode_batch: this rank's SST cut points and blocks. */
typedef struct {
  const uint8_t* lo;  /* device bytes; used when has_lo */
  const uint8_t* hi;  /* device bytes; used when has_hi (exclusive) */
  uint32_t lo_len, hi_len;
  uint32_t has_lo, has_hi;
} lsmblk_key_range;

/* Halo length: a block that starts before a range end can take at most block_size / 16 entries
 * after it, plus the entry it rejects. */
uint64_t lsmblk_shard_halo_entries(uint32_t block_size);

/* lsmblk_compact_batch's merge + rules + gather, restricted to keys in *range (NULL: all keys;
 * opts->merge_mode must be LSMBLK_MERGE_RUNS here; both modes: lsmblk_compact_merge_batch_ex):
 * kept receives this range's entries handed to SsTableBuilder::add.  stats: [0] kept entries [1] key
 * bytes [2] value bytes [3] error flags [4] merged entries.  Asynchronous. */
int lsmblk_compact_merge_batch(lsmblk_ctx* ctx, const lsmblk_kv_stream* in, const uint32_t* run_start, uint32_t nrun,
                               const lsmblk_compact_opts* opts, const lsmblk_key_range* range,
                               const lsmblk_kv_stream* kept, uint64_t* stats, void* stream);

/* The same in either merge mode.  LSMBLK_MERGE_TWO_LEVEL (TwoMergeIterator as written, run nrun-1 = b):
 * the stream ends at b's last key kb over the WHOLE compaction (two_merge_iterator.rs:32-42,60-66), so
 * each range says where kb lies (the caller all-gathers every range's local b-run end):
 *   LSMBLK_TWO_END_IN_RANGE  kb is in this range (or range is NULL): b's local last key is kb;
 *   LSMBLK_TWO_END_ABOVE     the range lies wholly below kb: no cut-off in it;
 *   LSMBLK_TWO_END_BELOW     kb lies below the range, or b is empty everywhere: no a-entry survives;
 * and kept_same (device u8[kept->entry_cap]) receives every kept entry's same_as_last_key of the
 * compact_generate_sst loop (src/compact.rs:279; with the two-level order it is not "same key as the
 * previous kept entry"), which the rotation needs: lsmblk_shard_rotation_prepare_ex.  LSMBLK_MERGE_RUNS:
 * two_end is ignored and kept_same may be NULL. */
#define LSMBLK_TWO_END_IN_RANGE 0u
#define LSMBLK_TWO_END_ABOVE 1u
#define LSMBLK_TWO_END_BELOW 2u
int lsmblk_compact_merge_batch_ex(lsmblk_ctx* ctx, const lsmblk_kv_stream* in, const uint32_t* run_start,
                                  uint32_t nrun, const lsmblk_compact_opts* opts, const lsmblk_key_range* range,
                                  uint32_t two_end, const lsmblk_kv_stream* kept, uint8_t* kept_same, uint64_t* stats,
                                  void* stream);

/* Rotation state of one range over `ext` = its n_own kept entries followed by the halo (ext->n
 * entries in all).  flags: LSMBLK_SHARD_LAST when ext ends where the whole compaction's stream ends
 * (the last rank, or a halo that reached the end).  sst_cap bounds the SSTs that start in the range.
 * The state stays on the context for the next two calls (same context, no other compaction call on
 * it in between).  Asynchronous. */
#define LSMBLK_SHARD_LAST 1u
int lsmblk_shard_rotation_prepare(lsmblk_ctx* ctx, const lsmblk_kv_stream* ext, uint64_t n_own, uint32_t flags,
                                  uint32_t block_size, uint64_t target_sst_size, uint32_t sst_cap, void* stream);
/* The same with ext_same (device u8[ext->n], two-level merges): every ext entry's same_as_last_key,
 * the range's own from lsmblk_compact_merge_batch_ex's kept_same, the halo's from the ranks that
 * own it.  NULL: "same key as the previous entry" (LSMBLK_MERGE_RUNS). */
int lsmblk_shard_rotation_prepare_ex(lsmblk_ctx* ctx, const lsmblk_kv_stream* ext, const uint8_t* ext_same,
                                     uint64_t n_own, uint32_t flags, uint32_t block_size, uint64_t target_sst_size,
                                     uint32_t sst_cap, void* stream);

/* carry_in (device u64[2]) -> carry_out (device u64[2]) for the next rank.  Asynchronous. */
int lsmblk_shard_rotation_carry(lsmblk_ctx* ctx, const uint64_t* carry_in, uint64_t* carry_out, void* stream);

/* The range's segments -- [p, first SST end, ..., last SST start, end), SST cut points of the whole
 * compaction, the first segment continuing the previous rank's open SST when carry_in.D > 0 and the
 * last one continued by the next rank when carry_out.D > 0 -- into seg_start (device u32[seg_cap]:
 * nseg + 1 entry indices of ext) and their blocks, packed, into out / blk_off as lsmblk_encode_batch
 * writes them; seg_blk (u32[seg_cap]) receives every segment's first block.  stats (u64[8]): [0]
 * blocks [1] bytes [2] segments [3] error flags [4] first segment continues [5] last segment
 * continues [6] first entry [7] end entry.  Asynchronous. */
int lsmblk_shard_encode_batch(lsmblk_ctx* ctx, const lsmblk_kv_stream* ext, uint8_t* out, uint64_t out_cap,
                              uint64_t* blk_off, uint64_t blk_cap, uint32_t* seg_start, uint32_t* seg_blk,
                              uint32_t seg_cap, uint64_t* stats, void* stream);

/* ------------------------------------------------------------------ memtable (§8 f row 4, host) */
/* MemTable (src/mem_table.rs:55-158): an ordered map keyed by the key bytes only (Key's Ord ignores
 * the ts, src/key.rs:63-81), so put() of a present key replaces the entry; flush() (:131-136) yields
 * the entries in key order -- the flush source the device encoder consumes (lsmblk_encode_batch,
 * then lsmblk_sst_files_batch).  Host memory; every call takes the memtable's lock (see _get). */
typedef struct lsmblk_memtable lsmblk_memtable;
lsmblk_memtable* lsmblk_memtable_new(void);
void lsmblk_memtable_free(lsmblk_memtable* m);
int lsmblk_memtable_put(lsmblk_memtable* m, const uint8_t* key, size_t klen, uint64_t ts, const uint8_t* val,
                        size_t vlen);                                                  /* :113-127 */
/* 1 = found, 0 = absent (:93-99).  *val points into the memtable: valid only while no put of the same
 * key can run (single-writer use); concurrent readers use lsmblk_memtable_get_copy. */
int lsmblk_memtable_get(lsmblk_memtable* m, const uint8_t* key, size_t klen, const uint8_t** val, size_t* vlen,
                        uint64_t* ts);
/* get() that copies the value into val[0 .. cap) under the memtable's lock (safe against concurrent
 * puts).  1 = found, 0 = absent, LSMBLK_E_CAPACITY = cap < *vlen (nothing copied; *vlen, *ts set). */
int lsmblk_memtable_get_copy(lsmblk_memtable* m, const uint8_t* key, size_t klen, uint8_t* val, size_t cap,
                             size_t* vlen, uint64_t* ts);
size_t lsmblk_memtable_len(lsmblk_memtable* m);
size_t lsmblk_memtable_approximate_size(lsmblk_memtable* m);                          /* :154-157 */
/* The entries in key order as a SoA KV stream in host buffers (flush, :131-136); *n / *kbytes /
 * *vbytes report the sizes (LSMBLK_E_CAPACITY when a buffer is too small). */
int lsmblk_memtable_flush(lsmblk_memtable* m, uint8_t* keys, uint32_t* key_off, uint8_t* vals, uint32_t* val_off,
                          uint64_t* ts, uint64_t entry_cap, uint64_t key_cap, uint64_t val_cap, uint64_t* n,
                          uint64_t* kbytes, uint64_t* vbytes);

/* ------------------------------------------------------------------ SST container (§8 f row 3) */
/* Whole SST files as SsTableBuilder::build writes them (src/table/builder.rs:68-98), for the nsst
 * SSTs of an encode or compaction: SST s = blocks [sst_blk[s], sst_blk[s+1]) of (blocks, blk_off)
 * (packed, as lsmblk_encode_batch / lsmblk_compact_batch write them), holding the entries
 * [sst_ent[s], sst_ent[s+1]) of `kv` -- the entries handed to SsTableBuilder::add, whose
 * fingerprint32 hashes fill the bloom filter (:53, src/table/bloom.rs:72-101).  File s =
 * files[file_off[s] .. file_off[s+1]) (file_off: device u64[nsst+1]):
 *   every block followed by its BE u32 crc32fast | BlockMeta section | BE u32 meta_offset |
 *   filter | k | BE u32 crc32fast(filter | k) | BE u32 bloom_offset.
 * sst_blk / sst_ent: device u32[nsst+1].  stats: [0] nsst [1] bytes (required on CAPACITY)
 * [3] error flags.  Synchronizes once (reads the key arena size to bound the workspace). */
int lsmblk_sst_files_batch(lsmblk_ctx* ctx, const uint8_t* blocks, const uint64_t* blk_off, uint64_t nblk,
                           const uint32_t* sst_blk, const uint32_t* sst_ent, uint32_t nsst,
                           const lsmblk_kv_stream* kv, uint8_t* files, uint64_t files_cap, uint64_t* file_off,
                           uint64_t* stats, void* stream);
/* BlockIterator::create_and_seek_to_key (src/block/iterator.rs:73-94) for a batch of point
 * lookups (§8 a row 13): lookup q seeks key qkeys[qkey_off[q] .. qkey_off[q+1]) in block q_blk[q]
 * of (blocks, blk_off, tail as for lsmblk_decode_batch_ex).  idx[q] = the entry index the
 * iterator lands on -- its binary search with ts-agnostic key order, stopping at the first probe
 * that compares equal -- or the block's entry count when the iterator ends invalid.  All device
 * pointers (qkey_off: u32[nq+1], q_blk, idx: u32[nq]).  stats[3]: MALFORMED for a block that does
 * not parse (idx = its entry count), SEGMENTS for a block index out of range.  Asynchronous. */
int lsmblk_seek_batch(lsmblk_ctx* ctx, const uint8_t* blocks, const uint64_t* blk_off, uint64_t nblk, uint32_t tail,
                      const uint8_t* qkeys, const uint32_t* qkey_off, const uint32_t* q_blk, uint64_t nq,
                      uint32_t* idx, uint64_t* stats, void* stream);
/* farmhash::fingerprint32 (the key hash of SsTableBuilder::add, src/table/builder.rs:53), host. */
uint32_t lsmblk_fingerprint32(const uint8_t* key, size_t klen);
/* Bloom::may_contain (src/table/bloom.rs:104-120) over a decoded filter, host. */
int lsmblk_bloom_may_contain(const uint8_t* filter, size_t nbytes, uint32_t k, uint32_t h);

#ifdef __cplusplus
}
#endif
#endif
