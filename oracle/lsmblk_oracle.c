/*
 * lsmblk_oracle.c -- CPU restatement of the CrystalAnalyst/Lsm SSTable block codec.
 *
 * TEST INFRASTRUCTURE ONLY (checker + timed CPU baseline).  The product (lsm_amd/,
 * liblsmblk.so) never links or calls this file.
 *
 * What it restates (reference paths relative to /root/reference):
 *   BlockBuilder          src/block/builder.rs:8-89  (common_prefix :19-33, add :54-73)
 *   Block::encode/decode  src/block.rs:14-34
 *   BlockIterator         src/block/iterator.rs:23-139, with seek_to_offset CORRECTED
 *                         (skip the 8-byte ts, set the key's ts); the verbatim buggy form
 *                         is kept as orc_block_entry_verbatim for documentation tests.
 *   Key ordering          src/key.rs:63-81 (ts-agnostic), raw_len src/key.rs:29-31
 *   SsTableBuilder driver src/table/builder.rs:48-65,105-123
 *   SST rotation          src/compact.rs:278-289
 *   crc32fast             == zlib CRC-32 (pinned by lsm.db/MANIFEST, see tests)
 *
 * Third-party arithmetic: `bytes` 1.5.0 put_u16/put_u64/get_u16/get_u64 are big-endian.
 *
 * Pinning: the reference is Rust and cannot be built here (no cargo/rustc, crates not
 * vendored), so no reference-produced byte vectors exist.  The restatement is pinned by
 * the reference's own test assertions -- src/tests/week1_day3.rs (builder accept/reject,
 * encode/decode round trip, iterator and seek expectations), week1_day4.rs (>= 2 blocks),
 * week1_day7.rs (<= 34 blocks at block_size 128 with ts), week3_day1.rs (multi-version
 * data) -- and by lsm.db/MANIFEST's CRC records; an independent pure-Python restatement
 * (oracle/pyref.py) must agree byte for byte (tests/test_oracle.py).
 */
#include "lsmblk_oracle.h"

#include <stdlib.h>
#include <string.h>

static inline void put_u16(uint8_t* p, uint32_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }
static inline uint32_t get_u16(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }
static inline void put_u64(uint8_t* p, uint64_t v) {
  for (int i = 0; i < 8; ++i) p[i] = (uint8_t)(v >> (56 - 8 * i));
}
static inline uint64_t get_u64(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 0; i < 8; ++i) v = (v << 8) | p[i];
  return v;
}

/* ------------------------------------------------------------------ builder */
struct orc_builder {
  uint8_t* data; size_t len, cap;          /* data: Vec<u8>            builder.rs:10 */
  uint16_t* offsets; size_t n, ocap;       /* offsets: Vec<u16>        builder.rs:11 */
  uint8_t* first_key; size_t fk_len;       /* first_key: KeyVec        builder.rs:13 */
  size_t block_size;                       /*                          builder.rs:14 */
};

static int reserve(void** p, size_t* cap, size_t need, size_t elt) {
  if (need <= *cap) return 0;
  size_t nc = *cap ? *cap : 64;
  while (nc < need) nc *= 2;
  void* q = realloc(*p, nc * elt);
  if (!q) return -1;
  *p = q; *cap = nc;
  return 0;
}

orc_builder* orc_builder_new(size_t block_size) {   /* builder.rs:37-44 */
  orc_builder* b = (orc_builder*)calloc(1, sizeof(*b));
  if (b) b->block_size = block_size;
  return b;
}

void orc_builder_free(orc_builder* b) {
  if (!b) return;
  free(b->data); free(b->offsets); free(b->first_key); free(b);
}

/* common_prefix, builder.rs:19-33: byte-wise LCP of key vs the block's FIRST key. */
static size_t common_prefix(const uint8_t* a, size_t alen, const uint8_t* b, size_t blen) {
  size_t i = 0;
  while (i < alen && i < blen && a[i] == b[i]) ++i;
  return i;
}

int orc_builder_is_empty(const orc_builder* b) { return b->n == 0; }   /* builder.rs:76-78 */

size_t orc_builder_estimated_size(const orc_builder* b) {              /* builder.rs:48-50 */
  return b->len + b->n * 2 + 2;
}

/* add, builder.rs:54-73 */
int orc_builder_add(orc_builder* b, const uint8_t* key, size_t klen, uint64_t ts,
                    const uint8_t* val, size_t vlen) {
  if (klen == 0) return ORC_E_INVAL;                         /* assert! :55 */
  size_t add_on = (klen + 8) + vlen + 2 * 3;                 /* raw_len + value + 3*u16 :56 */
  if (orc_builder_estimated_size(b) + add_on > b->block_size && !orc_builder_is_empty(b))
    return 0;                                                /* :57-60 */
  size_t p = common_prefix(b->first_key, b->fk_len, key, klen);   /* :62 */
  size_t grow = 4 + (klen - p) + 8 + 2 + vlen;
  if (reserve((void**)&b->offsets, &b->ocap, b->n + 1, 2)) return ORC_E_INVAL;
  if (reserve((void**)&b->data, &b->cap, b->len + grow, 1)) return ORC_E_INVAL;
  b->offsets[b->n++] = (uint16_t)b->len;                     /* data.len() as u16 :61 */
  uint8_t* d = b->data + b->len;
  put_u16(d, (uint32_t)(p & 0xFFFF));                        /* prefix as u16 :63 */
  put_u16(d + 2, (uint32_t)((klen - p) & 0xFFFF));           /* (klen-prefix) as u16 :64 */
  memcpy(d + 4, key + p, klen - p);                          /* key[prefix..] :65 */
  put_u64(d + 4 + (klen - p), ts);                           /* put_u64(ts) :66 */
  put_u16(d + 12 + (klen - p), (uint32_t)(vlen & 0xFFFF));   /* value.len() as u16 :67 */
  memcpy(d + 14 + (klen - p), val, vlen);                    /* value :68 */
  b->len += grow;
  if (b->fk_len == 0) {                                      /* :69-71 */
    b->first_key = (uint8_t*)malloc(klen);
    memcpy(b->first_key, key, klen);
    b->fk_len = klen;
  }
  return 1;
}

/* build (builder.rs:81-89) + Block::encode (block.rs:14-22); resets like SsTableBuilder's
 * std::mem::replace (table/builder.rs:113). */
int orc_builder_finish(orc_builder* b, uint8_t* out, size_t cap, size_t* len) {
  if (orc_builder_is_empty(b)) return ORC_E_INVAL;          /* panic :82-83 */
  size_t total = b->len + 2 * b->n + 2;
  *len = total;
  if (total > cap) return ORC_E_CAPACITY;
  memcpy(out, b->data, b->len);
  for (size_t i = 0; i < b->n; ++i) put_u16(out + b->len + 2 * i, b->offsets[i]);
  put_u16(out + b->len + 2 * b->n, (uint32_t)(b->n & 0xFFFF));   /* offsets_len as u16 */
  b->len = 0; b->n = 0;
  free(b->first_key); b->first_key = NULL; b->fk_len = 0;
  return ORC_OK;
}

/* ------------------------------------------------------------------ decode */
/* Block::decode, block.rs:24-34.  The reference panics on len < 2 or an oversized count;
 * that becomes ORC_E_MALFORMED. */
int orc_block_decode(const uint8_t* blk, size_t len, size_t* data_len, uint16_t* offsets,
                     size_t offsets_cap, size_t* n) {
  if (len < 2) return ORC_E_MALFORMED;
  size_t cnt = get_u16(blk + len - 2);
  if (2 + 2 * cnt > len) return ORC_E_MALFORMED;
  size_t data_end = len - 2 - 2 * cnt;
  *n = cnt; *data_len = data_end;
  if (cnt > offsets_cap) return ORC_E_CAPACITY;
  for (size_t i = 0; i < cnt; ++i) offsets[i] = (uint16_t)get_u16(blk + data_end + 2 * i);
  return ORC_OK;
}

/* Block::get_first_key, iterator.rs:23-34: parses the entry at DATA POSITION 0 (not
 * offsets[0]); skips the prefix field, reads key_len, the key and the ts. */
static int first_key_of(const uint8_t* blk, size_t data_end, const uint8_t** fk, uint32_t* fkl) {
  if (data_end < 4) return ORC_E_MALFORMED;
  uint32_t s = get_u16(blk + 2);
  if ((size_t)4 + s + 8 > data_end) return ORC_E_MALFORMED;
  *fk = blk + 4; *fkl = s;
  return ORC_OK;
}

/* Corrected seek_to_offset (iterator.rs:125-139 with the ts skipped and set). */
int orc_block_entry(const uint8_t* blk, size_t len, size_t idx, orc_entry* e,
                    const uint8_t** first_key, uint32_t* first_klen) {
  if (len < 2) return ORC_E_MALFORMED;
  size_t cnt = get_u16(blk + len - 2);
  if (2 + 2 * cnt > len) return ORC_E_MALFORMED;
  size_t data_end = len - 2 - 2 * cnt;
  if (idx >= cnt) return ORC_E_INVAL;
  const uint8_t* fk; uint32_t fkl;
  int rc = first_key_of(blk, data_end, &fk, &fkl);
  if (rc) return rc;
  size_t off = get_u16(blk + data_end + 2 * idx);
  if (off + 4 > data_end) return ORC_E_MALFORMED;
  uint32_t p = get_u16(blk + off), s = get_u16(blk + off + 2);
  if (off + 4 + s + 10 > data_end) return ORC_E_MALFORMED;
  if (p > fkl) return ORC_E_MALFORMED;               /* first_key[..prefix] would panic */
  if (p + s == 0) return ORC_E_MALFORMED;            /* empty key == "invalid" iterator */
  uint32_t vlen = get_u16(blk + off + 12 + s);
  if (off + 14 + s + vlen > data_end) return ORC_E_MALFORMED;
  e->prefix = p; e->suffix = s; e->key_suffix = blk + off + 4;
  e->ts = get_u64(blk + off + 4 + s);
  e->vlen = vlen; e->value = blk + off + 14 + s;
  if (first_key) *first_key = fk;
  if (first_klen) *first_klen = fkl;
  return ORC_OK;
}

/* The reference's seek_to_offset exactly as written (iterator.rs:125-139). */
int orc_block_entry_verbatim(const uint8_t* blk, size_t len, size_t idx, uint32_t* prefix,
                             uint32_t* suffix, size_t* value_begin, size_t* value_end) {
  if (len < 2) return ORC_E_MALFORMED;
  size_t cnt = get_u16(blk + len - 2);
  size_t data_end = len - 2 - 2 * cnt;
  if (idx >= cnt) return ORC_E_INVAL;
  size_t off = get_u16(blk + data_end + 2 * idx);
  uint32_t p = get_u16(blk + off), s = get_u16(blk + off + 2);   /* :127-128 */
  uint32_t vlen = get_u16(blk + off + 4 + s);                     /* :133, reads ts bytes */
  *prefix = p; *suffix = s;
  *value_begin = off + 2 + 2 + s + 2;                             /* :134 */
  *value_end = *value_begin + vlen;                               /* :135 */
  return ORC_OK;
}

static int key_cmp(const uint8_t* a, size_t al, const uint8_t* b, size_t bl) {
  size_t m = al < bl ? al : bl;
  int c = memcmp(a, b, m);
  if (c) return c;
  return al < bl ? -1 : (al > bl ? 1 : 0);
}

/* seek_to_key, iterator.rs:80-94 (binary search, ts-agnostic compare key.rs:77-81). */
size_t orc_block_seek_key(const uint8_t* blk, size_t len, const uint8_t* key, size_t klen) {
  size_t cnt = get_u16(blk + len - 2);
  size_t lo = 0, hi = cnt;
  uint8_t buf[1 << 17];
  while (lo < hi) {
    size_t mid = lo + (hi - lo) / 2;
    orc_entry e; const uint8_t* fk; uint32_t fkl;
    if (orc_block_entry(blk, len, mid, &e, &fk, &fkl)) return cnt;
    memcpy(buf, fk, e.prefix);
    memcpy(buf + e.prefix, e.key_suffix, e.suffix);
    int c = key_cmp(buf, e.prefix + e.suffix, key, klen);
    if (c < 0) lo = mid + 1;
    else if (c > 0) hi = mid;
    else return mid;
  }
  return lo;
}

/* ------------------------------------------------------------------ batch */
int orc_encode_segments(const orc_kv* kv, const uint32_t* seg_start, uint32_t nseg,
                        size_t block_size, uint8_t* out, uint64_t out_cap, uint64_t* blk_off,
                        uint64_t blk_cap, uint64_t* nblk, uint64_t* nbytes) {
  if (nseg > 0 && (seg_start[0] != 0 || seg_start[nseg] != kv->n)) return ORC_E_INVAL;
  for (uint32_t g = 0; g < nseg; ++g)
    if (seg_start[g] > seg_start[g + 1]) return ORC_E_INVAL;
  orc_builder* b = orc_builder_new(block_size);
  uint64_t pos = 0, nb = 0;
  int rc = ORC_OK;
  size_t scratch_cap = 1 << 16;
  uint8_t* scratch = (uint8_t*)malloc(scratch_cap);
#define FINISH()                                                                      \
  do {                                                                                \
    size_t need = orc_builder_estimated_size(b), l;                                   \
    if (need > scratch_cap) { scratch_cap = need; scratch = (uint8_t*)realloc(scratch, need); } \
    orc_builder_finish(b, scratch, scratch_cap, &l);                                  \
    if (nb < blk_cap) blk_off[nb] = pos;                                              \
    if (pos + l <= out_cap) memcpy(out + pos, scratch, l); else rc = ORC_E_CAPACITY;  \
    pos += l; ++nb;                                                                   \
  } while (0)
  for (uint32_t g = 0; g < nseg; ++g) {
    for (uint64_t i = seg_start[g]; i < seg_start[g + 1]; ++i) {
      const uint8_t* k = kv->keys + kv->key_off[i];
      size_t kl = kv->key_off[i + 1] - kv->key_off[i];
      const uint8_t* v = kv->vals + kv->val_off[i];
      size_t vl = kv->val_off[i + 1] - kv->val_off[i];
      int a = orc_builder_add(b, k, kl, kv->ts[i], v, vl);        /* table/builder.rs:55 */
      if (a < 0) { rc = a; goto done; }
      if (a == 0) {                                                /* :60-62 */
        FINISH();
        a = orc_builder_add(b, k, kl, kv->ts[i], v, vl);
        if (a != 1) { rc = ORC_E_INVAL; goto done; }
      }
    }
    if (!orc_builder_is_empty(b)) FINISH();                        /* build() :74 */
  }
#undef FINISH
  if (nb < blk_cap) blk_off[nb] = pos;
  if (nb + 1 > blk_cap) rc = ORC_E_CAPACITY;
done:
  *nblk = nb; *nbytes = pos;
  free(scratch);
  orc_builder_free(b);
  return rc;
}

int orc_decode_blocks(const uint8_t* blocks, const uint64_t* blk_off, uint64_t nblk,
                      orc_kv* out, uint64_t entry_cap, uint64_t key_cap, uint64_t val_cap,
                      uint64_t* n_out, uint64_t* kbytes, uint64_t* vbytes) {
  uint64_t n = 0, K = 0, V = 0;
  int rc = ORC_OK;
  for (uint64_t b = 0; b < nblk; ++b) {
    const uint8_t* blk = blocks + blk_off[b];
    size_t len = blk_off[b + 1] - blk_off[b];
    if (len < 2) return ORC_E_MALFORMED;
    size_t cnt = get_u16(blk + len - 2);
    for (size_t i = 0; i < cnt; ++i) {
      orc_entry e; const uint8_t* fk; uint32_t fkl;
      int r = orc_block_entry(blk, len, i, &e, &fk, &fkl);
      if (r) return r;
      uint32_t kl = e.prefix + e.suffix;
      if (n < entry_cap && K + kl <= key_cap && V + e.vlen <= val_cap) {
        out->key_off[n] = (uint32_t)K;
        out->val_off[n] = (uint32_t)V;
        out->ts[n] = e.ts;
        memcpy(out->keys + K, fk, e.prefix);
        memcpy(out->keys + K + e.prefix, e.key_suffix, e.suffix);
        memcpy(out->vals + V, e.value, e.vlen);
      } else {
        rc = ORC_E_CAPACITY;
      }
      ++n; K += kl; V += e.vlen;
    }
  }
  if (K > 0xFFFFFFFFull || V > 0xFFFFFFFFull) return ORC_E_OVERFLOW;
  if (n > entry_cap) rc = ORC_E_CAPACITY;
  if (rc == ORC_OK && out->key_off) { out->key_off[n] = (uint32_t)K; out->val_off[n] = (uint32_t)V; }
  out->n = n;
  *n_out = n; *kbytes = K; *vbytes = V;
  return rc;
}

int orc_segment_like_compaction(const orc_kv* kv, size_t block_size, uint64_t target,
                                uint32_t* seg_start, uint64_t seg_cap, uint64_t* nseg) {
  orc_builder* b = orc_builder_new(block_size);
  uint64_t est = 0;   /* SsTableBuilder::estimate_size() == data.len() (blocks + CRCs) */
  uint64_t g = 0;
  if (kv->n == 0) { *nseg = 0; if (seg_cap) seg_start[0] = 0; orc_builder_free(b); return ORC_OK; }
  if (seg_cap) seg_start[0] = 0;
  for (uint64_t i = 0; i < kv->n; ++i) {
    const uint8_t* k = kv->keys + kv->key_off[i];
    size_t kl = kv->key_off[i + 1] - kv->key_off[i];
    int same_as_last = 0;
    if (i > 0) {
      const uint8_t* pk = kv->keys + kv->key_off[i - 1];
      size_t pl = kv->key_off[i] - kv->key_off[i - 1];
      same_as_last = (pl == kl && memcmp(pk, k, kl) == 0);
    }
    if (i > 0 && est >= target && !same_as_last) {           /* compact.rs:279 */
      ++g;
      if (g < seg_cap) seg_start[g] = (uint32_t)i;
      est = 0;
      orc_builder_free(b);
      b = orc_builder_new(block_size);
    }
    const uint8_t* v = kv->vals + kv->val_off[i];
    size_t vl = kv->val_off[i + 1] - kv->val_off[i];
    int a = orc_builder_add(b, k, kl, kv->ts[i], v, vl);
    if (a < 0) { orc_builder_free(b); return a; }
    if (a == 0) {                                            /* finish_block: +block +crc */
      est += orc_builder_estimated_size(b) + 4;
      size_t l;
      uint8_t* tmp = (uint8_t*)malloc(orc_builder_estimated_size(b));
      orc_builder_finish(b, tmp, orc_builder_estimated_size(b), &l);
      free(tmp);
      orc_builder_add(b, k, kl, kv->ts[i], v, vl);
    }
  }
  ++g;
  if (g < seg_cap) seg_start[g] = (uint32_t)kv->n;
  *nseg = g;
  orc_builder_free(b);
  return g + 1 <= seg_cap ? ORC_OK : ORC_E_CAPACITY;
}

/* ------------------------------------------------------------------ merge */
/* MergeIterator (src/iterators/merge_iterator.rs:59-184) over nrun sorted runs of one KV stream,
 * run r = entries [run_start[r], run_start[r+1]), run 0 the highest priority.  The BinaryHeap of
 * HeapWrapper(idx, iter) orders by (user key, idx) reversed (:21-33, key.rs:63-81 ignores ts), so
 * it is kept here as a binary min-heap on (head key, run index). */
typedef struct { const orc_kv* kv; uint64_t* pos; const uint32_t* end; } merge_ctx;

static int head_cmp(const merge_ctx* m, uint32_t a, uint32_t b) {
  const orc_kv* kv = m->kv;
  uint64_t ia = m->pos[a], ib = m->pos[b];
  int c = key_cmp(kv->keys + kv->key_off[ia], kv->key_off[ia + 1] - kv->key_off[ia],
                  kv->keys + kv->key_off[ib], kv->key_off[ib + 1] - kv->key_off[ib]);
  if (c) return c;
  return a < b ? -1 : (a > b ? 1 : 0);
}
static void sift_down(const merge_ctx* m, uint32_t* h, uint32_t n, uint32_t i) {
  for (;;) {
    uint32_t l = 2 * i + 1, r = l + 1, s = i;
    if (l < n && head_cmp(m, h[l], h[s]) < 0) s = l;
    if (r < n && head_cmp(m, h[r], h[s]) < 0) s = r;
    if (s == i) return;
    uint32_t t = h[i]; h[i] = h[s]; h[s] = t; i = s;
  }
}
static void sift_up(const merge_ctx* m, uint32_t* h, uint32_t i) {
  while (i) {
    uint32_t p = (i - 1) / 2;
    if (head_cmp(m, h[i], h[p]) >= 0) return;
    uint32_t t = h[i]; h[i] = h[p]; h[p] = t; i = p;
  }
}
static int same_key(const orc_kv* kv, uint64_t a, uint64_t b) {
  uint32_t al = kv->key_off[a + 1] - kv->key_off[a], bl = kv->key_off[b + 1] - kv->key_off[b];
  return al == bl && memcmp(kv->keys + kv->key_off[a], kv->keys + kv->key_off[b], al) == 0;
}

int orc_merge_runs(const orc_kv* in, const uint32_t* run_start, uint32_t nrun, uint32_t* src,
                   uint64_t src_cap, uint64_t* n_out) {
  uint64_t* pos = (uint64_t*)malloc((nrun + 1) * sizeof(uint64_t));
  uint32_t* heap = (uint32_t*)malloc((nrun + 1) * sizeof(uint32_t));
  merge_ctx m = {in, pos, run_start + 1};
  uint32_t hn = 0, cur = 0;
  int have = 0;
  uint64_t n = 0;
  for (uint32_t r = 0; r < nrun; ++r) {          /* create, :93-100: push the valid iterators */
    pos[r] = run_start[r];
    if (run_start[r] < run_start[r + 1]) { heap[hn] = r; sift_up(&m, heap, hn); ++hn; }
  }
  if (hn) { cur = heap[0]; heap[0] = heap[--hn]; sift_down(&m, heap, hn, 0); have = 1; }
  while (have) {                                  /* is_valid, :123-128 */
    if (n < src_cap) src[n] = (uint32_t)pos[cur];
    ++n;
    /* next(), :130-169: advance every heap iterator whose head equals the current key */
    while (hn && same_key(in, pos[heap[0]], pos[cur])) {
      uint32_t t = heap[0];
      if (++pos[t] < run_start[t + 1]) sift_down(&m, heap, hn, 0);
      else { heap[0] = heap[--hn]; sift_down(&m, heap, hn, 0); }
    }
    if (++pos[cur] >= run_start[cur + 1]) {       /* :156-161 */
      if (hn) { cur = heap[0]; heap[0] = heap[--hn]; sift_down(&m, heap, hn, 0); }
      else have = 0;
      continue;
    }
    if (hn && head_cmp(&m, cur, heap[0]) > 0) {   /* :163-167: swap with the top */
      uint32_t t = heap[0]; heap[0] = cur; cur = t; sift_down(&m, heap, hn, 0);
    }
  }
  free(pos); free(heap);
  *n_out = n;
  return n <= src_cap ? ORC_OK : ORC_E_CAPACITY;
}

/* compact_generate_sst (src/compact.rs:223-311) over a merged stream given as src[0..n) indices
 * into `in`: the keep/drop rules (:239-276), the SST rotation (:278-289) and SsTableBuilder::add
 * (table/builder.rs:48-65) with estimate_size() = data.len() (finished blocks + 4-B CRC each,
 * :105-123).  Outputs the blocks packed (no CRC), blk_off[nblk+1], for every SST its first
 * block sst_blk[s] and its first kept entry sst_ent[s] (nsst+1 values each), and kept[] = the
 * src positions handed to SsTableBuilder::add.  If nothing is kept the reference panics
 * building an empty SST; here nsst = 0. */
int orc_compact(const orc_kv* in, const uint32_t* src, uint64_t n, uint64_t watermark, int bottom,
                const uint8_t* const* prefixes, const size_t* prefix_len, uint32_t nprefix,
                size_t block_size, uint64_t target, uint8_t* out, uint64_t out_cap, uint64_t* blk_off,
                uint64_t blk_cap, uint32_t* sst_blk, uint32_t* sst_ent, uint64_t sst_cap, uint32_t* kept,
                uint64_t kept_cap, uint64_t* nblk_out, uint64_t* nbytes_out, uint64_t* nsst_out,
                uint64_t* nkept_out) {
  orc_builder* b = NULL;
  uint64_t data_len = 0, nb = 0, pos = 0, nsst = 0, nk = 0;
  const uint8_t* last_key = NULL;
  size_t last_len = 0;
  int first_below = 0, rc = ORC_OK;
  size_t scratch_cap = 1 << 16;
  uint8_t* scratch = (uint8_t*)malloc(scratch_cap);
#define EMIT_BLOCK()                                                                   \
  do {                                                                                  \
    size_t need = orc_builder_estimated_size(b), l;                                     \
    if (need > scratch_cap) { scratch_cap = need; scratch = (uint8_t*)realloc(scratch, need); } \
    orc_builder_finish(b, scratch, scratch_cap, &l);                                    \
    if (nb < blk_cap) blk_off[nb] = pos;                                                \
    if (pos + l <= out_cap) memcpy(out + pos, scratch, l); else rc = ORC_E_CAPACITY;    \
    pos += l; ++nb; data_len += l + 4;                                                  \
  } while (0)
  for (uint64_t j = 0; j < n; ++j) {
    uint64_t i = src[j];
    const uint8_t* k = in->keys + in->key_off[i];
    size_t kl = in->key_off[i + 1] - in->key_off[i];
    const uint8_t* v = in->vals + in->val_off[i];
    size_t vl = in->val_off[i + 1] - in->val_off[i];
    uint64_t ts = in->ts[i];
    if (!b) {                                                   /* :235-237 */
      b = orc_builder_new(block_size);
      data_len = 0;
      if (nsst < sst_cap) { sst_blk[nsst] = (uint32_t)nb; sst_ent[nsst] = (uint32_t)nk; }
      ++nsst;
    }
    int same = last_key && last_len == kl && memcmp(last_key, k, kl) == 0;   /* :239 */
    if (!same) first_below = 1;
    if (bottom && !same && ts <= watermark && vl == 0) {       /* :244-254 */
      last_key = k; last_len = kl; first_below = 0;
      continue;
    }
    if (ts <= watermark) {                                      /* :256-276 */
      if (same && !first_below) continue;
      first_below = 0;
      int drop = 0;
      for (uint32_t f = 0; f < nprefix && !drop; ++f)
        drop = prefix_len[f] <= kl && memcmp(prefixes[f], k, prefix_len[f]) == 0;
      if (drop) continue;
    }
    if (data_len >= target && !same) {                          /* :278-289 */
      if (!orc_builder_is_empty(b)) EMIT_BLOCK();               /* build() -> finish_block */
      data_len = 0;
      if (nsst < sst_cap) { sst_blk[nsst] = (uint32_t)nb; sst_ent[nsst] = (uint32_t)nk; }
      ++nsst;
    }
    int a = orc_builder_add(b, k, kl, ts, v, vl);               /* SsTableBuilder::add */
    if (a < 0) { rc = a; goto done; }
    if (a == 0) {
      EMIT_BLOCK();                                             /* finish_block */
      if (orc_builder_add(b, k, kl, ts, v, vl) != 1) { rc = ORC_E_INVAL; goto done; }
    }
    if (nk < kept_cap) kept[nk] = (uint32_t)j;
    ++nk;
    if (!same) { last_key = k; last_len = kl; }                 /* :294-297 */
  }
  if (b && !orc_builder_is_empty(b)) EMIT_BLOCK();
  if (b && nk == 0) nsst = 0;   /* the reference would panic: build() of an empty SST */
#undef EMIT_BLOCK
  if (nb < blk_cap) blk_off[nb] = pos;
  if (nsst < sst_cap) { sst_blk[nsst] = (uint32_t)nb; sst_ent[nsst] = (uint32_t)nk; }
  if (nb + 1 > blk_cap || nsst + 1 > sst_cap || nk > kept_cap) rc = rc ? rc : ORC_E_CAPACITY;
done:
  *nblk_out = nb; *nbytes_out = pos; *nsst_out = nsst; *nkept_out = nk;
  free(scratch);
  orc_builder_free(b);
  return rc;
}

/* compact_generate_sst resumed from a range's carry-in (see the header).  The loop is the one of
 * orc_compact with the rules already applied (ext holds the entries handed to SsTableBuilder::add;
 * "same as last key" is then the previous ext entry's key): before adding entry e, a new SST starts
 * when data_len >= target and key(e) != key(e-1) (:278-289); adding e finishes the open block when
 * BlockBuilder rejects it (builder.rs:55-64), data_len += block + 4.  Entry p itself was already
 * checked with the data before its block's predecessor was finished. */
int orc_shard_rotation(const orc_kv* ext, uint64_t m, int last, uint64_t p, uint64_t d0, size_t block_size,
                       uint64_t target, uint32_t* seg_start, uint64_t seg_cap, uint64_t* nseg, uint64_t* p_out,
                       uint64_t* d_out) {
  return orc_shard_rotation_ex(ext, NULL, m, last, p, d0, block_size, target, seg_start, seg_cap, nseg, p_out, d_out);
}

/* The same with the loop's own same_as_last_key per ext entry (same != NULL): a two-level
 * (TwoMergeIterator) compaction, where a dropped bottom-level tombstone moves last_key
 * (src/compact.rs:244-254) so that "same" is not the previous kept entry's key. */
int orc_shard_rotation_ex(const orc_kv* ext, const uint8_t* same_in, uint64_t m, int last, uint64_t p, uint64_t d0,
                          size_t block_size, uint64_t target, uint32_t* seg_start, uint64_t seg_cap, uint64_t* nseg,
                          uint64_t* p_out, uint64_t* d_out) {
  const uint64_t n = ext->n;
  uint64_t g = 0, data_len = d0;
  *nseg = 0;
  if (p >= m) { *p_out = p - m; *d_out = d0; return ORC_OK; }
  if (m > n) return ORC_E_INVAL;
  orc_builder* b = orc_builder_new(block_size);
  if (seg_cap) seg_start[0] = (uint32_t)p;
  int rc = ORC_E_INVAL;   /* the halo ran out before the first event at or after m */
  for (uint64_t e = p; e < n; ++e) {
    const uint8_t* k = ext->keys + ext->key_off[e];
    size_t kl = ext->key_off[e + 1] - ext->key_off[e];
    int same = same_in ? same_in[e] != 0 : (e > 0 && same_key(ext, e - 1, e));
    if (e > p && data_len >= target && !same) {              /* a new SST starts at e */
      if (e >= m) { *p_out = e - m; *d_out = 0; rc = ORC_OK; break; }
      ++g;
      if (g < seg_cap) seg_start[g] = (uint32_t)e;
      data_len = 0;
      orc_builder_free(b);
      b = orc_builder_new(block_size);
    }
    const uint8_t* v = ext->vals + ext->val_off[e];
    size_t vl = ext->val_off[e + 1] - ext->val_off[e];
    int a = orc_builder_add(b, k, kl, ext->ts[e], v, vl);
    if (a < 0) { rc = a; break; }
    if (a == 0) {                                             /* finish_block: a block starts at e */
      data_len += orc_builder_estimated_size(b) + 4;
      if (e >= m) { *p_out = e - m; *d_out = data_len; rc = ORC_OK; break; }
      orc_builder_free(b);
      b = orc_builder_new(block_size);
      orc_builder_add(b, k, kl, ext->ts[e], v, vl);
    }
  }
  if (rc == ORC_E_INVAL && last) {                            /* the stream ended inside the range's SST */
    uint64_t end = n;
    *p_out = end - m; *d_out = 0; rc = ORC_OK;
  }
  orc_builder_free(b);
  if (rc) return rc;
  ++g;
  if (g < seg_cap) seg_start[g] = (uint32_t)(m + *p_out);
  *nseg = g;
  return g + 1 <= seg_cap ? ORC_OK : ORC_E_CAPACITY;
}

/* ------------------------------------------------------------------ crc32 */
uint32_t orc_crc32(const uint8_t* p, size_t n) {
  static uint32_t table[256];
  static int init = 0;
  if (!init) {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      table[i] = c;
    }
    init = 1;
  }
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) c = table[(c ^ p[i]) & 0xFF] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}
