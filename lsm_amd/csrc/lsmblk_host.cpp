// lsmblk_host.cpp -- per-entry half of the C ABI (include/lsmblk.h): BlockBuilder, Block and
// BlockIterator semantics of CrystalAnalyst/Lsm, synchronous on the host.
//
// Reference: src/block/builder.rs:8-89, src/block.rs:7-34, src/block/iterator.rs:11-139,
// src/key.rs:63-81 (ts-agnostic key order).  Unlike the reference, builder storage is
// reserved up front to the block size (the reference's Vec::new() doubles ~10 times per
// 4 KiB block), and errors are status codes instead of panics.
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "lsmblk.h"

namespace {

inline void be16(uint8_t* p, uint32_t v) {
  p[0] = uint8_t(v >> 8);
  p[1] = uint8_t(v);
}
inline uint32_t rd16(const uint8_t* p) { return (uint32_t(p[0]) << 8) | p[1]; }
inline uint64_t rd64(const uint8_t* p) {
  uint64_t v;
  std::memcpy(&v, p, 8);
  return __builtin_bswap64(v);
}

}  // namespace

struct lsmblk_builder {
  std::vector<uint8_t> data;        // builder.rs:10
  std::vector<uint16_t> offsets;    // builder.rs:11
  std::vector<uint8_t> first_key;   // builder.rs:13 (ts of the first key is never read back)
  size_t block_size;                // builder.rs:14
};

struct lsmblk_block {
  std::vector<uint8_t> data;        // block.rs:8
  std::vector<uint16_t> offsets;    // block.rs:9
  std::atomic<int> refs{1};         // Arc<Block>
};

struct lsmblk_iter {
  lsmblk_block* block;              // iterator.rs:12
  size_t idx = 0;                   // :14
  std::vector<uint8_t> first_key;   // :15
  uint64_t first_ts = 0;
  size_t vbegin = 0, vend = 0;      // :16 value_range
  std::vector<uint8_t> key;         // :18 (empty == invalid)
  uint64_t ts = 0;
};

extern "C" {

int lsmblk_abi_version(void) { return LSMBLK_ABI_VERSION; }

const char* lsmblk_strerror(int s) {
  switch (s) {
    case LSMBLK_OK: return "ok";
    case LSMBLK_E_INVAL: return "invalid argument";
    case LSMBLK_E_MALFORMED: return "malformed block";
    case LSMBLK_E_CAPACITY: return "output capacity exceeded";
    case LSMBLK_E_NOMEM: return "out of memory";
    case LSMBLK_E_HIP: return "HIP runtime error";
    case LSMBLK_E_TIMEOUT: return "device look-back timeout";
    case LSMBLK_E_OVERFLOW: return "batch exceeds u32 KV-stream offsets";
    case LSMBLK_E_INTERNAL: return "device self-check failed";
    case LSMBLK_E_CHECKSUM: return "block checksum mismatched";
    default: return "unknown status";
  }
}

int lsmblk_stats_status(uint64_t f) {
  if (f & LSMBLK_ERR_TIMEOUT) return LSMBLK_E_TIMEOUT;
  if (f & LSMBLK_ERR_INTERNAL) return LSMBLK_E_INTERNAL;
  if (f & LSMBLK_ERR_SEGMENTS) return LSMBLK_E_INVAL;
  if (f & LSMBLK_ERR_EMPTY_KEY) return LSMBLK_E_INVAL;
  if (f & LSMBLK_ERR_CHECKSUM) return LSMBLK_E_CHECKSUM;
  if (f & LSMBLK_ERR_MALFORMED) return LSMBLK_E_MALFORMED;
  if (f & LSMBLK_ERR_OVERFLOW) return LSMBLK_E_OVERFLOW;
  if (f & LSMBLK_ERR_CAPACITY) return LSMBLK_E_CAPACITY;
  return LSMBLK_OK;
}

// ---------------------------------------------------------------- builder
lsmblk_builder* lsmblk_builder_new(size_t block_size) {
  auto* b = new (std::nothrow) lsmblk_builder();
  if (!b) return nullptr;
  b->block_size = block_size;
  b->data.reserve(block_size < (1u << 20) ? block_size : (1u << 20));
  return b;
}

void lsmblk_builder_free(lsmblk_builder* b) { delete b; }

int lsmblk_builder_is_empty(const lsmblk_builder* b) { return b->offsets.empty() ? 1 : 0; }

size_t lsmblk_builder_estimated_size(const lsmblk_builder* b) {
  return b->data.size() + 2 * b->offsets.size() + 2;  // builder.rs:48-50
}

int lsmblk_builder_add(lsmblk_builder* b, const uint8_t* key, size_t klen, uint64_t ts,
                       const uint8_t* val, size_t vlen, int* accepted) {
  if (!b || !accepted || klen == 0) return LSMBLK_E_INVAL;  // builder.rs:55
  // builder.rs:56-60: the size test uses the FULL key length (raw_len = klen + 8).
  if (lsmblk_builder_estimated_size(b) + klen + 8 + vlen + 6 > b->block_size && !b->offsets.empty()) {
    *accepted = 0;
    return LSMBLK_OK;
  }
  size_t p = 0;  // common_prefix vs first key, builder.rs:19-33
  const size_t m = klen < b->first_key.size() ? klen : b->first_key.size();
  while (p < m && b->first_key[p] == key[p]) ++p;
  const size_t s = klen - p;
  const size_t at = b->data.size();
  b->offsets.push_back(uint16_t(at));  // `as u16`, :61
  b->data.resize(at + 14 + s + vlen);
  uint8_t* d = b->data.data() + at;
  be16(d, uint32_t(p));                // :63
  be16(d + 2, uint32_t(s));            // :64
  std::memcpy(d + 4, key + p, s);      // :65
  uint64_t tbe = __builtin_bswap64(ts);
  std::memcpy(d + 4 + s, &tbe, 8);     // :66
  be16(d + 12 + s, uint32_t(vlen));    // :67
  if (vlen) std::memcpy(d + 14 + s, val, vlen);  // :68
  if (b->first_key.empty()) b->first_key.assign(key, key + klen);  // :69-71
  *accepted = 1;
  return LSMBLK_OK;
}

static void reset_builder(lsmblk_builder* b) {
  b->data.clear();
  b->offsets.clear();
  b->first_key.clear();
}

int lsmblk_builder_finish(lsmblk_builder* b, uint8_t* out, size_t cap, size_t* len) {
  if (!b || !len) return LSMBLK_E_INVAL;
  if (b->offsets.empty()) return LSMBLK_E_INVAL;  // builder.rs:82-83
  const size_t n = b->offsets.size(), dl = b->data.size(), total = dl + 2 * n + 2;
  *len = total;
  if (!out || cap < total) return LSMBLK_E_CAPACITY;
  std::memcpy(out, b->data.data(), dl);  // block.rs:15
  for (size_t i = 0; i < n; ++i) be16(out + dl + 2 * i, b->offsets[i]);  // :17-19
  be16(out + dl + 2 * n, uint32_t(n));  // :20
  reset_builder(b);
  return LSMBLK_OK;
}

int lsmblk_builder_build(lsmblk_builder* b, lsmblk_block** out) {
  if (!b || !out) return LSMBLK_E_INVAL;
  if (b->offsets.empty()) return LSMBLK_E_INVAL;
  auto* blk = new (std::nothrow) lsmblk_block();
  if (!blk) return LSMBLK_E_NOMEM;
  blk->data.swap(b->data);
  blk->offsets.swap(b->offsets);
  reset_builder(b);
  *out = blk;
  return LSMBLK_OK;
}

// ---------------------------------------------------------------- block
int lsmblk_block_decode(const uint8_t* buf, size_t len, lsmblk_block** out) {
  if (!out || (!buf && len)) return LSMBLK_E_INVAL;
  if (len < 2) return LSMBLK_E_MALFORMED;  // block.rs:25 would panic
  const size_t n = rd16(buf + len - 2);
  if (2 + 2 * n > len) return LSMBLK_E_MALFORMED;  // :26 underflow
  const size_t data_end = len - 2 - 2 * n;
  auto* blk = new (std::nothrow) lsmblk_block();
  if (!blk) return LSMBLK_E_NOMEM;
  blk->data.assign(buf, buf + data_end);  // :32
  blk->offsets.resize(n);
  for (size_t i = 0; i < n; ++i) blk->offsets[i] = uint16_t(rd16(buf + data_end + 2 * i));  // :27-31
  *out = blk;
  return LSMBLK_OK;
}

size_t lsmblk_block_encoded_len(const lsmblk_block* blk) {
  return blk->data.size() + 2 * blk->offsets.size() + 2;
}

int lsmblk_block_encode(const lsmblk_block* blk, uint8_t* out, size_t cap, size_t* len) {
  if (!blk || !len) return LSMBLK_E_INVAL;
  const size_t total = lsmblk_block_encoded_len(blk);
  *len = total;
  if (!out || cap < total) return LSMBLK_E_CAPACITY;
  const size_t dl = blk->data.size(), n = blk->offsets.size();
  std::memcpy(out, blk->data.data(), dl);
  for (size_t i = 0; i < n; ++i) be16(out + dl + 2 * i, blk->offsets[i]);
  be16(out + dl + 2 * n, uint32_t(n));
  return LSMBLK_OK;
}

int lsmblk_block_data(const lsmblk_block* blk, const uint8_t** data, size_t* len) {
  if (!blk || !data || !len) return LSMBLK_E_INVAL;
  *data = blk->data.data();
  *len = blk->data.size();
  return LSMBLK_OK;
}

int lsmblk_block_offsets(const lsmblk_block* blk, const uint16_t** offsets, size_t* n) {
  if (!blk || !offsets || !n) return LSMBLK_E_INVAL;
  *offsets = blk->offsets.data();
  *n = blk->offsets.size();
  return LSMBLK_OK;
}

void lsmblk_block_free(lsmblk_block* blk) {
  if (blk && blk->refs.fetch_sub(1) == 1) delete blk;
}

// ---------------------------------------------------------------- iterator
// get_first_key, iterator.rs:23-34: entry at data position 0; skip u16 prefix, u16 key_len,
// key, u64 ts.
static int first_key(lsmblk_iter* it) {
  const auto& d = it->block->data;
  it->first_key.clear();
  if (it->block->offsets.empty()) return LSMBLK_OK;
  if (d.size() < 4) return LSMBLK_E_MALFORMED;
  const size_t s = rd16(d.data() + 2);
  if (4 + s + 8 > d.size()) return LSMBLK_E_MALFORMED;
  it->first_key.assign(d.begin() + 4, d.begin() + 4 + s);
  it->first_ts = rd64(d.data() + 4 + s);
  return LSMBLK_OK;
}

// seek_to_offset, iterator.rs:125-139, corrected: ts is skipped and kept.
static int seek_to_offset(lsmblk_iter* it, size_t off) {
  const auto& d = it->block->data;
  if (off + 4 > d.size()) return LSMBLK_E_MALFORMED;
  const size_t p = rd16(d.data() + off), s = rd16(d.data() + off + 2);
  if (off + 4 + s + 10 > d.size() || p > it->first_key.size()) return LSMBLK_E_MALFORMED;
  const size_t vlen = rd16(d.data() + off + 12 + s);
  if (off + 14 + s + vlen > d.size()) return LSMBLK_E_MALFORMED;
  it->key.assign(it->first_key.begin(), it->first_key.begin() + p);
  it->key.insert(it->key.end(), d.begin() + off + 4, d.begin() + off + 4 + s);
  it->ts = rd64(d.data() + off + 4 + s);
  it->vbegin = off + 14 + s;
  it->vend = it->vbegin + vlen;
  return LSMBLK_OK;
}

// seek_to, iterator.rs:110-121.
static int seek_to(lsmblk_iter* it, size_t idx) {
  if (idx >= it->block->offsets.size()) {
    it->key.clear();
    it->vbegin = it->vend = 0;
    it->idx = idx;
    return LSMBLK_OK;
  }
  int rc = seek_to_offset(it, it->block->offsets[idx]);
  if (rc) {
    it->key.clear();
    return rc;
  }
  it->idx = idx;
  return LSMBLK_OK;
}

static int key_cmp(const std::vector<uint8_t>& a, const uint8_t* b, size_t bl) {
  const size_t m = a.size() < bl ? a.size() : bl;
  const int c = m ? std::memcmp(a.data(), b, m) : 0;
  if (c) return c;
  return a.size() < bl ? -1 : (a.size() > bl ? 1 : 0);
}

int lsmblk_iter_seek_to_first(lsmblk_iter* it) { return it ? seek_to(it, 0) : LSMBLK_E_INVAL; }

int lsmblk_iter_next(lsmblk_iter* it) { return it ? seek_to(it, it->idx + 1) : LSMBLK_E_INVAL; }

// seek_to_key, iterator.rs:80-94: first entry whose key >= target (ts-agnostic, key.rs:77-81).
int lsmblk_iter_seek_to_key(lsmblk_iter* it, const uint8_t* key, size_t klen) {
  if (!it || (!key && klen)) return LSMBLK_E_INVAL;
  size_t lo = 0, hi = it->block->offsets.size();
  while (lo < hi) {
    const size_t mid = lo + (hi - lo) / 2;
    int rc = seek_to(it, mid);
    if (rc) return rc;
    const int c = key_cmp(it->key, key, klen);
    if (c < 0) lo = mid + 1;
    else if (c > 0) hi = mid;
    else return LSMBLK_OK;
  }
  return seek_to(it, lo);
}

static int make_iter(lsmblk_block* blk, lsmblk_iter** out) {
  if (!blk || !out) return LSMBLK_E_INVAL;
  auto* it = new (std::nothrow) lsmblk_iter();
  if (!it) return LSMBLK_E_NOMEM;
  blk->refs.fetch_add(1);
  it->block = blk;
  int rc = first_key(it);
  if (rc) {
    lsmblk_iter_free(it);
    return rc;
  }
  *out = it;
  return LSMBLK_OK;
}

int lsmblk_iter_create_and_seek_to_first(lsmblk_block* blk, lsmblk_iter** out) {
  int rc = make_iter(blk, out);
  if (rc) return rc;
  rc = lsmblk_iter_seek_to_first(*out);
  if (rc) {
    lsmblk_iter_free(*out);
    *out = nullptr;
  }
  return rc;
}

int lsmblk_iter_create_and_seek_to_key(lsmblk_block* blk, const uint8_t* key, size_t klen,
                                       lsmblk_iter** out) {
  int rc = make_iter(blk, out);
  if (rc) return rc;
  rc = lsmblk_iter_seek_to_key(*out, key, klen);
  if (rc) {
    lsmblk_iter_free(*out);
    *out = nullptr;
  }
  return rc;
}

int lsmblk_iter_is_valid(const lsmblk_iter* it) { return it && !it->key.empty() ? 1 : 0; }

int lsmblk_iter_key(const lsmblk_iter* it, const uint8_t** key, size_t* klen, uint64_t* ts) {
  if (!it || !key || !klen) return LSMBLK_E_INVAL;
  *key = it->key.data();
  *klen = it->key.size();
  if (ts) *ts = it->ts;
  return LSMBLK_OK;
}

int lsmblk_iter_value(const lsmblk_iter* it, const uint8_t** val, size_t* vlen) {
  if (!it || !val || !vlen) return LSMBLK_E_INVAL;
  *val = it->block->data.data() + it->vbegin;
  *vlen = it->vend - it->vbegin;
  return LSMBLK_OK;
}

void lsmblk_iter_free(lsmblk_iter* it) {
  if (!it) return;
  lsmblk_block_free(it->block);
  delete it;
}

}  // extern "C"

// ---------------------------------------------------------------- memtable (flush source)
// MemTable (src/mem_table.rs:55-158): a crossbeam SkipMap<KeyBytes, Bytes> whose key order
// ignores the ts (src/key.rs:63-81), so a put of a key that is present replaces the entry (key,
// ts and value); flush (:131-136) walks the map in key order into SsTableBuilder::add.  Here an
// ordered map of byte strings (unsigned lexicographic order) held on the host: the memtable is
// a random-insert structure; what it feeds -- the flush batch -- goes to the device encoder.
#include <map>
#include <mutex>
#include <string>

struct lsmblk_memtable {
  struct Ent {
    uint64_t ts;
    std::string val;
  };
  std::map<std::string, Ent> map;
  size_t approximate_size = 0;
  std::mutex mu;
};

extern "C" {

lsmblk_memtable* lsmblk_memtable_new(void) { return new (std::nothrow) lsmblk_memtable(); }
void lsmblk_memtable_free(lsmblk_memtable* m) { delete m; }

int lsmblk_memtable_put(lsmblk_memtable* m, const uint8_t* key, size_t klen, uint64_t ts, const uint8_t* val,
                        size_t vlen) {
  if (!m || (klen && !key) || (vlen && !val)) return LSMBLK_E_INVAL;
  std::lock_guard<std::mutex> g(m->mu);
  std::string k(reinterpret_cast<const char*>(key), klen);
  auto& e = m->map[k];  // insert replaces the entry with an equal key (mem_table.rs:120-123)
  e.ts = ts;
  e.val.assign(reinterpret_cast<const char*>(val), vlen);
  m->approximate_size += klen + 8 + vlen;  // key.raw_len() + value.len(), :119,124-125
  return LSMBLK_OK;
}

int lsmblk_memtable_get(lsmblk_memtable* m, const uint8_t* key, size_t klen, const uint8_t** val, size_t* vlen,
                        uint64_t* ts) {
  if (!m || (klen && !key) || !val || !vlen) return LSMBLK_E_INVAL;
  std::lock_guard<std::mutex> g(m->mu);
  auto it = m->map.find(std::string(reinterpret_cast<const char*>(key), klen));
  if (it == m->map.end()) {
    *val = nullptr;
    *vlen = 0;
    return 0;
  }
  *val = reinterpret_cast<const uint8_t*>(it->second.val.data());
  *vlen = it->second.val.size();
  if (ts) *ts = it->second.ts;
  return 1;
}

int lsmblk_memtable_get_copy(lsmblk_memtable* m, const uint8_t* key, size_t klen, uint8_t* val, size_t cap,
                             size_t* vlen, uint64_t* ts) {
  if (!m || (klen && !key) || !vlen || (cap && !val)) return LSMBLK_E_INVAL;
  std::lock_guard<std::mutex> g(m->mu);
  auto it = m->map.find(std::string(reinterpret_cast<const char*>(key), klen));
  if (it == m->map.end()) {
    *vlen = 0;
    return 0;
  }
  const std::string& v = it->second.val;
  *vlen = v.size();
  if (ts) *ts = it->second.ts;
  if (v.size() > cap) return LSMBLK_E_CAPACITY;
  if (!v.empty()) std::memcpy(val, v.data(), v.size());  // under the lock: a put may replace it
  return 1;
}

size_t lsmblk_memtable_len(lsmblk_memtable* m) {
  if (!m) return 0;
  std::lock_guard<std::mutex> g(m->mu);
  return m->map.size();
}

size_t lsmblk_memtable_approximate_size(lsmblk_memtable* m) {
  if (!m) return 0;
  std::lock_guard<std::mutex> g(m->mu);
  return m->approximate_size;
}

int lsmblk_memtable_flush(lsmblk_memtable* m, uint8_t* keys, uint32_t* key_off, uint8_t* vals, uint32_t* val_off,
                          uint64_t* ts, uint64_t entry_cap, uint64_t key_cap, uint64_t val_cap, uint64_t* n,
                          uint64_t* kbytes, uint64_t* vbytes) {
  if (!m || !n || !kbytes || !vbytes) return LSMBLK_E_INVAL;
  std::lock_guard<std::mutex> g(m->mu);
  uint64_t N = m->map.size(), K = 0, V = 0;
  for (const auto& kv : m->map) {
    K += kv.first.size();
    V += kv.second.val.size();
  }
  *n = N;
  *kbytes = K;
  *vbytes = V;
  if (K > 0xFFFFFFFFull || V > 0xFFFFFFFFull) return LSMBLK_E_OVERFLOW;
  if (N > entry_cap || K > key_cap || V > val_cap || !key_off || !val_off || (N && !ts)) return LSMBLK_E_CAPACITY;
  uint64_t i = 0, kp = 0, vp = 0;
  for (const auto& kv : m->map) {  // key order (mem_table.rs:132-134)
    key_off[i] = uint32_t(kp);
    val_off[i] = uint32_t(vp);
    ts[i] = kv.second.ts;
    if (!kv.first.empty()) std::memcpy(keys + kp, kv.first.data(), kv.first.size());
    if (!kv.second.val.empty()) std::memcpy(vals + vp, kv.second.val.data(), kv.second.val.size());
    kp += kv.first.size();
    vp += kv.second.val.size();
    ++i;
  }
  key_off[N] = uint32_t(kp);
  val_off[N] = uint32_t(vp);
  return LSMBLK_OK;
}

}  // extern "C"
