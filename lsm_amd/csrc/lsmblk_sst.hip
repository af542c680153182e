// lsmblk_sst.hip -- SST container of the batch C ABI (include/lsmblk.h), gfx950 (SURVEY.md §8 f, row 3):
//
//   lsmblk_sst_files_batch   whole SST files, as SsTableBuilder::build writes them
//                            (src/table/builder.rs:68-98), for every SST of an encode / compaction:
//     data section   every block followed by its crc32fast as a BE u32   (finish_block, :112-123)
//     meta section   BlockMeta::encode_block_meta                          (src/table.rs:29-63)
//     u32 BE meta_offset
//     bloom          filter | k | BE u32 crc32fast(filter | k)             (src/table/bloom.rs:63-69)
//     u32 BE bloom_offset
//   The bloom filter holds farmhash::fingerprint32 of every key handed to SsTableBuilder::add
//   (:53), bits per key Bloom::bloom_bits_per_key(n, 0.01), k = bits_per_key * 0.69 (:72-101).
//
// Kernels: per-block CRCs (crc_kernel) and the BlockMeta sections (meta kernels) are reused; then
//   sst_layout_kernel   file sizes per SST (data + CRCs, meta, bloom) and their exclusive scan
//   sst_data_kernel     one wave per block: block bytes + BE CRC into its file (whole-wave copies)
//   sst_meta_kernel     one wave per SST: the meta section and meta_offset
//   sst_bloom_kernel    one workgroup per SST: the key fingerprints set k bits each in an LDS
//                       bitmap (LDS atomics), CRC of filter | k by the lane-parallel CRC, the
//                       filter, k, CRC and bloom_offset written into the file.
// and the read side's point lookup inside a block:
//   lsmblk_seek_batch   BlockIterator::seek_to_key for a batch of (block, key) lookups
#include "lsmblk_dev.hpp"

namespace {

// ---------------------------------------------------------------- farmhash fingerprint32
// farmhash 1.1.5 fingerprint32 = farmhashmk::Hash32 of Google's FarmHash (a CityHash descendant):
// restated from the published algorithm (oracle/pyref.py has the same restatement; parity with
// the crate itself is unpinned here -- DESIGN.md).  Rotate is a right rotation; Fetch a
// little-endian u32 load at any byte offset.
constexpr uint32_t kF1 = 0xcc9e2d51u, kF2 = 0x1b873593u;

__host__ __device__ __forceinline__ uint32_t frot(uint32_t v, uint32_t s) { return s ? (v >> s) | (v << (32 - s)) : v; }
__host__ __device__ __forceinline__ uint32_t ffmix(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}
__host__ __device__ __forceinline__ uint32_t fmur(uint32_t a, uint32_t h) {
  a *= kF1;
  a = frot(a, 17);
  a *= kF2;
  h ^= a;
  h = frot(h, 19);
  return h * 5 + 0xe6546b64u;
}

// Src: a byte source with u32 fetches at arbitrary offsets (bytes [i, i + 4), little-endian)
// and single bytes.
template <class Src>
__host__ __device__ uint32_t fingerprint32(const Src& S, uint32_t len) {
  if (len <= 4) {
    uint32_t b = 0, c = 9;
    for (uint32_t i = 0; i < len; ++i) {
      const int32_t v = int32_t(int8_t(S.byte(i)));  // signed char
      b = b * kF1 + uint32_t(v);
      c ^= b;
    }
    return ffmix(fmur(b, fmur(len, c)));
  }
  if (len <= 12) {
    uint32_t a = len, b = len * 5, c = 9, d = b;
    a += S.fetch(0);
    b += S.fetch(len - 4);
    c += S.fetch((len >> 1) & 4);
    return ffmix(fmur(c, fmur(b, fmur(a, d))));
  }
  if (len <= 24) {
    uint32_t a = S.fetch((len >> 1) - 4), b = S.fetch(4), c = S.fetch(len - 8), d = S.fetch(len >> 1);
    const uint32_t e = S.fetch(0), f = S.fetch(len - 4);
    uint32_t h = d * kF1 + len;
    a = frot(a, 12) + f;
    h = fmur(c, h) + a;
    a = frot(a, 3) + c;
    h = fmur(e, h) + a;
    a = frot(a + f, 12) + d;
    h = fmur(b, h) + a;
    return ffmix(h);
  }
  uint32_t h = len, g = kF1 * len, f = g;
  const uint32_t a0 = frot(S.fetch(len - 4) * kF1, 17) * kF2, a1 = frot(S.fetch(len - 8) * kF1, 17) * kF2;
  const uint32_t a2 = frot(S.fetch(len - 16) * kF1, 17) * kF2, a3 = frot(S.fetch(len - 12) * kF1, 17) * kF2;
  const uint32_t a4 = frot(S.fetch(len - 20) * kF1, 17) * kF2;
  h ^= a0;
  h = frot(h, 19);
  h = h * 5 + 0xe6546b64u;
  h ^= a2;
  h = frot(h, 19);
  h = h * 5 + 0xe6546b64u;
  g ^= a1;
  g = frot(g, 19);
  g = g * 5 + 0xe6546b64u;
  g ^= a3;
  g = frot(g, 19);
  g = g * 5 + 0xe6546b64u;
  f += a4;
  f = frot(f, 19) + 113;
  uint32_t iters = (len - 1) / 20, p = 0;
  do {
    const uint32_t a = S.fetch(p), b = S.fetch(p + 4), c = S.fetch(p + 8), d = S.fetch(p + 12), e = S.fetch(p + 16);
    h += a;
    g += b;
    f += c;
    h = fmur(d, h) + e;
    g = fmur(c, g) + a;
    f = fmur(b + e * kF1, f) + d;
    f += g;
    g += f;
    p += 20;
  } while (--iters != 0);
  g = frot(g, 11) * kF1;
  g = frot(g, 17) * kF1;
  f = frot(f, 11) * kF1;
  f = frot(f, 17) * kF1;
  h = frot(h + g, 19);
  h = h * 5 + 0xe6546b64u;
  h = frot(h, 17) * kF1;
  h = frot(h + f, 19);
  h = h * 5 + 0xe6546b64u;
  h = frot(h, 17) * kF1;
  return h;
}

// A key in the KV stream's arena through a bounds-checked descriptor (aligned dword loads).
struct DevKey {
  rsrc_t r;
  uint32_t x;  // descriptor byte of the key's first byte
  __device__ __forceinline__ uint32_t fetch(uint32_t i) const {
    const uint32_t y = x + i, al = y & ~3u;
    return __builtin_amdgcn_alignbyte(__builtin_amdgcn_raw_buffer_load_b32(r, al + 4, 0, 0),
                                      __builtin_amdgcn_raw_buffer_load_b32(r, al, 0, 0), y & 3);
  }
  __device__ __forceinline__ uint32_t byte(uint32_t i) const { return __builtin_amdgcn_raw_buffer_load_b8(r, x + i, 0, 0); }
};
struct HostKey {
  const uint8_t* p;
  uint32_t fetch(uint32_t i) const {
    uint32_t v;
    memcpy(&v, p + i, 4);
    return v;
  }
  uint32_t byte(uint32_t i) const { return p[i]; }
};

// ---------------------------------------------------------------- bloom geometry
// Bloom::bloom_bits_per_key(n, 0.01) (bloom.rs:72-77) in f64 as the reference computes it, then
// build_from_key_hashes's k and filter size (:80-87).
struct BloomGeom {
  uint32_t k, nbytes;
  uint64_t nbits;
};
__host__ __device__ __forceinline__ BloomGeom bloom_geom(uint64_t n) {
  const double ln2 = 0.6931471805599453;    // std::f64::consts::LN_2
  const double lnfpr = -4.605170185988091;  // (0.01f64).ln()
  uint64_t bpk = 0;
  if (n) {
    const double size = -1.0 * double(n) * lnfpr / (ln2 * ln2);
    bpk = uint64_t(ceil(size / double(n)));
  }
  uint32_t k = uint32_t(double(bpk) * 0.69);
  k = k < 1 ? 1 : (k > 30 ? 30 : k);
  uint64_t nbits = n * bpk;
  if (nbits < 64) nbits = 64;
  BloomGeom g;
  g.nbytes = uint32_t((nbits + 7) / 8);
  g.nbits = uint64_t(g.nbytes) * 8;
  g.k = k;
  return g;
}

// ---------------------------------------------------------------- SST files
struct SstArgs {
  const uint8_t* blocks;
  const uint64_t* blk_off;
  uint64_t nblk;
  const uint32_t* sst_blk;  // nsst + 1
  const uint32_t* sst_ent;  // nsst + 1
  uint32_t nsst;
  const uint8_t* keys;
  const uint32_t* key_off;
  uint64_t n;               // entries of the KV stream (key arena = key_off[n])
  const uint32_t* crc;      // per block
  const uint8_t* meta;
  const uint64_t* meta_off; // nsst + 1
  uint8_t* files;
  uint64_t files_cap;
  uint64_t* file_off;       // nsst + 1
  uint64_t* data_len;       // nsst: data section bytes (= meta_offset)
  const CrcTabs* tabs;
  uint64_t* stats;          // [0] nsst [1] bytes [3] error flags
  const uint64_t* mstats;   // BlockMeta stage stats
  const uint64_t* cstats;   // block CRC stage stats
};

// One workgroup: file sizes and their exclusive scan (rounds of 1024 SSTs).
__global__ __launch_bounds__(1024) void sst_layout_kernel(SstArgs a) {
  const uint32_t t = threadIdx.x, w = t >> 6;
  __shared__ uint64_t wsum[16];
  uint64_t carry = 0;
  uint32_t err = 0;
  if (t == 0) err = uint32_t(a.mstats[3] | a.cstats[3]);
  for (uint32_t r = 0; r < a.nsst; r += 1024) {
    const uint32_t s = r + t;
    uint64_t len = 0;
    if (s < a.nsst) {
      const uint32_t b0 = a.sst_blk[s], b1 = a.sst_blk[s + 1];
      const uint64_t dl = a.blk_off[b1] - a.blk_off[b0] + 4ull * (b1 - b0);
      a.data_len[s] = dl;
      const uint64_t ml = a.meta_off[s + 1] - a.meta_off[s];
      len = dl + ml + 4 + bloom_geom(a.sst_ent[s + 1] - a.sst_ent[s]).nbytes + 1 + 4 + 4;
      if (dl > 0xFFFFFFFFull || dl + ml + 4 > 0xFFFFFFFFull) err |= LSMBLK_ERR_OVERFLOW;  // u32 offsets
    }
    const uint64_t inc = wave_incl_scan<uint64_t>(len);
    if (lane_id() == 63) wsum[w] = inc;
    __syncthreads();
    uint64_t base = carry, tot = carry;
    for (uint32_t x = 0; x < 16; ++x) {
      if (x < w) base += wsum[x];
      tot += wsum[x];
    }
    if (s < a.nsst) a.file_off[s] = base + inc - len;
    carry = tot;
    __syncthreads();
  }
  for (uint32_t d = 32; d >= 1; d >>= 1) err |= __shfl_xor(err, d, 64);
  __shared__ uint32_t werr[16];
  if (lane_id() == 0) werr[w] = err;
  __syncthreads();
  if (t == 0) {
    uint32_t e = 0;
    for (uint32_t x = 0; x < 16; ++x) e |= werr[x];
    a.file_off[a.nsst] = carry;
    a.stats[0] = a.nsst;
    a.stats[1] = carry;
    if (carry > a.files_cap) e |= LSMBLK_ERR_CAPACITY;
    if (e) atomicOr(reinterpret_cast<unsigned long long*>(a.stats + 3), (unsigned long long)e);
  }
}

__device__ __forceinline__ void put_be32(uint8_t* d, uint32_t v) {
  d[0] = uint8_t(v >> 24);
  d[1] = uint8_t(v >> 16);
  d[2] = uint8_t(v >> 8);
  d[3] = uint8_t(v);
}

// len bytes src -> dst by the whole wave, any alignment (16-B pieces, 1 KiB per instruction).
__device__ __forceinline__ void wave_copy_bytes(uint8_t* dst, const uint8_t* src, uint64_t len) {
  for (uint64_t o = 16ull * lane_id(); o < len; o += 1024) {
    if (o + 16 <= len) {
      *reinterpret_cast<u32x4*>(dst + o) = *reinterpret_cast<const u32x4*>(src + o);
    } else {
      for (uint64_t x = o; x < len; ++x) dst[x] = src[x];
    }
  }
}

__device__ __forceinline__ uint32_t sst_of_block(const SstArgs& a, uint64_t b) {
  uint32_t lo = 0, hi = a.nsst;  // largest s with sst_blk[s] <= b
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a.sst_blk[mid] <= b) lo = mid;
    else hi = mid;
  }
  return lo;
}

// One wave per block: block bytes, then its BE crc32fast (finish_block, builder.rs:118-122).
__global__ __launch_bounds__(256) void sst_data_kernel(SstArgs a) {
  if (a.stats[3]) return;
  const uint64_t b = uint64_t(blockIdx.x) * 4 + wave_id();
  if (b >= a.nblk) return;
  const uint32_t s = sst_of_block(a, b);
  const uint32_t b0 = a.sst_blk[s];
  const uint64_t st = a.blk_off[b], en = a.blk_off[b + 1];
  uint8_t* d = a.files + a.file_off[s] + (st - a.blk_off[b0]) + 4ull * (b - b0);
  wave_copy_bytes(d, a.blocks + st, en - st);
  if (lane_id() == 0) put_be32(d + (en - st), a.crc[b]);
}

// One wave per SST: the BlockMeta section and the u32 meta_offset (builder.rs:76-78).
__global__ __launch_bounds__(256) void sst_meta_kernel(SstArgs a) {
  if (a.stats[3]) return;
  const uint64_t s = uint64_t(blockIdx.x) * 4 + wave_id();
  if (s >= a.nsst) return;
  const uint64_t dl = a.data_len[s], m0 = a.meta_off[s], ml = a.meta_off[s + 1] - m0;
  uint8_t* d = a.files + a.file_off[s] + dl;
  wave_copy_bytes(d, a.meta + m0, ml);
  if (lane_id() == 0) put_be32(d + ml, uint32_t(dl));
}

constexpr uint32_t kBloomLds = 32768;  // filters up to 32 KiB (~26 K keys) are built in LDS

// crc32fast of LDS bytes p[0, len), p[-kCrcPad, 0) zero: chunks of 64 whole 68-B windows
// (the first holds the remainder), so only the first chunk's windows reach before its start;
// combined with Z(., 4352) = Z(., 68 << 5) twice.  Every lane of the wave returns the CRC.
__device__ uint32_t crc_lds(const CrcTabs& T, const uint8_t* p, uint32_t len) {
  constexpr uint32_t kW = 64 * kCrcSeg;
  if (len == 0) return 0;
  const uint32_t nch = (len + kW - 1) / kW, h = len - kW * (nch - 1);
  uint32_t acc = crc_chunk(T, p, h, true);
  for (uint32_t c = 1; c < nch; ++c)
    acc = crc_apply(T.shift[5], crc_apply(T.shift[5], acc)) ^ crc_chunk(T, p + h + kW * (c - 1), kW, false);
  return ~acc;
}

// One workgroup per SST: the bloom filter of its keys' fingerprints (build_from_key_hashes,
// bloom.rs:80-101), encoded as filter | k | crc (:63-69), then bloom_offset (builder.rs:83-85).
__global__ __launch_bounds__(256) void sst_bloom_kernel(SstArgs a) {
  __shared__ CrcTabs T;
  __shared__ __attribute__((aligned(16))) uint32_t bitbuf[kCrcPad / 4 + kBloomLds / 4 + 4];
  uint32_t* const bits = bitbuf + kCrcPad / 4;  // after the zeros crc_chunk reads before a chunk
  if (a.stats[3]) return;
  const uint32_t s = blockIdx.x;
  if (s >= a.nsst) return;
  const uint32_t e0 = a.sst_ent[s], e1 = a.sst_ent[s + 1];
  const BloomGeom G = bloom_geom(e1 - e0);
  const uint64_t boff = a.data_len[s] + (a.meta_off[s + 1] - a.meta_off[s]) + 4;  // bloom_offset
  uint8_t* d = a.files + a.file_off[s] + boff;
  const bool lds = G.nbytes + 1 <= kBloomLds;
  for (uint32_t i = threadIdx.x; i < sizeof(CrcTabs) / 16; i += 256)
    reinterpret_cast<u32x4*>(&T)[i] = reinterpret_cast<const u32x4*>(a.tabs)[i];
  const uint32_t nw = (G.nbytes + 1 + 3) / 4;
  if (threadIdx.x < kCrcPad / 4) bitbuf[threadIdx.x] = 0;
  if (lds) {
    for (uint32_t i = threadIdx.x; i < nw; i += 256) bits[i] = 0;
  } else {
    for (uint32_t i = threadIdx.x; i < G.nbytes; i += 256) d[i] = 0;
    __threadfence();  // the zeros reach L2 before any thread's atomics
  }
  __syncthreads();
  const uint32_t lead = uint32_t(reinterpret_cast<uintptr_t>(a.keys) & 15);
  const rsrc_t R = make_rsrc(a.keys - lead, lead + a.key_off[a.n]);
  // global path: OR into the file bytes through the aligned words that hold them
  uint8_t* const dal = reinterpret_cast<uint8_t*>(reinterpret_cast<uintptr_t>(d) & ~uintptr_t(3));
  const uint32_t dsh = uint32_t(reinterpret_cast<uintptr_t>(d) & 3);
  for (uint32_t e = e0 + threadIdx.x; e < e1; e += 256) {
    const uint32_t kp = a.key_off[e], kl = a.key_off[e + 1] - kp;
    uint32_t h = fingerprint32(DevKey{R, lead + kp}, kl);
    const uint32_t delta = (h >> 17) | (h << 15);
    for (uint32_t i = 0; i < G.k; ++i) {
      const uint32_t bit = uint32_t(uint64_t(h) % G.nbits);
      if (lds) {
        atomicOr(&bits[bit >> 5], 1u << (bit & 31));
      } else {
        const uint32_t x = dsh * 8 + bit;  // bit index from the aligned word base
        atomicOr(reinterpret_cast<uint32_t*>(dal) + (x >> 5), 1u << (x & 31));
      }
      h += delta;
    }
  }
  __syncthreads();
  if (lds) {
    if (threadIdx.x == 0) reinterpret_cast<uint8_t*>(bits)[G.nbytes] = uint8_t(G.k);
    __syncthreads();
    uint32_t crc = 0;
    if (threadIdx.x < 64) crc = crc_lds(T, reinterpret_cast<const uint8_t*>(bits), G.nbytes + 1);
    const uint8_t* src = reinterpret_cast<const uint8_t*>(bits);
    for (uint32_t i = threadIdx.x; i < G.nbytes + 1; i += 256) d[i] = src[i];
    if (threadIdx.x == 0) {
      put_be32(d + G.nbytes + 1, crc);
      put_be32(d + G.nbytes + 5, uint32_t(boff));
    }
  } else {
    // large filter: k byte, then the CRC over the file bytes staged through LDS by wave 0
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) d[G.nbytes] = uint8_t(G.k);
    __threadfence();
    __syncthreads();
    if (threadIdx.x < 64) {
      uint8_t* stage = reinterpret_cast<uint8_t*>(bits);
      const uint32_t len = G.nbytes + 1;
      const uint32_t nch = (len + kCrcChunk - 1) / kCrcChunk, h0 = len - kCrcChunk * (nch - 1);
      uint32_t acc = 0;
      for (uint32_t c = 0; c < nch; ++c) {
        const uint32_t off = c == 0 ? 0u : h0 + kCrcChunk * (c - 1), sz = c == 0 ? h0 : kCrcChunk;
        for (uint32_t i = lane_id(); i < sz; i += 64) stage[i] = __hip_atomic_load(d + off + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        wave_sync();
        const uint32_t part = crc_chunk(T, stage, sz, c == 0);
        acc = c == 0 ? part : crc_apply(T.shift[6], acc) ^ part;
        wave_sync();
      }
      if (lane_id() == 0) {
        put_be32(d + len, ~acc);
        put_be32(d + len + 4, uint32_t(boff));
      }
    }
  }
}

// ---------------------------------------------------------------- batched seek_to_key
// BlockIterator::seek_to_key (src/block/iterator.rs:80-94), one lane per point lookup: the same
// binary search (mid = low + (high - low) / 2, returning at the first probe whose key compares
// equal -- with several versions of a user key in the block that is not necessarily the first of
// them), keys reconstructed as first_key[..prefix] || suffix (seek_to_offset :125-132) and compared
// ts-agnostically (src/key.rs:77-81).  A block or probed entry that breaks the decode rules
//  reports LSMBLK_ERR_MALFORMED and the block's entry count.
struct SeekArgs {
  const uint8_t* blocks;
  const uint64_t* blk_off;
  uint64_t nblk;
  uint32_t tail;
  const uint8_t* qkeys;
  const uint32_t* qkey_off;
  const uint32_t* q_blk;
  uint64_t nq;
  uint32_t* idx;
  uint64_t* stats;
};

__device__ __forceinline__ uint32_t be16_at(const uint8_t* p, uint32_t i) { return (uint32_t(p[i]) << 8) | p[i + 1]; }

__global__ __launch_bounds__(256) void seek_kernel(SeekArgs a) {
  const uint64_t q = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  if (q >= a.nq) return;
  uint32_t err = 0, res = 0;
  const uint32_t b = a.q_blk[q];
  const uint8_t* key = a.qkeys + a.qkey_off[q];
  const uint32_t klen = a.qkey_off[q + 1] - a.qkey_off[q];
  do {
    if (b >= a.nblk) {
      err = LSMBLK_ERR_SEGMENTS;
      break;
    }
    const uint64_t start = a.blk_off[b], end = a.blk_off[b + 1];
    if (end < start + a.tail || end - start > 0x7FFFFFF0ull || end - start - a.tail < 2) {
      err = LSMBLK_ERR_MALFORMED;
      break;
    }
    const uint32_t len = uint32_t(end - start) - a.tail;
    const uint8_t* p = a.blocks + start;
    const uint32_t n = be16_at(p, len - 2);
    res = n;
    if (2 + 2 * n > len) {
      err = LSMBLK_ERR_MALFORMED;
      break;
    }
    const uint32_t data_end = len - 2 - 2 * n;
    uint32_t fks = 0;
    if (n) {
      if (data_end < 4 || 4 + (fks = be16_at(p, 2)) + 8 > data_end) {
        err = LSMBLK_ERR_MALFORMED;
        break;
      }
    }
    uint32_t lo = 0, hi = n;
    bool found = false;
    while (lo < hi) {
      const uint32_t mid = lo + (hi - lo) / 2;
      const uint32_t off = be16_at(p, data_end + 2 * mid);
      if (off + 4 > data_end) {
        err = LSMBLK_ERR_MALFORMED;
        break;
      }
      const uint32_t pf = be16_at(p, off), sf = be16_at(p, off + 2);
      if (!(off + 4 + sf + 10 <= data_end && pf <= fks && pf + sf > 0) ||
          off + 14 + sf + be16_at(p, off + 12 + sf) > data_end) {
        err = LSMBLK_ERR_MALFORMED;
        break;
      }
      // key order of first_key[..pf] || suffix against the target
      const uint32_t kl = pf + sf, m = kl < klen ? kl : klen;
      int c = 0;
      for (uint32_t i = 0; i < m && !c; ++i) {
        const uint32_t x = i < pf ? p[4 + i] : p[off + 4 + i - pf];
        if (x != key[i]) c = x < key[i] ? -1 : 1;
      }
      if (!c) c = kl < klen ? -1 : (kl > klen ? 1 : 0);
      if (c < 0) {
        lo = mid + 1;
      } else if (c > 0) {
        hi = mid;
      } else {
        res = mid;
        found = true;
        break;
      }
    }
    if (err) {
      res = n;
      break;
    }
    if (!found) res = lo;
  } while (false);
  a.idx[q] = res;
  if (err) atomicOr(reinterpret_cast<unsigned long long*>(a.stats + 3), (unsigned long long)err);
}

}  // namespace

extern "C" {

int lsmblk_seek_batch(lsmblk_ctx* c, const uint8_t* blocks, const uint64_t* blk_off, uint64_t nblk, uint32_t tail,
                      const uint8_t* qkeys, const uint32_t* qkey_off, const uint32_t* q_blk, uint64_t nq, uint32_t* idx,
                      uint64_t* stats, void* stream) {
  if (!c || !blk_off || !stats || (nq && (!qkey_off || !q_blk || !idx)) || tail > 16) return LSMBLK_E_INVAL;
  std::lock_guard<std::mutex> g(c->mu);
  DeviceGuard dg(c->device, c);
  if (!dg.ok) return LSMBLK_E_HIP;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (hipMemsetAsync(stats, 0, LSMBLK_STATS_WORDS * 8, st) != hipSuccess) return LSMBLK_E_HIP;
  if (nq == 0) return LSMBLK_OK;
  SeekArgs a{blocks, blk_off, nblk, tail, qkeys, qkey_off, q_blk, nq, idx, stats};
  LSM_LAUNCH(seek_kernel, dim3(uint32_t((nq + 255) / 256)), dim3(256), 0, st, a);
  return hipGetLastError() == hipSuccess ? LSMBLK_OK : LSMBLK_E_HIP;
}

uint32_t lsmblk_fingerprint32(const uint8_t* key, size_t klen) {
  return fingerprint32(HostKey{key}, uint32_t(klen));
}

int lsmblk_bloom_may_contain(const uint8_t* filter, size_t nbytes, uint32_t k, uint32_t h) {
  if (k > 30) return 1;  // bloom.rs:105-107
  const uint64_t nbits = uint64_t(nbytes) * 8;
  if (!filter || nbits == 0) return 0;
  const uint32_t delta = (h >> 17) | (h << 15);
  for (uint32_t i = 0; i < k; ++i) {
    const uint64_t bit = h % uint32_t(nbits);  // `h % (nbits as u32)`, bloom.rs:112
    if (!((filter[bit / 8] >> (bit % 8)) & 1)) return 0;
    h += delta;
  }
  return 1;
}

int lsmblk_sst_files_batch(lsmblk_ctx* c, const uint8_t* blocks, const uint64_t* blk_off, uint64_t nblk,
                           const uint32_t* sst_blk, const uint32_t* sst_ent, uint32_t nsst,
                           const lsmblk_kv_stream* kv, uint8_t* files, uint64_t files_cap, uint64_t* file_off,
                           uint64_t* stats, void* stream) {
  if (!c || !blk_off || !sst_blk || !sst_ent || !kv || !kv->key_off || !file_off || !stats) return LSMBLK_E_INVAL;
  if (nsst == 0 || nblk >= 0xFFFFFFFFull || (files_cap && !files)) return LSMBLK_E_INVAL;
  std::lock_guard<std::mutex> g(c->mu);
  DeviceGuard dg(c->device, c);
  if (!dg.ok) return LSMBLK_E_HIP;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int rc;
  if ((rc = lsmblk_impl::ensure_crc_tabs(c, st))) return rc;
  // workspace: block CRCs, BlockMeta sections, section offsets, data-section lengths, stats
  struct Ws {
    uint32_t* crc;
    uint64_t* meta_off;
    uint64_t* data_len;
    uint64_t* st;  // 3 x 4 stats: crc, meta, (spare)
    uint8_t* meta;
  };
  auto carve = [&](uint8_t* base, uint64_t meta_bytes, Ws& w) -> uint64_t {
    uint64_t off = 0;
    auto take = [&](uint64_t bytes) {
      uint8_t* p = base + off;
      off = (off + bytes + 255) & ~uint64_t(255);
      return p;
    };
    w.crc = reinterpret_cast<uint32_t*>(take(4 * (nblk + 1)));
    w.meta_off = reinterpret_cast<uint64_t*>(take(8ull * (nsst + 1)));
    w.data_len = reinterpret_cast<uint64_t*>(take(8ull * (nsst + 1)));
    w.st = reinterpret_cast<uint64_t*>(take(8 * 12));
    w.meta = take(meta_bytes + 16);
    return off;
  };
  // a block's BlockMeta record is 24 B + its first and last keys, two distinct entries of the
  // stream (or one twice): 16 B per section + 24 B per block + twice the key arena bounds them
  Ws w{};
  uint64_t meta_bytes = 16ull * nsst + 24ull * nblk;
  {
    uint32_t karena = 0;
    if (hipMemcpyAsync(&karena, kv->key_off + kv->n, 4, hipMemcpyDeviceToHost, st) != hipSuccess) return LSMBLK_E_HIP;
    if (hipStreamSynchronize(st) != hipSuccess) return LSMBLK_E_HIP;
    meta_bytes += 2ull * karena;
  }
  const uint64_t need = carve(nullptr, meta_bytes, w);
  if (need > c->sws_cap && (rc = grow(st, &c->sws, &c->sws_cap, need, 1))) return rc;
  carve(c->sws, meta_bytes, w);
  if (hipMemsetAsync(w.st, 0, 8 * 12, st) != hipSuccess) return LSMBLK_E_HIP;
  if (hipMemsetAsync(stats, 0, LSMBLK_STATS_WORDS * 8, st) != hipSuccess) return LSMBLK_E_HIP;
  if (nblk && (rc = lsmblk_impl::launch_crc(c, blocks, blk_off, nblk, 0, w.crc, w.st, st))) return rc;
  if ((rc = lsmblk_impl::block_meta_locked(c, blocks, blk_off, nblk, 0, sst_blk, nsst, w.meta, meta_bytes + 16,
                                           w.meta_off, w.st + 4, st)))
    return rc;
  SstArgs a;
  a.blocks = blocks;
  a.blk_off = blk_off;
  a.nblk = nblk;
  a.sst_blk = sst_blk;
  a.sst_ent = sst_ent;
  a.nsst = nsst;
  a.keys = kv->keys;
  a.key_off = kv->key_off;
  a.n = kv->n;
  a.crc = w.crc;
  a.meta = w.meta;
  a.meta_off = w.meta_off;
  a.files = files;
  a.files_cap = files_cap;
  a.file_off = file_off;
  a.data_len = w.data_len;
  a.tabs = static_cast<const CrcTabs*>(c->crc_tabs);
  a.stats = stats;
  a.mstats = w.st + 4;
  a.cstats = w.st;
  LSM_LAUNCH(sst_layout_kernel, dim3(1), dim3(1024), 0, st, a);
  if (nblk) LSM_LAUNCH(sst_data_kernel, dim3(uint32_t((nblk + 3) / 4)), dim3(256), 0, st, a);
  LSM_LAUNCH(sst_meta_kernel, dim3((nsst + 3) / 4), dim3(256), 0, st, a);
  LSM_LAUNCH(sst_bloom_kernel, dim3(nsst), dim3(256), 0, st, a);
  return hipGetLastError() == hipSuccess ? LSMBLK_OK : LSMBLK_E_HIP;
}

}  // extern "C"
