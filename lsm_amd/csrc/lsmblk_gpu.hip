// lsmblk_gpu.hip -- batch half of the C ABI (include/lsmblk.h): SSTable block decode and
// encode as hand-written HIP kernels for gfx950 (MI355X, CDNA4, wave64).
//
// Reference semantics (paths relative to the reference repository):
//   encode: BlockBuilder::add / build / Block::encode  src/block/builder.rs:54-89,
//           src/block.rs:14-22, driven per segment like SsTableBuilder::add
//           src/table/builder.rs:48-65, 112-123
//   decode: Block::decode src/block.rs:24-34 + the corrected BlockIterator walk
//           src/block/iterator.rs:23-34, 99-139
//
// Kernels (DESIGN.md has the data layout and the roofline of each):
//   decode_kernel   one wave per block (4 blocks per 256-thread workgroup).  The block is
//                   staged into LDS with 16-B buffer loads, entries are parsed one per lane,
//                   the block's (entries, key bytes, value bytes) are published and the
//                   output bases found by a wave-parallel decoupled look-back over
//                   data-tagged 8-byte granules; keys, values and per-entry metadata are
//                   then written with coalesced, aligned stores.
//   plan_kernel     one wave per segment: the greedy block-boundary walk (the only serial
//                   dependency of the format) 64 candidate entries per step with a wave
//                   prefix sum + ballot; segment totals via the same look-back.
//   emit_kernel     one wave per output block: keys/values staged into LDS, headers written
//                   by entry lanes, value bytes moved as aligned dwords, the block image
//                   flushed with 16-B stores.
// Blocks or batches that exceed the LDS fast paths take per-entry-lane "simple" paths
// that read/write global memory directly (same results, slower).
#include "lsmblk_dev.hpp"

namespace {


// ================================================================ decode
struct DecodeArgs {
  const uint8_t* blocks;
  const uint64_t* blk_off;
  uint64_t nblk;
  uint8_t* keys;
  uint32_t* key_off;
  uint8_t* vals;
  uint32_t* val_off;
  uint64_t* ts;
  uint64_t entry_cap, key_cap, val_cap;
  uint64_t* stats;
  const uint32_t* agg;        // per-block (entries, key bytes, value bytes), from the count pass (dec_count_staged_kernel or the CRC pass)
  const uint64_t* tile_pre;   // per-tile exclusive prefix (entries, key bytes, value bytes)
  uint32_t tail;              // bytes after each block inside its range (4: the framing CRC)
  uint64_t* blk_ent;          // optional: first entry index of every block
  uint32_t skip;  // ablation mask (lsmblk_debug_set, timing experiments only): 2 keys,
                  // 4 values, 8 per-entry metadata, 256 stop after staging, 512 after the tables;
                  // lagged decode: 1024 no count (aggregates 0), 2048 no wait for the base
  // lagged decode (decode_lag_kernel): uncached granules tagged with `tag`
  uint64_t* bagg;             // 3 per block: the block's (entries, key bytes, value bytes), from its count
  uint64_t* bbase;            // 3 per block: the block's output base (entries, key bytes, value bytes)
  uint64_t* tagg;             // 3 per kTile-block tile: the tile's aggregate
  uint64_t* tinc;             // 3 per tile: inclusive prefix through the tile
  uint64_t lag;               // workgroup j counts block j and decodes block j - lag (at most)
  uint64_t lag_bytes;         // nonzero: the lag is lag_bytes of blocks at the batch's mean block size
  uint64_t* dbg;              // optional realtime trace per tile (lsmblk_debug_counters)
  uint32_t tag, poll;
};

constexpr uint32_t kTile = 64;  // blocks per count tile
// debug buffer (LSMBLK_DEBUG_COUNTERS): 16 reserved words, then an 8-word s_memrealtime (100 MHz)
// trace per tile for the first kDbgTiles tiles: [0] finish start [1] bases published [2] first
// decoder's base wait begins [3] ends [4] the tile's first count starts [5] its first decoder starts
constexpr uint32_t kDbgTiles = 32768, kDbgWords = 16 + 8 * kDbgTiles;
__device__ __forceinline__ void dbg_trace(uint64_t* dbg, uint64_t t, uint32_t k) {  // diagnostics builds only
  if (kDiag && dbg && t < kDbgTiles && lane_id() == 0) dbg[16 + 8 * t + k] = __builtin_amdgcn_s_memrealtime();
}


// LDS reads per lane issued together before their uses (one LDS round trip per batch instead
// of one per read): flushes, value copies, chunk moves.
constexpr uint32_t kLB = 2;  // decode: 2 measured 1 % faster per step than 1, 4 slower (1.64 vs 1.58 ms)
#ifndef LSMBLK_XEB
#define LSMBLK_XEB 4
#endif
// Chunk groups per batch in emit's value moves and flush (all of a batch's LDS reads issued before
// its uses).  Round 2: 2 and 4 spilled beside the next block's prefetch; round 6: 124 / 128 VGPRs, no
// spill, emit 1.715 / 1.705 / 1.698 ms at 1 / 2 / 4 (alternating, one box).
constexpr uint32_t kEB = LSMBLK_XEB;


// LDS per single-wave workgroup is exactly 8 KiB, so 20 blocks are resident per CU (5 waves per
// SIMD; 10.3 KiB gave 15).  A 4 KiB block (up to 4098 B: the builder overshoots by 2) at any
// 16-B lead, plus the 16-B staging round-up, fits the image.
constexpr uint32_t kDecImg = 4128;  // staged block bytes per wave
constexpr uint32_t kDecMaxE = 128;  // entries of a fast-path block (tables in registers, 2 per lane)
constexpr uint32_t kDecOut = 4032;  // LDS output image (keys + values) of a fast-path block

struct alignas(16) DecLds {
  uint8_t img[kDecImg];
  alignas(16) uint8_t out[kDecOut];  // decoded key run, then (16-B aligned) value run
};
static_assert(sizeof(DecLds) == 8160, "decode LDS: 20 blocks per CU");

// Entry tables of a large block (kDecMaxE entries at a time).  A large block is not staged, so
// the tables live in the unused image.
struct DecTables {
  uint16_t epos[kDecMaxE], pfx[kDecMaxE], sfx[kDecMaxE];
  uint32_t kout[kDecMaxE + 1], vout[kDecMaxE + 1];
};
static_assert(sizeof(DecTables) <= kDecImg, "large-block tables overlay the image");

// One fast-path entry, held by its lane in registers (entries l and l + 64 of the block).
struct DecEnt {
  uint32_t epos, p, s, kout, vout, vl;
};

// 16 bytes at LDS byte offset x (any alignment): one unaligned ds_read_b128 (the gfx9 unaligned
// access mode).  Three aligned ds_read_b64 + four v_alignbyte (round 1) cost emit 4 % more time.
__device__ __forceinline__ void lds_read16(const uint8_t* base, uint32_t x, uint32_t (&v)[4]) {
  const u32x4 q = *reinterpret_cast<const u32x4*>(base + x);
  v[0] = q.x, v[1] = q.y, v[2] = q.z, v[3] = q.w;
}

// cache policy of the staging loads (default; nt loads measured no gain)
constexpr int kLdAux = 0;

struct BlockHdr {
  uint32_t len, n, data_end, fks;
  bool ok;
};

template <class Img>
__device__ __forceinline__ BlockHdr parse_hdr(const Img& im, uint32_t len) {
  BlockHdr h{len, 0, 0, 0, true};
  if (len < 2) { h.ok = false; return h; }
  h.n = im.u16(len - 2);
  if (2 + 2 * h.n > len) { h.ok = false; h.n = 0; return h; }
  h.data_end = len - 2 - 2 * h.n;
  if (h.n) {
    // get_first_key (iterator.rs:23-34) parses the entry at data position 0.
    if (h.data_end < 4) { h.ok = false; return h; }
    h.fks = im.u16(2);
    if (4 + h.fks + 8 > h.data_end) h.ok = false;
  }
  return h;
}

// Corrected seek_to_offset (iterator.rs:125-139) with the validation rules of DESIGN.md.
template <class Img>
__device__ __forceinline__ bool parse_entry(const Img& im, const BlockHdr& h, uint32_t k,
                                            uint32_t& off, uint32_t& p, uint32_t& s, uint32_t& vl) {
  off = im.u16(h.data_end + 2 * k);
  bool ok = off + 4 <= h.data_end;
  const uint32_t w = im.le32(off);  // BE16 p | BE16 s
  p = bswap16(w & 0xFFFF);
  s = bswap16(w >> 16);
  ok = ok && (off + 4 + s + 10 <= h.data_end) && (p <= h.fks) && (p + s > 0);
  vl = im.u16(off + 12 + s);
  ok = ok && (off + 14 + s + vl <= h.data_end);
  if (!ok) { p = s = vl = 0; }
  return ok;
}

// Simple path: per-entry lanes, any block size / entry count, byte-granular stores.
template <class Img>
__device__ void dec_simple_outputs(const DecodeArgs& a, const Img& im, const BlockHdr& h,
                                   uint64_t E0, uint64_t K0, uint64_t V0) {
  const uint32_t l = lane_id();
  uint64_t kc = 0, vc = 0;
  for (uint32_t c = 0; c < h.n; c += 64) {
    const uint32_t k = c + l;
    uint32_t off = 0, p = 0, s = 0, vl = 0;
    if (k < h.n) parse_entry(im, h, k, off, p, s, vl);
    const uint64_t kl = p + s;
    const uint64_t ki = wave_incl_scan<uint64_t>(kl), vi = wave_incl_scan<uint64_t>(vl);
    const uint64_t kpos = K0 + kc + ki - kl, vpos = V0 + vc + vi - vl;
    kc += __shfl(ki, 63, 64);
    vc += __shfl(vi, 63, 64);
    if (k < h.n) {
      const uint64_t e = E0 + k;
      if (e < a.entry_cap) {
        a.ts[e] = im.u64(off + 4 + s);
        a.key_off[e] = uint32_t(kpos);
        a.val_off[e] = uint32_t(vpos);
      }
      for (uint32_t t = 0; t < p; ++t)
        if (kpos + t < a.key_cap) a.keys[kpos + t] = uint8_t(im.u8(4 + t));
      for (uint32_t t = 0; t < s; ++t)
        if (kpos + p + t < a.key_cap) a.keys[kpos + p + t] = uint8_t(im.u8(off + 4 + t));
      for (uint32_t t = 0; t < vl; ++t)
        if (vpos + t < a.val_cap) a.vals[vpos + t] = uint8_t(im.u8(off + 14 + s + t));
    }
  }
}

// Unaligned 16-B / 8-B / 4-B / 1-B stores through a buffer descriptor whose base is 16-B
// aligned (the gfx9 unaligned access mode: a dword store needs only byte alignment).
__device__ __forceinline__ void st16(const rsrc_t& R, uint32_t off, const uint32_t (&v)[4]) {
  const u32x4 q = {v[0], v[1], v[2], v[3]};
  __builtin_amdgcn_raw_buffer_store_b128(q, R, off, 0, 0);
}

// Store bytes [0, len) of a run (len < 16) whose first 16 bytes are v: overlapping stores of
// the widest size that fits (8+8, 4+4, or single bytes), never past len.
__device__ __forceinline__ void st_short(const rsrc_t& R, uint32_t off, uint32_t len, const uint32_t (&v)[4]) {
  if (len >= 8) {
    __builtin_amdgcn_raw_buffer_store_b64(u32x2{v[0], v[1]}, R, off, 0, 0);
    // bytes [len - 8, len)
    const uint32_t x = len - 8, sh = x & 3;
    const uint32_t w0 = x < 4 ? v[0] : v[1], w1 = x < 4 ? v[1] : v[2], w2 = x < 4 ? v[2] : v[3];
    __builtin_amdgcn_raw_buffer_store_b64(
        u32x2{__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh)}, R, off + x, 0, 0);
  } else if (len >= 4) {
    __builtin_amdgcn_raw_buffer_store_b32(v[0], R, off, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_amdgcn_alignbyte(v[1], v[0], len - 4), R, off + len - 4, 0, 0);
  } else {
    for (uint32_t i = 0; i < len; ++i)
      __builtin_amdgcn_raw_buffer_store_b8(uint8_t(v[0] >> (8 * i)), R, off + i, 0, 0);
  }
}

// Output sinks of the lane-per-entry decode: unaligned runs either go straight to global
// memory (GlbSink, buffer stores) or are composed in the wave's LDS output image (LdsSink)
// that is then flushed with aligned, coalesced 16-B stores (one HBM write request per 64-B
// line instead of one per lane).
struct GlbSink {
  rsrc_t RK, RV;
  uint32_t kb, vb;  // byte of the first key / value in its descriptor (16-B aligned base)
  __device__ __forceinline__ void put16(bool val, uint32_t off, const uint32_t (&v)[4]) const {
    st16(val ? RV : RK, (val ? vb : kb) + off, v);
  }
  __device__ __forceinline__ void put_short(bool val, uint32_t off, uint32_t len, const uint32_t (&v)[4]) const {
    st_short(val ? RV : RK, (val ? vb : kb) + off, len, v);
  }
};
struct LdsSink {
  uint8_t* out;
  uint32_t kb, vb;  // LDS byte of the first key / value
  __device__ __forceinline__ void put16(bool val, uint32_t off, const uint32_t (&v)[4]) const {
    *reinterpret_cast<u32x4*>(out + (val ? vb : kb) + off) = u32x4{v[0], v[1], v[2], v[3]};
  }
  __device__ __forceinline__ void put_short(bool val, uint32_t off, uint32_t len, const uint32_t (&v)[4]) const {
    uint8_t* p = out + (val ? vb : kb) + off;
    if (len >= 8) {
      const uint32_t x = len - 8, sh = x & 3;
      const uint32_t w0 = x < 4 ? v[0] : v[1], w1 = x < 4 ? v[1] : v[2], w2 = x < 4 ? v[2] : v[3];
      *reinterpret_cast<u32x2*>(p) = u32x2{v[0], v[1]};
      *reinterpret_cast<u32x2*>(p + x) =
          u32x2{__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh)};
    } else if (len >= 4) {
      *reinterpret_cast<uint32_t*>(p) = v[0];
      *reinterpret_cast<uint32_t*>(p + len - 4) = __builtin_amdgcn_alignbyte(v[1], v[0], len - 4);
    } else {
      for (uint32_t i = 0; i < len; ++i) p[i] = uint8_t(v[0] >> (8 * i));
    }
  }
};

// Value copies of a staged (LDS) wave as 16-B-aligned output chunks, each funnel-shifted from
// 8-B-aligned image reads (LSMBLK_XDEC_VALN, round 6; 0 = the unaligned 16-B pieces below).
// PMC at U (profiles/r06_pmc_lds_decode_{old,new}.txt): unaligned-LDS stall cycles 8.2e8 -> 3.6e8,
// LDS issue waits 4.7e8 -> 1.2e8 (0.60 -> 0.20 of all instruction waits), bank conflicts 2.2e7 ->
// 3.0e8 (the staged values sit at a ~128-B stride, so lanes reading the same chunk of their values
// share banks), VALU +46 %; decode 2.050 against 2.060 ms (three alternating pairs, one box).
// Rotating each lane's chunk order spreads the banks (1.2e8) but its VALU made the kernel 2-6 %
// slower (not kept).
#ifndef LSMBLK_XDEC_VALN
#define LSMBLK_XDEC_VALN 1
#endif
// Fast path, lane per entry: every entry lane writes its own key and value as contiguous
// runs of 16-B pieces (the last piece overlaps the previous one), so runs of adjacent
// entries abut and no lane needs a chunk -> entry search.
// The piece loops run a wave-uniform trip count (the wave's longest run) with each lane's piece
// index clamped to its last piece, so no per-piece exec mask is needed (PMC: the scalar unit,
// which runs those masks, is the decode's busiest pipe).  Lanes past the block's entries are
// masked off once per iteration (mirroring lane 0's entry instead made up to 63 lanes write the
// same LDS words: bank-conflicted, the decode lost a third of its rate).  Keys under 16 B,
// suffixes before the image start and values under 16 B keep per-lane paths.
template <class Sink>
__device__ __forceinline__ void dec_entry_runs(const DecodeArgs& a, DecLds& L, uint32_t lead, uint32_t n,
                                               const DecEnt (&ent)[2], uint64_t E0, uint64_t K0, uint64_t V0,
                                               const Sink& out, uint32_t skip) {
  const uint32_t l = lane_id();
  const uint8_t* img = L.img;
  const uint32_t fk = lead + 4;  // image byte of the first key
#pragma unroll
  for (uint32_t it = 0; it < 2; ++it) {
    if (64 * it >= n) break;  // wave-uniform
    const uint32_t k = 64 * it + l;
    const bool live = k < n;
    const uint32_t epos = ent[it].epos, p = ent[it].p, s = ent[it].s;
    const uint32_t kout = ent[it].kout, vout = ent[it].vout, vl = ent[it].vl;
    const uint32_t sb = lead + epos + 4;  // image byte of the suffix
    const uint32_t kl = p + s;
    // wave-uniform trip counts and path choice, over the live lanes (all lanes active here)
    const bool kirr = live && (kl < 16 || sb < p);
    const bool kuni = !__ballot(kirr);
    const uint32_t nkmax = __builtin_amdgcn_readlane(wave_incl_max32(live ? (kl + 15) >> 4 : 0u), 63);
    const uint32_t nvmax = __builtin_amdgcn_readlane(wave_incl_max32(live && vl >= 16 ? (vl + 15) >> 4 : 0u), 63);
    // Aligned value path (values composed in the LDS output image, at most 64 entries, every value
    // >= 16 B): lane k writes the 16-B-aligned image chunks that start inside its value, each built
    // from 8-B-aligned reads of the staged image and a byte funnel shift; the chunk that runs past
    // the value's end takes the rest from the next value (lane k + 1).  The misaligned 16-B LDS reads
    // and writes of the piece copies below cost the LDS array extra passes (PMC SQ_LDS_UNALIGNED_STALL;
    // the same accesses moved to aligned addresses, a timing probe: decode 2.14 -> 1.96 ms at U).
    const uint32_t vS = sb + s + 10, vD = out.vb + vout;  // the value's image / output-image bytes
    bool valn = false;
    uint32_t vm = 0, vmmax = 0, vS1 = 0, vD1 = 0;
    if constexpr (std::is_same_v<Sink, LdsSink>) {
      // (lane 0 also writes the chunk holding the run's first byte, read from vS - (vD & 15) on)
      valn = LSMBLK_XDEC_VALN && it == 0 && n <= 64 && !__ballot(live && (vl < 16 || (l == 0 && vS < (vD & 15)))) &&
             !(skip & (4 | 32 | 64));
      if (valn) {  // (wave-uniform)
        const uint32_t cs = l == 0 ? (vD >> 4) : ((vD + 15) >> 4), ce = (vD + vl - 1) >> 4;
        vm = live ? ce - cs + 1 : 0u;
        vmmax = __builtin_amdgcn_readlane(wave_incl_max32(vm), 63);
        vS1 = uint32_t(__shfl(int(vS), int(min(l + 1, 63u)), 64));
        vD1 = uint32_t(__shfl(int(vD), int(min(l + 1, 63u)), 64));
      }
    }
    if (!live) continue;
    if (!(skip & 8)) {
      const uint64_t e = E0 + k;
      const u32x2 q = LSMBLK_XALIGNED_LDS ? lds_qw_al(img, sb + s) : *reinterpret_cast<const u32x2*>(img + sb + s);
      a.ts[e] = __builtin_bswap64((uint64_t(q.y) << 32) | q.x);
      a.key_off[e] = uint32_t(K0 + kout);
      a.val_off[e] = uint32_t(V0 + vout);
    }
    if (!(skip & 2)) {
      // key byte x = first key byte x (x < p) or suffix byte x - p: a 16-B piece is one
      // unaligned read of each, merged under a per-dword byte mask
      auto merged = [&](uint32_t o, uint32_t (&v)[4]) {
        const u32x4 sq = *reinterpret_cast<const u32x4*>(img + sb + o - p);
        const u32x4 fq = *reinterpret_cast<const u32x4*>(img + fk + o);
        const uint32_t sv[4] = {sq.x, sq.y, sq.z, sq.w}, fv[4] = {fq.x, fq.y, fq.z, fq.w};
#pragma unroll
        for (uint32_t d = 0; d < 4; ++d) {
          const int32_t nf = int32_t(p) - int32_t(o + 4 * d);  // leading bytes from the first key
          const uint32_t m = nf <= 0 ? 0u : nf >= 4 ? ~0u : (1u << (8 * nf)) - 1;
          v[d] = (fv[d] & m) | (sv[d] & ~m);
        }
      };
      if (kuni) {  // every live key >= 16 B, its suffix in the image
        for (uint32_t t = 0; t < nkmax; ++t) {
          const uint32_t o = min(16 * t, kl - 16);
          uint32_t v[4];
          merged(o, v);
          out.put16(false, kout + o, v);
        }
      } else {
        for (uint32_t t = 0; t < kl; t += 16) {
          const uint32_t o = kl >= 16 ? min(t, kl - 16) : 0u;
          uint32_t v[4];
          if (sb + o >= p) {
            merged(o, v);
          } else {  // suffix before the image start (a prefix longer than the entry offset)
#pragma unroll
            for (uint32_t d = 0; d < 4; ++d) {
              uint32_t wd = 0;
              for (uint32_t i = 0; i < 4; ++i) {
                const uint32_t x = o + 4 * d + i;
                wd |= uint32_t(x < p ? img[fk + x] : img[sb + x - p]) << (8 * i);
              }
              v[d] = wd;
            }
          }
          if (kl >= 16) out.put16(false, kout + o, v);
          else out.put_short(false, kout, kl, v);
        }
      }
    }
    if (valn) {
      uint8_t* const ob = L.out;
      // 16 bytes of the staged image at byte x (any alignment) from the 8-B-aligned dwords d[0..5]
      // that start at x & ~7: a dword select by bit 2, then v_alignbyte by x & 3
      // (the dword select by mask, not `b2 ? d[j + 1] : d[j]`: the compiler turned that into a
      // dynamically indexed array in scratch memory -- decode 3.35 ms)
      auto funnel = [](const uint32_t (&d)[6], uint32_t x, uint32_t (&v)[4]) {
        const uint32_t m = (x & 4) ? ~0u : 0u;
        uint32_t y[5];
#pragma unroll
        for (uint32_t j = 0; j < 5; ++j) y[j] = __builtin_amdgcn_bitop3_b32(m, d[j + 1], d[j], 0xCA);  // m ? d[j + 1] : d[j]
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i) v[i] = __builtin_amdgcn_alignbyte(y[i + 1], y[i], x & 3);
      };
      auto rd8 = [&](uint32_t x, uint32_t& lo, uint32_t& hi) {  // (x 8-B aligned)
        const u32x2 q = *reinterpret_cast<const u32x2*>(img + x);
        lo = q.x, hi = q.y;
      };
      const uint32_t cs = l == 0 ? (vD >> 4) : ((vD + 15) >> 4);
      const uint32_t a0 = vS + 16 * cs - vD;  // image byte of chunk cs's first byte (>= 0, see valn)
      uint32_t d[6], x8 = a0 & ~7u;
      rd8(x8, d[0], d[1]);
      rd8(x8 + 8, d[2], d[3]);
      rd8(x8 + 16, d[4], d[5]);
      for (uint32_t i = 0; i < vmmax; ++i) {
        if (i < vm) {
          uint32_t v[4];
          funnel(d, a0, v);
          const uint32_t c = cs + i, cut = vD + vl - 16 * c;  // bytes of the chunk from this value
          if (cut < 16 && k + 1 < n) {  // the rest from the next value
            const uint32_t a1 = vS1 + 16 * c - vD1, y8 = a1 & ~7u;
            uint32_t e[6], w[4];
            rd8(y8, e[0], e[1]);
            rd8(y8 + 8, e[2], e[3]);
            rd8(y8 + 16, e[4], e[5]);
            funnel(e, a1, w);
#pragma unroll
            for (uint32_t q = 0; q < 4; ++q) {
              const int32_t nb = int32_t(cut) - int32_t(4 * q);  // leading bytes of dword q from this value
              const uint32_t msk = nb <= 0 ? 0u : nb >= 4 ? ~0u : (1u << (8 * nb)) - 1;
              v[q] = (v[q] & msk) | (w[q] & ~msk);
            }
          }
          *reinterpret_cast<u32x4*>(ob + 16 * c) = u32x4{v[0], v[1], v[2], v[3]};
          d[0] = d[4], d[1] = d[5];
          x8 += 16;
          rd8(x8 + 8, d[2], d[3]);
          rd8(x8 + 16, d[4], d[5]);
        }
      }
    } else if (!(skip & 4)) {
      const uint32_t src = sb + s + 10;  // image byte of the value
      if (vl >= 16) {
        for (uint32_t i0 = 0; i0 < nvmax; i0 += kLB) {  // uniform trip count, pieces clamped
          u32x4 q[kLB];
          uint32_t o[kLB];
          // (diagnostics builds, ablation masks 32 / 64: the same accesses moved to 16- / 4-byte
          // aligned addresses -- timing probes of the misaligned accesses' cost, bytes wrong)
          const uint32_t am = (skip & 32) ? 15u : (skip & 64) ? 3u : 0u;
#pragma unroll
          for (uint32_t j = 0; j < kLB; ++j) {
            o[j] = min(16 * (i0 + j), vl - 16);
            q[j] = *reinterpret_cast<const u32x4*>(img + ((src + o[j]) & ~am));
          }
#pragma unroll
          for (uint32_t j = 0; j < kLB; ++j) {
            const uint32_t v[4] = {q[j].x, q[j].y, q[j].z, q[j].w};
            const uint32_t xa = (out.vb + vout + o[j]) & ~am;
            out.put16(true, xa >= out.vb ? xa - out.vb : xa + am + 1 - out.vb, v);
          }
        }
      } else if (vl) {
        const u32x4 q = *reinterpret_cast<const u32x4*>(img + src);
        const uint32_t v[4] = {q.x, q.y, q.z, q.w};
        out.put_short(true, vout, vl, v);
      }
    }
  }
}

// Aligned flush of an LDS output run by the wave: LDS bytes [lo, lo + len) -> global bytes at
// gdst_aligned + lo, the LDS run mirroring the global 16-B alignment (flush_chunks).
template <uint32_t B = kLB>
__device__ __forceinline__ void flush_run(uint8_t* gdst_aligned, const uint8_t* lds, uint32_t lo, uint32_t len) {
  flush_chunks<B, LSMBLK_XDEC_STORE>(gdst_aligned, lds, lo, len, lane_id(), 64);
}

// The same flush with the edge chunks byte-masked inside the chunk loop (emit: its register
// budget has no room for flush_chunks' separate edge pass).
template <uint32_t B>
__device__ __forceinline__ void flush_run_masked(uint8_t* gdst_aligned, const uint8_t* lds, uint32_t lo, uint32_t len) {
  const uint32_t end = lo + len, nc = (end + 15) >> 4;
  const uint32_t l = lane_id();
  for (uint32_t c0 = 0; c0 < nc; c0 += 64 * B) {
    u32x4 q[B];
#pragma unroll
    for (uint32_t j = 0; j < B; ++j) {
      const uint32_t c = c0 + 64 * j + l;
      if (c < nc) q[j] = *reinterpret_cast<const u32x4*>(lds + 16 * c);
    }
#pragma unroll
    for (uint32_t j = 0; j < B; ++j) {
      const uint32_t c = c0 + 64 * j + l;
      if (c < nc) {
        const uint32_t v[4] = {q[j].x, q[j].y, q[j].z, q[j].w};
        const uint32_t a0 = 16 * c < lo ? lo - 16 * c : 0u;
        const uint32_t a1 = min(end - 16 * c, 16u);
        store_chunk(gdst_aligned + 16 * c, v, a0, a1);
      }
    }
  }
}

__device__ void dec_fast_outputs(const DecodeArgs& a, DecLds& L, uint32_t lead, const BlockHdr& h,
                                 const DecEnt (&ent)[2], uint64_t E0, uint64_t K0, uint64_t V0, uint32_t K,
                                 uint32_t V, uint32_t skip) {
  const uint32_t kb = uint32_t(K0 & 15), vb = uint32_t(V0 & 15);
  const uint32_t vrun = (kb + K + 15) & ~15u;  // LDS start of the value run's first chunk
  // the flush reads whole 16-B chunks: the value run's last chunk must lie in the image
  if (vrun + ((vb + V + 15) & ~15u) <= kDecOut) {
    dec_entry_runs(a, L, lead, h.n, ent, E0, K0, V0, LdsSink{L.out, kb, vrun + vb}, skip);
    wave_sync();
    flush_run(a.keys + (K0 - kb), L.out, kb, K);
    flush_run(a.vals + (V0 - vb), L.out + vrun, vb, V);
  } else {
    const GlbSink g{make_rsrc_exact(a.keys + (K0 - kb), kb + K), make_rsrc_exact(a.vals + (V0 - vb), vb + V), kb, vb};
    dec_entry_runs(a, L, lead, h.n, ent, E0, K0, V0, g, skip);
  }
}

// ---------------------------------------------------------------- large blocks
// Blocks over the LDS image (config M: 64 KiB blocks, values up to 4 KiB) keep their entry
// tables in LDS, kDecMaxE entries at a time, and move bytes HBM -> HBM: every entry lane copies
// its key and value as 16-B unaligned buffer loads/stores (last piece overlapping), with
// kBigB pieces' loads issued before their stores (one memory round trip per kBigB pieces).
constexpr uint32_t kBigB = 8;

__device__ __forceinline__ u32x4 gload16(const rsrc_t& R, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(R, off, 0, 0);
}

// bytes [so, so + len) of RS -> bytes [dof, dof + len) of RD, any alignment on either side.
// RS bytes past lim are not the block's: a short run near the end is read byte by byte, so
// no 16-B load straddles the block end (the descriptor bound may zero a whole load).
__device__ __forceinline__ void copy_run(const rsrc_t& RS, uint32_t so, uint32_t lim, const rsrc_t& RD, uint32_t dof,
                                         uint32_t len) {
  if (len == 0) return;
  if (len < 16) {
    uint32_t v[4] = {0, 0, 0, 0};
    if (so + 16 <= lim) {
      const u32x4 q = gload16(RS, so);
      v[0] = q.x, v[1] = q.y, v[2] = q.z, v[3] = q.w;
    } else {
      for (uint32_t i = 0; i < len; ++i) v[i >> 2] |= __builtin_amdgcn_raw_buffer_load_b8(RS, so + i, 0, 0) << (8 * (i & 3));
    }
    st_short(RD, dof, len, v);
    return;
  }
  const uint32_t np = (len + 15) >> 4, last = len - 16;
  for (uint32_t j0 = 0; j0 < np; j0 += kBigB) {
    u32x4 q[kBigB];
#pragma unroll
    for (uint32_t j = 0; j < kBigB; ++j)
      if (j0 + j < np) q[j] = gload16(RS, so + min(16 * (j0 + j), last));
#pragma unroll
    for (uint32_t j = 0; j < kBigB; ++j)
      if (j0 + j < np) {
        const uint32_t v[4] = {q[j].x, q[j].y, q[j].z, q[j].w};
        st16(RD, dof + min(16 * (j0 + j), last), v);
      }
  }
}

// copy_run one 16-B piece at a time (few registers: for copies inside another loop's live range)
__device__ __forceinline__ void copy_run1(const rsrc_t& RS, uint32_t so, uint32_t lim, const rsrc_t& RD, uint32_t dof,
                                          uint32_t len) {
  if (len < 16) {
    copy_run(RS, so, lim, RD, dof, len);
    return;
  }
  const uint32_t last = len - 16;
  for (uint32_t o = 0;; o += 16) {
    const uint32_t x = min(o, last);
    const u32x4 q = gload16(RS, so + x);
    const uint32_t v[4] = {q.x, q.y, q.z, q.w};
    st16(RD, dof + x, v);
    if (x == last) break;
  }
}

// The same copy by the whole wave (len >= 16, wave-uniform arguments): lane j moves pieces
// j, j + 64, ... so a wave instruction moves 1 KiB of contiguous bytes.  Values of
// kCoop bytes or more go this way: one long value no longer keeps 63 lanes idle.
constexpr uint32_t kCoop = 16;  // M: 799 / 830-846 / 840 GiB/s at 256 / 32 / 16 (every run of 16 B or more packed)
__device__ __forceinline__ void copy_run_wave(const rsrc_t& RS, uint32_t so, const rsrc_t& RD, uint32_t dof,
                                              uint32_t len) {
  const uint32_t l = lane_id();
  const uint32_t np = (len + 15) >> 4, last = len - 16;
  for (uint32_t j0 = 0; j0 < np; j0 += 64 * kBigB) {
    u32x4 q[kBigB];
#pragma unroll
    for (uint32_t j = 0; j < kBigB; ++j) {
      const uint32_t idx = j0 + 64 * j + l;
      if (idx < np) q[j] = gload16(RS, so + min(16 * idx, last));
    }
#pragma unroll
    for (uint32_t j = 0; j < kBigB; ++j) {
      const uint32_t idx = j0 + 64 * j + l;
      if (idx < np) {
        const uint32_t v[4] = {q[j].x, q[j].y, q[j].z, q[j].w};
        st16(RD, dof + min(16 * idx, last), v);
      }
    }
  }
}

// Copies of every lane's run of kCoop bytes or more by the whole wave, packed: the runs' 16-B
// pieces are numbered consecutively over the lanes (wave scan of the piece counts) and each
// lane moves pieces lane, lane + 64, ... of that numbering, kBigB loads in flight per lane --
// so a wave round trip moves 8 KiB whatever the run lengths.  (One run after another cost a
// round trip per run: ~46 per 64 KiB block of config M.)  A run's last piece overlaps the one
// before, so any length >= 16 is covered exactly.
// A piece finds its run through the wave-private LDS scratch sc (kCopyScratch words): per row of
// 64 pieces, each run starting in the row marks its slot with its lane + 1, and an inclusive
// max-scan over the slots (carried from row to row) gives every piece its owner; the owner's
// {source, destination, length - 16, first piece} is one 16-B LDS read.  (Round 2 searched the
// lanes' first-piece numbers with 6 dependent ds_bpermutes and read the owner's fields with 4
// more; the copies are most of M's large-block encode.)
constexpr uint32_t kCopyScratch = 4 * 64 + 64;
static_assert(4 * kCopyScratch <= kDecOut, "the decode's large-block path lends its output image");

template <uint32_t B>
struct CopyBatch {
  u32x4 q[B];
  uint32_t dst[B];
};

// Rows g0 .. g0 + 64 B of the piece numbering: owners, then the pieces' loads.
template <uint32_t B>
__device__ __forceinline__ void copy_issue(const rsrc_t& RS, uint32_t g0, uint32_t total, uint32_t np, uint32_t first,
                                           uint32_t* sc, uint32_t& carry, CopyBatch<B>& c) {
  const uint32_t l = lane_id();
  const u32x4* rec = reinterpret_cast<const u32x4*>(sc);
  uint32_t* mark = sc + 4 * 64;
  uint32_t own[B];
#pragma unroll
  for (uint32_t j = 0; j < B; ++j) {
    const uint32_t G = g0 + 64 * j;
    own[j] = 0;
    if (G < total) {  // wave-uniform
      mark[l] = 0;
      wave_sync();
      if (np != 0 && first - G < 64u) mark[first - G] = l + 1;  // run starts are distinct pieces
      wave_sync();
      const uint32_t m = max(wave_incl_max32(mark[l]), carry);
      carry = __builtin_amdgcn_readlane(m, 63);
      own[j] = m - 1;
      wave_sync();  // this row's slot reads are done before the next row clears them
    }
  }
#pragma unroll
  for (uint32_t j = 0; j < B; ++j) {
    const uint32_t g = g0 + 64 * j + l;
    c.dst[j] = ~0u;
    if (g < total) {
      const u32x4 r = rec[own[j]];
      const uint32_t off = min(16 * (g - r.w), r.z);
      c.q[j] = gload16(RS, r.x + off);
      c.dst[j] = r.y + off;
    }
  }
}

template <uint32_t B>
__device__ __forceinline__ void copy_store(const rsrc_t& RD, const CopyBatch<B>& c) {
#pragma unroll
  for (uint32_t j = 0; j < B; ++j)
    if (c.dst[j] != ~0u) {
      const uint32_t v[4] = {c.q[j].x, c.q[j].y, c.q[j].z, c.q[j].w};
      st16(RD, c.dst[j], v);
    }
}

// after(lo, hi), if given, runs after each round's stores with the round's piece range [lo, hi)
// (hi = ~0u on the last round; once with [0, ~0u) when no lane has a run): lanes whose first
// piece number falls in it can store the bytes next to those pieces while their lines are hot.
struct NoAfter {
  __device__ void operator()(uint32_t, uint32_t, uint32_t) const {}
};
template <uint32_t B = kBigB, class After = NoAfter>
__device__ __forceinline__ void copy_long_runs(bool longrun, const rsrc_t& RS, uint32_t so, const rsrc_t& RD,
                                               uint32_t dof, uint32_t len, uint32_t* sc, const After& after = After()) {
  const uint32_t l = lane_id();
  const uint32_t np = longrun ? (len + 15) >> 4 : 0u;
  const uint32_t incl = wave_incl_scan32(np);
  const uint32_t total = __builtin_amdgcn_readlane(incl, 63);
  const uint32_t first = incl - np;  // this lane's first piece number
  if (total == 0) {
    after(first, 0u, ~0u);
    return;
  }
  wave_sync();                       // the scratch's previous readers are done
  reinterpret_cast<u32x4*>(sc)[l] = u32x4{so, dof, len - 16, first};  // read only for lanes with a run
  uint32_t carry = 0;  // owner + 1 of the previous row's last piece
  for (uint32_t g0 = 0; g0 < total; g0 += 64 * B) {
    CopyBatch<B> c;
    copy_issue(RS, g0, total, np, first, sc, carry, c);
    copy_store(RD, c);
    after(first, g0, g0 + 64 * B >= total ? ~0u : g0 + 64 * B);
  }
}

// One entry of a large block: ts / key_off / val_off, and the key (first-key bytes below p,
// suffix bytes from there on, one 16-B load of each source per piece, merged under byte
// masks; byte loads where a piece would read past the block end).
__device__ __forceinline__ void dec_big_entry(const DecodeArgs& a, const DecTables& L, const GlbImg& im, uint32_t k,
                                              uint32_t lim, const rsrc_t& RK, uint32_t kb, uint64_t E0, uint64_t K0,
                                              uint64_t V0) {
  const rsrc_t& R = im.r;
  const uint32_t lead = im.lead, fk = lead + 4;  // descriptor byte of the first key
  const uint32_t epos = L.epos[k], p = L.pfx[k], s = L.sfx[k], kout = L.kout[k];
  const uint32_t sb = lead + epos + 4, kl = p + s;  // descriptor byte of the suffix
  const uint64_t e = E0 + k;
  a.ts[e] = im.u64(epos + 4 + s);
  a.key_off[e] = uint32_t(K0 + kout);
  a.val_off[e] = uint32_t(V0 + L.vout[k]);
  for (uint32_t t = 0; t < kl; t += 16) {
    const uint32_t o = kl >= 16 ? min(t, kl - 16) : 0u;
    uint32_t v[4];
    if (sb + o >= p && sb + o - p + 16 <= lim && fk + o + 16 <= lim) {
      const u32x4 sq = gload16(R, sb + o - p), fq = gload16(R, fk + o);
      const uint32_t sv[4] = {sq.x, sq.y, sq.z, sq.w}, fv[4] = {fq.x, fq.y, fq.z, fq.w};
#pragma unroll
      for (uint32_t d = 0; d < 4; ++d) {
        const int32_t nf = int32_t(p) - int32_t(o + 4 * d);  // leading bytes from the first key
        const uint32_t m = nf <= 0 ? 0u : nf >= 4 ? ~0u : (1u << (8 * nf)) - 1;
        v[d] = (fv[d] & m) | (sv[d] & ~m);
      }
    } else {
#pragma unroll
      for (uint32_t d = 0; d < 4; ++d) {
        uint32_t wd = 0;
        for (uint32_t i = 0; i < 4; ++i) {
          const uint32_t x = o + 4 * d + i;
          wd |= (x < p ? im.u8(4 + x) : im.u8(epos + 4 + x - p)) << (8 * i);
        }
        v[d] = wd;
      }
    }
    if (kl >= 16) st16(RK, kb + kout + o, v);
    else st_short(RK, kb + kout, kl, v);
  }
}

#ifndef LSMBLK_XDBB
#define LSMBLK_XDBB 8
#endif
constexpr uint32_t kDecBigB = LSMBLK_XDBB;  // (experiment) pieces per lane per copy round, large-block decode

// Outputs of the n entries whose tables are in L (block entries Eb - E0 .. + n), large block.
__device__ void dec_big_outputs(const DecodeArgs& a, const DecTables& L, const rsrc_t& R, uint32_t lead,
                                const BlockHdr& h, uint32_t n, uint64_t Eb, uint64_t K0, uint64_t V0, uint32_t K,
                                uint32_t V, uint32_t* sc) {
  const uint32_t l = lane_id();
  const uint32_t kb = uint32_t(K0 & 15), vb = uint32_t(V0 & 15);
  const rsrc_t RK = make_rsrc_exact(a.keys + (K0 - kb), kb + K), RV = make_rsrc_exact(a.vals + (V0 - vb), vb + V);
  const GlbImg im{R, lead};
  const uint32_t lim = lead + h.len;  // descriptor byte of the block end
  for (uint32_t c = 0; c < n; c += 64) {  // uniform trip count: the wave copies long values
    const uint32_t k = c + l;
    const bool live = k < n;
    uint32_t vsrc = 0, vdst = 0, vl = 0;
    if (live) {
      dec_big_entry(a, L, im, k, lim, RK, kb, Eb, K0, V0);
      vsrc = lead + L.epos[k] + 14 + L.sfx[k];
      vdst = vb + L.vout[k];
      vl = L.vout[k + 1] - L.vout[k];
      if (vl < kCoop) copy_run(R, vsrc, lim, RV, vdst, vl);
    }
    copy_long_runs<kDecBigB>(live && vl >= kCoop, R, vsrc, RV, vdst, vl, sc);
  }
}

// Decode block b = [start, end) of the block stream.  mid() runs after the block's staging loads
// are issued and before they are written to LDS (the lagged decode counts another block through
// the image there, its loads issued before these).
// post() runs once the staging has landed, pre_wait() before the wait for the output base.
template <bool lagm, class Mid, class Post, class PreWait>
__device__ void decode_block(const DecodeArgs& a, DecLds& L, uint64_t b, uint64_t start, uint64_t end, Mid&& mid,
                             Post&& post, PreWait&& pre_wait) {
  const uint32_t l = lane_id();
  uint32_t err = 0;
  // Output-base loads depend only on b.  Two-pass: the tile prefix + the aggregates of the tile's
  // earlier blocks, issued first, they land during staging + parse.  Lagged decode: the block's
  // base granules (lanes 0-2), issued after the landing, under the entry parse: issued first they
  // returned before the tile finisher had published them about half the time (trace: the finish
  // ends ~1.6 us after the tile's first decoder starts), and the decoder then waited a re-poll
  // round trip (~1 us median); moved, decode 2.09 -> 2.05 ms at U (A/B, one box).
  const uint64_t tb = b / kTile, jb = b % kTile;
  uint32_t cn = 0, ck = 0, cv = 0;
  uint64_t tp0 = 0, tp1 = 0, tp2 = 0, gb = 0;
  if constexpr (!lagm) {
    if (l < jb) {
      const uint64_t q = tb * kTile + l;
      cn = a.agg[3 * q];
      ck = a.agg[3 * q + 1];
      cv = a.agg[3 * q + 2];
    }
    tp0 = a.tile_pre[3 * tb], tp1 = a.tile_pre[3 * tb + 1], tp2 = a.tile_pre[3 * tb + 2];
  }
  uint32_t len = 0;
  if (end < start + a.tail || end - start > 0x7FFFFFF0ull) err |= LSMBLK_ERR_MALFORMED;
  else len = uint32_t(end - start) - a.tail;
  const uint8_t* bp = a.blocks + start;
  const uint32_t lead = uni(uint32_t(reinterpret_cast<uintptr_t>(bp) & 15));
  const uint8_t* abase = bp - lead;
  const rsrc_t R = make_rsrc(abase, lead + len);
  const bool fits = lead + len + 15 <= kDecImg;  // the staging writes whole 16-B chunks

  BlockHdr h;
  if (fits) {
    // all loads in flight before the first LDS write (kDecImg / 1 KiB = at most 5 per lane)
    const uint32_t nchunk = (lead + len + 15) >> 4;
    u32x4 v[5];
    if constexpr (lagm) {
      // Issued by inline asm so that the compiler can neither sink them below mid() (it did, below
      // the whole count) nor wait for them inside it: mid()'s own waits count only the loads the
      // compiler issued, so they over-wait by these (safe: returns are in issue order).  Landed
      // by the explicit vmcnt(0) below, before any store is issued after them.
      const uint32_t o = 16 * l, o4 = o + 4096;
      // (one statement led by s_nop 4: a VALU write of R's SGPRs needs 5 wait states before a VMEM
      // read of them, which the compiler's hazard pass does not check inside asm)
      asm volatile(
          "s_nop 4\n\t"
          "buffer_load_dwordx4 %0, %5, %7, 0 offen\n\t"
          "buffer_load_dwordx4 %1, %5, %7, 0 offen offset:1024\n\t"
          "buffer_load_dwordx4 %2, %5, %7, 0 offen offset:2048\n\t"
          "buffer_load_dwordx4 %3, %5, %7, 0 offen offset:3072\n\t"
          "buffer_load_dwordx4 %4, %6, %7, 0 offen"
          : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4])
          : "v"(o), "v"(o4), "s"(R));
      mid();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (uint32_t i = 0; i < 5; ++i) asm volatile("" : "+v"(v[i]));  // defined here for the compiler
    } else {
#pragma unroll
      for (uint32_t i = 0; i < 5; ++i)
        v[i] = __builtin_amdgcn_raw_buffer_load_b128(R, (l + 64 * i) * 16, 0, kLdAux);  // 0 past the block
    }
#pragma unroll
    for (uint32_t i = 0; i < 5; ++i)
      if (l + 64 * i < nchunk) *reinterpret_cast<u32x4*>(L.img + (l + 64 * i) * 16) = v[i];
    wave_sync();
    post();
    if (lagm && l < 3 && !(diag_mask(a.skip) & 4096)) gb = gload(a.bbase + 3 * b + l, 0);  // (4096: ablation)
    h = parse_hdr(LdsImg{L.img, lead}, len);
  } else {
    mid();
    post();
    if (lagm && l < 3 && !(diag_mask(a.skip) & 4096)) gb = gload(a.bbase + 3 * b + l, 0);
    h = parse_hdr(GlbImg{R, lead}, len);
  }
  if (diag_mask(a.skip) & 256) return;  // ablation: staging only
  if (!h.ok) err |= LSMBLK_ERR_MALFORMED;
  const bool fast = fits && h.n <= kDecMaxE;
  // large block: entry tables in LDS, bytes HBM -> HBM; more than kDecMaxE entries are taken
  // kDecMaxE at a time (the tables of each chunk are built just before its outputs)
  const bool big = !fits;

  // phase 1: parse entries, block aggregates (entries, key bytes, value bytes)
  uint64_t K = 0, V = 0;
  bool bad = false;
  DecTables& T = *reinterpret_cast<DecTables*>(L.img);  // large blocks only (not staged)
  // tables of entries [c0, c0 + cn) (cn <= kDecMaxE) at table rows 0 .. cn, output offsets
  // from the block's key / value bytes before c0 (kr, vr)
  auto parse_tables = [&](const auto& im, uint32_t c0, uint32_t cn, uint64_t& kr, uint64_t& vr) {
    for (uint32_t c = 0; c < cn; c += 64) {
      const uint32_t k = c + l;
      uint32_t off = 0, p = 0, s = 0, vl = 0;
      bool ok = true;
      if (k < cn) ok = parse_entry(im, h, c0 + k, off, p, s, vl);
      bad = bad || !ok;
      const uint32_t kl = p + s;
      const uint32_t ki = wave_incl_scan<uint32_t>(kl), vi = wave_incl_scan<uint32_t>(vl);
      if (k < cn) {
        T.epos[k] = uint16_t(off);
        T.pfx[k] = uint16_t(p);
        T.sfx[k] = uint16_t(s);
        T.kout[k] = uint32_t(kr) + ki - kl;
        T.vout[k] = uint32_t(vr) + vi - vl;
      }
      kr += __shfl(ki, 63, 64);
      vr += __shfl(vi, 63, 64);
    }
    if (l == 0) {
      T.kout[cn] = uint32_t(kr);
      T.vout[cn] = uint32_t(vr);
    }
  };
  DecEnt ent[2] = {};
  if (fast) {  // entries l and l + 64 stay in this lane's registers
    const LdsImg im{L.img, lead};
#pragma unroll
    for (uint32_t it = 0; it < 2; ++it) {
      if (64 * it >= h.n) break;
      const uint32_t k = 64 * it + l;
      uint32_t off = 0, p = 0, s = 0, vl = 0;
      bool ok = true;
      if (k < h.n) ok = parse_entry(im, h, k, off, p, s, vl);
      bad = bad || !ok;
      const uint32_t kl = p + s;
      const uint32_t ki = wave_incl_scan<uint32_t>(kl), vi = wave_incl_scan<uint32_t>(vl);
      ent[it] = DecEnt{off, p, s, uint32_t(K) + ki - kl, uint32_t(V) + vi - vl, vl};
      K += __shfl(ki, 63, 64);
      V += __shfl(vi, 63, 64);
    }
  } else if (big && h.n <= kDecMaxE) {
    parse_tables(GlbImg{R, lead}, 0, h.n, K, V);
  } else {
    for (uint32_t c = 0; c < h.n; c += 64) {
      const uint32_t k = c + l;
      uint32_t off = 0, p = 0, s = 0, vl = 0;
      bool ok = true;
      if (k < h.n) {
        if (fits) ok = parse_entry(LdsImg{L.img, lead}, h, k, off, p, s, vl);
        else ok = parse_entry(GlbImg{R, lead}, h, k, off, p, s, vl);
      }
      bad = bad || !ok;
      K += wave_sum<uint64_t>(p + s);
      V += wave_sum<uint64_t>(vl);
    }
  }
  if (diag_mask(a.skip) & 512) return;  // ablation: staging + entry tables only
  if (__ballot(bad)) err |= LSMBLK_ERR_MALFORMED;
  uint64_t agg[3] = {h.n, K, V};
  if (err) agg[0] = agg[1] = agg[2] = 0;

  pre_wait();
  // output bases: tile prefix + this tile's earlier blocks
  uint64_t excl[3];
  if constexpr (lagm) {
    // the block's base, published by its tile's last counter (normally long since there)
    const uint64_t want = (uint64_t(a.tag) << 2) | 2;
    uint32_t spins = 0;
    if (b % kTile == 0) dbg_trace(a.dbg, b / kTile, 2);
    while (!(diag_mask(a.skip) & 2048) && __ballot(l < 3 && (gb & 0xFFFF) != want)) {  // (2048: ablation, no wait)
      if (++spins > kSpinLimit) {
        err |= LSMBLK_ERR_TIMEOUT;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      if (l < 3 && (gb & 0xFFFF) != want) gb = gload(a.bbase + 3 * b + l, a.poll);
    }
#pragma unroll
    for (uint32_t q = 0; q < 3; ++q)
      excl[q] = uint64_t(uint32_t(__builtin_amdgcn_readlane(uint32_t(gb >> 16), q))) |
                (uint64_t(uint32_t(__builtin_amdgcn_readlane(uint32_t(gb >> 48), q))) << 32);
    if (b % kTile == 0) dbg_trace(a.dbg, b / kTile, 3);
  } else {
    excl[0] = tp0 + wave_sum(cn);
    excl[1] = tp1 + wave_sum(ck);
    excl[2] = tp2 + wave_sum(cv);
  }
  wave_sync();
  const uint64_t E0 = excl[0], K0 = excl[1], V0 = excl[2];
  if (a.blk_ent && l == 0) a.blk_ent[b] = E0;
  const uint64_t Et = E0 + agg[0], Kt = K0 + agg[1], Vt = V0 + agg[2];
  if (Kt > 0xFFFFFFFFull || Vt > 0xFFFFFFFFull) err |= LSMBLK_ERR_OVERFLOW;
  if (Et > a.entry_cap || Kt > a.key_cap || Vt > a.val_cap) err |= LSMBLK_ERR_CAPACITY;
  if (lagm && b + 1 == a.nblk && l == 0) {  // totals, required sizes and the sentinels (as dec_scan_kernel)
    if (a.blk_ent) a.blk_ent[a.nblk] = Et;
    a.stats[0] = Et;
    a.stats[1] = Kt;
    a.stats[2] = Vt;
    if (Et <= a.entry_cap) {
      a.key_off[Et] = uint32_t(Kt);
      a.val_off[Et] = uint32_t(Vt);
    }
  }

  if (!(err & (LSMBLK_ERR_MALFORMED | LSMBLK_ERR_TIMEOUT | LSMBLK_ERR_OVERFLOW | LSMBLK_ERR_CAPACITY)) && h.n) {
    if (fast) {
      dec_fast_outputs(a, L, lead, h, ent, E0, K0, V0, uint32_t(K), uint32_t(V), diag_mask(a.skip));
    } else if (big && h.n <= kDecMaxE) {
      dec_big_outputs(a, T, R, lead, h, h.n, E0, K0, V0, uint32_t(K), uint32_t(V), reinterpret_cast<uint32_t*>(L.out));
    } else if (big) {
      uint64_t kr = 0, vr = 0;
      for (uint32_t c0 = 0; c0 < h.n; c0 += kDecMaxE) {
        const uint32_t nc = min(kDecMaxE, h.n - c0);
        wave_sync();  // the previous chunk's table reads are done
        parse_tables(GlbImg{R, lead}, c0, nc, kr, vr);
        wave_sync();
        dec_big_outputs(a, T, R, lead, h, nc, E0 + c0, K0, V0, uint32_t(K), uint32_t(V), reinterpret_cast<uint32_t*>(L.out));
      }
    } else if (fits) {
      dec_simple_outputs(a, LdsImg{L.img, lead}, h, E0, K0, V0);
    } else {
      dec_simple_outputs(a, GlbImg{R, lead}, h, E0, K0, V0);
    }
  }
  raise_err(a.stats, err);
}

// One wave per block, no inter-wave waiting: the bases come from the count + scan passes.
// One single-wave workgroup per block (LDS, not waves, bounds the residency: single-wave
// workgroups pack the CU's LDS best).  No inter-wave waiting: the output bases come from the
// count + scan passes.
__global__ __launch_bounds__(64) void decode_kernel(DecodeArgs a) {
  __shared__ DecLds lds;
  const uint64_t b = blockIdx.x;
  decode_block<false>(a, lds, b, uni64(a.blk_off[b]), uni64(a.blk_off[b + 1]), [] {}, [] {}, [] {});
}

// ---------------------------------------------------------------- lagged decode (one launch)
// E is read from HBM once.  Workgroup j counts block j (stages it, parses its headers with decode's
// rules, publishes its (entries, key bytes, value bytes) as a tagged granule) and then decodes
// block j - lag.  The counts run `lag` blocks ahead of the decodes, so:
//   * a block's output base is ready long before its decode starts: the last counter of each
//     64-block tile sums the tile, finds the tile's prefix by a decoupled look-back over tiles and
//     publishes every block's base (one granule triple per block, read by its decoder);
//   * the decode's second read of the block comes from the Infinity Cache: between the two reads
//     the chip reads `lag` further blocks and writes their decoded bytes (~8 KiB each; lag 10240
//     = 84 MB of the 256 MB cache; lag 8192 / 10240 / 12288: decode 2.11 / 2.08-2.09 / 2.10 ms).
// Every wait is on lower-indexed workgroups (dispatch is in index order), bounded by kSpinLimit
// (then TIMEOUT).  The two-pass path (count, tile scan, decode: three launches) remains for the
// CRC-verifying read and as the A/B diagnostic.
// Measured before: a single pass holding each block in LDS across its
// look-back (tiles of 4 blocks, one wave each) took 3.4 ms against 2.3 for the two passes -- the
// look-back waits idle the LDS that bounds decode's residency.

__device__ __forceinline__ uint64_t sat47(uint64_t v) { return v > (1ull << 47) - 1 ? (1ull << 47) - 1 : v; }

// Lanes 0..2 publish (x0, x1, x2) as three granules (scalars, not an array the lane would index:
// that compiled to a scratch round trip).
__device__ __forceinline__ void publish3(uint64_t* arr, uint64_t idx, uint64_t x0, uint64_t x1, uint64_t x2,
                                         uint32_t tag, uint32_t flag, uint32_t poll) {
  const uint32_t l = lane_id();
  const uint64_t x = l == 0 ? x0 : (l == 1 ? x1 : x2);
  if (l < 3) gstore(arr + 3 * idx + l, (sat47(x) << 16) | (uint64_t(tag) << 2) | flag, poll);
}

// (entries, key bytes, value bytes) of block [start, end) with decode's rules; malformed ->
// (0, 0, 0), bad.  cnt_issue issues the staging loads (a block that fits the image), cnt_finish
// lands them in img and parses there (else parses from global memory).
struct BlkCount {
  uint32_t n;
  uint64_t K, V;
  bool bad;
};
struct CntPre {
  rsrc_t R;
  uint32_t len, lead;
  bool ok, staged;
  u32x4 v[5];
};
__device__ __forceinline__ CntPre cnt_issue(const uint8_t* blocks, uint32_t tail, uint64_t start, uint64_t end) {
  const uint32_t l = lane_id();
  CntPre C;
  C.ok = !(end < start + tail || end - start > 0x7FFFFFF0ull);
  C.len = C.ok ? uint32_t(end - start) - tail : 0u;
  const uint8_t* bp = blocks + start;
  C.lead = uni(uint32_t(reinterpret_cast<uintptr_t>(bp) & 15));
  C.R = make_rsrc(bp - C.lead, C.lead + C.len);
  C.staged = C.ok && C.lead + C.len + 15 <= kDecImg;
  if (C.staged) {
#pragma unroll
    for (uint32_t i = 0; i < 5; ++i)
      C.v[i] = __builtin_amdgcn_raw_buffer_load_b128(C.R, (l + 64 * i) * 16, 0, kLdAux);  // 0 past the block
  }
  return C;
}
__device__ __forceinline__ BlkCount cnt_finish(const CntPre& C, uint8_t* img) {
  const uint32_t l = lane_id();
  BlkCount r{0, 0, 0, false};
  bool bad = false;
  auto count = [&](const auto& im) {
    const BlockHdr h = parse_hdr(im, C.len);
    if (!h.ok) {
      bad = true;
      return;
    }
    r.n = h.n;
    if constexpr (std::is_same_v<std::decay_t<decltype(im)>, GlbImg>) {
      // a large block's headers from global memory: entries l and l + 64 parsed side by side
      // (indices clamped, so both dependent load chains are straight-line code and overlap)
      for (uint32_t c = 0; c < h.n; c += 128) {
        const uint32_t k0 = c + l, k1 = c + 64 + l;
        const bool l0 = k0 < h.n, l1 = k1 < h.n;
        uint32_t o0, p0, s0, v0, o1, p1, s1, v1;
        const bool ok0 = parse_entry(im, h, l0 ? k0 : h.n - 1, o0, p0, s0, v0);
        const bool ok1 = parse_entry(im, h, l1 ? k1 : h.n - 1, o1, p1, s1, v1);
        if ((l0 && !ok0) || (l1 && !ok1)) bad = true;
        r.K += wave_sum<uint32_t>((l0 ? p0 + s0 : 0u) + (l1 ? p1 + s1 : 0u));
        r.V += wave_sum<uint32_t>((l0 ? v0 : 0u) + (l1 ? v1 : 0u));
      }
    } else {
      for (uint32_t c = 0; c < h.n; c += 64) {
        const uint32_t k = c + l;
        uint32_t off = 0, p = 0, s = 0, vl = 0;
        if (k < h.n && !parse_entry(im, h, k, off, p, s, vl)) bad = true;
        r.K += wave_sum<uint32_t>(p + s);
        r.V += wave_sum<uint32_t>(vl);
      }
    }
  };
  if (C.staged) {
    const uint32_t nchunk = (C.lead + C.len + 15) >> 4;
#pragma unroll
    for (uint32_t i = 0; i < 5; ++i)
      if (l + 64 * i < nchunk) *reinterpret_cast<u32x4*>(img + (l + 64 * i) * 16) = C.v[i];
    wave_sync();
    count(LdsImg{img, C.lead});
  } else if (C.ok) {
    count(GlbImg{C.R, C.lead});
  }
  if (!C.ok || __ballot(bad)) {
    r.bad = true;
    r.n = 0;
    r.K = r.V = 0;
  }
  return r;
}

// The last counter of tile t: waits for the tile's aggregates, publishes the tile aggregate, looks
// back over the tiles for its prefix, publishes the inclusive prefix and every block's base.
struct FinPf {
  uint64_t g0, g1, g2;
};
__device__ __forceinline__ FinPf fin_prefetch(const DecodeArgs& a, uint64_t t) {
  const uint32_t l = lane_id();
  const uint64_t b0 = t * kTile, nb = min(uint64_t(kTile), a.nblk - b0);
  const uint64_t want = (uint64_t(a.tag) << 2) | 1;
  FinPf f{want, want, want};  // lanes >= nb read as present zeros
  if (l < nb) {
    f.g0 = gload(a.bagg + 3 * (b0 + l), 0);
    f.g1 = gload(a.bagg + 3 * (b0 + l) + 1, 0);
    f.g2 = gload(a.bagg + 3 * (b0 + l) + 2, 0);
  }
  return f;
}
__device__ void lag_tile_finish(const DecodeArgs& a, uint64_t t, uint32_t& err, const FinPf* pf = nullptr) {
  const uint32_t l = lane_id();
  dbg_trace(a.dbg, t, 0);
  const uint64_t b0 = t * kTile, nb = min(uint64_t(kTile), a.nblk - b0);
  const uint64_t want = (uint64_t(a.tag) << 2) | 1;
  const bool mine = l < nb;
  const FinPf f0 = pf ? *pf : fin_prefetch(a, t);
  uint64_t g0 = f0.g0, g1 = f0.g1, g2 = f0.g2;
  uint32_t spins = 0;
  for (;;) {
    const bool here = (g0 & 0xFFFF) == want && (g1 & 0xFFFF) == want && (g2 & 0xFFFF) == want;
    if (!__ballot(!here)) break;
    if (++spins > kSpinLimit) {
      err |= LSMBLK_ERR_TIMEOUT;
      return;  // the decoders of this tile time out too: the call reports TIMEOUT
    }
    __builtin_amdgcn_s_sleep(1);
    if (!here) {
      g0 = gload(a.bagg + 3 * (b0 + l), a.poll);
      g1 = gload(a.bagg + 3 * (b0 + l) + 1, a.poll);
      g2 = gload(a.bagg + 3 * (b0 + l) + 2, a.poll);
    }
  }
  const uint64_t x0 = mine ? g0 >> 16 : 0, x1 = mine ? g1 >> 16 : 0, x2 = mine ? g2 >> 16 : 0;
  const uint64_t i0 = wave_incl_scan<uint64_t>(x0), i1 = wave_incl_scan<uint64_t>(x1), i2 = wave_incl_scan<uint64_t>(x2);
  const uint64_t A[3] = {lane64(i0, 63), lane64(i1, 63), lane64(i2, 63)};
  uint64_t X[3] = {0, 0, 0};
  if (t == 0) {
    publish3(a.tinc, t, A[0], A[1], A[2], a.tag, 2, a.poll);
  } else {
    publish3(a.tagg, t, A[0], A[1], A[2], a.tag, 1, a.poll);
    // tile t-1's inclusive prefix if it is there at once, else the wave-parallel look-back
    const uint64_t wi = (uint64_t(a.tag) << 2) | 2;
    uint64_t g = wi;
    if (l < 3) g = gload(a.tinc + 3 * (t - 1) + l, 0);
    if (!__ballot(l < 3 && (g & 0xFFFF) != wi)) {
#pragma unroll
      for (uint32_t q = 0; q < 3; ++q)
        X[q] = uint64_t(uint32_t(__builtin_amdgcn_readlane(uint32_t(g >> 16), q))) |
               (uint64_t(uint32_t(__builtin_amdgcn_readlane(uint32_t(g >> 48), q))) << 32);
    } else {
      if (!lookback<3>(a.tagg, a.tinc, t, a.tag, a.poll, X)) {
        err |= LSMBLK_ERR_TIMEOUT;
        return;
      }
    }
    publish3(a.tinc, t, X[0] + A[0], X[1] + A[1], X[2] + A[2], a.tag, 2, a.poll);
  }
  if (mine) {
    const uint64_t tg = (uint64_t(a.tag) << 2) | 2;
    gstore(a.bbase + 3 * (b0 + l), (sat47(X[0] + i0 - x0) << 16) | tg, a.poll);
    gstore(a.bbase + 3 * (b0 + l) + 1, (sat47(X[1] + i1 - x1) << 16) | tg, a.poll);
    gstore(a.bbase + 3 * (b0 + l) + 2, (sat47(X[2] + i2 - x2) << 16) | tg, a.poll);
  }
  if (kDiag && a.dbg) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    dbg_trace(a.dbg, t, 1);
  }
}

__global__ __launch_bounds__(64) void decode_lag_kernel(DecodeArgs a) {
  __shared__ DecLds lds;
  // Workgroup indices, the lag and the block count are below 2^31 (lsmblk_decode_batch_ex), so the
  // per-workgroup bookkeeping is 32-bit: the scalar unit, not the vector one, is the decode's most
  // loaded pipe (PMC), and 64-bit scalar math costs it two to four times more.
  const uint32_t j = blockIdx.x, nblk = uint32_t(a.nblk), lag0 = uint32_t(a.lag);
  const bool cnt = j < nblk;
  // both blocks' ranges first, then the count's staging loads, then (inside decode_block) the
  // decode's: the count waits only for its own loads
  // (one load instruction: lanes 0-1 the count's range, lanes 2-3 the decode's at the largest lag)
  // The lag scales with the block size (lag_bytes): the decode re-reads its block's bytes lag
  // blocks after the count did (the parse of a large block, the whole staged image of a small
  // one), and those reads should come from the Infinity Cache.  Measured on config M (64 KiB
  // blocks): decode 2.11 ms at lag 10240 (640 MiB apart, headers re-read from HBM: 6.2 GB
  // fetched for 4.3 GB of blocks), 2.02 at 640 (40 MiB, as 10240 x 4 KiB) and 2.01 at 320.
  const uint32_t l = lane_id();
  uint64_t o = 0;
  if ((l < 2 && cnt) || (l >= 2 && l < 4 && j >= lag0)) o = a.blk_off[(l < 2 ? j : j - lag0) + (l & 1)];
  // the batch's first and last offsets: scalar loads (as vector-load lanes they cost U's decode ~1 %)
  const uint64_t o0 = a.lag_bytes ? a.blk_off[0] : 0, o1 = a.lag_bytes ? a.blk_off[nblk] : 0;
  const uint64_t cs = lane64(o, 0), ce = lane64(o, 1);
  CntPre C;
  const bool do_cnt = cnt && !(diag_mask(a.skip) & 1024);  // (1024: ablation, aggregates 0 without the count)
  if (do_cnt) C = cnt_issue(a.blocks, a.tail, cs, ce);
  uint32_t lag = lag0;  // (worked out under the count's loads)
  if (a.lag_bytes) {
    // lag_bytes / mean block size < lag?  (4 KiB units: 32 x 32-bit products; the divide only then)
    const uint32_t tot = uint32_t(min((o1 - o0) >> 12, uint64_t(0xFFFFFFFFu))), lb = uint32_t(a.lag_bytes >> 12);
    if (uint64_t(lb) * nblk < uint64_t(lag) * tot) {
      const uint32_t want = uint32_t(float(lb) * (float(nblk) / float(tot)));
      lag = want < 2 * kTile ? 2 * kTile : want;
    }
  }
  if (j >= nblk + lag) return;  // (the grid is sized for the largest lag; no count was issued here)
  const bool dec = j >= lag;
  if (j % kTile == 0) dbg_trace(a.dbg, j / kTile, 4);                       // the tile's first count starts
  if (dec && (j - lag) % kTile == 0) dbg_trace(a.dbg, (j - lag) / kTile, 5);  // its first decoder starts
  const uint32_t b = j - lag;
  if (lag != lag0 && dec && l >= 2 && l < 4) o = a.blk_off[b + (l & 1)];  // (wave-uniform branch)
  const uint64_t ds = lane64(o, 2), de = lane64(o, 3);
  uint32_t err = 0;
  BlkCount r{0, 0, 0, false};
  auto count = [&] {
    if (!do_cnt) return;
    r = cnt_finish(C, lds.img);
    wave_sync();  // the count's image reads are done before the decode stages into it
  };
  // (the count's aggregate is published after the decode's staging has landed: a store issued
  // before the landing's vmcnt(0) would be waited for there)
  // Tile t's bases are published by workgroup f(t) = 64 t + 63 + lag / 2 - (t & 7), after its own
  // block's entry parse and before its own decode waits for a base.  By then the tile's counts
  // have long been published (no waiting on a slow XCD's tile-mates), f(t) < f(t + 1) (the tile
  // look-back finds its predecessors' aggregates), f(t) is far below the tile's first decoder
  // (64 t + lag), and the finishers rotate over the XCDs (workgroup j runs on XCD j mod 8).
  // Measured before: the tile's last-arriving count finishing it (an arrival counter) put every
  // tile finish on the slowest XCD -- which then stayed `lag` behind, the other XCDs' decoders
  // waiting (2.8 ms at every lag); the tile's last block finishing it after its own decode
  // chained the tiles `lag` apart into one serial sequence (2.7 ms).
  const uint32_t D = lag / 2 + 63;
  const uint32_t ft = j >= D ? (j - D + 8) / kTile : ~0u;  // the tile workgroup j finishes, if any
  const bool fin = j >= D && ft * kTile + D - (ft & 7) == j && ft * kTile < nblk;
  auto publish = [&] {
    if (!cnt || (diag_mask(a.skip) & 16384)) return;  // (16384: ablation, no publish)
    // (a malformed block is reported by its decoder; its aggregate is 0 there too)
    publish3(a.bagg, j, r.n, r.K, r.V, a.tag, 1, a.poll);
    if (r.K > 0xFFFFFFFFull || r.V > 0xFFFFFFFFull) err |= LSMBLK_ERR_OVERFLOW;
  };
  // a finisher loads its tile's aggregates now, under its own staging and count (they are
  // normally all there: the tile's counts ran lag / 2 workgroups earlier); its finish re-polls
  // only those that were not
  FinPf fpf{};
  if (fin) fpf = fin_prefetch(a, ft);
  auto finish = [&] {
    if (fin && !(diag_mask(a.skip) & (8192 | 16384))) lag_tile_finish(a, ft, err, &fpf);  // (8192: ablation, no tile finish)
  };
  if (dec) {
    decode_block<true>(a, lds, b, ds, de, count, publish, finish);
  } else {
    count();
    publish();
    finish();
  }
  raise_err(a.stats, err);
}

// ---------------------------------------------------------------- decode pass 1: count
// (the two-pass decode: the CRC-verifying read path and the A/B diagnostic)
struct CountArgs {
  const uint8_t* blocks;
  const uint64_t* blk_off;
  uint64_t nblk;
  uint32_t* agg;        // 3 per block
  uint64_t* tile_sum;   // 3 per tile
  uint64_t* stats;
  uint32_t tail;        // bytes after each block inside its range (4: the framing CRC)
};

// Count pass: one single-wave workgroup per block streams the whole block into LDS with
// coalesced 16-B loads (4 KiB of LDS: up to 32 waves per CU) and parses every header there with
// decode's own rules (parse_hdr / parse_entry).  Reading all of E in full lines costs less than
// a header-only parse with byte loads (round 1: 0.86 against 0.75 ms): those touch a 64-B sector
// per entry, which at U's 128-B entries is most of E anyway, in scattered requests.  Blocks over
// the image parse from global memory.  Tile sums: agg_tile_kernel.
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(8))) void dec_count_staged_kernel(CountArgs a) {
  __shared__ alignas(16) uint8_t img[kDecImg];
  const uint64_t b = blockIdx.x;
  const BlkCount r = cnt_finish(cnt_issue(a.blocks, a.tail, uni64(a.blk_off[b]), uni64(a.blk_off[b + 1])), img);
  uint32_t err = r.bad ? LSMBLK_ERR_MALFORMED : 0u;
  if (lane_id() == 0) {
    a.agg[3 * b] = r.n;
    a.agg[3 * b + 1] = uint32_t(r.K > 0xFFFFFFFFull ? 0xFFFFFFFFull : r.K);
    a.agg[3 * b + 2] = uint32_t(r.V > 0xFFFFFFFFull ? 0xFFFFFFFFull : r.V);
    if (r.K > 0xFFFFFFFFull || r.V > 0xFFFFFFFFull) err |= LSMBLK_ERR_OVERFLOW;
  }
  raise_err(a.stats, err);
}

// ---------------------------------------------------------------- decode pass 2: tile scan
// One workgroup: exclusive scan of the per-tile sums; totals, capacity / overflow checks and
// the key_off[N] / val_off[N] sentinels.
struct ScanArgs {
  const uint64_t* tile_sum;
  uint64_t* tile_pre;
  uint64_t ntiles;
  uint32_t* key_off;
  uint32_t* val_off;
  uint64_t entry_cap, key_cap, val_cap;
  uint64_t* stats;
  uint64_t* blk_ent;   // optional: [nblk] = total entries
  uint64_t nblk;
};

__global__ __launch_bounds__(1024) void dec_scan_kernel(ScanArgs a) {
  __shared__ uint64_t part[32][3];  // wave totals, then wave bases
  const uint32_t t = threadIdx.x;
  const uint64_t per = (a.ntiles + 1023) / 1024, lo = t * per, hi = lo + per < a.ntiles ? lo + per : a.ntiles;
  uint64_t s0 = 0, s1 = 0, s2 = 0;
#pragma unroll 8
  for (uint64_t i = lo; i < hi; ++i) {  // (unrolled: the tiles' loads in flight together)
    s0 += a.tile_sum[3 * i];
    s1 += a.tile_sum[3 * i + 1];
    s2 += a.tile_sum[3 * i + 2];
  }
  // block scan of the 1024 partials: wave scans, then one wave over the 16 wave totals (two
  // barriers; a Hillis-Steele scan over LDS took twenty)
  const uint32_t l = t & 63, w = t >> 6;
  uint64_t i0 = wave_incl_scan<uint64_t>(s0), i1 = wave_incl_scan<uint64_t>(s1), i2 = wave_incl_scan<uint64_t>(s2);
  if (l == 63) {
    part[w][0] = i0;
    part[w][1] = i1;
    part[w][2] = i2;
  }
  __syncthreads();
  if (w == 0) {
    uint64_t x0 = l < 16 ? part[l][0] : 0, x1 = l < 16 ? part[l][1] : 0, x2 = l < 16 ? part[l][2] : 0;
    const uint64_t y0 = wave_incl_scan<uint64_t>(x0), y1 = wave_incl_scan<uint64_t>(x1), y2 = wave_incl_scan<uint64_t>(x2);
    if (l < 16) {
      part[16 + l][0] = y0 - x0;  // exclusive wave bases
      part[16 + l][1] = y1 - x1;
      part[16 + l][2] = y2 - x2;
    }
  }
  __syncthreads();
  i0 += part[16 + w][0];
  i1 += part[16 + w][1];
  i2 += part[16 + w][2];
  uint64_t e0 = i0 - s0, e1 = i1 - s1, e2 = i2 - s2;
  for (uint64_t i = lo; i < hi; ++i) {
    a.tile_pre[3 * i] = e0;
    a.tile_pre[3 * i + 1] = e1;
    a.tile_pre[3 * i + 2] = e2;
    e0 += a.tile_sum[3 * i];
    e1 += a.tile_sum[3 * i + 1];
    e2 += a.tile_sum[3 * i + 2];
  }
  if (t == 1023) {
    const uint64_t N = i0, K = i1, V = i2;
    if (a.blk_ent) a.blk_ent[a.nblk] = N;
    a.stats[0] = N;
    a.stats[1] = K;
    a.stats[2] = V;
    uint32_t err = 0;
    if (K > 0xFFFFFFFFull || V > 0xFFFFFFFFull) err |= LSMBLK_ERR_OVERFLOW;
    if (N > a.entry_cap || K > a.key_cap || V > a.val_cap) err |= LSMBLK_ERR_CAPACITY;
    if (N <= a.entry_cap) {
      a.key_off[N] = uint32_t(K);
      a.val_off[N] = uint32_t(V);
    }
    if (err) atomicOr(reinterpret_cast<unsigned long long*>(a.stats + 3), (unsigned long long)err);
  }
}

// ================================================================ encode: plan
// The greedy block walk of SsTableBuilder (table/builder.rs:48-65 over BlockBuilder::add,
// block/builder.rs:54-73), plan_walk_kernel: one walker wave per segment walks the blocks over
// an LDS ring of per-entry (rec = klen + vlen, alcp = LCP with the predecessor key, bit 31 set
// when the pair is out of order) that a helper wave of the same workgroup computes just ahead of
// it.  For non-decreasing keys LCP(first key, key_e) = min of alcp over (first, e], so each block
// boundary is a min-scan, a sum-scan and a ballot over 64 candidate entries; a block holding an
// out-of-order pair compares with its first key directly.  Segment totals by decoupled look-back,
// then the dense block tables.
struct PlanArgs {
  const uint8_t* keys;
  const uint32_t* key_off;
  const uint32_t* val_off;
  uint64_t n;
  const uint32_t* seg_start;
  uint32_t nseg;
  uint32_t block_size;
  uint32_t* sz;         // scratch, n+1: encoded size per (segment-local) block
  uint32_t* rec_first;  // scratch, n+1
  uint32_t* blk_first;  // dense, n+1
  uint64_t* blk_off;    // user, blk_cap
  uint64_t blk_cap, out_cap;
  uint64_t* stats;
  uint32_t* ticket;
  uint64_t* agg;
  uint64_t* inc;
  uint32_t tag;
  uint32_t poll;
  const uint64_t* dn;      // optional: n read from device memory (overrides n)
  const uint32_t* dnseg;   // optional: nseg read from device memory (overrides nseg)
  uint32_t span;           // segments cover [seg_start[0], seg_start[nseg]) of the stream, not all of it
  uint64_t* dbg;           // optional realtime trace per segment (LSMBLK_DEBUG_COUNTERS)
  uint32_t skip;           // ablation (timing only, emit not launched): 1 << 16 helpers skip the key
                           // loads and LCPs, 1 << 17 walkers skip the scans (one block per window)
  // per-segment slot output (LSMBLK_ENCODE_SEG_SLOTS; encode_fused_kernel has the layout): segment
  // g's blocks at seg_slot(g) on; seg_out[2 g] = that slot, [2 g + 1] = its bytes; blk_sz = the
  // blocks' sizes (a segment's last block does not end where the next one starts)
  uint64_t* seg_out;
  uint32_t* blk_sz;
  uint32_t pipe_helper;    // the helper's loads pipelined over chunks (plan_produce_pipe)
  uint32_t frame;          // LSMBLK_ENCODE_FRAMED: 4 bytes (the block's CRC) after every block, else 0
};

__device__ __forceinline__ PlanArgs resolve(const PlanArgs& a0) {
  PlanArgs a = a0;
  if (a.dn) a.n = uni64(*a.dn);
  if (a.dnseg) a.nseg = uni(*a.dnseg);
  return a;
}

// First byte of segment g's slot in the per-segment output (LSMBLK_ENCODE_SEG_SLOTS): the keys and
// values of the segments before it plus 18 bytes per entry, an upper bound of their encoded size
// (encode_fused_kernel).
// Callers pass validated entry indices b = seg_start[0] and s = seg_start[g] (b <= s <= n): the
// table's raw entries are never used as array indices here (a table like
// [0, 0xFFFFFFFF, n] made the walker of segment 1 read key_off[0xFFFFFFFF] after flagging it).
// Framed output (LSMBLK_ENCODE_FRAMED) adds 4 bytes per block, at most one block per entry: 22 per entry.
__device__ __forceinline__ uint64_t seg_slot(const uint32_t* key_off, const uint32_t* val_off, uint32_t b, uint32_t s,
                                             uint32_t frame = 0) {
  if (s <= b) return 0;
  return uint64_t(key_off[s] - key_off[b]) + uint64_t(val_off[s] - val_off[b]) + (18ull + frame) * (s - b);
}

constexpr uint32_t kAlcpUnsorted = 0x80000000u;
constexpr uint32_t kAlcpLcp = 0x7FFFFFFFu;

// Key bytes of the batch through one descriptor over the whole key arena.
struct PlanKeys {
  rsrc_t gk;       // whole key arena, base aligned down to 16
  uint32_t glead;  // keys pointer & 15
  __device__ __forceinline__ uint32_t dword(uint32_t pos) const {  // 4 bytes at arena pos
    const uint32_t x = glead + pos, al = x & ~3u;
    const uint32_t w0 = __builtin_amdgcn_raw_buffer_load_b32(gk, al, 0, 0);
    const uint32_t w1 = __builtin_amdgcn_raw_buffer_load_b32(gk, al + 4, 0, 0);
    return __builtin_amdgcn_alignbyte(w1, w0, x & 3);
  }
};

__device__ __forceinline__ PlanKeys plan_keys(const PlanArgs& a) {
  PlanKeys K;
  K.glead = uint32_t(reinterpret_cast<uintptr_t>(a.keys) & 15);
  K.gk = make_rsrc(a.keys - K.glead, K.glead + uni(a.key_off[a.n]));
  return K;
}

// LCP of keys (pp, pl) and (kp, kl); *w0 / *w1 = the dwords holding the first difference.
__device__ __forceinline__ uint32_t key_lcp(const PlanKeys& K, uint32_t pp, uint32_t pl, uint32_t kp, uint32_t kl,
                                            uint32_t& w0, uint32_t& w1) {
  const uint32_t m = pl < kl ? pl : kl;
  uint32_t lcp = m;
  w0 = w1 = 0;
  for (uint32_t d = 0; 4 * d < m; ++d) {
    const uint32_t x0 = K.dword(pp + 4 * d), x1 = K.dword(kp + 4 * d);
    if (x0 != x1) {
      const uint32_t z = 4 * d + (__builtin_ctz(x0 ^ x1) >> 3);
      if (z < m) {
        lcp = z;
        w0 = x0;
        w1 = x1;
      }
      break;
    }
  }
  return lcp;
}


constexpr uint32_t kWalkThreads = 512;  // 4 walker waves + their 4 helper (producer) waves
constexpr uint32_t kSpinMax = 1u << 24;  // LDS hand-off polls before a wave gives up (TIMEOUT)
constexpr uint32_t kProdBatch = 4;       // entries per helper lane with loads in flight together (2: 0.41 ms,
                                         // 8: 128 VGPRs and a spill, against 0.39)
constexpr uint32_t kRing = 1024;         // (rec, alcp) ring entries per walker (power of two, >= 2 chunks):
                                         // 32 KiB per workgroup, three per CU
constexpr uint32_t kChunk = 256;         // entries per producer hand-off (1024 / 512 / 256: 0.39 / 0.376 /
                                         // 0.371 ms)

// Helper wave of a walker: plan_adj's per-entry values for the walker's segment [s0, s1),
// written chunk by chunk into the walker's ring (slot (e - s0) % kRing), never to HBM.
// A chunk may overwrite the ring's older half once the walker's window has left it;
// prod[0] = entries produced (relative to s0), cons[0] = walker's window start (relative).
__device__ void plan_produce(const PlanArgs& a, const PlanKeys& K, uint32_t s0, uint32_t s1, uint32_t* CR,
                             uint32_t* CA, uint32_t* prod, const uint32_t* cons, uint32_t& err, uint64_t* tr) {
  const uint32_t l = lane_id();
  uint64_t waited = 0;
  if (tr && l == 0) tr[4] = __builtin_amdgcn_s_memrealtime();
  const uint32_t klim = K.glead + uni(a.key_off[a.n]);
  for (uint32_t c = s0; c < s1; c += kChunk) {
    const uint32_t cend = s1 - c < kChunk ? s1 : c + kChunk;
    if (c - s0 + kChunk > kRing) {  // ring space: the walker's window must have passed c + kChunk - kRing
      const uint32_t need = c - s0 + kChunk - kRing;
      uint32_t spins = 0;
      const uint64_t w0 = tr ? __builtin_amdgcn_s_memrealtime() : 0;
      while (__hip_atomic_load(cons, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < need) {
        if (++spins > kSpinMax) {
          err |= LSMBLK_ERR_TIMEOUT;
          return;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (tr) waited += __builtin_amdgcn_s_memrealtime() - w0;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
#pragma unroll 1
    for (uint32_t h = 0; h < kChunk / 64; h += kProdBatch) {  // kProdBatch entries per lane at a time
      uint32_t kp[kProdBatch], kn[kProdBatch], pp[kProdBatch], v0[kProdBatch], v1[kProdBatch];
#pragma unroll
      for (uint32_t i = 0; i < kProdBatch; ++i) {
        const uint32_t e = c + 64 * (h + i) + l;
        kp[i] = kn[i] = pp[i] = v0[i] = v1[i] = 0;
        if (e < cend) {
          kp[i] = a.key_off[e];
          kn[i] = a.key_off[e + 1];
          pp[i] = e > 0 ? a.key_off[e - 1] : 0u;
          v0[i] = a.val_off[e];
          v1[i] = a.val_off[e + 1];
        }
      }
      u32x4 xk[kProdBatch], xp[kProdBatch];
      const bool nokeys = diag_mask(a.skip) & (1u << 16);
#pragma unroll
      for (uint32_t i = 0; i < kProdBatch; ++i) {
        const uint32_t e = c + 64 * (h + i) + l;
        if (e < cend && e != s0 && !nokeys) {
          xk[i] = __builtin_amdgcn_raw_buffer_load_b128(K.gk, K.glead + kp[i], 0, 0);
          xp[i] = __builtin_amdgcn_raw_buffer_load_b128(K.gk, K.glead + pp[i], 0, 0);
        }
      }
#pragma unroll
      for (uint32_t i = 0; i < kProdBatch; ++i) {
        const uint32_t e = c + 64 * (h + i) + l;
        if (e >= cend) continue;
        // offsets that decrease (a corrupt stream) are refused, and the entry is walked as a
        // 1-byte key and an empty value so that no loop below runs over a wrapped length
        const bool inv = kn[i] < kp[i] || v1[i] < v0[i];
        if (inv) err |= LSMBLK_ERR_MALFORMED;
        const uint32_t kl = inv ? 1u : kn[i] - kp[i], x = (e - s0) & (kRing - 1);
        if (kl == 0) err |= LSMBLK_ERR_EMPTY_KEY;
        uint32_t al = 0;
        if (e != s0 && !nokeys) {  // as plan_adj_kernel: LCP with the predecessor, bit 31 = out of order
          const uint32_t pl = kp[i] - pp[i], m = pl < kl ? pl : kl;
          uint32_t lcp = m, w0 = 0, w1 = 0;
          bool done = false;
          if (K.glead + kp[i] + 16 <= klim && K.glead + pp[i] + 16 <= klim) {
            // first differing byte z of the 16 loaded (16: none), by selects instead of a branch per
            // dword (the helper shares its SIMD with the walker: its instructions are the walk's time)
            const uint32_t P[4] = {xp[i].x, xp[i].y, xp[i].z, xp[i].w}, Q[4] = {xk[i].x, xk[i].y, xk[i].z, xk[i].w};
            uint32_t t[4];
#pragma unroll
            for (uint32_t d = 0; d < 4; ++d) t[d] = uint32_t(__builtin_ctzg(P[d] ^ Q[d], 32)) >> 3;  // 4: equal
            const uint32_t z16 = t[0] < 4 ? t[0] : t[1] < 4 ? 4 + t[1] : t[2] < 4 ? 8 + t[2] : 12 + t[3];
            const uint32_t zd = z16 >> 2;  // (z16 < 16 only)
            if (z16 < m) {
              lcp = z16;
              w0 = zd == 0 ? P[0] : zd == 1 ? P[1] : zd == 2 ? P[2] : P[3];
              w1 = zd == 0 ? Q[0] : zd == 1 ? Q[1] : zd == 2 ? Q[2] : Q[3];
            }
            done = z16 < m || m <= 16;
            if (!done) {  // equal first 16 bytes: the rest by dwords
              for (uint32_t d = 4; 4 * d < m; ++d) {
                const uint32_t y0 = K.dword(pp[i] + 4 * d), y1 = K.dword(kp[i] + 4 * d);
                if (y0 != y1) {
                  const uint32_t z = 4 * d + (__builtin_ctz(y0 ^ y1) >> 3);
                  if (z < m) {
                    lcp = z;
                    w0 = y0;
                    w1 = y1;
                  }
                  break;
                }
              }
            }
          } else {
            lcp = key_lcp(K, pp[i], pl, kp[i], kl, w0, w1);
          }
          const uint32_t sh = 8 * (lcp & 3);
          const bool sorted = lcp == m ? pl <= kl : ((w0 >> sh) & 0xFF) < ((w1 >> sh) & 0xFF);
          al = (lcp < kAlcpLcp ? lcp : kAlcpLcp) | (sorted ? 0u : kAlcpUnsorted);
        }
        CR[x] = inv ? kl : kl + (v1[i] - v0[i]);
        CA[x] = al;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (l == 0) __hip_atomic_store(prod, cend - s0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  if (tr && l == 0) {
    tr[5] = __builtin_amdgcn_s_memrealtime();
    tr[6] = waited;
  }
}

// The walker's side of the ring hand-off: its window start, and the producer's count.
struct WalkRing {
  const uint32_t* CR;   // rec per entry, slot (e - S0) % kRing
  const uint32_t* CA;   // alcp per entry
  uint32_t* cons;       // walker's window start (relative to S0)
  const uint32_t* prod; // entries produced (relative to S0)
  uint32_t S0;          // the ring's base entry (the first entry of the walker's first segment)
  uint32_t known = 0;   // entries the producer has finished (relative to S0)
  bool stalled = false; // a poll gave up: the walk goes on over stale data, the call reports TIMEOUT
};

// The greedy block walk of one segment [s0, s1) over the helper's ring (SsTableBuilder::add over
// BlockBuilder::add: src/table/builder.rs:48-65, src/block/builder.rs:54-73).  Every block, in
// order, goes to sink(first entry, end entry, encoded size, blocks before it in the segment,
// bytes before it in the segment) (wave-uniform arguments); returns (blocks, bytes).
template <class Sink>
__device__ __forceinline__ void walk_segment(const PlanArgs& a, const PlanKeys& K, WalkRing& R, uint32_t s0, uint32_t s1,
                                             uint32_t& err, uint32_t& nb, uint64_t& bytes, Sink&& sink, uint64_t* tr,
                                             uint64_t& waited, uint64_t& windows) {
  const uint32_t l = lane_id();
  // (rec, alcp) of entry e at LDS slot (e - S0) % kRing, written by the helper wave; `need` waits
  // until the window's entries are in and tells the helper where the window starts.
  auto need = [&](uint32_t j0, uint32_t wend) {
    __hip_atomic_store(R.cons, j0 - R.S0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (tr) ++windows;
    if (wend - R.S0 > R.known && !R.stalled) {
      const uint64_t w0 = tr ? __builtin_amdgcn_s_memrealtime() : 0;
      uint32_t spins = 0;
      while ((R.known = __hip_atomic_load(R.prod, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < wend - R.S0) {
        if (++spins > kSpinMax) {
          err |= LSMBLK_ERR_TIMEOUT;
          R.stalled = true;  // walk on over stale ring data: the call fails with TIMEOUT
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (tr) waited += __builtin_amdgcn_s_memrealtime() - w0;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
  };
  const uint32_t* const CR = R.CR;
  const uint32_t* const CA = R.CA;
  const uint32_t S0 = R.S0;
  nb = 0;
  bytes = 0;
  const uint64_t bs = a.block_size;
  const bool narrow = bs < (1ull << 30);
  for (uint32_t s = s0; s < s1;) {
    uint64_t carry = 2;           // estimated_size() of an empty builder
    uint32_t pmin = kAlcpLcp;     // running min of alcp over (s, window start)
    bool direct = false;
    uint32_t sp = 0, sl = 0;      // key_s (direct compares only)
    for (uint32_t j0 = s;; j0 += 64) {
      const uint32_t wend = s1 - j0 < 64 ? s1 : j0 + 64;
      need(j0, wend);
      if (diag_mask(a.skip) & (1u << 17)) {  // ablation: consume the window as one block, no scans
        const uint32_t x = (j0 + l - S0) & (kRing - 1);
        const uint32_t rr = j0 + l < s1 ? CR[x] + CA[x] : 0u;
        sink(s, wend, uint32_t(__builtin_amdgcn_readfirstlane(rr)), nb, bytes);
        ++nb;
        s = wend;
        break;
      }
      const uint32_t e = j0 + l;
      const bool valid = e < s1;
      uint32_t r = 0, al = kAlcpLcp;
      if (valid) {
        const uint32_t x = (e - S0) & (kRing - 1);
        r = CR[x];
        if (e != s) al = CA[x];
      }
      if (!direct && __ballot(al & kAlcpUnsorted)) {  // an out-of-order pair inside this block
        direct = true;
        sp = a.key_off[s];
        sl = a.key_off[s + 1] >= sp ? a.key_off[s + 1] - sp : 0u;  // (decreasing offsets: refused by the helper)
      }
      uint32_t p = 0;
      if (!direct) {
        p = min(pmin, wave_incl_min31(al & kAlcpLcp));
        pmin = __builtin_amdgcn_readlane(p, 63);
      } else if (valid && e != s) {
        const uint32_t kp = a.key_off[e], kl = a.key_off[e + 1] >= kp ? a.key_off[e + 1] - kp : 0u;
        uint32_t w0, w1;
        p = key_lcp(K, sp, sl, kp, kl, w0, w1);
      }
      if (e == s) p = 0;
      // data growth + offset slot, its inclusive scan and estimated_size() before adding e.  u32
      // throughout when the block size is < 2^30 and every lane's growth < 2^25 (then carry <= bs +
      // 2, the scan < 2^31 and before + r + 14 < 2^32: exact), else 64-bit.
      uint64_t before, incl_all;
      bool stop;
      if (narrow && __ballot(valid && r >= (1u << 25) - 16) == 0) {
        const uint32_t g32 = valid ? r + 16 - p : 0u;
        const uint32_t i32 = wave_incl_scan32(g32);
        const uint32_t b32 = uint32_t(carry) + i32 - g32;
        // builder.rs:56-60: reject when est + raw_len + vlen + 6 > block_size (not first entry)
        stop = !valid || (e != s && b32 + r + 14 > uint32_t(bs));
        before = b32;
        incl_all = uint32_t(__builtin_amdgcn_readlane(i32, 63));
      } else {
        const uint64_t gr = valid ? uint64_t(r) + 16 - p : 0;
        const uint64_t incl = __ballot(gr >= (1u << 25)) == 0 ? uint64_t(wave_incl_scan32(uint32_t(gr)))
                                                               : wave_incl_scan<uint64_t>(gr);
        before = carry + incl - gr;
        stop = !valid || (e != s && before + r + 14 > bs);
        incl_all = lane64(incl, 63);
      }
      const uint64_t m = __ballot(stop);
      if (m) {
        uint32_t f = uint32_t(__builtin_ctzll(m));
        const uint64_t size = lane64(before, f);
        sink(s, j0 + f, uint32_t(size), nb, bytes);
        ++nb;
        bytes += size;
        s = j0 + f;
        // Further blocks from entry s on the same window's lanes f..63 (the window held no
        // out-of-order pair, or direct would be set): LCP with entry s = min of alcp over
        // (f, e] (lanes <= f read the min identity); growth and estimated_size restart at s.
        // Every block ending in the window is found here; a block still open at the window's
        // end carries (estimated_size, running LCP) into the next window instead of restarting
        // the walk at its first entry.
        bool open = false;
        while (!direct && s < s1) {
          const uint32_t mn = wave_incl_min31(l <= f ? kAlcpLcp : (al & kAlcpLcp));  // all lanes (DPP)
          const uint32_t p2 = l <= f ? 0u : mn;
          const uint32_t g2 = (valid && l >= f) ? r + 16 - p2 : 0u;
          if (__ballot(g2 >= (1u << 25)) != 0) break;  // huge entries: restart at s (64-bit path)
          const uint32_t incl2 = wave_incl_scan32(g2);
          const uint32_t before2 = 2 + incl2 - g2;
          const uint64_t m2 = __ballot(l > f && (!valid || uint64_t(before2) + r + 14 > bs));
          if (!m2) {  // block s runs past this window
            carry = 2 + uint64_t(uint32_t(__builtin_amdgcn_readlane(incl2, 63)));
            pmin = uint32_t(__builtin_amdgcn_readlane(mn, 63));
            open = true;
            break;
          }
          const uint32_t f2 = uint32_t(__builtin_ctzll(m2));
          const uint32_t size2 = uint32_t(__builtin_amdgcn_readlane(before2, f2));
          sink(s, j0 + f2, size2, nb, bytes);
          ++nb;
          bytes += size2;
          s = j0 + f2;
          f = f2;
        }
        if (open) continue;  // next window, same block
        break;
      }
      carry += incl_all;
    }
  }
}

// plan_produce, software-pipelined over batches of kPipeB entries per lane (64 kPipeB entries): a
// batch's key loads go out, then the next batch's entry-offset loads (5 per entry), and only then
// does the batch wait for its keys (vmcnt(5 kPipeB)) -- one memory round trip per batch instead of
// two.  Both sets are issued by inline asm so that the compiler neither sinks the key loads into
// the per-entry branch (it did) nor waits for the offsets there; registers loaded by asm are
// landed by explicit waits and then redefined for the compiler.  (The fused walk + emit launch's
// helper: beside emit's stream the round trips are long, and the unpipelined helper held its
// walker to ~2.5 us per window.  The standalone walk: M's short segments wait on its round trips.)
// Two entries per lane per batch keep the plan walk at 3 workgroups (24 waves) per CU.
constexpr uint32_t kPipeB = 2;
constexpr uint32_t kPipeE = 64 * kPipeB;  // entries per batch
static_assert(kRing % kPipeE == 0 && kRing >= 2 * kPipeE, "ring holds whole batches");
struct ProdOffs {
  uint32_t kp[kPipeB], kn[kPipeB], pp[kPipeB], v0[kPipeB], v1[kPipeB];
};
// the 5 offset loads of entry lane l's i-th entry of batch [c, cend) (indices clamped: always issued)
__device__ __forceinline__ void prod_offs_issue(const rsrc_t& RKO, const rsrc_t& RVO, uint32_t c, uint32_t cend,
                                                ProdOffs& P) {
  const uint32_t l = lane_id();
#pragma unroll
  for (uint32_t i = 0; i < kPipeB; ++i) {
    uint32_t e = c + 64 * i + l;
    e = e < cend ? e : cend - 1;
    const uint32_t oe = 4 * e, op = 4 * (e > 0 ? e - 1 : 0u);
    asm volatile(
        "buffer_load_dword %0, %5, %7, 0 offen\n\t"
        "buffer_load_dword %1, %5, %7, 0 offen offset:4\n\t"
        "buffer_load_dword %2, %6, %7, 0 offen\n\t"
        "buffer_load_dword %3, %5, %8, 0 offen\n\t"
        "buffer_load_dword %4, %5, %8, 0 offen offset:4"
        : "=&v"(P.kp[i]), "=&v"(P.kn[i]), "=&v"(P.pp[i]), "=&v"(P.v0[i]), "=&v"(P.v1[i])
        : "v"(oe), "v"(op), "s"(RKO), "s"(RVO));
  }
}
__device__ __forceinline__ void prod_offs_land(ProdOffs& P) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (uint32_t i = 0; i < kPipeB; ++i)
    asm volatile("" : "+v"(P.kp[i]), "+v"(P.kn[i]), "+v"(P.pp[i]), "+v"(P.v0[i]), "+v"(P.v1[i]));
}
__device__ void plan_produce_pipe(const PlanArgs& a, const PlanKeys& K, uint32_t s0, uint32_t s1, uint32_t* CR,
                                  uint32_t* CA, uint32_t* prod, const uint32_t* cons, uint32_t& err,
                                  uint64_t* tr = nullptr) {
  static_assert(kPipeB == 2, "the vmcnt below counts 5 kPipeB offset loads");
  const uint32_t l = lane_id();
  const uint32_t klim = K.glead + uni(a.key_off[a.n]);
  uint64_t waited = 0;
  if (tr && l == 0) tr[4] = __builtin_amdgcn_s_memrealtime();
  if (s0 >= s1) return;
  const uint32_t nb4 = uint32_t(min(uint64_t(a.n + 1) * 4, uint64_t(0xFFFFFFF0u)));
  const rsrc_t RKO = make_rsrc(a.key_off, nb4), RVO = make_rsrc(a.val_off, nb4);
  ProdOffs P;
  asm volatile("s_nop 4" ::: "memory");  // (VALU-written descriptor SGPRs before a VMEM read of them, inside asm)
  prod_offs_issue(RKO, RVO, s0, s1 - s0 < kPipeE ? s1 : s0 + kPipeE, P);
  prod_offs_land(P);
  for (uint32_t c = s0; c < s1; c += kPipeE) {
    const uint32_t cend = s1 - c < kPipeE ? s1 : c + kPipeE;
    if (c - s0 + kPipeE > kRing) {  // ring space: the walker's window must have passed c + kPipeE - kRing
      const uint32_t need = c - s0 + kPipeE - kRing;
      uint32_t spins = 0;
      const uint64_t w0 = tr ? __builtin_amdgcn_s_memrealtime() : 0;
      while (__hip_atomic_load(cons, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < need) {
        if (++spins > kSpinMax) {
          err |= LSMBLK_ERR_TIMEOUT;
          return;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (tr) waited += __builtin_amdgcn_s_memrealtime() - w0;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
    u32x4 xk[kPipeB], xp[kPipeB];
#pragma unroll
    for (uint32_t i = 0; i < kPipeB; ++i) {
      const uint32_t ok = K.glead + P.kp[i], op = K.glead + P.pp[i];
      asm volatile(
          "buffer_load_dwordx4 %0, %2, %4, 0 offen\n\t"
          "buffer_load_dwordx4 %1, %3, %4, 0 offen"
          : "=&v"(xk[i]), "=&v"(xp[i])
          : "v"(ok), "v"(op), "s"(K.gk));
    }
    // the next batch's offsets (after the last batch: its own again -- always 5 kPipeB loads)
    const uint32_t cn = c + kPipeE < s1 ? c + kPipeE : c;
    ProdOffs Pn;
    prod_offs_issue(RKO, RVO, cn, s1 - cn < kPipeE ? s1 : cn + kPipeE, Pn);
    asm volatile("s_waitcnt vmcnt(10)" ::: "memory");  // this batch's keys (issued before the 10)
#pragma unroll
    for (uint32_t i = 0; i < kPipeB; ++i) asm volatile("" : "+v"(xk[i]), "+v"(xp[i]));
#pragma unroll
    for (uint32_t i = 0; i < kPipeB; ++i) {
      const uint32_t e = c + 64 * i + l;
      if (e >= cend) continue;
      const bool inv = P.kn[i] < P.kp[i] || P.v1[i] < P.v0[i];  // (refused, as plan_produce)
      if (inv) err |= LSMBLK_ERR_MALFORMED;
      const uint32_t kp = P.kp[i], pp = P.pp[i], kl = inv ? 1u : P.kn[i] - kp, x = (e - s0) & (kRing - 1);
      if (kl == 0) err |= LSMBLK_ERR_EMPTY_KEY;
      uint32_t al = 0;
      if (e != s0) {  // LCP with the predecessor, bit 31 = out of order (as plan_produce)
        const uint32_t pl = kp - pp, m = pl < kl ? pl : kl;
        uint32_t lcp = m, w0 = 0, w1 = 0;
        if (K.glead + kp + 16 <= klim && K.glead + pp + 16 <= klim) {
          const uint32_t Pw[4] = {xp[i].x, xp[i].y, xp[i].z, xp[i].w}, Qw[4] = {xk[i].x, xk[i].y, xk[i].z, xk[i].w};
          uint32_t t[4];
#pragma unroll
          for (uint32_t d = 0; d < 4; ++d) t[d] = uint32_t(__builtin_ctzg(Pw[d] ^ Qw[d], 32)) >> 3;  // 4: equal
          const uint32_t z16 = t[0] < 4 ? t[0] : t[1] < 4 ? 4 + t[1] : t[2] < 4 ? 8 + t[2] : 12 + t[3];
          const uint32_t zd = z16 >> 2;
          if (z16 < m) {
            lcp = z16;
            w0 = zd == 0 ? Pw[0] : zd == 1 ? Pw[1] : zd == 2 ? Pw[2] : Pw[3];
            w1 = zd == 0 ? Qw[0] : zd == 1 ? Qw[1] : zd == 2 ? Qw[2] : Qw[3];
          }
          if (!(z16 < m || m <= 16)) {  // equal first 16 bytes: the rest by dwords
            for (uint32_t d = 4; 4 * d < m; ++d) {
              const uint32_t y0 = K.dword(pp + 4 * d), y1 = K.dword(kp + 4 * d);
              if (y0 != y1) {
                const uint32_t z = 4 * d + (__builtin_ctz(y0 ^ y1) >> 3);
                if (z < m) {
                  lcp = z;
                  w0 = y0;
                  w1 = y1;
                }
                break;
              }
            }
          }
        } else {
          lcp = key_lcp(K, pp, pl, kp, kl, w0, w1);
        }
        const uint32_t sh = 8 * (lcp & 3);
        const bool sorted = lcp == m ? pl <= kl : ((w0 >> sh) & 0xFF) < ((w1 >> sh) & 0xFF);
        al = (lcp < kAlcpLcp ? lcp : kAlcpLcp) | (sorted ? 0u : kAlcpUnsorted);
      }
      CR[x] = inv ? kl : kl + (P.v1[i] - P.v0[i]);
      CA[x] = al;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (l == 0) __hip_atomic_store(prod, cend - s0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    prod_offs_land(Pn);
    P = Pn;
  }
  if (tr && l == 0) {
    tr[5] = __builtin_amdgcn_s_memrealtime();
    tr[6] = waited;
  }
}

// (fused: three workgroups of 8 waves per CU, so that up to 3 K segments walk at once)
__global__ __launch_bounds__(kWalkThreads) __attribute__((amdgpu_waves_per_eu(4))) void plan_walk_kernel(PlanArgs a0) {
  const PlanArgs a = resolve(a0);
  static_assert(kRing >= 2 * kChunk && (kRing & (kRing - 1)) == 0, "plan ring size");
  __shared__ uint32_t crec[4][kRing], calcp[4][kRing];
  const uint32_t l = lane_id();
  // waves 0-3 walk segments, wave 4 + w produces (rec, alcp) into walker w's ring
  __shared__ uint32_t hand_g[4], hand_prod[4], hand_cons[4];
  const uint32_t wv = wave_id(), ww = wv & 3;
  if (wv < 4) {
    const uint32_t t = take_ticket(a.ticket);
    if (l == 0) {
      hand_g[wv] = t;
      hand_prod[wv] = 0;
      hand_cons[wv] = 0;
    }
  }
  __syncthreads();
  const uint32_t g = uni(hand_g[ww]);
  uint32_t* CR = crec[ww];
  uint32_t* CA = calcp[ww];
  if (g >= a.nseg) return;
  uint32_t err = 0;
  uint32_t s0 = uni(a.seg_start[g]), s1 = uni(a.seg_start[g + 1]);
  if ((!a.span && g == 0 && s0 != 0) || (!a.span && g == a.nseg - 1 && uint64_t(s1) != a.n) || s0 > s1 ||
      uint64_t(s1) > a.n) {
    err |= LSMBLK_ERR_SEGMENTS;
    s1 = s0 = (s0 > a.n ? uint32_t(a.n) : s0);
    if (s1 < s0) s1 = s0;
  }
  const PlanKeys K = plan_keys(a);
  uint64_t* const tr = kDiag && a.dbg && g < kDbgTiles ? a.dbg + 16 + 8 * uint64_t(g) : nullptr;  // (diagnostics)
  if (wv >= 4) {
    if (a.pipe_helper) plan_produce_pipe(a, K, s0, s1, CR, CA, &hand_prod[ww], &hand_cons[ww], err, tr);
    else plan_produce(a, K, s0, s1, CR, CA, &hand_prod[ww], &hand_cons[ww], err, tr);
    const uint32_t werr = (__ballot(err & LSMBLK_ERR_EMPTY_KEY) ? LSMBLK_ERR_EMPTY_KEY : 0u) |
                          (__ballot(err & LSMBLK_ERR_MALFORMED) ? LSMBLK_ERR_MALFORMED : 0u) |
                          (__ballot(err & LSMBLK_ERR_TIMEOUT) ? LSMBLK_ERR_TIMEOUT : 0u);
    raise_err(a.stats, werr);
    return;
  }
  uint64_t waited = 0, windows = 0;
  if (tr && l == 0) tr[0] = __builtin_amdgcn_s_memrealtime();
  WalkRing R{CR, CA, &hand_cons[ww], &hand_prod[ww], s0};
  uint32_t nb = 0;
  uint64_t bytes = 0;
  walk_segment(a, K, R, s0, s1, err, nb, bytes,
               [&](uint32_t first, uint32_t, uint32_t size, uint32_t i, uint64_t) {
                 if (l == 0) {
                   a.rec_first[s0 + i] = first;
                   a.sz[s0 + i] = size;
                 }
               },
               tr, waited, windows);
  if (tr && l == 0) {
    tr[1] = __builtin_amdgcn_s_memrealtime();
    tr[2] = waited;
    tr[3] = windows;
    // blocks | HW_ID (wave, SIMD, CU, SE) << 32 | XCC_ID << 56: where the walker ran
    tr[7] = nb | (uint64_t(__builtin_amdgcn_s_getreg(0xF804)) << 32) | (uint64_t(__builtin_amdgcn_s_getreg(0x1814) & 0xF) << 56);
  }
  bytes += uint64_t(a.frame) * nb;  // (framed: every block's CRC after it, written by the CRC pass)
  // make this wave's record stores visible to its own later loads
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  // segment totals -> dense block numbering and output offsets
  uint64_t agg[2] = {nb, bytes};
  uint64_t excl[2] = {0, 0};
  if (g == 0) {
    publish<2>(a.inc, g, agg, a.tag, 2, a.poll);
  } else {
    publish<2>(a.agg, g, agg, a.tag, 1, a.poll);
    if (!lookback<2>(a.agg, a.inc, g, a.tag, a.poll, excl)) err |= LSMBLK_ERR_TIMEOUT;
    const uint64_t inc[2] = {excl[0] + agg[0], excl[1] + agg[1]};
    publish<2>(a.inc, g, inc, a.tag, 2, a.poll);
  }
  // slot mode: segment 0 starts at 0 (checked by its own walker, err SEGMENTS otherwise); a
  // segment whose own bounds were refused gets slot 0 and writes nothing (emit: kPlanFatal)
  uint64_t O0 = excl[1];
  if (a.seg_out) O0 = (err & LSMBLK_ERR_SEGMENTS) ? 0ull : seg_slot(a.key_off, a.val_off, 0u, s0, a.frame);
  const uint64_t B0 = excl[0];
  if (a.seg_out && l == 0) {
    a.seg_out[2ull * g] = O0;
    a.seg_out[2ull * g + 1] = bytes;
  }
  uint64_t oc = O0;
  for (uint32_t c = 0; c < nb; c += 64) {
    const uint32_t i = c + l;
    uint32_t sz = 0, first = 0;
    if (i < nb) {
      first = a.rec_first[s0 + i];
      sz = a.sz[s0 + i];
    }
    const uint64_t ext = i < nb ? uint64_t(sz) + a.frame : 0ull;  // the block and its frame
    const uint64_t incl = wave_incl_scan<uint64_t>(ext);
    if (i < nb) {
      const uint64_t bi = B0 + i;
      a.blk_first[bi] = first;
      if (a.blk_sz) a.blk_sz[bi] = sz;
      if (bi < a.blk_cap) a.blk_off[bi] = oc + incl - ext;
    }
    oc += __shfl(incl, 63, 64);
  }
  if (g == a.nseg - 1 && l == 0) {
    const uint64_t Bt = B0 + nb, Ot = O0 + bytes;
    a.blk_first[Bt] = a.span ? s1 : uint32_t(a.n);
    if (Bt < a.blk_cap) a.blk_off[Bt] = Ot;
    a.stats[0] = Bt;
    a.stats[1] = excl[1] + bytes;  // (the encoded bytes; in slot mode Ot is where they end)
    if (Bt + 1 > a.blk_cap || Ot > a.out_cap) err |= LSMBLK_ERR_CAPACITY;
  }
  raise_err(a.stats, err);
}

// ================================================================ encode: emit
struct EmitArgs {
  const uint8_t* keys;
  const uint32_t* key_off;
  const uint8_t* vals;
  const uint32_t* val_off;
  const uint64_t* ts;
  const uint32_t* blk_first;
  const uint64_t* blk_off;
  uint8_t* out;
  uint64_t out_cap, blk_cap;
  uint64_t n;  // entries; arena sizes are key_off[n], val_off[n]
  uint64_t* stats;
  // per block: 1 = beyond the LDS image, left by emit_kernel for emit_big_kernel (a flag per
  // block, not a list: appending through one shared counter cost 0.6 ms on 64 Ki big blocks)
  uint8_t* big_flag;
  // optional: every block's encoded size (per-segment slot output, LSMBLK_ENCODE_SEG_SLOTS: a
  // segment's last block does not end where the next block starts); else blk_off[bi + 1] - blk_off[bi]
  const uint32_t* blk_sz;
  uint32_t skip;  // ablation mask (timing experiments only): 16 entry-lane byte writes,
                  // 32 bulk value copy, 64 flush, 128 LCP
  const uint64_t* dn;  // optional: n read from device memory (overrides n)
};

__device__ __forceinline__ EmitArgs resolve(const EmitArgs& a0) {
  EmitArgs a = a0;
  if (a.dn) a.n = uni64(*a.dn);
  return a;
}

constexpr uint32_t kEmitWaves = 4;
constexpr uint32_t kEmitKCap = 1088;
constexpr uint32_t kEmitICap = 4224;  // block image: staged values, then the encoded block (33 swizzle rows)
constexpr uint32_t kEmitMaxE = 128;

struct alignas(16) EmitLds {
  uint8_t kimg[kEmitKCap];
  uint8_t img[kEmitICap];
  alignas(16) uint32_t cent[kEmitICap / 16 + 4];  // chunk -> its source byte in the staged values, ~0 if not wholly inside one value
  alignas(16) uint32_t erec[4 * kEmitMaxE];  // per entry: record start | prefix << 16, suffix in kimg | value length << 16, suffix length
  uint64_t ts[kEmitMaxE];
};

// bytes [0, len) (len < 16) of v at an unaligned LDS address: overlapping stores of the widest
// size that fits (8 + 8, 4 + 4, or single bytes)
__device__ __forceinline__ void lds_st_short(uint8_t* p, uint32_t len, const uint32_t (&v)[4]) {
  if (len >= 8) {
    const uint32_t x = len - 8, sh = x & 3;
    const uint32_t w0 = x < 4 ? v[0] : v[1], w1 = x < 4 ? v[1] : v[2], w2 = x < 4 ? v[2] : v[3];
    *reinterpret_cast<u32x2*>(p) = u32x2{v[0], v[1]};
    *reinterpret_cast<u32x2*>(p + x) = u32x2{__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh)};
  } else if (len >= 4) {
    *reinterpret_cast<uint32_t*>(p) = v[0];
    *reinterpret_cast<uint32_t*>(p + len - 4) = __builtin_amdgcn_alignbyte(v[1], v[0], len - 4);
  } else {
    for (uint32_t i = 0; i < len; ++i) p[i] = uint8_t(v[0] >> (8 * i));
  }
}

#ifndef LSMBLK_XEBB
#define LSMBLK_XEBB 4
#endif
constexpr uint32_t kEmitBigB = LSMBLK_XEBB;  // (experiment) pieces per lane per copy round in emit_big

// Blocks beyond the LDS image (config M's 64 KiB blocks, oversize entries, > kEmitMaxE
// entries), one wave per block, 64 entries (a chunk) at a time: entry lanes write their records
// straight to HBM.  LCP against the first key in 16-B compares; suffix and value as 16-B
// unaligned buffer loads/stores (long values by the wave's packed copy); header, ts and
// value_len as single unaligned stores; the offset slot at data_len + 2k, data_len = size - 2n - 2
// known from the plan (checked at the end).
//
// The chunks of a wave's blocks are software-pipelined (emit_big_kernel): a chunk's entry offsets
// (level 1) are loaded while the chunk before it is processed, and its first 16 key bytes and the
// block's first key (level 2, the LCP's operands) right after that chunk's first copy round --
// without it each chunk waited two round trips before its copies (M: 0.40 of 1.93 ms with the
// copies ablated, none of it overlapped).
struct BigBlk {
  uint64_t bi, O, size;
  uint32_t s, n;
};
struct BigL1 {  // lane k: key_off[s + k], key_off[s + k + 1], val_off[s + k], val_off[s + k + 1]
  uint32_t ko0, ko1, vo0, vo1;
};
struct BigL2 {  // lane k: its key's first 16 bytes; the block's first key's first 16 bytes
  u32x4 own, first;
};

// Block metadata of one emit unit: two levels of dependent loads (block tables, then the
// entry offsets of its first/last entry).
struct EmitMeta {
  uint64_t bi;
  uint32_t s, e, n;
  uint64_t O, size;
  uint32_t kb0, kb1, vb0, vb1;
  bool bad;  // the block table entry is not s <= e <= n: refused (LSMBLK_ERR_INTERNAL), never read
};

// The plan's error flags that leave its block tables unusable: emit then writes nothing (a
// refused segment table gave blocks whose end entry precedes their start, which emit_big walked
// as ~2^32 entries).  CAPACITY is not one: every block that fits is still written.
constexpr uint64_t kPlanFatal =
    LSMBLK_ERR_SEGMENTS | LSMBLK_ERR_TIMEOUT | LSMBLK_ERR_INTERNAL | LSMBLK_ERR_EMPTY_KEY | LSMBLK_ERR_MALFORMED;

// One fast-path block of emit (wave-uniform): entries [s, s + n), output [O, O + size), its keys
// staged at kimg[klead], its values at img[vlead], fl = its first key's length.
struct EmitBlk {
  uint32_t s, n;
  uint64_t O, size;
  uint32_t kb0, vb0, klead, vlead, olead, fl, kb1, vb1;
};
// The first 64 entries' offsets and ts of a block, loaded by entry lane k one block ahead.
struct EmitPf {
  uint32_t ko0 = 0, ko1 = 0, vo0 = 0, vo1 = 0;
  uint64_t ts = 0;
};

// (diagnostics builds, ablation mask 1: emit's misaligned LDS accesses moved to aligned addresses --
// a timing probe of their cost, the bytes are wrong)
#define EAL(x, m) ((diag_mask(a.skip) & 1u) ? ((x) & ~uint32_t(m)) : (x))
// Phase 1 of emit_kernel for block B (staged and landed): returns the block's data length, ncs =
// its image chunks; eh / et = the first / last 16 bytes of the value of entries l, l + 64.
// kChk: check every entry against its block's byte ranges (the fused launch, which emits while the
// plan's helper may still be finding a corrupt stream; emit_kernel runs only after a plan without
// fatal flags, whose helper has checked every entry's offsets).
template <bool kChk>
__device__ __forceinline__ uint32_t emit_phase1(const EmitArgs& a, EmitLds& L, const EmitBlk& B, const EmitPf& pf,
                                                uint32_t (&eh)[2][4], uint32_t (&et)[2][4], uint32_t& ncs, uint32_t& err) {
  const uint32_t l = lane_id();
  const uint32_t s = B.s, n = B.n, kb0 = B.kb0, vb0 = B.vb0, klead = B.klead, vlead = B.vlead, olead = B.olead, fl = B.fl;
  const uint64_t size = B.size;
  // Phase 1, entry lanes: LCP against the first key, record positions (wave scan), tables,
  // and the value bytes of each value's two partial edge chunks (captured in registers: the
  // in-place move below overwrites the staged values).
  ncs = (olead + uint32_t(size) + 15) >> 4;  // image chunks of the encoded block
  for (uint32_t j = 4 * l; j < ncs; j += 256) *reinterpret_cast<u32x4*>(L.cent + j) = u32x4{~0u, ~0u, ~0u, ~0u};
  uint32_t fkw[4];  // first 16 bytes of the first key (LDS broadcast reads)
#pragma unroll
  for (int i = 0; i < 4; ++i) fkw[i] = lds_dword_at(L.kimg, klead + 4 * i);
  uint32_t dc = 0;
#pragma unroll
  for (uint32_t it = 0; it < 2; ++it) {
    const uint32_t c = 64 * it;
    if (c >= n) break;
    const uint32_t k = c + l;
    uint32_t kp = 0, kl = 0, vp = 0, vl = 0, p = 0;
    if (k < n) {
      uint32_t ko0, ko1, vo0, vo1;
      if (it == 0) {  // prefetched one block ahead
        ko0 = pf.ko0; ko1 = pf.ko1; vo0 = pf.vo0; vo1 = pf.vo1;
        L.ts[k] = pf.ts;
      } else {
        ko0 = a.key_off[s + k]; ko1 = a.key_off[s + k + 1];
        vo0 = a.val_off[s + k]; vo1 = a.val_off[s + k + 1];
        L.ts[k] = a.ts[s + k];
      }
      // (kChk) an entry outside its block's byte ranges or of negative length (offsets that
      // decrease: the plan helper refuses such a stream, but the fused launch emits while it
      // walks) is emptied and reported, so no loop below runs over a wrapped length
      const bool inv = kChk && (ko0 < kb0 || ko1 < ko0 || ko1 - kb0 > B.kb1 - kb0 || vo0 < vb0 || vo1 < vo0 ||
                                vo1 - vb0 > B.vb1 - vb0);
      if (inv) err |= LSMBLK_ERR_MALFORMED;
      kp = inv ? 0u : ko0 - kb0;
      kl = inv ? 0u : ko1 - ko0;
      vp = inv ? 0u : vo0 - vb0;
      vl = inv ? 0u : vo1 - vo0;
      if (k != 0 && !inv && !(diag_mask(a.skip) & 128)) {
        // the first 16 bytes by selects, no branches: z = the first differing byte (16 if none);
        // bytes read past either key do not matter, p is capped at m (the key image has 16 B
        // of slack before the value image, which is LDS too)
        const uint32_t m = fl < kl ? fl : kl;
        uint32_t z = 16;
#pragma unroll
        for (int i = 3; i >= 0; --i) {
          const uint32_t x = fkw[i] ^ lds_dword_at(L.kimg, EAL(klead + kp + 4 * i, 3));
          z = x ? 4 * i + (__builtin_ctz(x) >> 3) : z;
        }
        p = z < 16 && z < m ? z : m;  // (z == 16: m unless the loop below finds a difference)
        bool done = z < 16 || m <= 16;
        for (uint32_t q = 16; !done && q < m; q += 4) {
          const uint32_t x = lds_dword_at(L.kimg, klead + q) ^ lds_dword_at(L.kimg, klead + kp + q);
          if (x) {
            const uint32_t zq = q + (__builtin_ctz(x) >> 3);
            p = zq < m ? zq : m;
            done = true;
          }
        }
      }
      const uint32_t vs = vlead + vp;
      lds_read16(L.img, EAL(vs, 15), eh[it]);
      lds_read16(L.img, EAL(vs + (vl > 16 ? vl - 16 : 0u), 15), et[it]);
    }
    const uint32_t dg = k < n ? kl + vl + 14 - p : 0;
    const uint32_t incl = wave_incl_scan<uint32_t>(dg);
    const uint32_t pos = dc + incl - dg;
    dc += __shfl(incl, 63, 64);
    if (k < n) {
      const uint32_t sfx = kl - p;
      *reinterpret_cast<u32x4*>(L.erec + 4 * k) = u32x4{pos | (p << 16), (klead + kp + p) | (vl << 16), sfx, 0u};
      // the image chunks lying wholly inside this value -> their source bytes in the staged
      // values (every other chunk keeps ~0)
      {
        const uint32_t vdb = olead + pos + 14 + sfx;  // image byte of the value
        const uint32_t srcb = vlead + vp - vdb;       // + image byte = staged byte (mod 2^32)
        for (uint32_t cc = (vdb + 15) >> 4; 16 * cc + 16 <= vdb + vl; ++cc) L.cent[cc] = srcb + 16 * cc;
      }
    }
  }
  // (a block holding an emptied entry has the wrong length by construction: MALFORMED says why)
  if (uint64_t(dc) + 2ull * n + 2 != size && !(err & LSMBLK_ERR_MALFORMED)) err |= LSMBLK_ERR_INTERNAL;
  return dc;
}

// Phases 2b-3 of emit_kernel, the offsets table and the flush of block B's image.
template <uint32_t EB>
__device__ __forceinline__ void emit_finish(const EmitArgs& a, EmitLds& L, const EmitBlk& B, uint32_t data_len,
                                            uint32_t ncs, const uint32_t (&eh)[2][4], const uint32_t (&et)[2][4]) {
  const uint32_t l = lane_id();
  const uint32_t n = B.n, olead = B.olead;
  const uint64_t O = B.O, size = B.size;
  // Phase 2a (ascending): image chunk -> source byte of a chunk lying wholly inside one
  // value, else ~0 (the last entry whose value starts at or before the chunk by max-scan).
  // EB chunk groups per batch: every LDS read of the batch is issued before its uses.
  // (EMIT_DIRECT_CENT: the entry lanes wrote the map in phase 1)
  wave_sync();
  // Phase 2b (descending): move whole-value chunks to their place in the encoded block.
  // A value only moves up (its destination follows its own header and every earlier
  // record), so a chunk's source lies below the chunk's end: walking batches of chunks from
  // the top, with all of a batch's reads before its writes, never overwrites a source still
  // unread.
  if (!(diag_mask(a.skip) & 32)) {
    const int32_t top = int32_t((ncs + 63) & ~63u);
    for (int32_t c0 = top; c0 > 0; c0 -= int32_t(64 * EB)) {
      uint32_t src[EB];
      u32x4 v[EB];
#pragma unroll
      for (uint32_t j = 0; j < EB; ++j) {
        const int32_t c = c0 - int32_t(64 * (j + 1)) + int32_t(l);
        src[j] = (c0 >= int32_t(64 * (j + 1)) && uint32_t(c) < ncs) ? L.cent[c] : ~0u;
      }
#pragma unroll
      for (uint32_t j = 0; j < EB; ++j)
        if (src[j] != ~0u) v[j] = *reinterpret_cast<const u32x4*>(L.img + EAL(src[j], 15));
#pragma unroll
      for (uint32_t j = 0; j < EB; ++j)
        if (src[j] != ~0u) *reinterpret_cast<u32x4*>(L.img + 16 * (c0 - int32_t(64 * (j + 1)) + int32_t(l))) = v[j];
    }
  }
  wave_sync();
  // Phase 3, entry lanes: header, key suffix, ts, value_len, and the value bytes of the
  // partial edge chunks (from the registers captured in phase 1).
  if (!(diag_mask(a.skip) & 16)) {
#pragma unroll
    for (uint32_t it = 0; it < 2; ++it) {
      const uint32_t k = 64 * it + l;
      if (64 * it >= n) break;
      if (k >= n) continue;
      const u32x4 er = *reinterpret_cast<const u32x4*>(L.erec + 4 * k);
      const uint32_t pos = er.x & 0xFFFF, p = er.x >> 16, ks = er.y & 0xFFFF, vl = er.y >> 16, sfx = er.z;
      const uint32_t vd = pos + 14 + sfx;
      const uint64_t tsv = L.ts[k];
      // unaligned LDS stores (the image is not swizzled): every field is one or two stores
      uint8_t* o = L.img;
      const uint32_t ox = olead + pos;
      *reinterpret_cast<uint32_t*>(o + EAL(ox, 3)) = bswap16(p & 0xFFFF) | (bswap16(sfx & 0xFFFF) << 16);
      for (uint32_t t = 0; t < sfx; t += 16) {
        const uint32_t o2 = sfx >= 16 ? min(t, sfx - 16) : 0u;
        uint32_t v[4];
        lds_read16(L.kimg, EAL(ks + o2, 15), v);
        if (sfx >= 16) *reinterpret_cast<u32x4*>(o + EAL(ox + 4 + o2, 15)) = u32x4{v[0], v[1], v[2], v[3]};
        else lds_st_short(o + ox + 4, sfx, v);
      }
      const uint64_t tbe = __builtin_bswap64(tsv);
      *reinterpret_cast<u32x2*>(o + EAL(ox + 4 + sfx, 7)) = u32x2{uint32_t(tbe), uint32_t(tbe >> 32)};
      *reinterpret_cast<uint16_t*>(o + EAL(ox + 12 + sfx, 1)) = uint16_t(bswap16(vl & 0xFFFF));
      // value bytes outside whole chunks: a value of >= 16 bytes rewrites its first and last
      // 16 (the bytes inside whole chunks are rewritten with what the move put there)
      const uint32_t A = olead + vd;
      if (vl >= 16) {
        *reinterpret_cast<u32x4*>(o + EAL(A, 15)) = u32x4{eh[it][0], eh[it][1], eh[it][2], eh[it][3]};
        *reinterpret_cast<u32x4*>(o + EAL(A + vl - 16, 15)) = u32x4{et[it][0], et[it][1], et[it][2], et[it][3]};
      } else if (vl) {
        lds_st_short(o + A, vl, eh[it]);
      }
    }
  }
  wave_sync();
  // offsets table + entry count (u16 BE, `as u16`)
  for (uint32_t k = l; k < n; k += 64)
    *reinterpret_cast<uint16_t*>(L.img + olead + data_len + 2 * k) = uint16_t(bswap16(L.erec[4 * k] & 0xFFFF));
  if (l == 0) *reinterpret_cast<uint16_t*>(L.img + olead + data_len + 2 * n) = uint16_t(bswap16(n & 0xFFFF));
  wave_sync();
  // flush the image: 16-B chunks; only the two end chunks can be partial
  // (a block past out_cap writes nothing: the plan pass has raised CAPACITY)
  if (!(diag_mask(a.skip) & 64) && O + size <= a.out_cap) flush_run_masked<EB>(a.out + (O - olead), L.img, olead, uint32_t(size));
  wave_sync();
}

// Persistent waves, software-pipelined one block ahead: while block i is processed, the
// metadata, the key/value staging loads and the first 64 entries' offsets/ts of block i+1
// are already in flight (the wave is latency-bound otherwise: ~3 dependent global round
// trips per block).  LDS caps occupancy at 3 waves/SIMD, so the prefetch registers are free.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void emit_kernel(EmitArgs a0) {
  const EmitArgs a = resolve(a0);
  __shared__ EmitLds lds[kEmitWaves];
  EmitLds& L = lds[threadIdx.x >> 6];  // (a VGPR LDS base: readfirstlane here costs the kernel 4 spilled VGPRs)
  const uint32_t l = lane_id();
  const uint64_t nblk = uni64(a.stats[3]) & kPlanFatal ? 0 : uni64(a.stats[0]);
  const uint64_t nwaves = uint64_t(gridDim.x) * kEmitWaves;
  uint32_t err = 0;
  const uintptr_t kaddr = reinterpret_cast<uintptr_t>(a.keys), vaddr = reinterpret_cast<uintptr_t>(a.vals);
  const uint64_t lim = nblk < a.blk_cap ? nblk : (a.blk_cap ? a.blk_cap - 1 : 0);  // blk_off[bi+1] must exist

  // block metadata by scalar loads (written by the plan kernels / the caller, read-only here):
  // they wait on lgkmcnt, not behind the staging loads in flight
  cu32_t* const kfirst = kconst(a.blk_first);
  cu64_t* const koff = kconst(a.blk_off);
  // A block whose entry range is not s <= e <= n is refused with LSMBLK_ERR_INTERNAL and none of
  // its entries is read: its wrapped entry count would otherwise send it to emit_big_kernel's
  // per-entry walk, ~2^32 entries of unchecked global loads (the single-block emit
  // experiment's illegal address).  A valid plan never writes such a block.
  auto meta1 = [&](uint64_t bi, EmitMeta& m) {
    m.bi = bi;
    m.s = kfirst[bi];
    m.e = kfirst[bi + 1];
    m.bad = m.e < m.s || uint64_t(m.e) > a.n;
    if (m.bad) m.s = m.e = 0;  // (meta2's loads stay in bounds)
    m.n = m.e - m.s;
    m.O = koff[bi];
    m.size = a.blk_sz ? uint64_t(kconst(a.blk_sz)[bi]) : koff[bi + 1] - m.O;
  };
  auto meta2 = [&](EmitMeta& m) {
    m.kb0 = uni(a.key_off[m.s]);
    m.kb1 = uni(a.key_off[m.e]);
    m.vb0 = uni(a.val_off[m.s]);
    m.vb1 = uni(a.val_off[m.e]);
  };
  auto is_fast = [&](const EmitMeta& m) {
    const uint32_t klead = uint32_t((kaddr + m.kb0) & 15), vlead = uint32_t((vaddr + m.vb0) & 15);
    // the staged values and the encoded block share the image (24 B of read slack)
    return !m.bad && m.n <= kEmitMaxE && m.kb1 >= m.kb0 && m.vb1 >= m.vb0 && klead + (m.kb1 - m.kb0) + 8 <= kEmitKCap &&
           vlead + (m.vb1 - m.vb0) + 24 <= kEmitICap && uint32_t(m.O & 15) + m.size + 8 <= kEmitICap;
  };
  // a block off the fast path: beyond the LDS image -> flagged for emit_big_kernel; refused -> error
  auto not_fast = [&](const EmitMeta& m) {
    if (m.bad) err |= LSMBLK_ERR_INTERNAL;
    else if (l == 0) a.big_flag[m.bi] = 1;
  };
  u32x4 kq[2], vq[5];
  EmitPf pf;
  auto issue = [&](const EmitMeta& m) {  // staging + first-chunk entry loads of block m
    const uint32_t klead = uint32_t((kaddr + m.kb0) & 15), vlead = uint32_t((vaddr + m.vb0) & 15);
    const rsrc_t RK = make_rsrc(a.keys + m.kb0 - klead, klead + (m.kb1 - m.kb0));
    const uint32_t nk = (klead + (m.kb1 - m.kb0) + 15) >> 4;
    const rsrc_t RV = make_rsrc(a.vals + m.vb0 - vlead, vlead + (m.vb1 - m.vb0));
    const uint32_t nv = (vlead + (m.vb1 - m.vb0) + 15) >> 4;
#pragma unroll
    for (uint32_t i = 0; i < 2; ++i)
      if (l + 64 * i < nk) kq[i] = __builtin_amdgcn_raw_buffer_load_b128(RK, (l + 64 * i) * 16, 0, kLdAux);
#pragma unroll
    for (uint32_t i = 0; i < 5; ++i)
      if (l + 64 * i < nv) vq[i] = __builtin_amdgcn_raw_buffer_load_b128(RV, (l + 64 * i) * 16, 0, kLdAux);
    if (l < m.n) {
      pf.ko0 = a.key_off[m.s + l];
      pf.ko1 = a.key_off[m.s + l + 1];
      pf.vo0 = a.val_off[m.s + l];
      pf.vo1 = a.val_off[m.s + l + 1];
      pf.ts = a.ts[m.s + l];
    }
  };

  // The wave's next block on the fast path from bi on: blocks beyond the LDS image are flagged
  // for emit_big_kernel on the way (rare, so their dependent metadata loads are not hidden).
  // The prefetch of a fast block is issued in exactly two places (before the loop, and after
  // phase 1 for the next block): a third issue site in the loop (the flagged-block path used
  // to have one) gave the prefetch registers a second register assignment, and the waitcnt
  // pass then drained every load in flight (vmcnt(0)) inside the chunk move of each block.
  auto find_fast = [&](uint64_t bi, EmitMeta& m) -> bool {
    for (; bi < lim; bi += nwaves) {
      meta1(bi, m);
      meta2(m);
      if (is_fast(m)) return true;
      not_fast(m);
    }
    return false;
  };
  EmitMeta cur;
  if (!find_fast(uni64(uint64_t(blockIdx.x) * kEmitWaves + wave_id()), cur)) {
    raise_err(a.stats, err);
    return;
  }
  issue(cur);
  for (;;) {
    const uint64_t bn = cur.bi + nwaves;
    bool has_next = bn < lim;
    EmitMeta nxt;
    if (has_next) meta1(bn, nxt);  // level-1 of the next block (scalar loads)
    const uint32_t s = cur.s, n = cur.n;
    const uint64_t O = cur.O, size = cur.size;
    const uint32_t kb0 = cur.kb0, kb1 = cur.kb1, vb0 = cur.vb0, vb1 = cur.vb1;
    const uint32_t klead = uint32_t((kaddr + kb0) & 15), vlead = uint32_t((vaddr + vb0) & 15);
    const uint32_t olead = uint32_t(O & 15);
    // first key length at kimg[klead]: made uniform before the next block's level-2 loads are
    // issued (read after them, its wait would also cover the first of them: vmcnt is in order)
    const uint32_t fl = __builtin_amdgcn_readfirstlane(pf.ko1) - kb0;
    {  // land the staged keys (plain) and values (swizzled block image at vlead)
      const uint32_t nk = (klead + (kb1 - kb0) + 15) >> 4;
      const uint32_t nv = (vlead + (vb1 - vb0) + 15) >> 4;
#pragma unroll
      for (uint32_t i = 0; i < 2; ++i)
        if (l + 64 * i < nk) *reinterpret_cast<u32x4*>(L.kimg + (l + 64 * i) * 16) = kq[i];
#pragma unroll
      for (uint32_t i = 0; i < 5; ++i)
        if (l + 64 * i < nv) *reinterpret_cast<u32x4*>(L.img + (l + 64 * i) * 16) = vq[i];
    }
    // Every prefetched register has landed: say so to the waitcnt pass, whose own waits in the
    // exec-skippable landing stores do not cover all paths -- it would otherwise wait for
    // vmcnt(0) at the first use of a prefetched entry register in phase 1, i.e. for the
    // level-2 loads below as well.
    __builtin_amdgcn_s_waitcnt(0x0F70);  // s_waitcnt vmcnt(0)
    // level-2 of the next block: loaded now into VGPRs, made uniform after phase 1 (a
    // readfirstlane here would stall on the loads' round trip)
    uint32_t r_kb0 = 0, r_kb1 = 0, r_vb0 = 0, r_vb1 = 0;
    __builtin_amdgcn_sched_barrier(0);  // (not hoisted into the landing: its waits would cover them)
    if (has_next) {
      r_kb0 = a.key_off[nxt.s];
      r_kb1 = a.key_off[nxt.e];
      r_vb0 = a.val_off[nxt.s];
      r_vb1 = a.val_off[nxt.e];
    }
    wave_sync();
    const EmitBlk B{s, n, O, size, kb0, vb0, klead, vlead, olead, fl, kb1, vb1};
    uint32_t eh[2][4], et[2][4];  // first / last 16 bytes of the value of entries l, l + 64
    uint32_t ncs;
    const uint32_t data_len = emit_phase1<false>(a, L, B, pf, eh, et, ncs, err);
    // the level-2 loads have landed on every path (on the !has_next path there were none):
    // without this the waitcnt pass keeps them pending past the branch below and waits for
    // the next block's whole prefetch before the chunk moves reuse their registers
    __builtin_amdgcn_s_waitcnt(0x0F70);  // s_waitcnt vmcnt(0)
    if (has_next) {  // next block's staging loads overlap the rest of this block
      nxt.kb0 = uni(r_kb0);
      nxt.kb1 = uni(r_kb1);
      nxt.vb0 = uni(r_vb0);
      nxt.vb1 = uni(r_vb1);
      if (!is_fast(nxt)) {
        not_fast(nxt);
        has_next = find_fast(nxt.bi + nwaves, nxt);
      }
      if (has_next) issue(nxt);
    }
    wave_sync();
    emit_finish<kEB>(a, L, B, data_len, ncs, eh, et);
    if (!has_next) break;
    cur = nxt;
  }
  raise_err(a.stats, err);
}

// The blocks emit_kernel flagged as beyond its LDS image, one wave per block: wave j checks
// blocks j, j + nw, j + 2 nw, ... 64 at a time (a flag per lane, then a ballot).
__global__ __launch_bounds__(256) void emit_big_kernel(EmitArgs a0) {
  const EmitArgs a = resolve(a0);
  const uint64_t nblk = uni64(a.stats[3]) & kPlanFatal ? 0 : uni64(a.stats[0]);
  const uint64_t lim = nblk < a.blk_cap ? nblk : (a.blk_cap ? a.blk_cap - 1 : 0);
  const uint64_t nw = uint64_t(gridDim.x) * 4;
  const uint32_t l = lane_id();
  __shared__ alignas(16) uint32_t scratch[4][kCopyScratch];
  uint32_t* const sc = scratch[wave_id()];
  uint32_t err = 0;
  const uint32_t kg = uint32_t(reinterpret_cast<uintptr_t>(a.keys) & 15), vg = uint32_t(reinterpret_cast<uintptr_t>(a.vals) & 15);
  const uint32_t klim = kg + uni(a.key_off[a.n]), vlim = vg + uni(a.val_off[a.n]);  // valid descriptor bytes
  const rsrc_t RK = make_rsrc(a.keys - kg, klim), RV = make_rsrc(a.vals - vg, vlim);
  // this wave's flagged blocks, in order
  uint64_t wbase = uint64_t(blockIdx.x) * 4 + wave_id(), cbase = 0, bits = 0;
  // (a flagged block whose entry range is not s <= e <= n is refused with LSMBLK_ERR_INTERNAL, as in
  // emit_kernel: a wrapped entry count would walk ~2^32 entries of unchecked global loads)
  auto next_block = [&](BigBlk& B) -> bool {
    for (;;) {
      while (bits == 0) {
        if (wbase >= lim) return false;
        const uint64_t mine = wbase + nw * l;
        bits = __ballot(mine < lim && a.big_flag[mine]);
        cbase = wbase;
        wbase += nw * 64;
      }
      const uint32_t i = uint32_t(__builtin_ctzll(bits));
      bits &= bits - 1;
      B.bi = cbase + nw * i;
      B.s = uni(a.blk_first[B.bi]);
      const uint32_t e = uni(a.blk_first[B.bi + 1]);
      if (e < B.s || uint64_t(e) > a.n) {
        err |= LSMBLK_ERR_INTERNAL;
        continue;
      }
      B.n = e - B.s;
      B.O = uni64(a.blk_off[B.bi]);
      B.size = a.blk_sz ? uint64_t(uni(a.blk_sz[B.bi])) : uni64(a.blk_off[B.bi + 1]) - B.O;
      return true;
    }
  };
  auto issue_l1 = [&](const BigBlk& B, uint32_t c) -> BigL1 {
    BigL1 x{0u, 0u, 0u, 0u};
    const uint32_t k = c + l;
    if (k < B.n) {
      x.ko0 = a.key_off[B.s + k];
      x.ko1 = a.key_off[B.s + k + 1];
      x.vo0 = a.val_off[B.s + k];
      x.vo1 = a.val_off[B.s + k + 1];
    }
    return x;
  };
  // fp: descriptor byte of the block's first key (a 16-B load only where it stays in the keys)
  auto issue_l2 = [&](const BigL1& x, uint32_t fp) -> BigL2 {
    BigL2 y{u32x4{0u, 0u, 0u, 0u}, u32x4{0u, 0u, 0u, 0u}};
    const uint32_t kp = kg + x.ko0;
    if (kp + 16 <= klim) y.own = gload16(RK, kp);
    if (fp + 16 <= klim) y.first = gload16(RK, fp);
    return y;
  };
  BigBlk B;
  if (!next_block(B)) {
    raise_err(a.stats, err);
    return;
  }
  BigL1 x = issue_l1(B, 0);
  uint32_t fp = kg + uint32_t(__builtin_amdgcn_readlane(x.ko0, 0));        // key_off[s]
  uint32_t fl = uint32_t(__builtin_amdgcn_readlane(x.ko1, 0)) - (fp - kg);  // its length
  BigL2 y = issue_l2(x, fp);
  uint32_t c = 0;
  uint64_t dc = 0;
  for (;;) {
    // the next chunk: its entry offsets in flight during this one
    BigBlk NB = B;
    uint32_t nc = c + 64;
    bool more = true;
    if (nc >= B.n) {
      more = next_block(NB);
      nc = 0;
    }
    BigL1 nx{0u, 0u, 0u, 0u};
    if (more) nx = issue_l1(NB, nc);
    BigL2 ny{u32x4{0u, 0u, 0u, 0u}, u32x4{0u, 0u, 0u, 0u}};
    uint32_t nfp = fp, nfl = fl;
    bool ny_done = !more;
    auto issue_next_l2 = [&]() {
      if (ny_done) return;
      if (nc == 0) {
        nfp = kg + uint32_t(__builtin_amdgcn_readlane(nx.ko0, 0));
        nfl = uint32_t(__builtin_amdgcn_readlane(nx.ko1, 0)) - (nfp - kg);
      }
      ny = issue_l2(nx, nfp);
      ny_done = true;
    };
    // this chunk
    const uint32_t s = B.s, n = B.n, k = c + l;
    const uint32_t ob = uint32_t(B.O & 15);
    const uint64_t room = B.O < a.out_cap ? a.out_cap - B.O : 0;  // never store past out_cap
    const rsrc_t RO = make_rsrc_exact(a.out + (B.O - ob), ob + uint32_t(B.size < room ? B.size : room));
    const uint64_t data_len = B.size - 2ull * n - 2;
    uint32_t kp = 0, kl = 0, vp = 0, vl = 0, p = 0;
    uint64_t tsv = 0;
    if (k < n) {
      tsv = a.ts[s + k];  // (used after the copy rounds)
      kp = kg + x.ko0;
      kl = x.ko1 - x.ko0;
      vp = vg + x.vo0;
      vl = x.vo1 - x.vo0;
      if (k != 0 && !(diag_mask(a.skip) & 128)) {  // builder.rs:62 common_prefix(first_key, key)
        const uint32_t m = fl < kl ? fl : kl;
        p = m;
        uint32_t q = 0;
        if (fp + 16 <= klim && kp + 16 <= klim) {  // the first 16 bytes from the prefetch
          const uint32_t d[4] = {y.first.x ^ y.own.x, y.first.y ^ y.own.y, y.first.z ^ y.own.z, y.first.w ^ y.own.w};
          uint32_t z = 16;
          for (uint32_t i = 0; i < 4 && z == 16; ++i)
            if (d[i]) z = 4 * i + (__builtin_ctz(d[i]) >> 3);
          q = z < 16 || m <= 16 ? m : 16u;
          if (z < 16) p = min(z, m);
        }
        for (; q < m; q += 16) {
          uint32_t z = 16;  // first differing byte in [q, q + 16)
          if (fp + q + 16 <= klim && kp + q + 16 <= klim) {
            const u32x4 xa = gload16(RK, fp + q), ya = gload16(RK, kp + q);
            const uint32_t d[4] = {xa.x ^ ya.x, xa.y ^ ya.y, xa.z ^ ya.z, xa.w ^ ya.w};
            for (uint32_t i = 0; i < 4 && z == 16; ++i)
              if (d[i]) z = 4 * i + (__builtin_ctz(d[i]) >> 3);
          } else {
            for (uint32_t i = 0; i < 16 && z == 16 && q + i < m; ++i)
              if (__builtin_amdgcn_raw_buffer_load_b8(RK, fp + q + i, 0, 0) !=
                  __builtin_amdgcn_raw_buffer_load_b8(RK, kp + q + i, 0, 0))
                z = i;
          }
          if (z < 16) {
            p = min(q + z, m);
            break;
          }
        }
      }
    }
    const uint64_t dg = k < n ? uint64_t(kl) + vl + 14 - p : 0;
    const uint64_t incl = wave_incl_scan<uint64_t>(dg);
    const uint64_t pos = dc + incl - dg;
    dc += __shfl(incl, 63, 64);
    const uint32_t sfx = kl - p, at = ob + uint32_t(pos), vdst = at + 14 + sfx;
    // builder.rs:71: offsets.push(data.len() as u16), BE (the table's stores are contiguous)
    if (k < n && !(diag_mask(a.skip) & 16))
      __builtin_amdgcn_raw_buffer_store_b16(uint16_t(bswap16(uint32_t(pos) & 0xFFFF)), RO, ob + uint32_t(data_len) + 2 * k, 0, 0);
    // builder.rs:63-70: BE u16 prefix, BE u16 suffix len, suffix, BE u64 ts, BE u16 value len, value.
    // A record's fields (and a short value) are stored right after the copy round that stores the
    // first piece of its long value (or the next long value), so the partial lines they share with
    // the value pieces around them are written close together in time: written up front, the
    // fields' lines were evicted from L2 half-written before the pieces came (M: WRITE_SIZE 1.165x
    // the encoded bytes).  The next chunk's level-2 loads go out after the first round.
    auto fields = [&](uint32_t first, uint32_t lo, uint32_t hi) {
      if (k < n && first >= lo && first < hi && !(diag_mask(a.skip) & 16)) {
        __builtin_amdgcn_raw_buffer_store_b32(bswap16(p & 0xFFFF) | (bswap16(sfx & 0xFFFF) << 16), RO, at, 0, 0);
        copy_run1(RK, kp + p, klim, RO, at + 4, sfx);
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{__builtin_bswap32(uint32_t(tsv >> 32)), __builtin_bswap32(uint32_t(tsv))},
                                              RO, at + 4 + sfx, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b16(uint16_t(bswap16(vl & 0xFFFF)), RO, at + 12 + sfx, 0, 0);
        if (vl < kCoop) copy_run1(RV, vp, vlim, RO, vdst, vl);
      }
      issue_next_l2();
    };
    if (!(diag_mask(a.skip) & 32)) copy_long_runs<kEmitBigB>(k < n && vl >= kCoop, RV, vp, RO, vdst, vl, sc, fields);
    else fields(0u, 0u, ~0u);
    if (c + 64 >= n) {  // the block's last chunk
      if (dc != data_len) err |= LSMBLK_ERR_INTERNAL;
      if (l == 0) __builtin_amdgcn_raw_buffer_store_b16(uint16_t(bswap16(n & 0xFFFF)), RO, ob + uint32_t(B.size) - 2, 0, 0);
      dc = 0;
    }
    if (!more) break;
    B = NB;
    c = nc;
    x = nx;
    y = ny;
    fp = nfp;
    fl = nfl;
  }
  raise_err(a.stats, err);
}

// Fault injection (LSMBLK_DEBUG_EMIT_POISON, diagnostics builds): after the plan walk, block b = 1,
// 6, 11, ... gets first entry blk_first[b + 1] + 1, so block b's end precedes its start and block
// b - 1 ends one entry later (past n when b is the last block).  Thread t writes only b = 1 + 5 t
// and reads only b + 1, which no thread writes.
__global__ __launch_bounds__(256) void emit_poison_kernel(uint32_t* blk_first, const uint64_t* stats) {
  if (stats[3] & kPlanFatal) return;
  const uint64_t nblk = stats[0], b = 1 + 5 * (uint64_t(blockIdx.x) * 256 + threadIdx.x);
  if (b < nblk) blk_first[b] = blk_first[b + 1] + 1;
}

// ================================================================ encode: fused walk + emit
// LSMBLK_ENCODE_SEG_SLOTS (per-segment output) with blocks no larger than emit's LDS image, under
// LSMBLK_DEBUG_ENCODE_FUSED: the plan walk and emit run in one launch.  Measured (DESIGN.md section
// 8): correct, but 2.16-2.18 ms against 2.08 for the two launches at U -- the walkers finish at 1.2
// ms and the emitters almost never wait for a record, yet emit slows by the walk's instructions,
// which need the same SIMD issue slots (both are issue-bound).  Segment g's blocks go back to back to its own slot,
//   slot(g) = (key_off[s_g] - key_off[s_0]) + (val_off[s_g] - val_off[s_0]) + 18 (s_g - s_0),
// the bytes of every earlier segment's keys and values plus 18 per entry: an upper bound of those
// segments' encoded size (an entry costs 2 + 2 + 8 + 2 header bytes + its 2-byte offset slot + its
// key and value minus the shared prefix, a block 2 more for its count, and a block holds at least
// one entry).  So no block's position depends on another segment's walk, and a block can be
// emitted as soon as its segment's walker has found it -- the walk leaves the critical path.
//   * Workgroups [0, walk_wgs): two walkers and their two helpers (plan_walk_kernel's waves; their
//     rings in the workgroup's LDS).  Walker w walks segments [w spw, (w + 1) spw) one after
//     another and publishes every block as a record of four tagged granules {first entry, end
//     entry, output offset, size} at R(w, i) = s_(w spw) - s_0 + w + i (a walker has at most one
//     block per entry), then its block count (wdone[w]).
//   * The other workgroups: emit_kernel's waves.  Emitter e takes walker (e mod nwalk)'s blocks
//     i = e / nwalk, + r, + 2 r, ... (r emitters per walker) until the walker's count says there
//     are no more; the record of its next block is loaded while a block is emitted (landed by the
//     landing's vmcnt(0)).
// Emitters wait only on walkers and walkers only on their helpers, all in lower-indexed (earlier
// dispatched) workgroups; every wait is bounded (TIMEOUT).  emit_kernel measured the same at 12
// and 16 waves per CU, so the walkers take one of a CU's four slots.
struct FuseArgs {
  PlanArgs p;
  EmitArgs e;
  uint64_t* rec;       // uncached: 4 granules per block record
  uint64_t* wdone;     // uncached: per walker, its block count (flag 2)
  uint32_t* wnb;       // per walker, its block count (plain: slot_tables_kernel)
  uint64_t* seg_out;   // per segment: slot start, encoded bytes
  uint8_t* bigr;       // per record: the block is beyond the LDS image (emit_big_kernel)
  uint32_t nwalk;      // walkers (2 per walker workgroup)
  uint32_t spw;        // segments per walker
  uint32_t walk_wgs;   // workgroups [0, walk_wgs) walk
  uint32_t per_walker; // emitters per walker (r)
};
static_assert(4 * kRing * 4 + 16 <= sizeof(EmitLds) * kEmitWaves, "two walkers' rings fit emit's LDS");

__device__ __forceinline__ uint32_t walker_first_seg(const FuseArgs& f, uint32_t w) {
  return uint32_t(min(uint64_t(w) * f.spw, uint64_t(f.p.nseg)));
}
// Record index of walker w's first block.
__device__ __forceinline__ uint32_t walker_rbase(const FuseArgs& f, uint32_t w) {
  return f.p.seg_start[walker_first_seg(f, w)] - f.p.seg_start[0] + w;
}

__device__ void fuse_walk(const FuseArgs& f, uint32_t* ring) {
  const PlanArgs& a = f.p;
  const uint32_t l = lane_id(), wv = wave_id(), ww = wv & 1;
  uint32_t* CR = ring + ww * kRing;
  uint32_t* CA = ring + (2 + ww) * kRing;
  uint32_t* prod = ring + 4 * kRing + ww;
  uint32_t* cons = ring + 4 * kRing + 2 + ww;
  const uint32_t w = 2 * blockIdx.x + ww;
  const uint32_t g0 = walker_first_seg(f, w), g1 = uint32_t(min(uint64_t(g0) + f.spw, uint64_t(a.nseg)));
  uint32_t err = 0;
  // the walker's segments must be a non-decreasing run inside the stream (seg_start[0] = 0,
  // seg_start[nseg] = n); otherwise neither wave walks and the call fails with SEGMENTS
  bool ok = uni(a.seg_start[0]) == 0;
  for (uint32_t g = g0; g < g1; ++g) {
    const uint32_t s0 = uni(a.seg_start[g]), s1 = uni(a.seg_start[g + 1]);
    if ((g == 0 && s0 != 0) || (g == a.nseg - 1 && uint64_t(s1) != a.n) || s0 > s1 || uint64_t(s1) > a.n) ok = false;
  }
  const uint32_t S0 = ok ? uni(a.seg_start[g0]) : 0u, S1 = ok ? uni(a.seg_start[g1]) : 0u;
  const PlanKeys K = plan_keys(a);
  if (wv >= 2) {
    plan_produce_pipe(a, K, S0, S1, CR, CA, prod, cons, err);
    const uint32_t werr = (__ballot(err & LSMBLK_ERR_EMPTY_KEY) ? LSMBLK_ERR_EMPTY_KEY : 0u) |
                          (__ballot(err & LSMBLK_ERR_MALFORMED) ? LSMBLK_ERR_MALFORMED : 0u) |
                          (__ballot(err & LSMBLK_ERR_TIMEOUT) ? LSMBLK_ERR_TIMEOUT : 0u);
    raise_err(a.stats, werr);
    return;
  }
  if (!ok) err |= LSMBLK_ERR_SEGMENTS;
  WalkRing R{CR, CA, cons, prod, S0};
  const uint32_t rb = walker_rbase(f, w);
  const uint64_t tagb = uint64_t(a.tag) << 2;
  uint32_t nbw = 0;
  uint64_t waited = 0, windows = 0;
  // (diagnostics: per-walker realtime trace, bench.py --trace-fused)
  uint64_t* const tr = kDiag && a.dbg && w < kDbgTiles ? a.dbg + 16 + 8 * uint64_t(w) : nullptr;
  if (tr && l == 0) tr[0] = __builtin_amdgcn_s_memrealtime();
  for (uint32_t g = g0; ok && g < g1; ++g) {
    const uint32_t s0 = uni(a.seg_start[g]), s1 = uni(a.seg_start[g + 1]);
    const uint64_t slot = seg_slot(a.key_off, a.val_off, 0u, s0);  // (ok: seg_start[0] = 0, s0 <= n)
    uint32_t nb = 0;
    uint64_t bytes = 0;
    walk_segment(a, K, R, s0, s1, err, nb, bytes,
                 [&](uint32_t first, uint32_t end, uint32_t size, uint32_t i, uint64_t before) {
                   const uint64_t v = l == 0 ? first : (l == 1 ? end : (l == 2 ? slot + before : size));
                   if (l < 4) gstore(f.rec + 4ull * (rb + nbw + i) + l, (v << 16) | tagb | 1, a.poll);
                 },
                 tr, waited, windows);
    if (l == 0) {
      f.seg_out[2ull * g] = slot;
      f.seg_out[2ull * g + 1] = bytes;
    }
    nbw += nb;
  }
  if (l == 0) {
    f.wnb[w] = nbw;
    gstore(f.wdone + w, (uint64_t(nbw) << 16) | tagb | 2, a.poll);
    if (tr) {
      tr[1] = __builtin_amdgcn_s_memrealtime();
      tr[2] = waited;
      tr[3] = windows;
      tr[4] = nbw;
    }
  }
  raise_err(a.stats, err);
}

__device__ void fuse_emit(const FuseArgs& f, EmitLds& L) {
  const EmitArgs& a = f.e;
  const uint32_t l = lane_id();
  const uint32_t eidx = (blockIdx.x - f.walk_wgs) * kEmitWaves + wave_id();
  const uint32_t w = eidx % f.nwalk, r = f.per_walker;
  uint32_t it = eidx / f.nwalk;  // this emitter's first block of walker w
  if (it >= r) return;           // (grid rounding)
  // walker w's entries bound its blocks: records [rb, rb + cap) are its own
  const uint32_t g0 = walker_first_seg(f, w), g1 = uint32_t(min(uint64_t(g0) + f.spw, uint64_t(f.p.nseg)));
  const uint32_t S0 = uni(f.p.seg_start[g0]), S1 = uni(f.p.seg_start[g1]);
  // (a segment table the walkers refuse -- SEGMENTS -- gives the emitters no records to poll)
  const bool sane = uni(f.p.seg_start[0]) == 0 && S0 <= S1 && uint64_t(S1) <= f.p.n;
  const uint32_t cap = sane ? S1 - S0 : 0u, rb = S0 + w;
  const uint64_t want1 = (uint64_t(f.p.tag) << 2) | 1, want2 = (uint64_t(f.p.tag) << 2) | 2;
  uint32_t err = 0;
  const uintptr_t kaddr = reinterpret_cast<uintptr_t>(a.keys), vaddr = reinterpret_cast<uintptr_t>(a.vals);
  // The record of block x of walker w: lanes 0-3 its granules, the others the walker's block count
  // (agent-coherent sc1 loads of uncached memory, as gload).  Every record load is inline asm: the
  // in-loop prefetch (the block after next) is landed by the landing's explicit vmcnt(0), the
  // others by their own wait.  Issued as compiler loads, their destinations stayed "pending" for
  // the waitcnt pass into the block's LDS loops, which then began with vmcnt(0) -- draining the
  // next block's staging loads (2.5 ms against emit_kernel's 1.7).
  auto rec_issue_asm = [&](uint32_t x) -> uint64_t {
    const uint64_t* p = x < cap && l < 4 ? f.rec + 4ull * (rb + x) + l : f.wdone + w;
    uint64_t g;
    asm volatile("global_load_dwordx2 %0, %1, off sc1" : "=&v"(g) : "v"(p));
    return g;
  };
  auto rec_poll = [&](uint32_t x) -> uint64_t {
    uint64_t g = rec_issue_asm(x);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("" : "+v"(g));
    return g;
  };
  uint64_t* const dbg = kDiag ? f.p.dbg : nullptr;  // (diagnostics: record-wait ticks, bench.py --trace-fused)
  uint64_t wait_t = 0, nwait = 0, nitems = 0;
  // 1: m is block x; 0: walker w has no block x (the emitter is done); -1: timeout
  auto rec_resolve = [&](uint64_t g, uint32_t x, EmitMeta& m) -> int {
    if (x >= cap) return 0;
    const uint64_t t0 = dbg ? __builtin_amdgcn_s_memrealtime() : 0;
    if (dbg) ++nitems;
    for (uint32_t spins = 0;; ++spins) {
      const uint64_t okm = __ballot((l < 4 && (g & 0xFFFF) == want1) || (l == 4 && (g & 0xFFFF) == want2));
      if ((okm & 0xF) == 0xF) {
        m.bi = x;
        m.s = uint32_t(lane64(g, 0) >> 16);
        m.e = uint32_t(lane64(g, 1) >> 16);
        m.bad = false;  // (the walker's own records: s < e <= n)
        m.n = m.e - m.s;
        m.O = lane64(g, 2) >> 16;
        m.size = lane64(g, 3) >> 16;
        if (dbg && spins) {
          wait_t += __builtin_amdgcn_s_memrealtime() - t0;
          ++nwait;
        }
        return 1;
      }
      if ((okm & 0x10) && x >= uint32_t(lane64(g, 4) >> 16)) return 0;
      if (spins > kSpinLimit) return -1;
      __builtin_amdgcn_s_sleep(1);
      g = rec_poll(x);
    }
  };
  auto meta2 = [&](EmitMeta& m) {
    m.kb0 = uni(a.key_off[m.s]);
    m.kb1 = uni(a.key_off[m.e]);
    m.vb0 = uni(a.val_off[m.s]);
    m.vb1 = uni(a.val_off[m.e]);
  };
  auto is_fast = [&](const EmitMeta& m) {
    const uint32_t klead = uint32_t((kaddr + m.kb0) & 15), vlead = uint32_t((vaddr + m.vb0) & 15);
    // (decreasing bounds: not fast; the helper has refused the stream, so emit_big writes nothing)
    return m.n <= kEmitMaxE && m.kb1 >= m.kb0 && m.vb1 >= m.vb0 && klead + (m.kb1 - m.kb0) + 8 <= kEmitKCap &&
           vlead + (m.vb1 - m.vb0) + 24 <= kEmitICap && uint32_t(m.O & 15) + m.size + 8 <= kEmitICap;
  };
  u32x4 kq[2], vq[5];
  EmitPf pf;
  auto issue = [&](const EmitMeta& m) {  // staging + first-chunk entry loads of block m
    const uint32_t klead = uint32_t((kaddr + m.kb0) & 15), vlead = uint32_t((vaddr + m.vb0) & 15);
    const rsrc_t RK = make_rsrc(a.keys + m.kb0 - klead, klead + (m.kb1 - m.kb0));
    const uint32_t nk = (klead + (m.kb1 - m.kb0) + 15) >> 4;
    const rsrc_t RV = make_rsrc(a.vals + m.vb0 - vlead, vlead + (m.vb1 - m.vb0));
    const uint32_t nv = (vlead + (m.vb1 - m.vb0) + 15) >> 4;
#pragma unroll
    for (uint32_t i = 0; i < 2; ++i)
      if (l + 64 * i < nk) kq[i] = __builtin_amdgcn_raw_buffer_load_b128(RK, (l + 64 * i) * 16, 0, kLdAux);
#pragma unroll
    for (uint32_t i = 0; i < 5; ++i)
      if (l + 64 * i < nv) vq[i] = __builtin_amdgcn_raw_buffer_load_b128(RV, (l + 64 * i) * 16, 0, kLdAux);
    if (l < m.n) {
      pf.ko0 = a.key_off[m.s + l];
      pf.ko1 = a.key_off[m.s + l + 1];
      pf.vo0 = a.val_off[m.s + l];
      pf.vo1 = a.val_off[m.s + l + 1];
      pf.ts = a.ts[m.s + l];
    }
  };
  // from block x on (x advanced), the first on the fast path; the others are flagged for
  // emit_big_kernel.  Waits for each record (before the loop, and after a flagged block).
  auto find_fast = [&](uint32_t& x, EmitMeta& m) -> bool {
    for (;; x += r) {
      const int st = rec_resolve(rec_poll(x), x, m);
      if (st <= 0) {
        if (st < 0) err |= LSMBLK_ERR_TIMEOUT;
        return false;
      }
      meta2(m);
      if (is_fast(m)) return true;
      if (l == 0) f.bigr[rb + x] = 1;
    }
  };
  EmitMeta cur;
  if (!find_fast(it, cur)) {
    raise_err(a.stats, err);
    return;
  }
  issue(cur);
  uint32_t in = it + r;        // the next block: its record loads in flight
  uint64_t pg = rec_issue_asm(in);
  for (;;) {
    const uint32_t s = cur.s, n = cur.n;
    const uint64_t O = cur.O, size = cur.size;
    const uint32_t kb0 = cur.kb0, kb1 = cur.kb1, vb0 = cur.vb0, vb1 = cur.vb1;
    const uint32_t klead = uint32_t((kaddr + kb0) & 15), vlead = uint32_t((vaddr + vb0) & 15);
    const uint32_t olead = uint32_t(O & 15);
    const uint32_t fl = __builtin_amdgcn_readfirstlane(pf.ko1) - kb0;
    {  // land the staged keys (plain) and values (block image at vlead)
      const uint32_t nk = (klead + (kb1 - kb0) + 15) >> 4;
      const uint32_t nv = (vlead + (vb1 - vb0) + 15) >> 4;
#pragma unroll
      for (uint32_t i = 0; i < 2; ++i)
        if (l + 64 * i < nk) *reinterpret_cast<u32x4*>(L.kimg + (l + 64 * i) * 16) = kq[i];
#pragma unroll
      for (uint32_t i = 0; i < 5; ++i)
        if (l + 64 * i < nv) *reinterpret_cast<u32x4*>(L.img + (l + 64 * i) * 16) = vq[i];
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // s_waitcnt vmcnt(0): the staging and the next record
    asm volatile("" : "+v"(pg));         // (landed: defined here for the compiler)
    EmitMeta nxt;
    const int st = rec_resolve(pg, in, nxt);
    bool has_next = st > 0;
    if (st < 0) err |= LSMBLK_ERR_TIMEOUT;
    uint32_t r_kb0 = 0, r_kb1 = 0, r_vb0 = 0, r_vb1 = 0;
    __builtin_amdgcn_sched_barrier(0);
    if (has_next) {
      r_kb0 = a.key_off[nxt.s];
      r_kb1 = a.key_off[nxt.e];
      r_vb0 = a.val_off[nxt.s];
      r_vb1 = a.val_off[nxt.e];
    }
    wave_sync();
    const EmitBlk B{s, n, O, size, kb0, vb0, klead, vlead, olead, fl, kb1, vb1};
    uint32_t eh[2][4], et[2][4];
    uint32_t ncs;
    const uint32_t data_len = emit_phase1<true>(a, L, B, pf, eh, et, ncs, err);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // s_waitcnt vmcnt(0)
    if (has_next) {
      nxt.kb0 = uni(r_kb0);
      nxt.kb1 = uni(r_kb1);
      nxt.vb0 = uni(r_vb0);
      nxt.vb1 = uni(r_vb1);
      if (!is_fast(nxt)) {
        if (l == 0) f.bigr[rb + in] = 1;
        in += r;
        has_next = find_fast(in, nxt);
      }
      if (has_next) {
        issue(nxt);
        in += r;
        pg = rec_issue_asm(in);
      }
    }
    wave_sync();
    emit_finish<1>(a, L, B, data_len, ncs, eh, et);  // (one chunk group: four spill beside the fused launch's walk state)
    if (!has_next) break;
    cur = nxt;
  }
  if (dbg && l == 0) {
    atomicAdd(reinterpret_cast<unsigned long long*>(dbg + 0), (unsigned long long)wait_t);
    atomicAdd(reinterpret_cast<unsigned long long*>(dbg + 1), (unsigned long long)nwait);
    atomicAdd(reinterpret_cast<unsigned long long*>(dbg + 2), (unsigned long long)nitems);
    atomicMax(reinterpret_cast<unsigned long long*>(dbg + 3), (unsigned long long)__builtin_amdgcn_s_memrealtime());
  }
  raise_err(a.stats, err);
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void encode_fused_kernel(FuseArgs f) {
  __shared__ EmitLds lds[kEmitWaves];
  if (blockIdx.x < f.walk_wgs) {
    // the walk is the serial part: its waves win the issue arbitration against the emitters
    // sharing their SIMDs
    __builtin_amdgcn_s_setprio(3);
    uint32_t* ring = reinterpret_cast<uint32_t*>(lds);
    if (threadIdx.x < 4) ring[4 * kRing + threadIdx.x] = 0;  // the hand-off counters
    __syncthreads();
    fuse_walk(f, ring);
  } else {
    fuse_emit(f, lds[threadIdx.x >> 6]);
  }
}

// After encode_fused_kernel: the dense block tables of the slot output -- blk_first, blk_off (every
// block's position), blk_sz, the big-block flags -- stats[0] / [1], and the capacity checks.
// Workgroup w takes walker w's blocks: dense indices B_w + i (a walker's segments are consecutive).
// blk_off[nblk] = the end of the last segment's data.
__global__ __launch_bounds__(256) void slot_tables_kernel(FuseArgs f, uint32_t* blk_first, uint32_t* blk_sz,
                                                          uint8_t* big_flag, uint64_t* blk_off, uint64_t blk_cap,
                                                          uint64_t out_cap) {
  __shared__ uint64_t part[4];
  const uint32_t w = blockIdx.x, tid = threadIdx.x, l = lane_id();
  uint64_t acc = 0;
  for (uint32_t v = tid; v < w; v += 256) acc += f.wnb[v];
  acc = wave_sum<uint64_t>(acc);
  if (l == 0) part[tid >> 6] = acc;
  __syncthreads();
  const uint64_t B = part[0] + part[1] + part[2] + part[3];
  const uint32_t nb = f.wnb[w], rb = walker_rbase(f, w);
  for (uint32_t i = tid; i < nb; i += 256) {
    const uint64_t* g = f.rec + 4ull * (rb + i);
    const uint64_t bi = B + i;
    blk_first[bi] = uint32_t(g[0] >> 16);
    blk_sz[bi] = uint32_t(g[3] >> 16);
    big_flag[bi] = f.bigr[rb + i];
    f.bigr[rb + i] = 0;
    if (bi < blk_cap) blk_off[bi] = g[2] >> 16;
  }
  if (tid == 0) {
    uint32_t err = 0;
    uint64_t bytes = 0;
    const uint32_t g0 = walker_first_seg(f, w), g1 = uint32_t(min(uint64_t(g0) + f.spw, uint64_t(f.p.nseg)));
    for (uint32_t g = g0; g < g1; ++g) {
      bytes += f.seg_out[2ull * g + 1];
      if (f.seg_out[2ull * g] + f.seg_out[2ull * g + 1] > out_cap) err |= LSMBLK_ERR_CAPACITY;
    }
    if (bytes) atomicAdd(reinterpret_cast<unsigned long long*>(f.p.stats + 1), (unsigned long long)bytes);
    if (w == f.nwalk - 1) {
      const uint64_t nblk = B + nb, gl = f.p.nseg - 1;
      blk_first[nblk] = uint32_t(f.p.n);
      if (nblk < blk_cap) blk_off[nblk] = f.seg_out[2 * gl] + f.seg_out[2 * gl + 1];
      f.p.stats[0] = nblk;
      if (nblk + 1 > blk_cap) err |= LSMBLK_ERR_CAPACITY;
    }
    if (err) atomicOr(reinterpret_cast<unsigned long long*>(f.p.stats + 3), (unsigned long long)err);
  }
}

// read_block's check (src/table.rs:226-230): the BE u32 after every block must equal the
// block's crc32fast.  A mismatch raises LSMBLK_ERR_CHECKSUM in the decode stats.
__global__ __launch_bounds__(256) void crc_verify_kernel(const uint8_t* blocks, const uint64_t* blk_off, uint64_t nblk,
                                                         const uint32_t* crc, const uint64_t* cstats, uint64_t* stats) {
  const uint64_t b = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  uint32_t err = 0;
  if (b == 0) err |= uint32_t(cstats[3]);  // MALFORMED ranges, and the fused count's flags
  if (b < nblk) {
    const uint64_t e = blk_off[b + 1];
    if (e >= blk_off[b] + 4) {
      const uint8_t* q = blocks + e - 4;
      const uint32_t stored = (uint32_t(q[0]) << 24) | (uint32_t(q[1]) << 16) | (uint32_t(q[2]) << 8) | q[3];
      if (stored != crc[b]) err |= LSMBLK_ERR_CHECKSUM;
    }
  }
  for (uint32_t d = 32; d >= 1; d >>= 1) err |= __shfl_xor(err, d, 64);
  raise_err(stats, err);
}

// Per-64-block tile sums of agg (the count pass writes agg), one wave per tile.
__global__ __launch_bounds__(256) void agg_tile_kernel(const uint32_t* agg, uint64_t nblk, uint64_t* tile_sum) {
  const uint64_t tile = uint64_t(blockIdx.x) * 4 + wave_id(), b = tile * kTile + lane_id();
  if (tile * kTile >= nblk) return;
  uint64_t x[3] = {0, 0, 0};
  if (b < nblk) {
    x[0] = agg[3 * b];
    x[1] = agg[3 * b + 1];
    x[2] = agg[3 * b + 2];
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const uint64_t t = wave_sum(x[i]);
    if (lane_id() == 0) tile_sum[3 * tile + i] = t;
  }
}

__global__ void finish_empty_decode(uint32_t* key_off, uint32_t* val_off, uint64_t cap) {
  if (threadIdx.x == 0 && cap + 1 > 0) {
    key_off[0] = 0;
    val_off[0] = 0;
  }
}

// ================================================================ CRC-32 (SST block framing)
// crc32fast::hash of every block: the checksum SsTableBuilder::finish_block appends
// (src/table/builder.rs:120-122) and SsTable::read_block verifies (src/table.rs:226-230).
// CRC-32/ISO-HDLC: reflected polynomial 0xEDB88320, init and xorout 0xFFFFFFFF.
//
// CRC is a serial recurrence per block, so a wave splits each 4-KiB chunk into (at most 61)
// segments of kCrcSeg = 68 B, one per lane, and recombines them by linearity.  With R_x(M)
// the CRC register after feeding M from state x and Z(x, n) = R_x(n zero bytes) (linear in x):
//   R_x(A || B) = Z(R_x(A), |B|) ^ R_0(B).
// The chunk is right-aligned on the lanes -- its one short segment (sz mod 68) is the
// first -- so the segment of lane l is followed by exactly 63 - l full segments and
// contributes Z(R(seg_l), 68 (63 - l)): the binary digits of 63 - l select up to six of the
// precomputed maps Z(., 68 << j).  (68 = 17 dwords keeps the 32 lanes of an LDS read group on
// 32 distinct banks; 64-B segments measured 2.5 ms per 4.2 GB, 16-way conflicted.)  The
// block's init 0xFFFFFFFF rides in its first segment;
// chunk after chunk, acc = Z(acc, 4096) ^ R_0(chunk).
//
// Every linear map (the 4-byte fold step and each Z) is applied as eight 16-entry NIBBLE
// tables in LDS: all 64 lanes of one lookup instruction then address 16 dwords in 16
// distinct banks (repeats broadcast), so lookups are conflict-free.  256-entry byte tables
// put 64 random lanes on 32 banks and measured 1.6 TB/s; 4 KiB of nibble tables also leave
// room for more resident workgroups.
struct CrcArgs {
  const uint8_t* blocks;
  const uint64_t* blk_off;
  uint64_t nblk;
  uint32_t tail;  // bytes of each range that are not block (4: the framing CRC itself)
  uint32_t* crc;
  const CrcTabs* tabs;
  uint64_t* stats;
  // optional (the verifying decode): per-block (entries, key bytes, value bytes) exactly as
  // the count pass computes them, parsed from the staged block -- one read of E for both
  uint32_t* agg;
};

// (entries, key bytes, value bytes) of one block with decode_block's parse rules; 0s and
// MALFORMED for a block that breaks them, OVERFLOW past u32.  Written by lane 0.
template <class Img>
__device__ void count_block(const Img& im, uint32_t len, bool len_ok, uint32_t* agg, uint32_t& err) {
  const uint32_t l = lane_id();
  BlockHdr h = parse_hdr(im, len);
  bool bad = !len_ok || !h.ok;
  uint64_t K = 0, V = 0;
  const uint32_t n = bad ? 0u : h.n;
  for (uint32_t c = 0; c < n; c += 64) {
    const uint32_t k = c + l;
    uint32_t off = 0, p = 0, s = 0, vl = 0;
    if (k < n) bad = bad || !parse_entry(im, h, k, off, p, s, vl);
    K += wave_sum<uint64_t>(p + s);
    V += wave_sum<uint64_t>(vl);
  }
  bad = __ballot(bad) != 0;
  if (bad) err |= LSMBLK_ERR_MALFORMED;
  if (K > 0xFFFFFFFFull || V > 0xFFFFFFFFull) err |= LSMBLK_ERR_OVERFLOW;
  if (l == 0) {
    agg[0] = bad ? 0u : n;
    agg[1] = bad ? 0u : uint32_t(K > 0xFFFFFFFFull ? 0xFFFFFFFFull : K);
    agg[2] = bad ? 0u : uint32_t(V > 0xFFFFFFFFull ? 0xFFFFFFFFull : V);
  }
}

// COUNT: also the per-block counts into a.agg (the verifying decode); a separate instantiation
// so the plain CRC keeps its registers (and occupancy)
template <bool COUNT>
__global__ __launch_bounds__(256) void crc_kernel(CrcArgs a) {
  __shared__ CrcTabs T;
  __shared__ __attribute__((aligned(16))) uint8_t stage[4][kCrcStage];
  const uint32_t t = threadIdx.x, w = t >> 6, l = lane_id();
  for (uint32_t i = t; i < sizeof(CrcTabs) / 16; i += 256)
    reinterpret_cast<u32x4*>(&T)[i] = reinterpret_cast<const u32x4*>(a.tabs)[i];
  if (t < 4 * kCrcPad / 16)  // the zero pad before each wave's chunk image (crc_chunk reads it)
    *reinterpret_cast<u32x4*>(stage[t / (kCrcPad / 16)] + 16 * (t % (kCrcPad / 16))) = u32x4{0, 0, 0, 0};
  if (blockIdx.x == 0 && t == 0) {
    a.stats[0] = a.nblk;
    a.stats[1] = a.blk_off[a.nblk] - a.blk_off[0];
  }
  __syncthreads();
  uint8_t* S = stage[w] + kCrcPad;
  const uint64_t stride = uint64_t(gridDim.x) * 4;
  // (readfirstlane: the compiler does not know threadIdx.x >> 6 is wave-uniform, and a block
  // index it thinks divergent makes the whole block loop an exec-masked one)
  uint64_t b = uni64(uint64_t(blockIdx.x) * 4 + w);
  if (b >= a.nblk) return;
  uint32_t err = 0;
  bool len_ok = true, len_okn = true;
  auto meta_of = [&](uint64_t s0, uint64_t e0, uint64_t& st, uint32_t& len, bool& lok) {
    const bool ok = e0 >= s0 + a.tail && e0 - s0 <= 0x7FFFFFF0ull;
    if (!ok) err |= LSMBLK_ERR_MALFORMED;
    st = s0;
    len = ok ? uint32_t(e0 - s0) - a.tail : 0u;
    lok = ok;
  };
  auto meta = [&](uint64_t bi, uint64_t& st, uint32_t& len, bool& lok) {
    meta_of(uni64(a.blk_off[bi]), uni64(a.blk_off[bi + 1]), st, len, lok);
  };
  // Always five 16-B loads per lane (bytes past the chunk come back 0 from the descriptor's
  // bound) and five LDS stores: no predicated loads, so the compiler counts the waits
  // exactly instead of draining everything (block metadata included) at the landing.
  u32x4 q[5];
  uint32_t qlead = 0;
  auto issue = [&](uint64_t cs, uint32_t sz) {  // loads of block bytes [cs, cs + sz)
    const uint32_t lead = uni(uint32_t(reinterpret_cast<uintptr_t>(a.blocks + cs) & 15));
    // (uniform base and size, so the descriptor lives in SGPRs: no waterfall loop per load)
    const rsrc_t R = make_rsrc(reinterpret_cast<const uint8_t*>(uni64(reinterpret_cast<uintptr_t>(a.blocks + cs - lead))),
                               uni(lead + sz));
#pragma unroll
    for (uint32_t i = 0; i < 5; ++i) q[i] = __builtin_amdgcn_raw_buffer_load_b128(R, (l + 64 * i) * 16, 0, 0);
    qlead = lead;
  };
  // block metadata runs two blocks ahead of the folding, chunk loads one chunk ahead
  uint64_t st, stn = 0;
  uint32_t len, lenn = 0;
  meta(b, st, len, len_ok);
  if (b + stride < a.nblk) meta(b + stride, stn, lenn, len_okn);
  uint32_t nch = (len + kCrcChunk - 1) / kCrcChunk;
  issue(st, nch ? len - kCrcChunk * (nch - 1) : 0u);
  for (;;) {
    const uint64_t bn = b + stride, b2 = bn + stride;
    const bool has_next = bn < a.nblk;
    // block b2's offsets: loaded after the first landing (so the landing never waits for them)
    // into VGPRs, made uniform only at the end of this block -- a readfirstlane right away would
    // wait (vmcnt counts in order) for a full memory round trip
    uint64_t r0 = 0, r1 = 0;
    const uint32_t nchn = (lenn + kCrcChunk - 1) / kCrcChunk;
    const uint32_t h = len - kCrcChunk * (nch ? nch - 1 : 0u);  // first chunk's size
    uint32_t acc = 0;
    for (uint32_t c = 0; c == 0 || c < nch; ++c) {  // an empty block still lands its (zero) loads
      const uint32_t sz = c == 0 ? h : kCrcChunk, lead = qlead;
      // land the chunk at S + lead; the lead bytes before it (lane l0's window reaches them) and
      // the t < 4 bytes after it (up to the next 4-aligned byte: crc_chunk's aligned windows)
      // are zeroed in registers first
      const uint32_t P = lead + sz, tz = (0u - P) & 3u;  // zero bytes after the chunk
      if (l == 0) {
        uint32_t* v = reinterpret_cast<uint32_t*>(&q[0]);
#pragma unroll
        for (uint32_t d = 0; d < 4; ++d) {
          const int32_t z = int32_t(lead) - int32_t(4 * d);  // lead bytes in this dword
          v[d] &= z <= 0 ? ~0u : z >= 4 ? 0u : ~0u << (8 * z);
        }
      }
      if (tz && l == ((P >> 4) & 63)) {
#pragma unroll
        for (uint32_t i = 0; i < 5; ++i) {
          if (i != (P >> 10)) continue;
          uint32_t* v = reinterpret_cast<uint32_t*>(&q[i]);
#pragma unroll
          for (uint32_t d = 0; d < 4; ++d) {
            const int32_t z = int32_t(P & 15) - int32_t(4 * d);  // chunk bytes in this dword
            v[d] &= z <= 0 ? 0u : z >= 4 ? ~0u : ~(~0u << (8 * z));
          }
        }
      }
#pragma unroll
      for (uint32_t i = 0; i < 5; ++i) *reinterpret_cast<u32x4*>(S + 16 * (l + 64 * i)) = q[i];
      if (c == 0 && b2 < a.nblk) {
        r0 = a.blk_off[b2];
        r1 = a.blk_off[b2 + 1];
      }
      wave_sync();
      {  // one issue site with uniform operands (two sites get merged into a divergent phi)
        const bool more = c + 1 < nch;
        const uint64_t ncs = more ? st + h + uint64_t(kCrcChunk) * c : stn;
        const uint32_t nsz = more ? kCrcChunk : nchn ? lenn - kCrcChunk * (nchn - 1) : 0u;
        if (more || has_next) issue(uni64(ncs), uni(nsz));
      }
      if (nch) {
        const uint32_t part = crc_chunk(T, S + lead, sz, c == 0, tz);
        acc = c == 0 ? part : crc_apply(T.shift[6], acc) ^ part;
      }
      if (COUNT && nch <= 1) count_block(LdsImg{S, lead}, len, len_ok, a.agg + 3 * b, err);
      wave_sync();  // the next landing overwrites S
    }
    if (COUNT && nch > 1) {  // a block over one chunk: its headers from global memory
      const uint32_t lead = uni(uint32_t(reinterpret_cast<uintptr_t>(a.blocks + st) & 15));
      const rsrc_t R = make_rsrc(reinterpret_cast<const uint8_t*>(uni64(reinterpret_cast<uintptr_t>(a.blocks + st - lead))),
                                 uni(lead + len));
      count_block(GlbImg{R, lead}, len, len_ok, a.agg + 3 * b, err);
    }
    if (l == 0) a.crc[b] = nch ? ~acc : 0u;
    if (!has_next) break;
    uint64_t st2 = 0;
    uint32_t len2 = 0;
    bool len_ok2 = true;
    if (b2 < a.nblk) meta_of(uni64(r0), uni64(r1), st2, len2, len_ok2);
    b = bn;
    st = stn;
    len = lenn;
    len_ok = len_okn;
    nch = nchn;
    stn = st2;
    lenn = len2;
    len_okn = len_ok2;
  }
  raise_err(a.stats, err);
}

// ---------------------------------------------------------------- streaming CRC (the plain pass)
// crc_kernel folds each lane's contiguous 68-B window, so it stages every chunk in LDS and pays
// eight nibble lookups per dword.  This kernel reads the blocks straight into registers
// with coalesced 16-B loads and folds them where they land:
//   * a wave takes 4 consecutive blocks, a 16-lane row each; a block of L bytes is cut into
//     4 KiB chunks of the padded message 0^P || M || 0^T (T = -L mod 16, P a multiple of 16 that
//     fills the first chunk), lane r of the row holding the 16-B pieces r, r + 16, ... of a chunk;
//   * dword i of every piece of a lane is one chain whose consecutive dwords lie 256 B apart, so
//     every chain step is c <- Z(c ^ d, 256), the same map for all chains: four byte tables,
//     replicated 32 times in LDS so that lane l reads copy l mod 32 (bank l mod 32: conflict-free),
//     4 lookups per dword instead of 8;
//   * a chain ends 16 r + 4 i bytes past the chunk end: the lane joins its four chains by
//     Z(., 4)^-1 (Horner), the row's lanes by a DPP tree over Z(., 16 << b)^-1;
//   * chunk after chunk acc = Z(acc, 4096) ^ R_0(chunk), starting from the init carried through
//     the first chunk's data, Z(0xFFFFFFFF, 4096 - P); the T tail zeros come off with Z(., T)^-1.
// Bytes outside a block are never read: padding pieces load from past the descriptor's bound
// (zeros), and the last piece -- the block's last 16 - T bytes and T zeros -- is loaded as the
// block's last 16 bytes and shifted down by T (byte loads when the block is shorter).
constexpr uint32_t kCsWaves = 16;
constexpr uint32_t kCsOob = 0x80000000u;  // a piece offset past every descriptor bound (range < 2^31)

struct CrcStreamArgs {
  const uint8_t* blocks;
  const uint64_t* blk_off;
  uint64_t nblk;
  uint32_t tail;
  uint32_t* crc;
  const CrcStreamTabs* tabs;
  uint64_t* stats;
  // framed encode (LSMBLK_ENCODE_FRAMED): the encode's own blocks, nblk read from the device (the
  // encode's stats[0]; none after any encode error), block b = [blk_off[b], + sz[b]), and its CRC
  // written big-endian right after it (finish_block, src/table/builder.rs:118-122) instead of to crc
  uint8_t* frame_out;
  const uint32_t* sz;
  const uint64_t* dnblk;
};

__global__ __launch_bounds__(1024) void crc_stream_kernel(CrcStreamArgs a) {
  __shared__ uint32_t rep[4 * 256 * 32];  // rep[(k * 256 + v) * 32 + r] = a256[k][v]
  __shared__ CrcStreamTabs S;
  const uint32_t t = threadIdx.x, w = t >> 6, l = lane_id(), g = l >> 4, lq = l & 15;
  for (uint32_t i = t; i < sizeof(CrcStreamTabs) / 16; i += 64 * kCsWaves)
    reinterpret_cast<u32x4*>(&S)[i] = reinterpret_cast<const u32x4*>(a.tabs)[i];
  for (uint32_t e = t; e < 4 * 256 * 32; e += 64 * kCsWaves) rep[e] = (&a.tabs->a256[0][0])[e >> 5];
  const uint64_t nblk = a.dnblk ? (a.stats[3] ? 0ull : *a.dnblk) : a.nblk;
  if (blockIdx.x == 0 && t == 0 && !a.frame_out) {
    a.stats[0] = nblk;
    a.stats[1] = nblk ? a.blk_off[nblk] - a.blk_off[0] : 0;
  }
  __syncthreads();
  const uint8_t* const R8 = reinterpret_cast<const uint8_t*>(rep);
  const uint32_t lane4 = (l & 31) << 2;
  // c <- Z(x, 256): byte k of x addresses copy (l mod 32) of table k
  auto step = [&](uint32_t x) -> uint32_t {
    const uint32_t a0 = *reinterpret_cast<const uint32_t*>(R8 + (((x << 7) & 0x7F80u) | lane4));
    const uint32_t a1 = *reinterpret_cast<const uint32_t*>(R8 + 32768 + (((x >> 1) & 0x7F80u) | lane4));
    const uint32_t a2 = *reinterpret_cast<const uint32_t*>(R8 + 65536 + (((x >> 9) & 0x7F80u) | lane4));
    const uint32_t a3 = *reinterpret_cast<const uint32_t*>(R8 + 98304 + (((x >> 17) & 0x7F80u) | lane4));
    return xor3(a0, a1, a2) ^ a3;
  };
  uint32_t err = 0;
  const uint64_t ngrp = (nblk + 3) / 4, nw = uint64_t(gridDim.x) * kCsWaves;
  // lanes 0..4: blk_off[4 G + lane], the group's block offsets (loaded one group ahead)
  auto offs = [&](uint64_t G) -> uint64_t {
    return G < ngrp && l <= 4 && 4 * G + l <= nblk ? a.blk_off[4 * G + l] : 0ull;
  };
  uint64_t G = uni64(uint64_t(blockIdx.x) * kCsWaves + w);
  uint64_t onext = offs(G);
  for (; G < ngrp; G += nw) {
    const uint64_t b0 = G * 4, nb = nblk - b0 < 4 ? nblk - b0 : 4;  // blocks of this wave
    uint64_t Sx[5];
#pragma unroll
    for (uint32_t k = 0; k < 5; ++k) Sx[k] = lane64(onext, k);
    onext = offs(G + nw);
    const bool have = g < nb;
    const uint64_t s = g == 0 ? Sx[0] : g == 1 ? Sx[1] : g == 2 ? Sx[2] : Sx[3];
    const uint64_t e = g == 0 ? Sx[1] : g == 1 ? Sx[2] : g == 2 ? Sx[3] : Sx[4];
    const uint32_t fsz = a.sz && have ? a.sz[b0 + g] : 0u;  // (framed: the block's size from the plan)
    const bool valid = have && (a.sz ? fsz <= 0x7FFFFFF0u : e >= s + a.tail && e - s <= 0x7FFFFFF0ull);
    if (have && !valid) err |= LSMBLK_ERR_MALFORMED;
    const uint32_t L = !valid ? 0u : a.sz ? fsz : uint32_t(e - s) - a.tail;
    const uint32_t T = (0u - L) & 15u, nch = (L + T + 4095) >> 12, P = (nch << 12) - L - T;
    const uint64_t S0 = Sx[0], Se = Sx[nb];
    // one descriptor over the wave's blocks when they lie inside [S0, Se) (adjacent ranges do)
    const bool wave_ok = Se >= S0 && Se - S0 <= 0x7FFFFFF0ull &&
                         __ballot(valid && (s < S0 || s + L > Se)) == 0;
    uint32_t maxnch = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) maxnch = max(maxnch, uint32_t(__builtin_amdgcn_readlane(nch, 16 * k)));
    uint32_t acc = S.zinit[(4096 - P) >> 4];
    for (uint32_t c = 0; c < maxnch; ++c) {
      const bool live = c < nch;
      const bool tailp = live && c + 1 == nch && lq == 15 && T != 0;
      u32x4 q[16];
      // piece j of this lane: padded position 4096 c + 256 j + 16 lq, data offset that - P; the
      // last piece of a block with tail zeros loads the block's last 16 bytes (shifted below)
      // (offsets by masks, not selects: selects let the compiler sink each load into branches)
      auto issue = [&](const rsrc_t& R, uint32_t rel) {
        const uint32_t m15 = tailp && L >= 16 ? ~0u : 0u;
#pragma unroll
        for (uint32_t j = 0; j < 16; ++j) {
          const uint32_t po = (c << 12) + 256 * j + 16 * lq, x = po - P;
          const uint32_t in = live && po >= P && x + 16 <= L ? ~0u : 0u;
          uint32_t off = kCsOob ^ ((kCsOob ^ (rel + x)) & in);
          if (j == 15) off ^= (off ^ (rel + L - 16)) & m15;
          q[j] = __builtin_amdgcn_raw_buffer_load_b128(R, off, 0, 0);
        }
      };
      if (wave_ok) {
        const rsrc_t R = make_rsrc_exact(const_cast<uint8_t*>(a.blocks + S0), uint32_t(Se - S0));
        issue(R, uint32_t(s - S0));
      } else {  // (non-adjacent or huge ranges: one descriptor per block, its row's lanes only)
        for (uint32_t k = 0; k < 4; ++k) {
          const uint64_t sk = lane64(s, 16 * k);
          const uint32_t Lk = uint32_t(__builtin_amdgcn_readlane(L, 16 * k));
          const rsrc_t R = make_rsrc_exact(const_cast<uint8_t*>(a.blocks + sk), Lk);
          if (g == k) issue(R, 0);
        }
      }
      uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
#pragma unroll
      for (uint32_t j = 0; j < 16; ++j) {
        if (j == 15) {  // (here, not before the loop: the fold of pieces 0..14 waits only for them)
          if (tailp) {
            uint32_t v[4] = {q[15].x, q[15].y, q[15].z, q[15].w};
            if (L < 16) {  // the whole block is the last piece: its L bytes, then zeros
              const rsrc_t R = make_rsrc_exact(const_cast<uint8_t*>(a.blocks + s), L);
              v[0] = v[1] = v[2] = v[3] = 0;
              for (uint32_t i = 0; i < L; ++i) v[i >> 2] |= uint32_t(__builtin_amdgcn_raw_buffer_load_b8(R, i, 0, 0)) << (8 * (i & 3));
            } else {  // the block's last 16 bytes, down by T
              for (uint32_t r = 0; r < 3; ++r)
                if ((T >> 2) > r) v[0] = v[1], v[1] = v[2], v[2] = v[3], v[3] = 0;
              const uint32_t sb = T & 3;
              v[0] = __builtin_amdgcn_alignbyte(v[1], v[0], sb);
              v[1] = __builtin_amdgcn_alignbyte(v[2], v[1], sb);
              v[2] = __builtin_amdgcn_alignbyte(v[3], v[2], sb);
              v[3] = __builtin_amdgcn_alignbyte(0u, v[3], sb);
            }
            q[15] = u32x4{v[0], v[1], v[2], v[3]};
          }
        }
        c0 = step(c0 ^ q[j].x);
        c1 = step(c1 ^ q[j].y);
        c2 = step(c2 ^ q[j].z);
        c3 = step(c3 ^ q[j].w);
      }
      // chain i of row lane r ends 16 r + 4 i bytes past the chunk end
      uint32_t x = crc_apply(S.unz4, c3) ^ c2;
      x = crc_apply(S.unz4, x) ^ c1;
      x = crc_apply(S.unz4, x) ^ c0;
      x ^= crc_apply(S.unzl[0], LSM_DPP(x, 0x101, 0xF));  // row_shl:1
      x ^= crc_apply(S.unzl[1], LSM_DPP(x, 0x102, 0xF));  // row_shl:2
      x ^= crc_apply(S.unzl[2], LSM_DPP(x, 0x104, 0xF));  // row_shl:4
      x ^= crc_apply(S.unzl[3], LSM_DPP(x, 0x108, 0xF));  // row_shl:8
      if (live) acc = c == 0 ? acc ^ x : crc_apply(S.z4096, acc) ^ x;  // (row lane 0's x is the chunk's)
    }
    if (have && lq == 0) {
      const uint32_t r = crc_apply(S.unzt[T], acc);
      const uint32_t v = L ? ~r : 0u;
      if (a.crc) a.crc[b0 + g] = v;
      if (a.frame_out && valid) {  // big-endian, as put_u32 writes it
        uint8_t* f = a.frame_out + s + L;
        f[0] = uint8_t(v >> 24), f[1] = uint8_t(v >> 16), f[2] = uint8_t(v >> 8), f[3] = uint8_t(v);
      }
    }
  }
#pragma unroll
  for (uint32_t d = 32; d >= 1; d >>= 1) err |= __shfl_xor(err, d, 64);
  raise_err(a.stats, err);
}

}  // namespace lsmblk_impl

// ---------------------------------------------------------------- SST BlockMeta section
// SsTableBuilder::build -> BlockMeta::encode_block_meta (src/table.rs:29-63), one section per
// segment (SST):
//   u32 num | { u32 offset | u16 flen | first_key | u64 0 | u16 llen | last_key | u64 0 }*
//   | u64 max_ts (0) | u32 crc32(section[4 .. len - 4])              (big-endian integers)
// The keys come from the encoded blocks themselves: entry 0 holds the whole first key
// (get_first_key, src/block/iterator.rs:23-34) and the last entry is first_key[..p] || suffix.
// BlockMeta keys carry ts 0 (KeyVec::set_from_slice copies key bytes only, src/key.rs:166-169)
// and SsTableBuilder never raises max_ts (src/table/builder.rs:41,77).  offset = the block's
// position in the SST data section, where every block is followed by its u32 CRC (:118-122).
// Four small launches: record sizes per block, one-workgroup tile scan, record writes (one
// lane per block), section headers; then crc_kernel over the sections and the CRC stores.
// The section is ~1.3 % of the block bytes at config U (56 B per 4 KiB block).
constexpr uint32_t kMetaTile = 256;  // blocks per workgroup (one lane each)

struct MetaArgs {
  const uint8_t* blocks;
  const uint64_t* blk_off;
  uint64_t nblk;
  uint32_t tail;            // bytes after each block inside its blk_off range (4 = framed)
  uint32_t nseg;
  const uint32_t* seg_blk;  // nseg + 1: segment s = blocks [seg_blk[s], seg_blk[s+1])
  uint8_t* meta;
  uint64_t meta_cap;
  uint64_t* meta_off;       // nseg + 1 (output)
  uint32_t* rec;            // nblk: record bytes
  uint64_t* tile_sum;       // per kMetaTile-block tile
  uint64_t* tile_pre;
  uint64_t* pos;            // nblk + 1: exclusive prefix of rec
  const uint32_t* crc;      // nseg: section CRCs (crc_kernel output)
  const uint64_t* crc_stats;
  uint64_t* stats;
};

struct MetaBlk {
  uint64_t base;
  uint32_t s0, loff, p, s;
  bool ok;
};

__device__ __forceinline__ void or_err(uint64_t* stats, uint32_t err) {
  if (err) atomicOr(reinterpret_cast<unsigned long long*>(stats + 3), (unsigned long long)err);
}

// Parse block b's first key length and last entry; ok = false where the reference would panic
// (no entries, trailer/offsets past the block, first or last entry past the data).
__device__ MetaBlk meta_parse(const MetaArgs& a, uint64_t b) {
  MetaBlk m{};
  const uint64_t base = a.blk_off[b], end = a.blk_off[b + 1];
  m.base = base;
  if (end < base || end - base < uint64_t(a.tail) + 2) return m;
  const uint64_t len = end - base - a.tail;
  const uint8_t* q = a.blocks + base;
  auto be16 = [&](uint64_t i) { return (uint32_t(q[i]) << 8) | q[i + 1]; };
  const uint32_t n = be16(len - 2);
  if (n == 0 || 2 + 2ull * n > len) return m;
  const uint64_t dend = len - 2 - 2ull * n;
  if (dend < 4) return m;
  m.s0 = be16(2);
  if (4ull + m.s0 + 8 > dend) return m;
  m.loff = be16(dend + 2ull * (n - 1));
  if (m.loff + 4ull > dend) return m;
  m.p = be16(m.loff);
  m.s = be16(m.loff + 2);
  if (m.loff + 4ull + m.s > dend || m.p > m.s0 || m.p + m.s == 0) return m;
  m.ok = true;
  return m;
}

__global__ __launch_bounds__(256) void meta_size_kernel(MetaArgs a) {
  const uint64_t b = uint64_t(blockIdx.x) * kMetaTile + threadIdx.x;
  uint32_t r = 0;
  if (b < a.nblk) {
    const MetaBlk m = meta_parse(a, b);
    if (!m.ok) or_err(a.stats, LSMBLK_ERR_MALFORMED);
    r = 24u + (m.ok ? m.s0 + m.p + m.s : 0u);
    a.rec[b] = r;
  }
  __shared__ uint32_t ws[4];
  const uint32_t t = wave_sum32(r);
  if (lane_id() == 0) ws[wave_id()] = t;
  __syncthreads();
  if (threadIdx.x == 0) a.tile_sum[blockIdx.x] = uint64_t(ws[0]) + ws[1] + ws[2] + ws[3];
}

// One workgroup: exclusive scan of the tile sums, the total, the capacity check and the
// segment-table check (seg_blk[0] = 0, non-decreasing, seg_blk[nseg] = nblk).
__global__ __launch_bounds__(1024) void meta_scan_kernel(MetaArgs a) {
  const uint32_t t = threadIdx.x;
  const uint64_t ntiles = (a.nblk + kMetaTile - 1) / kMetaTile;
  const uint64_t per = (ntiles + 1023) / 1024;
  const uint64_t lo = min(ntiles, t * per), hi = min(ntiles, lo + per);
  uint64_t s = 0;
  for (uint64_t i = lo; i < hi; ++i) s += a.tile_sum[i];
  __shared__ uint64_t wsum[16];
  const uint64_t inc = wave_incl_scan<uint64_t>(s);
  if (lane_id() == 63) wsum[t >> 6] = inc;
  __syncthreads();
  uint64_t base = 0;
  for (uint32_t w = 0; w < (t >> 6); ++w) base += wsum[w];
  uint64_t run = base + inc - s;
  for (uint64_t i = lo; i < hi; ++i) {
    a.tile_pre[i] = run;
    run += a.tile_sum[i];
  }
  uint32_t err = 0;
  if (t == 1023) {
    const uint64_t total = base + inc, need = total + 16ull * a.nseg;
    a.pos[a.nblk] = total;
    a.stats[0] = a.nseg;
    a.stats[1] = need;
    if (need > a.meta_cap) err |= LSMBLK_ERR_CAPACITY;
  }
  for (uint64_t g = t; g <= a.nseg; g += 1024) {
    const uint32_t v = a.seg_blk[g];
    if ((g == 0 && v != 0) || (g == a.nseg && v != a.nblk) || (g < a.nseg && v > a.seg_blk[g + 1]))
      err |= LSMBLK_ERR_SEGMENTS;
  }
  or_err(a.stats, err);
}

__device__ __forceinline__ void put_be(uint8_t* d, uint64_t v, uint32_t nbytes) {
  for (uint32_t i = 0; i < nbytes; ++i) d[i] = uint8_t(v >> (8 * (nbytes - 1 - i)));
}

// len bytes from global src to dst (LDS or global), any alignment: unaligned 16-B loads and
// stores (gfx9 unaligned access mode), the last piece overlapping the one before; byte copies
// under 16 bytes.  The source range must lie inside the block.
__device__ __forceinline__ void copy_bytes16(uint8_t* dst, const uint8_t* src, uint32_t len) {
  if (len < 16) {
    for (uint32_t i = 0; i < len; ++i) dst[i] = src[i];
    return;
  }
  for (uint32_t i = 0;; i += 16) {
    const uint32_t o = min(i, len - 16);
    *reinterpret_cast<u32x4*>(dst + o) = *reinterpret_cast<const u32x4*>(src + o);
    if (o == len - 16) break;
  }
}

// One BlockMeta record at d: u32 offset | u16 flen | first key | u64 0 | u16 llen | last key |
// u64 0 (table.rs:42-51).
__device__ __forceinline__ void meta_record(uint8_t* d, const uint8_t* q, const MetaBlk& m, uint32_t off) {
  put_be(d, off, 4);  // offset as u32 (table.rs:44)
  put_be(d + 4, m.s0, 2);
  copy_bytes16(d + 6, q + 4, m.s0);
  d += 6 + m.s0;
  put_be(d, 0, 8);
  put_be(d + 8, (m.p + m.s) & 0xFFFFu, 2);
  copy_bytes16(d + 10, q + 4, m.p);
  copy_bytes16(d + 10 + m.p, q + m.loff + 4, m.s);
  put_be(d + 10 + m.p + m.s, 0, 8);
}

// One lane per block: its position (tile prefix + in-workgroup scan), its segment (binary
// search of seg_blk) and the record.  A tile's records (and the section headers/footers
// between them, rewritten by the later kernels) span one contiguous range: it is composed in
// LDS and flushed with aligned 16-B stores, byte-masked only at the two ends.  A tile whose
// range exceeds the image (long keys) writes its records straight to HBM.
constexpr uint32_t kMetaImg = 24576;
__global__ __launch_bounds__(256) void meta_write_kernel(MetaArgs a) {
  if (a.stats[3]) return;
  __shared__ __attribute__((aligned(16))) uint8_t img[kMetaImg + 16];
  __shared__ uint32_t ws[4];
  __shared__ uint64_t ext[2];
  const uint64_t b = uint64_t(blockIdx.x) * kMetaTile + threadIdx.x;
  const uint64_t bend = min(a.nblk, uint64_t(blockIdx.x + 1) * kMetaTile);
  const bool live = b < a.nblk;
  const uint32_t r = live ? a.rec[b] : 0u;
  const uint32_t inc = wave_incl_scan32(r);
  const uint32_t w = wave_id();
  if (lane_id() == 63) ws[w] = inc;
  __syncthreads();
  uint64_t pos = a.tile_pre[blockIdx.x] + inc - r;
  for (uint32_t j = 0; j < w; ++j) pos += ws[j];
  uint32_t seg = 0;
  MetaBlk m{};
  uint64_t dst = 0;
  uint32_t off = 0;
  if (live) {
    a.pos[b] = pos;
    uint32_t lo = 0, hi = a.nseg;  // largest seg with seg_blk[seg] <= b
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (a.seg_blk[mid] <= b) lo = mid; else hi = mid;
    }
    seg = lo;
    const uint64_t first = a.seg_blk[seg];
    m = meta_parse(a, b);
    off = uint32_t(a.blk_off[b] - a.blk_off[first] + (4ull - a.tail) * (b - first));
    dst = pos + 16ull * seg + 4;
    if (b == uint64_t(blockIdx.x) * kMetaTile) ext[0] = dst;
    if (b == bend - 1) ext[1] = dst + r;
  }
  __syncthreads();
  const uint64_t t_lo = ext[0], t_hi = ext[1];
  uint8_t* gb = a.meta + t_lo;
  const uint32_t lead = uint32_t(reinterpret_cast<uintptr_t>(gb) & 15);
  const uint64_t span = lead + (t_hi - t_lo);
  const uint8_t* q = a.blocks + m.base;
  if (span > kMetaImg) {
    if (live) meta_record(a.meta + dst, q, m, off);
    return;
  }
  if (live) meta_record(img + lead + (dst - t_lo), q, m, off);
  __syncthreads();
  uint8_t* ga = gb - lead;
  const uint32_t nc = uint32_t((span + 15) >> 4);
  for (uint32_t c = threadIdx.x; c < nc; c += 256) {
    const u32x4 v4 = *reinterpret_cast<const u32x4*>(img + 16 * c);
    const uint32_t v[4] = {v4.x, v4.y, v4.z, v4.w};
    const uint32_t lo = c == 0 ? lead : 0u;
    const uint64_t rest = span - 16ull * c;  // (min<uint64_t> compiles to f64 compares)
    const uint32_t hi = rest < 16 ? uint32_t(rest) : 16u;
    store_chunk(ga + 16 * c, v, lo, hi);
  }
}

// One lane per segment: section offsets, u32 num and u64 max_ts.  After an error every offset
// is 0, so the CRC pass over the sections reads nothing.
__global__ __launch_bounds__(256) void meta_seg_kernel(MetaArgs a) {
  const uint64_t g = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  if (g >= a.nseg) return;
  if (a.stats[3]) {
    a.meta_off[g] = 0;
    if (g == a.nseg - 1) a.meta_off[a.nseg] = 0;
    return;
  }
  const uint32_t b0 = a.seg_blk[g], b1 = a.seg_blk[g + 1];
  const uint64_t st = a.pos[b0] + 16ull * g, en = a.pos[b1] + 16ull * (g + 1);
  a.meta_off[g] = st;
  if (g == a.nseg - 1) a.meta_off[a.nseg] = en;
  put_be(a.meta + st, b1 - b0, 4);
  put_be(a.meta + en - 12, 0, 8);
}

__global__ __launch_bounds__(256) void meta_crc_put_kernel(MetaArgs a) {
  const uint64_t g = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  if (a.stats[3]) return;
  if (g == 0) or_err(a.stats, uint32_t(a.crc_stats[3]));
  if (g >= a.nseg) return;
  put_be(a.meta + a.meta_off[g + 1] - 4, a.crc[g], 4);
}

// Segment -> first block after an encode: seg_blk[s] = lower_bound(blk_first[0 .. nblk),
// seg_start[s]) -- every non-empty segment starts a block (table/builder.rs:48-65).
__global__ __launch_bounds__(256) void seg_blocks_kernel(const uint32_t* blk_first, const uint64_t* enc_stats,
                                                        const uint32_t* seg_start, uint32_t nseg,
                                                        uint32_t* seg_blk) {
  const uint64_t g = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  if (g > nseg) return;
  if (enc_stats[3]) {
    seg_blk[g] = 0;
    return;
  }
  const uint32_t key = seg_start[g];
  uint32_t lo = 0, hi = uint32_t(enc_stats[0]);
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (blk_first[mid] < key) lo = mid + 1; else hi = mid;
  }
  seg_blk[g] = lo;
}

// ---------------------------------------------------------------- compaction filter
// The per-entry rules of compact_generate_sst (src/compact.rs:234-299) over a merged KV stream
// (user keys ascending, versions newest first, as MergeIterator yields them).  Walking the
// loop's state (last_key, first_key_below_watermark) through one key's versions gives a rule
// that needs only the entry and its predecessor, so every entry is decided independently:
//   start  = first version of its key (key differs from the previous entry's)
//   keep   = ts > watermark
//         || (first version at or below the watermark: start || prev.ts > watermark)
//            && !(bottom_level && start && value empty)       (:244-254, a tombstone with no
//                                                               newer version is dropped)
//            && !any prefix filter matches the key             (:264-275)
// Every later version at or below the watermark is dropped (:256-260).  The closed form is
// checked against a line-by-line restatement of the loop (tests/test_oracle.py).
// Three launches: keep flags + per-tile sums, a one-workgroup tile scan (totals, capacity),
// and the compaction into the output stream (16-B unaligned copies of keys and values).
constexpr uint32_t kFiltTile = 1024;  // entries per workgroup (4 rounds of 256 lanes)

struct FiltArgs {
  const uint8_t* keys;
  const uint32_t* key_off;
  const uint8_t* vals;
  const uint32_t* val_off;
  const uint64_t* ts;
  uint64_t n;
  uint64_t wm;
  uint32_t bottom;
  uint32_t npfx;
  const uint8_t* pfx;
  const uint32_t* pfx_off;
  uint8_t* okeys;
  uint32_t* okey_off;
  uint8_t* ovals;
  uint32_t* oval_off;
  uint64_t* ots;
  uint64_t entry_cap, key_cap, val_cap;
  uint32_t* keep;      // n
  uint64_t* tile_sum;  // 3 per tile: entries, key bytes, value bytes
  uint64_t* tile_pre;
  uint64_t* stats;
};

__device__ __forceinline__ bool filt_keep(const FiltArgs& a, uint64_t i) {
  const uint64_t t = a.ts[i];
  if (t > a.wm) return true;
  const uint32_t k0 = a.key_off[i], k1 = a.key_off[i + 1];
  bool start = true;
  if (i > 0) {
    const uint32_t p0 = a.key_off[i - 1];
    const uint32_t kl = k1 - k0;
    if (k0 - p0 == kl) {
      start = false;
      uint32_t j = 0;
      for (; j + 16 <= kl && !start; j += 16) {  // unaligned 16-B compares, then bytes
        const u32x4 x = *reinterpret_cast<const u32x4*>(a.keys + p0 + j);
        const u32x4 y = *reinterpret_cast<const u32x4*>(a.keys + k0 + j);
        start = x.x != y.x || x.y != y.y || x.z != y.z || x.w != y.w;
      }
      for (; j < kl && !start; ++j) start = a.keys[p0 + j] != a.keys[k0 + j];
    }
    if (!start && a.ts[i - 1] <= a.wm) return false;  // a later version below the watermark
  }
  if (a.bottom && start && a.val_off[i + 1] == a.val_off[i]) return false;
  for (uint32_t f = 0; f < a.npfx; ++f) {
    const uint32_t f0 = a.pfx_off[f], fl = a.pfx_off[f + 1] - f0;
    if (fl > k1 - k0) continue;
    bool m = true;
    for (uint32_t j = 0; j < fl && m; ++j) m = a.pfx[f0 + j] == a.keys[k0 + j];
    if (m) return false;
  }
  return true;
}

__global__ __launch_bounds__(256) void filt_flag_kernel(FiltArgs a) {
  uint32_t c = 0;
  uint64_t kb = 0, vb = 0;
#pragma unroll
  for (uint32_t sub = 0; sub < kFiltTile / 256; ++sub) {
    const uint64_t i = uint64_t(blockIdx.x) * kFiltTile + sub * 256 + threadIdx.x;
    if (i < a.n) {
      const bool k = filt_keep(a, i);
      a.keep[i] = k;
      if (k) {
        c += 1;
        kb += a.key_off[i + 1] - a.key_off[i];
        vb += a.val_off[i + 1] - a.val_off[i];
      }
    }
  }
  __shared__ uint64_t ws[4][3];
  const uint32_t w = wave_id();
  const uint32_t sc = wave_sum32(c);
  const uint64_t sk = wave_sum<uint64_t>(kb), sv = wave_sum<uint64_t>(vb);
  if (lane_id() == 0) ws[w][0] = sc, ws[w][1] = sk, ws[w][2] = sv;
  __syncthreads();
  if (threadIdx.x < 3) {
    const uint32_t q = threadIdx.x;
    a.tile_sum[3 * uint64_t(blockIdx.x) + q] = ws[0][q] + ws[1][q] + ws[2][q] + ws[3][q];
  }
}

// Rounds of 1024 consecutive tiles (coalesced loads), each a workgroup scan plus the carry.
__global__ __launch_bounds__(1024) void filt_scan_kernel(FiltArgs a) {
  const uint32_t t = threadIdx.x, w = t >> 6;
  const uint64_t ntiles = (a.n + kFiltTile - 1) / kFiltTile;
  __shared__ uint64_t wsum[16][3];
  uint64_t carry[3] = {0, 0, 0};
  for (uint64_t r = 0; r < ntiles; r += 1024) {
    const uint64_t i = r + t;
    uint64_t v[3], inc[3];
#pragma unroll
    for (uint32_t q = 0; q < 3; ++q) {
      v[q] = i < ntiles ? a.tile_sum[3 * i + q] : 0ull;
      inc[q] = wave_incl_scan<uint64_t>(v[q]);
      if (lane_id() == 63) wsum[w][q] = inc[q];
    }
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < 3; ++q) {
      uint64_t base = carry[q], tot = carry[q];
      for (uint32_t x = 0; x < 16; ++x) {
        if (x < w) base += wsum[x][q];
        tot += wsum[x][q];
      }
      if (i < ntiles) a.tile_pre[3 * i + q] = base + inc[q] - v[q];
      carry[q] = tot;
    }
    __syncthreads();
  }
  if (t == 1023) {
    const uint64_t tot[3] = {carry[0], carry[1], carry[2]};
#pragma unroll
    for (uint32_t q = 0; q < 3; ++q) a.stats[q] = tot[q];
    uint32_t err = 0;
    if (tot[1] > 0xFFFFFFFFull || tot[2] > 0xFFFFFFFFull) err |= LSMBLK_ERR_OVERFLOW;
    if (tot[0] > a.entry_cap || tot[1] > a.key_cap || tot[2] > a.val_cap) err |= LSMBLK_ERR_CAPACITY;
    if (!err) {
      a.okey_off[tot[0]] = uint32_t(tot[1]);
      a.oval_off[tot[0]] = uint32_t(tot[2]);
    }
    or_err(a.stats, err);
  }
}

// Copy len bytes src -> dst by the whole wave (wave-uniform arguments): lane l moves 16-B
// pieces l, l + 64, ... (unaligned loads/stores, 1 KiB of contiguous bytes per instruction);
// the lane holding a final piece under 16 bytes copies it bytewise.
__device__ __forceinline__ void wave_copy(uint8_t* dst, const uint8_t* src, uint64_t len) {
  for (uint64_t o = 16ull * lane_id(); o < len; o += 1024) {
    if (o + 16 <= len) {
      *reinterpret_cast<u32x4*>(dst + o) = *reinterpret_cast<const u32x4*>(src + o);
    } else {
      for (uint64_t x = o; x < len; ++x) dst[x] = src[x];
    }
  }
}

// Output offsets and ts per kept entry; key and value bytes by runs: consecutive kept entries
// are one contiguous range in the input arenas and in the output, so each wave copies its
// runs whole (one run per wave when nothing in it is dropped).
__global__ __launch_bounds__(256) void filt_write_kernel(FiltArgs a) {
  if (a.stats[3]) return;
  __shared__ uint64_t ws[4][3];
  const uint32_t w = wave_id();
  uint64_t carry[3] = {a.tile_pre[3 * uint64_t(blockIdx.x)], a.tile_pre[3 * uint64_t(blockIdx.x) + 1],
                       a.tile_pre[3 * uint64_t(blockIdx.x) + 2]};
  for (uint32_t sub = 0; sub < kFiltTile / 256; ++sub) {  // 256 entries per round, running carry
    const uint64_t i = uint64_t(blockIdx.x) * kFiltTile + sub * 256 + threadIdx.x;
    const bool k = i < a.n && a.keep[i];
    const uint32_t kl = k ? a.key_off[i + 1] - a.key_off[i] : 0u;
    const uint32_t vl = k ? a.val_off[i + 1] - a.val_off[i] : 0u;
    const uint32_t ic = wave_incl_scan32(k ? 1u : 0u);
    const uint64_t ik = wave_incl_scan<uint64_t>(kl), iv = wave_incl_scan<uint64_t>(vl);
    if (lane_id() == 63) ws[w][0] = ic, ws[w][1] = ik, ws[w][2] = iv;
    __syncthreads();
    uint64_t j = carry[0] + ic - 1, ko = carry[1] + ik - kl, vo = carry[2] + iv - vl;
    for (uint32_t q = 0; q < w; ++q) j += ws[q][0], ko += ws[q][1], vo += ws[q][2];
#pragma unroll
    for (uint32_t q = 0; q < 3; ++q) carry[q] += ws[0][q] + ws[1][q] + ws[2][q] + ws[3][q];
    __syncthreads();  // ws is rewritten by the next round
    uint32_t ki = 0, vi = 0;
    if (k) {
      ki = a.key_off[i];
      vi = a.val_off[i];
      a.okey_off[j] = uint32_t(ko);
      a.oval_off[j] = uint32_t(vo);
      a.ots[j] = a.ts[i];
    }
    for (uint64_t mask = __ballot(k); mask;) {
      const uint32_t s = uint32_t(__builtin_ctzll(mask));
      const uint64_t rest = ~(mask >> s);
      const uint32_t e = rest ? s + uint32_t(__builtin_ctzll(rest)) : 64u;  // run = lanes [s, e)
      const uint32_t ks = __builtin_amdgcn_readlane(ki, s), ke = __builtin_amdgcn_readlane(ki + kl, e - 1);
      const uint32_t vs = __builtin_amdgcn_readlane(vi, s), ve = __builtin_amdgcn_readlane(vi + vl, e - 1);
      wave_copy(a.okeys + lane64(ko, s), a.keys + ks, ke - ks);
      wave_copy(a.ovals + lane64(vo, s), a.vals + vs, ve - vs);
      mask = e >= 64 ? 0ull : mask & (~0ull << e);
    }
  }
}

// ================================================================ host side
namespace {

// per block 3 aggregate + 3 base granules; per tile 3 aggregate + 3 inclusive granules
uint64_t lag_words(uint64_t nb) { return 6 * nb + 6 * ((nb + kTile - 1) / kTile + 1); }

int reserve_locked(lsmblk_ctx* c, uint64_t blocks, uint64_t entries, uint64_t segs, hipStream_t st) {
  int rc;
  uint64_t cap;
  if (blocks > c->dec_cap) {
    if ((rc = grow(st, &c->dec_agg, &c->dec_cap, blocks, 3))) return rc;
  }
  const uint64_t tiles = (blocks + kTile - 1) / kTile;
  if (tiles > c->tile_cap) {
    cap = c->tile_cap;
    if ((rc = grow(st, &c->tile_sum, &cap, tiles, 3))) return rc;
    cap = c->tile_cap;
    if ((rc = grow(st, &c->tile_pre, &cap, tiles, 3))) return rc;
    c->tile_cap = cap;
  }
  if (blocks > c->lag_blk_cap) {
    // one arena: per block 3 aggregate + 3 base granules, then per tile 3 aggregate + 3 inclusive
    const uint64_t nb = blocks + blocks / 4 + 1024;
    cap = 0;  // (grow frees the old arena)
    if ((rc = grow(st, &c->lag_gran, &cap, lag_words(nb), 1, kStatusFlags))) {
      c->lag_blk_cap = 0;
      return rc;
    }
    c->lag_blk_cap = nb;
    c->epoch = 0;  // the fresh arena is zeroed; the next call starts a new epoch sequence
  }
  if (segs > c->seg_cap) {
    cap = c->seg_cap;
    if ((rc = grow(st, &c->seg_agg, &cap, segs, 2, kStatusFlags))) return rc;
    cap = c->seg_cap;
    if ((rc = grow(st, &c->seg_inc, &cap, segs, 2, kStatusFlags))) return rc;
    c->seg_cap = cap;
    c->epoch = 0;
  }
  if (entries + 1 > c->rec_cap) {
    cap = c->rec_cap;
    if ((rc = grow(st, &c->rec_first, &cap, entries + 1, 1))) return rc;
    cap = c->rec_cap;
    if ((rc = grow(st, &c->blk_first, &cap, entries + 1, 1))) return rc;
    cap = c->rec_cap;
    if ((rc = grow(st, &c->ent, &cap, entries + 1, 1))) return rc;
    cap = c->rec_cap;
    if ((rc = grow(st, &c->big_list, &cap, entries + 1, 1))) return rc;
    cap = c->rec_cap;
    if ((rc = grow(st, &c->blk_sz, &cap, entries + 1, 1))) return rc;
    c->rec_cap = cap;
  }
  return LSMBLK_OK;
}

// Next look-back epoch; on wrap the status arrays are cleared on the stream.
int next_epoch(lsmblk_ctx* c, hipStream_t st) {
  if (c->epoch == 0 || c->epoch >= 16383) {
    if (c->seg_cap) {
      if (hipMemsetAsync(c->seg_agg, 0, c->seg_cap * 2 * 8, st) != hipSuccess) return LSMBLK_E_HIP;
      if (hipMemsetAsync(c->seg_inc, 0, c->seg_cap * 2 * 8, st) != hipSuccess) return LSMBLK_E_HIP;
    }
    if (c->lag_blk_cap) {
      if (hipMemsetAsync(c->lag_gran, 0, lag_words(c->lag_blk_cap) * 8, st) != hipSuccess) return LSMBLK_E_HIP;
    }
    if (c->frec_cap && hipMemsetAsync(c->frec, 0, c->frec_cap * 4 * 8, st) != hipSuccess) return LSMBLK_E_HIP;
    if (c->fdone_cap && hipMemsetAsync(c->fdone, 0, c->fdone_cap * 8, st) != hipSuccess) return LSMBLK_E_HIP;
    c->epoch = 0;
  }
  ++c->epoch;
  return LSMBLK_OK;
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace lsmblk_impl

extern "C" {

int lsmblk_ctx_create(int device, lsmblk_ctx** out) {
  if (!out) return LSMBLK_E_INVAL;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return LSMBLK_E_HIP;
  auto* c = new (std::nothrow) lsmblk_ctx();
  if (!c) return LSMBLK_E_NOMEM;
  c->device = device;
  if (const char* e = getenv("LSMBLK_POLL_MODE")) c->poll = uint32_t(atoi(e));
  if (const char* e = getenv("LSMBLK_PLAN_PIPE")) c->plan_pipe = atoi(e) != 0;  // (A/B: LSMBLK_DEBUG_PLAN_PIPE)
  DeviceGuard dg(device);
  if (!dg.ok || hipMalloc(&c->counters, 2048) != hipSuccess) {
    delete c;
    return LSMBLK_E_HIP;
  }
  *out = c;
  return LSMBLK_OK;
}

void lsmblk_ctx_destroy(lsmblk_ctx* c) {
  if (!c) return;
  DeviceGuard dg(c->device, c);
  (void)hipDeviceSynchronize();
  if (c->aux) (void)hipStreamDestroy(c->aux);
  if (c->fork_ev) (void)hipEventDestroy(c->fork_ev);
  if (c->join_ev) (void)hipEventDestroy(c->join_ev);
  (void)hipFree(c->counters);
  release(c->dec_agg);
  release(c->tile_sum);
  release(c->tile_pre);
  release(c->seg_agg, kStatusFlags);
  release(c->seg_inc, kStatusFlags);
  release(c->rec_first);
  release(c->ent);
  release(c->big_list);
  release(c->blk_sz);
  release(c->frec, kStatusFlags);
  release(c->fdone, kStatusFlags);
  release(c->fwnb);
  release(c->fbig);
  release(c->blk_first);
  (void)hipFree(c->crc_tabs);
  release(c->meta_rec);
  release(c->meta_pos);
  release(c->meta_tile);
  release(c->meta_crc);
  (void)hipFree(c->meta_cstats);
  release(c->filt_keep);
  release(c->filt_tile);
  release(c->cws);
  release(c->vcrc);
  release(c->sws);
  release(c->rws);
  release(c->lag_gran, kStatusFlags);
  (void)hipStreamSynchronize(nullptr);  // (the pool frees above were queued on the null stream)
  (void)hipFree(c->dbg);
  for (auto& e : c->klog) {
    if (e.e0) (void)hipEventDestroy(e.e0);
    if (e.e1) (void)hipEventDestroy(e.e1);
  }
  delete c;
}

int lsmblk_debug_set(lsmblk_ctx* c, int key, uint32_t value) {
  if (!c) return LSMBLK_E_INVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (key == LSMBLK_DEBUG_POLL_MODE && value <= 2) {
    c->poll = value;
  } else if (key == LSMBLK_DEBUG_DECODE_SKIP && kDiag) {  // ablation masks: diagnostics builds only
    c->skip = value;
  } else if (key == LSMBLK_DEBUG_TWO_PASS_DECODE) {
    c->dec_two_pass = value != 0;
  } else if (key == LSMBLK_DEBUG_COUNTERS && kDiag) {  // realtime traces: diagnostics builds only
    if (value && !c->dbg) {
      DeviceGuard dg(c->device, c);
      if (!dg.ok || hipMalloc(reinterpret_cast<void**>(&c->dbg), kDbgWords * 8) != hipSuccess) {
        c->dbg = nullptr;
        return LSMBLK_E_NOMEM;
      }
    }
    c->dbg_on = value != 0;
  } else if (key == LSMBLK_DEBUG_ROT_POISON && kDiag) {  // fault injection: diagnostics builds only
    c->rot_poison = value;
  } else if (key == LSMBLK_DEBUG_EMIT_POISON && kDiag) {  // fault injection: diagnostics builds only
    c->emit_poison = value;
  } else if (key == LSMBLK_DEBUG_DECODE_LAG_BYTES) {
    c->dec_lag_bytes = value;
  } else if (key == LSMBLK_DEBUG_DECODE_LAG && value == 0) {  // the default
    c->dec_lag = kDecLagDefault;
    c->dec_lag_bytes = kDecLagBytesDefault;
  } else if (key == LSMBLK_DEBUG_DECODE_LAG && value >= 2 * kTile && value <= (1u << 24)) {
    c->dec_lag = value;
    c->dec_lag_bytes = 0;  // exactly this lag (experiments)
  } else if (key == LSMBLK_DEBUG_ENCODE_FUSED) {
    c->fuse_on = value != 0;
  } else if (key == LSMBLK_DEBUG_PLAN_PIPE) {
    c->plan_pipe = value != 0;
  } else if (key == LSMBLK_DEBUG_KERNEL_TIMING) {
    if (value && !c->timing) c->klog_n = 0;  // the log restarts with the timing
    c->timing = value != 0;
  } else {
    return LSMBLK_E_INVAL;
  }
  return LSMBLK_OK;
}

int lsmblk_debug_counters(lsmblk_ctx* c, uint64_t* out, uint32_t n) {
  if (!c || !out || n > kDbgWords) return LSMBLK_E_INVAL;
  std::lock_guard<std::mutex> g(c->mu);
  for (uint32_t i = 0; i < n; ++i) out[i] = 0;
  if (!c->dbg) return LSMBLK_OK;
  DeviceGuard dg(c->device, c);
  if (!dg.ok || hipDeviceSynchronize() != hipSuccess) return LSMBLK_E_HIP;
  return hipMemcpy(out, c->dbg, n * 8, hipMemcpyDeviceToHost) == hipSuccess ? LSMBLK_OK : LSMBLK_E_HIP;
}

int lsmblk_ctx_kernel_times(lsmblk_ctx* c, float* ms) {
  if (!c || !ms) return LSMBLK_E_INVAL;
  std::lock_guard<std::mutex> g(c->mu);
  for (int i = 0; i < LSMBLK_KERNELS; ++i) ms[i] = -1.f;  // a kernel the last call did not launch
  if (c->klog.empty()) return LSMBLK_OK;
  DeviceGuard dg(c->device);
  if (!dg.ok) return LSMBLK_E_HIP;
  // the last decode's and the last encode's launches (while still in the ring), summed by slot
  auto add = [&](uint64_t i0, uint64_t i1) -> int {
    if (c->klog_total - i0 > kKLogCap) return LSMBLK_OK;  // overwritten since
    for (uint64_t i = i0; i < i1; ++i) {
      const lsmblk_ctx::KLog& e = c->klog[i % kKLogCap];
      if (e.slot < 0 || e.slot >= LSMBLK_KERNELS) continue;
      float t = 0.f;
      if (hipEventSynchronize(e.e1) != hipSuccess || hipEventElapsedTime(&t, e.e0, e.e1) != hipSuccess)
        return LSMBLK_E_HIP;
      ms[e.slot] = (ms[e.slot] < 0.f ? 0.f : ms[e.slot]) + t;
    }
    return LSMBLK_OK;
  };
  const int rc = add(c->dec_log0, c->dec_log1);
  return rc ? rc : add(c->enc_log0, c->enc_log1);
}

int lsmblk_ctx_kernel_log(lsmblk_ctx* c, lsmblk_kernel_stat* out, uint32_t cap, uint32_t* n) {
  if (!c || !n || (cap && !out)) return LSMBLK_E_INVAL;
  std::lock_guard<std::mutex> g(c->mu);
  *n = 0;
  const uint64_t cnt = c->klog_n;
  c->klog_n = 0;
  if (cnt == 0) return LSMBLK_OK;
  if (cnt > kKLogCap) return LSMBLK_E_CAPACITY;  // the ring was overwritten: read it more often
  DeviceGuard dg(c->device);
  if (!dg.ok) return LSMBLK_E_HIP;
  for (uint64_t i = c->klog_total - cnt; i < c->klog_total; ++i) {
    const lsmblk_ctx::KLog& e = c->klog[i % kKLogCap];
    float t = 0.f;
    if (hipEventSynchronize(e.e1) != hipSuccess || hipEventElapsedTime(&t, e.e0, e.e1) != hipSuccess)
      return LSMBLK_E_HIP;
    uint32_t k = 0;
    while (k < *n && strncmp(out[k].name, e.name, sizeof(out[k].name) - 1) != 0) ++k;
    if (k == *n) {
      if (k == cap) return LSMBLK_E_CAPACITY;
      memset(&out[k], 0, sizeof(out[k]));
      strncpy(out[k].name, e.name, sizeof(out[k].name) - 1);
      ++*n;
    }
    out[k].launches += 1;
    out[k].ms += t;
  }
  return LSMBLK_OK;
}

int lsmblk_ctx_reserve(lsmblk_ctx* c, uint64_t max_blocks, uint64_t max_entries, uint64_t max_segments) {
  if (!c) return LSMBLK_E_INVAL;
  std::lock_guard<std::mutex> g(c->mu);
  DeviceGuard dg(c->device, c);
  if (!dg.ok) return LSMBLK_E_HIP;
  // (on the null stream, completed before returning: a later call may come on any stream)
  const int rc = reserve_locked(c, max_blocks, max_entries, max_segments, nullptr);
  if (rc) return rc;
  return hipStreamSynchronize(nullptr) == hipSuccess ? LSMBLK_OK : LSMBLK_E_HIP;
}

int lsmblk_decode_batch(lsmblk_ctx* c, const uint8_t* blocks, const uint64_t* blk_off, uint64_t nblk,
                        const lsmblk_kv_stream* out, uint64_t* stats, void* stream) {
  return lsmblk_decode_batch_ex(c, blocks, blk_off, nblk, 0, 0, out, nullptr, stats, stream);
}

int lsmblk_decode_batch_ex(lsmblk_ctx* c, const uint8_t* blocks, const uint64_t* blk_off, uint64_t nblk, uint32_t tail,
                           uint32_t flags, const lsmblk_kv_stream* out, uint64_t* blk_ent, uint64_t* stats,
                           void* stream) {
  if (!c || !blk_off || !out || !stats) return LSMBLK_E_INVAL;
  if (!aligned16(out->keys) || !aligned16(out->vals) || !out->key_off || !out->val_off) return LSMBLK_E_INVAL;
  if (nblk > 0x7FFFFFFFull || tail > 16) return LSMBLK_E_INVAL;  // one workgroup (or wave) per block
  if ((flags & LSMBLK_DECODE_VERIFY_CRC) && tail != 4) return LSMBLK_E_INVAL;
  std::lock_guard<std::mutex> g(c->mu);
  DeviceGuard dg(c->device, c);
  if (!dg.ok) return LSMBLK_E_HIP;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int rc = reserve_locked(c, nblk, 0, 0, st);
  if (rc) return rc;
  if (hipMemsetAsync(stats, 0, LSMBLK_STATS_WORDS * 8, st) != hipSuccess) return LSMBLK_E_HIP;
  if (nblk == 0) {
    LSM_LAUNCH(finish_empty_decode, dim3(1), dim3(64), 0, st, out->key_off, out->val_off, out->entry_cap);
    if (blk_ent && hipMemsetAsync(blk_ent, 0, 8, st) != hipSuccess) return LSMBLK_E_HIP;
    return hipGetLastError() == hipSuccess ? LSMBLK_OK : LSMBLK_E_HIP;
  }
  if (flags & LSMBLK_DECODE_VERIFY_CRC) {
    // read_block's checksum test (src/table.rs:226-230) over the framed ranges, then the decode
    if ((rc = lsmblk_impl::ensure_crc_tabs(c, st))) return rc;
    if ((rc = grow(st, &c->vcrc, &c->vcrc_cap, nblk + 1, 1))) return rc;
    if (!c->meta_cstats && hipMalloc(reinterpret_cast<void**>(&c->meta_cstats), LSMBLK_STATS_WORDS * 8) != hipSuccess) {
      c->meta_cstats = nullptr;
      return LSMBLK_E_NOMEM;
    }
    if (hipMemsetAsync(c->meta_cstats, 0, LSMBLK_STATS_WORDS * 8, st) != hipSuccess) return LSMBLK_E_HIP;
  }
  const uint64_t ntiles = (nblk + kTile - 1) / kTile;
  const KLogRange lr(c, &c->dec_log0, &c->dec_log1);
  DecodeArgs a;
  a.blocks = blocks;
  a.blk_off = blk_off;
  a.nblk = nblk;
  a.keys = out->keys;
  a.key_off = out->key_off;
  a.vals = out->vals;
  a.val_off = out->val_off;
  a.ts = out->ts;
  a.entry_cap = out->entry_cap;
  a.key_cap = out->key_cap;
  a.val_cap = out->val_cap;
  a.stats = stats;
  a.agg = c->dec_agg;
  a.tile_pre = c->tile_pre;
  a.tail = tail;
  a.blk_ent = blk_ent;
  a.skip = c->skip;
  a.bagg = a.bbase = a.tagg = a.tinc = a.dbg = nullptr;
  a.lag = a.lag_bytes = 0;
  a.tag = a.poll = 0;
  if (!c->dec_two_pass) {
    // lagged decode: E is read from HBM once, one launch (decode_lag_kernel).  The CRC-verifying
    // read runs the streaming CRC pass and the checksum test first, on the same stream (round 4:
    // the two-pass decode with the count folded into the old CRC pass, 4.0 ms at U; the lagged
    // decode beside that CRC pass on a second stream, 5.07 ms -- the persistent CRC grid and the
    // lagged decode's dispatch-order schedule got in each other's way).
    if (flags & LSMBLK_DECODE_VERIFY_CRC) {
      if ((rc = lsmblk_impl::launch_crc(c, blocks, blk_off, nblk, tail, c->vcrc, c->meta_cstats, st)))
        return rc;
      LSM_LAUNCH(crc_verify_kernel, dim3(uint32_t((nblk + 255) / 256)), dim3(256), 0, st, blocks, blk_off, nblk,
                 c->vcrc, c->meta_cstats, stats);
    }
    if ((rc = next_epoch(c, st))) return rc;
    a.bagg = c->lag_gran;
    a.bbase = a.bagg + 3 * c->lag_blk_cap;
    a.tagg = a.bbase + 3 * c->lag_blk_cap;
    a.tinc = a.tagg + 3 * ((c->lag_blk_cap + kTile - 1) / kTile + 1);
    // a batch shorter than the lag needs no more workgroups than blocks of lag: any lag >= 2 kTile
    // keeps the finisher schedule (decode_lag_kernel) deadlock-free, and lag >= nblk counts every
    // block before the first decode (one 4 KiB block launched 10 241 workgroups)
    a.lag = std::max<uint64_t>(2 * kTile, std::min<uint64_t>(c->dec_lag, nblk));
    a.lag_bytes = c->dec_lag_bytes;
    a.dbg = c->dbg_on ? c->dbg : nullptr;
    if (a.dbg && hipMemsetAsync(a.dbg, 0, kDbgWords * 8, st) != hipSuccess) return LSMBLK_E_HIP;
    a.tag = c->epoch;
    a.poll = c->poll;
    LSM_LAUNCH_SLOT(2, decode_lag_kernel, dim3(uint32_t(nblk + a.lag)), dim3(64), 0, st, a);
    return hipGetLastError() == hipSuccess ? LSMBLK_OK : LSMBLK_E_HIP;
  }
  if (flags & LSMBLK_DECODE_VERIFY_CRC) {
    // (two-pass A/B) one pass over E: the CRC of every block and its (entries, key bytes, value
    // bytes), in place of the count pass's second read of E
    if ((rc = lsmblk_impl::launch_crc(c, blocks, blk_off, nblk, tail, c->vcrc, c->meta_cstats, st, c->dec_agg)))
      return rc;
    LSM_LAUNCH(crc_verify_kernel, dim3(uint32_t((nblk + 255) / 256)), dim3(256), 0, st, blocks, blk_off, nblk,
                       c->vcrc, c->meta_cstats, stats);
    LSM_LAUNCH_SLOT(0, agg_tile_kernel, dim3(uint32_t((ntiles + 3) / 4)), dim3(256), 0, st, (const uint32_t*)c->dec_agg, nblk,
            c->tile_sum);
  } else {
    CountArgs ca;
    ca.blocks = blocks;
    ca.blk_off = blk_off;
    ca.nblk = nblk;
    ca.agg = c->dec_agg;
    ca.tile_sum = c->tile_sum;
    ca.stats = stats;
    ca.tail = tail;
    LSM_LAUNCH_SLOT(0, dec_count_staged_kernel, dim3(uint32_t(nblk)), dim3(64), 0, st, ca);
    LSM_LAUNCH_SLOT(0, agg_tile_kernel, dim3(uint32_t((ntiles + 3) / 4)), dim3(256), 0, st, (const uint32_t*)c->dec_agg,
            nblk, c->tile_sum);
  }
  ScanArgs sa;
  sa.tile_sum = c->tile_sum;
  sa.tile_pre = c->tile_pre;
  sa.ntiles = ntiles;
  sa.key_off = out->key_off;
  sa.val_off = out->val_off;
  sa.entry_cap = out->entry_cap;
  sa.key_cap = out->key_cap;
  sa.val_cap = out->val_cap;
  sa.stats = stats;
  sa.blk_ent = blk_ent;
  sa.nblk = nblk;
  LSM_LAUNCH_SLOT(1, dec_scan_kernel, dim3(1), dim3(1024), 0, st, sa);
  LSM_LAUNCH_SLOT(2, decode_kernel, dim3(uint32_t(nblk)), dim3(64), 0, st, a);
  return hipGetLastError() == hipSuccess ? LSMBLK_OK : LSMBLK_E_HIP;
}

int lsmblk_encode_batch(lsmblk_ctx* c, const lsmblk_kv_stream* in, const uint32_t* seg_start, uint32_t nseg,
                        uint32_t block_size, uint8_t* out, uint64_t out_cap, uint64_t* blk_off, uint64_t blk_cap,
                        uint64_t* stats, void* stream) {
  return lsmblk_encode_batch_ex(c, in, seg_start, nseg, block_size, 0, out, out_cap, blk_off, blk_cap, nullptr, stats,
                                stream);
}

int lsmblk_encode_batch_ex(lsmblk_ctx* c, const lsmblk_kv_stream* in, const uint32_t* seg_start, uint32_t nseg,
                           uint32_t block_size, uint32_t flags, uint8_t* out, uint64_t out_cap, uint64_t* blk_off,
                           uint64_t blk_cap, uint64_t* seg_out, uint64_t* stats, void* stream) {
  if (!c || !in || !seg_start || !blk_off || !stats || !aligned16(out)) return LSMBLK_E_INVAL;
  if (in->n >= 0xFFFFFFFFull || !in->key_off || !in->val_off) return LSMBLK_E_INVAL;
  if (block_size == 0 || (flags & ~uint32_t(LSMBLK_ENCODE_SEG_SLOTS | LSMBLK_ENCODE_FRAMED))) return LSMBLK_E_INVAL;
  if ((flags & LSMBLK_ENCODE_SEG_SLOTS) && !seg_out) return LSMBLK_E_INVAL;
  std::lock_guard<std::mutex> g(c->mu);
  DeviceGuard dg(c->device, c);
  if (!dg.ok) return LSMBLK_E_HIP;
  return lsmblk_impl::encode_locked(c, in, nullptr, seg_start, nullptr, nseg, block_size, out, out_cap, blk_off,
                                    blk_cap, stats, reinterpret_cast<hipStream_t>(stream), false, flags, seg_out);
}

}  // extern "C"

namespace lsmblk_impl {
int encode_locked(lsmblk_ctx* c, const lsmblk_kv_stream* in, const uint64_t* dn, const uint32_t* seg_start,
                  const uint32_t* dnseg, uint32_t nseg, uint32_t block_size, uint8_t* out, uint64_t out_cap,
                  uint64_t* blk_off, uint64_t blk_cap, uint64_t* stats, hipStream_t st, bool span, uint32_t flags,
                  uint64_t* seg_out) {
  const KLogRange lr(c, &c->enc_log0, &c->enc_log1);
  const bool slots = (flags & LSMBLK_ENCODE_SEG_SLOTS) != 0;
  const bool framed = (flags & LSMBLK_ENCODE_FRAMED) != 0;
  if (slots && (!seg_out || span || dn || dnseg)) return LSMBLK_E_INVAL;
  if (framed && (span || dn || dnseg)) return LSMBLK_E_INVAL;
  // in->n (and nseg) are upper bounds when dn (dnseg) point at the device-side values
  int rc = reserve_locked(c, 0, in->n, nseg, st);
  if (rc) return rc;
  if (hipMemsetAsync(stats, 0, LSMBLK_STATS_WORDS * 8, st) != hipSuccess) return LSMBLK_E_HIP;
  if (nseg == 0) {
    // no segments: zero blocks; blk_off[0] = 0
    if (in->n != 0) return LSMBLK_E_INVAL;
    if (blk_cap >= 1 && hipMemsetAsync(blk_off, 0, 8, st) != hipSuccess) return LSMBLK_E_HIP;
    return LSMBLK_OK;
  }
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device);
  // the fused walk + emit (A/B only: the walk's instructions compete with emit's for the same
  // issue slots): per-segment slots, blocks no larger than emit's LDS image
  const bool fused = slots && !framed && block_size <= 4096 && c->fuse_on;
  uint32_t walk_wgs = 0, nwalk = 0;
  if (fused) {
    walk_wgs = uint32_t(std::min<uint64_t>(uint64_t(cus), (uint64_t(nseg) + 1) / 2));
    walk_wgs += walk_wgs & 1;  // walkers a multiple of 4: emitters split evenly over them
    nwalk = 2 * walk_wgs;
    const uint64_t recs = in->n + nwalk + 1;
    const uint64_t fc = c->frec_cap, dc = c->fdone_cap;
    if ((rc = grow(st, &c->frec, &c->frec_cap, recs, 4, kStatusFlags))) return rc;
    if ((rc = grow(st, &c->fdone, &c->fdone_cap, nwalk, 1, kStatusFlags))) return rc;
    if ((rc = grow(st, &c->fwnb, &c->fwnb_cap, nwalk, 1))) return rc;
    if ((rc = grow(st, &c->fbig, &c->fbig_cap, recs, 1))) return rc;
    if (c->frec_cap != fc || c->fdone_cap != dc) c->epoch = 0;  // fresh granules: a new epoch sequence
  }
  if (framed && (rc = ensure_crc_tabs(c, st))) return rc;
  if ((rc = next_epoch(c, st))) return rc;
  if (hipMemsetAsync(c->counters, 0, 2048, st) != hipSuccess) return LSMBLK_E_HIP;
  PlanArgs p;
  p.keys = in->keys;
  p.key_off = in->key_off;
  p.val_off = in->val_off;
  p.n = in->n;
  p.seg_start = seg_start;
  p.nseg = nseg;
  p.block_size = block_size;
  p.sz = c->ent;
  p.rec_first = c->rec_first;
  p.blk_first = c->blk_first;
  p.blk_off = blk_off;
  p.blk_cap = blk_cap;
  p.out_cap = out_cap;
  p.stats = stats;
  p.ticket = c->counters + 256;
  p.agg = c->seg_agg;
  p.inc = c->seg_inc;
  p.tag = c->epoch;
  p.poll = c->poll;
  p.dn = dn;
  p.dnseg = dnseg;
  p.span = span ? 1u : 0u;
  p.skip = c->skip;
  p.dbg = c->dbg_on ? c->dbg : nullptr;
  p.seg_out = slots ? seg_out : nullptr;
  p.blk_sz = slots || framed ? c->blk_sz : nullptr;
  p.pipe_helper = c->plan_pipe ? 1u : 0u;
  p.frame = framed ? 4u : 0u;
  EmitArgs e;
  e.keys = in->keys;
  e.key_off = in->key_off;
  e.vals = in->vals;
  e.val_off = in->val_off;
  e.ts = in->ts;
  e.blk_first = c->blk_first;
  e.blk_off = blk_off;
  e.out = out;
  e.out_cap = out_cap;
  e.blk_cap = blk_cap;
  e.n = in->n;
  e.stats = stats;
  e.big_flag = reinterpret_cast<uint8_t*>(c->big_list);
  e.blk_sz = slots || framed ? c->blk_sz : nullptr;
  e.skip = c->skip;
  e.dn = dn;
  if (fused) {
    if (p.dbg && hipMemsetAsync(p.dbg, 0, kDbgWords * 8, st) != hipSuccess) return LSMBLK_E_HIP;
    FuseArgs f;
    f.p = p;
    f.e = e;
    f.rec = c->frec;
    f.wdone = c->fdone;
    f.wnb = c->fwnb;
    f.seg_out = seg_out;
    f.bigr = c->fbig;
    f.nwalk = nwalk;
    f.spw = uint32_t((uint64_t(nseg) + nwalk - 1) / nwalk);
    f.walk_wgs = walk_wgs;
    // three emit workgroups per CU beside the walkers' one, split evenly over the walkers
    f.per_walker = std::max<uint32_t>(1u, uint32_t(3ull * kEmitWaves * uint64_t(cus) / nwalk));
    const uint32_t emit_wgs = f.per_walker * nwalk / kEmitWaves;
    LSM_LAUNCH_SLOT(4, encode_fused_kernel, dim3(walk_wgs + emit_wgs), dim3(256), 0, st, f);
    LSM_LAUNCH(slot_tables_kernel, dim3(nwalk), dim3(256), 0, st, f, c->blk_first, c->blk_sz,
               reinterpret_cast<uint8_t*>(c->big_list), blk_off, blk_cap, out_cap);
  } else {
    if (p.dbg && hipMemsetAsync(p.dbg, 0, kDbgWords * 8, st) != hipSuccess) return LSMBLK_E_HIP;
    LSM_LAUNCH_SLOT(3, plan_walk_kernel, dim3((nseg + 3) / 4), dim3(kWalkThreads), 0, st, p);
    if (c->skip & (3u << 16)) {  // plan ablation: the block tables are wrong, emit is not launched
      return hipGetLastError() == hipSuccess ? LSMBLK_OK : LSMBLK_E_HIP;
    }
    if (kDiag && c->emit_poison)  // fault injection (diagnostics builds): a corrupt block table
      LSM_LAUNCH(emit_poison_kernel, dim3(uint32_t(in->n / (5 * 256) + 1)), dim3(256), 0, st, c->blk_first, stats);
    // the big-block flags are cleared before emit (the start of emit_kernel to the end of
    // emit_big_kernel is what bench.py's roofline divides by)
    const uint64_t nblk_max = blk_cap < in->n + 1 ? blk_cap : in->n + 1;  // blocks <= entries, <= blk_cap
    if (nblk_max && hipMemsetAsync(c->big_list, 0, nblk_max, st) != hipSuccess) return LSMBLK_E_HIP;
    if (hipGetLastError() != hipSuccess) return LSMBLK_E_HIP;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, emit_kernel, 256, 0) != hipSuccess || per_cu < 1)
      per_cu = 3;
    const uint32_t grid = uint32_t(cus) * uint32_t(per_cu);
    LSM_LAUNCH_SLOT(4, emit_kernel, dim3(grid), dim3(256), 0, st, e);
  }
  // (every workgroup resident at once: the flagged blocks are strided over the whole grid)
  int big_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&big_cu, emit_big_kernel, 256, 0) != hipSuccess || big_cu < 1)
    big_cu = 4;
  LSM_LAUNCH_SLOT(4, emit_big_kernel, dim3(uint32_t(cus) * uint32_t(big_cu)), dim3(256), 0, st, e);
  if (framed) {  // every block's CRC after it: the SST data section (src/table/builder.rs:112-123)
    const uint64_t nblk_max = blk_cap < in->n + 1 ? blk_cap : in->n + 1;
    if ((rc = launch_crc_frames(c, out, blk_off, c->blk_sz, nblk_max, stats, st))) return rc;
  }
  return hipGetLastError() == hipSuccess ? LSMBLK_OK : LSMBLK_E_HIP;
}

int segment_blocks_locked(lsmblk_ctx* c, const uint32_t* seg_start, uint32_t nseg_max, const uint64_t* enc_stats,
                          uint32_t* seg_blk, hipStream_t st) {
  LSM_LAUNCH(seg_blocks_kernel, dim3(uint32_t((uint64_t(nseg_max) + 256) / 256)), dim3(256), 0, st,
                     c->blk_first, enc_stats, seg_start, nseg_max, seg_blk);
  return hipGetLastError() == hipSuccess ? LSMBLK_OK : LSMBLK_E_HIP;
}
}  // namespace lsmblk_impl

extern "C" {

int lsmblk_crc32_batch(lsmblk_ctx* c, const uint8_t* blocks, const uint64_t* blk_off, uint64_t nblk, uint32_t tail,
                       uint32_t* crc, uint64_t* stats, void* stream) {
  if (!c || !blk_off || !stats || (nblk && !crc)) return LSMBLK_E_INVAL;
  std::lock_guard<std::mutex> g(c->mu);
  DeviceGuard dg(c->device, c);
  if (!dg.ok) return LSMBLK_E_HIP;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int rc = lsmblk_impl::ensure_crc_tabs(c, st);
  if (rc) return rc;
  if (hipMemsetAsync(stats, 0, LSMBLK_STATS_WORDS * 8, st) != hipSuccess) return LSMBLK_E_HIP;
  if (nblk == 0) return LSMBLK_OK;
  return lsmblk_impl::launch_crc(c, blocks, blk_off, nblk, tail, crc, stats, st);
}

int lsmblk_encode_segment_blocks(lsmblk_ctx* c, const uint32_t* seg_start, uint32_t nseg, const uint64_t* enc_stats,
                                 uint32_t* seg_blk, void* stream) {
  if (!c || !seg_start || !enc_stats || !seg_blk) return LSMBLK_E_INVAL;
  std::lock_guard<std::mutex> g(c->mu);
  DeviceGuard dg(c->device, c);
  if (!dg.ok) return LSMBLK_E_HIP;
  if (!c->blk_first) return LSMBLK_E_INVAL;  // no encode ran on this context
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  LSM_LAUNCH(seg_blocks_kernel, dim3(uint32_t((uint64_t(nseg) + 256) / 256)), dim3(256), 0, st,
                     c->blk_first, enc_stats, seg_start, nseg, seg_blk);
  return hipGetLastError() == hipSuccess ? LSMBLK_OK : LSMBLK_E_HIP;
}

int lsmblk_block_meta_batch(lsmblk_ctx* c, const uint8_t* blocks, const uint64_t* blk_off, uint64_t nblk,
                            uint32_t tail, const uint32_t* seg_blk, uint32_t nseg, uint8_t* meta, uint64_t meta_cap,
                            uint64_t* meta_off, uint64_t* stats, void* stream) {
  if (!c || !blk_off || !seg_blk || !meta_off || !stats || !meta || meta_cap < 16) return LSMBLK_E_INVAL;
  if (nseg == 0 || nblk >= 0xFFFFFFFFull) return LSMBLK_E_INVAL;
  std::lock_guard<std::mutex> g(c->mu);
  DeviceGuard dg(c->device, c);
  if (!dg.ok) return LSMBLK_E_HIP;
  return lsmblk_impl::block_meta_locked(c, blocks, blk_off, nblk, tail, seg_blk, nseg, meta, meta_cap, meta_off,
                                        stats, reinterpret_cast<hipStream_t>(stream));
}

}  // extern "C"

namespace lsmblk_impl {
int block_meta_locked(lsmblk_ctx* c, const uint8_t* blocks, const uint64_t* blk_off, uint64_t nblk, uint32_t tail,
                      const uint32_t* seg_blk, uint32_t nseg, uint8_t* meta, uint64_t meta_cap, uint64_t* meta_off,
                      uint64_t* stats, hipStream_t st) {
  int rc = lsmblk_impl::ensure_crc_tabs(c, st);
  if (rc) return rc;
  const uint64_t ntiles = (nblk + kMetaTile - 1) / kMetaTile;
  if (nblk + 1 > c->meta_blk_cap) {
    uint64_t cap = c->meta_blk_cap;
    if ((rc = grow(st, &c->meta_rec, &cap, nblk + 1, 1))) return rc;
    cap = c->meta_blk_cap;
    if ((rc = grow(st, &c->meta_pos, &cap, nblk + 1, 1))) return rc;
    c->meta_blk_cap = cap;
  }
  if ((rc = grow(st, &c->meta_tile, &c->meta_tile_cap, ntiles + 1, 2))) return rc;
  if ((rc = grow(st, &c->meta_crc, &c->meta_seg_cap, nseg, 1))) return rc;
  if (!c->meta_cstats && hipMalloc(reinterpret_cast<void**>(&c->meta_cstats), LSMBLK_STATS_WORDS * 8) != hipSuccess) {
    c->meta_cstats = nullptr;
    return LSMBLK_E_NOMEM;
  }
  if (hipMemsetAsync(stats, 0, LSMBLK_STATS_WORDS * 8, st) != hipSuccess) return LSMBLK_E_HIP;
  MetaArgs a;
  a.blocks = blocks;
  a.blk_off = blk_off;
  a.nblk = nblk;
  a.tail = tail;
  a.nseg = nseg;
  a.seg_blk = seg_blk;
  a.meta = meta;
  a.meta_cap = meta_cap;
  a.meta_off = meta_off;
  a.rec = c->meta_rec;
  a.tile_sum = c->meta_tile;
  a.tile_pre = c->meta_tile + c->meta_tile_cap;
  a.pos = c->meta_pos;
  a.crc = c->meta_crc;
  a.crc_stats = c->meta_cstats;
  a.stats = stats;
  const uint32_t sg = uint32_t((uint64_t(nseg) + 255) / 256);
  if (ntiles) LSM_LAUNCH(meta_size_kernel, dim3(uint32_t(ntiles)), dim3(256), 0, st, a);
  LSM_LAUNCH(meta_scan_kernel, dim3(1), dim3(1024), 0, st, a);
  if (ntiles) LSM_LAUNCH(meta_write_kernel, dim3(uint32_t(ntiles)), dim3(256), 0, st, a);
  LSM_LAUNCH(meta_seg_kernel, dim3(sg), dim3(256), 0, st, a);
  if (hipGetLastError() != hipSuccess) return LSMBLK_E_HIP;
  // section CRC over [meta_off[s] + 4, meta_off[s+1] - 4): blocks = meta + 4, tail = 8
  if (hipMemsetAsync(c->meta_cstats, 0, LSMBLK_STATS_WORDS * 8, st) != hipSuccess) return LSMBLK_E_HIP;
  if ((rc = lsmblk_impl::launch_crc(c, meta + 4, meta_off, nseg, 8, c->meta_crc, c->meta_cstats, st, nullptr, true)))
    return rc;
  LSM_LAUNCH(meta_crc_put_kernel, dim3(sg), dim3(256), 0, st, a);
  return hipGetLastError() == hipSuccess ? LSMBLK_OK : LSMBLK_E_HIP;
}
}  // namespace lsmblk_impl

extern "C" {

int lsmblk_compact_filter_batch(lsmblk_ctx* c, const lsmblk_kv_stream* in, uint64_t watermark, int bottom_level,
                                const uint8_t* prefixes, const uint32_t* prefix_off, uint32_t nprefix,
                                const lsmblk_kv_stream* out, uint64_t* stats, void* stream) {
  if (!c || !in || !out || !stats || !in->key_off || !in->val_off || !out->key_off || !out->val_off) return LSMBLK_E_INVAL;
  if (nprefix && (!prefixes || !prefix_off)) return LSMBLK_E_INVAL;
  if (in->n >= 0xFFFFFFFFull) return LSMBLK_E_INVAL;
  std::lock_guard<std::mutex> g(c->mu);
  DeviceGuard dg(c->device, c);
  if (!dg.ok) return LSMBLK_E_HIP;
  const uint64_t n = in->n, ntiles = (n + kFiltTile - 1) / kFiltTile;
  int rc;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if ((rc = grow(st, &c->filt_keep, &c->filt_cap, n + 1, 1))) return rc;
  if ((rc = grow(st, &c->filt_tile, &c->filt_tile_cap, ntiles + 1, 6))) return rc;
  if (hipMemsetAsync(stats, 0, LSMBLK_STATS_WORDS * 8, st) != hipSuccess) return LSMBLK_E_HIP;
  FiltArgs a;
  a.keys = in->keys;
  a.key_off = in->key_off;
  a.vals = in->vals;
  a.val_off = in->val_off;
  a.ts = in->ts;
  a.n = n;
  a.wm = watermark;
  a.bottom = bottom_level ? 1u : 0u;
  a.npfx = nprefix;
  a.pfx = prefixes;
  a.pfx_off = prefix_off;
  a.okeys = out->keys;
  a.okey_off = out->key_off;
  a.ovals = out->vals;
  a.oval_off = out->val_off;
  a.ots = out->ts;
  a.entry_cap = out->entry_cap;
  a.key_cap = out->key_cap;
  a.val_cap = out->val_cap;
  a.keep = c->filt_keep;
  a.tile_sum = c->filt_tile;
  a.tile_pre = c->filt_tile + 3 * c->filt_tile_cap;
  a.stats = stats;
  if (ntiles) LSM_LAUNCH(filt_flag_kernel, dim3(uint32_t(ntiles)), dim3(256), 0, st, a);
  LSM_LAUNCH(filt_scan_kernel, dim3(1), dim3(1024), 0, st, a);
  if (ntiles) LSM_LAUNCH(filt_write_kernel, dim3(uint32_t(ntiles)), dim3(256), 0, st, a);
  return hipGetLastError() == hipSuccess ? LSMBLK_OK : LSMBLK_E_HIP;
}

}  // extern "C"

namespace lsmblk_impl {
int fork_aux(lsmblk_ctx* c, hipStream_t st) {
  // (normal priority: a highest-priority second stream slowed every later kernel of the process
  // once several streams were in use)
  if (!c->aux && hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking) != hipSuccess) return LSMBLK_E_HIP;
  if (!c->fork_ev && hipEventCreateWithFlags(&c->fork_ev, hipEventDisableTiming) != hipSuccess) return LSMBLK_E_HIP;
  if (!c->join_ev && hipEventCreateWithFlags(&c->join_ev, hipEventDisableTiming) != hipSuccess) return LSMBLK_E_HIP;
  if (hipEventRecord(c->fork_ev, st) != hipSuccess || hipStreamWaitEvent(c->aux, c->fork_ev, 0) != hipSuccess)
    return LSMBLK_E_HIP;
  return LSMBLK_OK;
}

int join_aux(lsmblk_ctx* c, hipStream_t st) {
  if (hipEventRecord(c->join_ev, c->aux) != hipSuccess || hipStreamWaitEvent(st, c->join_ev, 0) != hipSuccess)
    return LSMBLK_E_HIP;
  return LSMBLK_OK;
}

int ensure_crc_tabs(lsmblk_ctx* c, hipStream_t st) {
  if (c->crc_tabs) return LSMBLK_OK;
  static CrcAllTabs h;  // (built once per process: the stream tables take ~40 M bit steps; never written after)
  static std::once_flag once;
  std::call_once(once, [] {
    crc_host_tables(h.t);
    crc_stream_host_tables(h.s);
  });
  void* d = nullptr;
  if (hipMalloc(&d, sizeof(CrcAllTabs)) != hipSuccess) return LSMBLK_E_NOMEM;
  // Copied on the call's stream and waited for there (first use only; a later call of the context
  // may come on another stream).  On any failure the tables are freed and c->crc_tabs stays null,
  // so no later call runs the CRC kernels over tables that were never filled.
  if (hipMemcpyAsync(d, &h, sizeof(CrcAllTabs), hipMemcpyHostToDevice, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess) {
    (void)hipFree(d);
    return LSMBLK_E_HIP;
  }
  c->crc_tabs = d;
  return LSMBLK_OK;
}

int launch_crc(lsmblk_ctx* c, const uint8_t* blocks, const uint64_t* blk_off, uint64_t nblk, uint32_t tail,
               uint32_t* crc, uint64_t* stats, hipStream_t st, uint32_t* agg, bool sections) {
  CrcArgs a;
  a.agg = agg;
  a.blocks = blocks;
  a.blk_off = blk_off;
  a.nblk = nblk;
  a.tail = tail;
  a.crc = crc;
  a.tabs = static_cast<const CrcTabs*>(c->crc_tabs);
  a.stats = stats;
  int cus = 256, per_cu = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device);
#ifndef LSMBLK_XCRC_OLD
  if (!agg && !sections) {  // the plain pass: one 16-wave workgroup per CU (the replicated tables fill the LDS)
    CrcStreamArgs b;
    b.blocks = blocks;
    b.blk_off = blk_off;
    b.nblk = nblk;
    b.tail = tail;
    b.crc = crc;
    b.tabs = &static_cast<const CrcAllTabs*>(c->crc_tabs)->s;
    b.stats = stats;
    b.frame_out = nullptr;
    b.sz = nullptr;
    b.dnblk = nullptr;
    const uint64_t want = (nblk + 4 * kCsWaves - 1) / (4 * kCsWaves);
    const uint32_t grid = uint32_t(want < uint64_t(cus) ? (want ? want : 1) : uint64_t(cus));
    LSM_LAUNCH(crc_stream_kernel, dim3(grid), dim3(64 * kCsWaves), 0, st, b);
    return hipGetLastError() == hipSuccess ? LSMBLK_OK : LSMBLK_E_HIP;
  }
#endif
  // persistent: as many workgroups as are resident at once (4 KiB tables + 4 x 4 KiB staging)
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, agg ? crc_kernel<true> : crc_kernel<false>, 256, 0) !=
          hipSuccess ||
      per_cu < 1)
    per_cu = 3;
  const uint64_t want = (nblk + 3) / 4, cap = uint64_t(cus > 0 ? cus : 256) * uint64_t(per_cu);
  const dim3 grid(uint32_t(want < cap ? want : cap));
  if (agg) LSM_LAUNCH(crc_kernel<true>, grid, dim3(256), 0, st, a);
  else LSM_LAUNCH(crc_kernel<false>, grid, dim3(256), 0, st, a);
  return hipGetLastError() == hipSuccess ? LSMBLK_OK : LSMBLK_E_HIP;
}

// The CRCs of a framed encode's blocks, written after each block (LSMBLK_ENCODE_FRAMED): the
// streaming CRC pass over the encode's own block table, its block count read on the device.
int launch_crc_frames(lsmblk_ctx* c, uint8_t* out, const uint64_t* blk_off, const uint32_t* blk_sz,
                      uint64_t nblk_max, uint64_t* stats, hipStream_t st) {
  CrcStreamArgs b;
  b.blocks = out;
  b.blk_off = blk_off;
  b.nblk = nblk_max;
  b.tail = 4;
  b.crc = nullptr;
  b.tabs = &static_cast<const CrcAllTabs*>(c->crc_tabs)->s;
  b.stats = stats;
  b.frame_out = out;
  b.sz = blk_sz;
  b.dnblk = stats;
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device);
  const uint64_t want = (nblk_max + 4 * kCsWaves - 1) / (4 * kCsWaves);
  const uint32_t grid = uint32_t(want < uint64_t(cus) ? (want ? want : 1) : uint64_t(cus));
  LSM_LAUNCH(crc_stream_kernel, dim3(grid), dim3(64 * kCsWaves), 0, st, b);
  return hipGetLastError() == hipSuccess ? LSMBLK_OK : LSMBLK_E_HIP;
}
}  // namespace lsmblk_impl lsmblk_impl
