// lsmblk_compact.hip -- compaction half of the batch C ABI (include/lsmblk.h), gfx950 (wave64):
//
//   lsmblk_merge_batch        MergeIterator over k sorted runs (src/iterators/merge_iterator.rs:59-184)
//   lsmblk_compact_batch      compact_generate_sst (src/compact.rs:223-311): merge -> keep/drop rules
//                             -> SST rotation -> SsTableBuilder block packing, on the device
//   lsmblk_sst_rotation_batch the SST cut points of compact_generate_sst (:278-289) over a stream
//                             that already holds exactly the entries handed to SsTableBuilder::add
//
// Merge semantics.  MergeIterator's heap orders heads by (user key, run index) -- Key's Ord ignores
// the ts (src/key.rs:63-81) -- and on every step advances each other run whose head has the
// current user key (:134-152).  Followed through, a user key's output is ALL the versions of the
// lowest-index run holding that key, in that run's order, and nothing of the other runs
// (tests/test_merge_oracle.py checks this closed form against a line-by-line heap simulation).
// So every entry is decided independently: it survives iff no lower-index run holds its key,
// and its merged position is the number of surviving entries with a smaller key plus its rank
// inside its own run's group.
//
// Kernels ("sample merge path"):
//   cand_rank_kernel   every kMS-th entry of every run is a candidate; its rank among all the
//                      candidates by (key, run, index) comes from binary searches in the other
//                      runs' candidate lists; candidates are scattered into sorted order
//   bounds_kernel      tile t = keys in [cand t, cand t+1): its sub-range in every run
//                      (lower bound via the candidate list, then within kMS entries)
//   merge_tile_kernel  one wave per tile: the tile's keys staged in LDS, survival (search the
//                      lower-index runs), survivor prefix, in-tile merged rank (search every
//                      other run); equal keys never straddle tiles (key-only lower bounds)
//   tscan_*_kernel     exclusive scan of per-tile survivor counts -> tile bases
//   perm_kernel        perm[tile base + in-tile rank] = input index
// Then, over the merged order:
//   mflag_kernel / mscan_*_kernel / mwrite_kernel   the compaction rules (or keep-all for a plain
//                      merge), output offsets, and the gather of the kept entries.
#include "lsmblk_dev.hpp"

namespace {

#ifndef LSMBLK_MS
#define LSMBLK_MS 128
#endif
#ifndef LSMBLK_MTE
#define LSMBLK_MTE 512
#endif
#ifndef LSMBLK_MTT
#define LSMBLK_MTT 128
#endif
constexpr uint32_t kMS = LSMBLK_MS;  // every kMS-th entry of a run is a merge candidate
constexpr uint32_t kMaxRuns = 64;   // runs per merge (one lane per run in the tile kernels)
// Tile entries with LDS tables.  Tile sizes average kMS (the gaps between consecutive candidates
// of all runs) with a long tail, so the limit trades residency against the share of tiles left
// to merge_big_kernel: merge_tile on config C took 5.3 / 3.1 / 2.8 / 2.8 / 3.5 / 6.9 ms at
// 256 / 384 / 512 / 640 / 1024 / 2048 entries when larger tiles went to the one-wave global path
// (and 3.2 / 3.8 ms at mean tile sizes 192 / 256 with the limit at 4x the mean).
constexpr uint32_t kMTE = LSMBLK_MTE;
constexpr uint32_t kMTT = LSMBLK_MTT;  // threads per tile workgroup
// merge_big_kernel: tiles of kMTE < total <= kBigTE entries (about 1 % of the tiles; 0.8 ms of
// config C's 2.9 ms merge_tile as a global-memory tail), workgroups of kBigTT threads
constexpr uint32_t kBigTE = 2048;
constexpr uint32_t kBigTT = 256;
constexpr uint32_t kBigGrid = 1024;
constexpr uint32_t kNone = 0xFFFFFFFFu;

// ---------------------------------------------------------------- key access
// Global keys through a bounds-checked descriptor over the key arena (reads past it give 0).
struct GKeys {
  rsrc_t r;
  uint32_t lead;
  __device__ __forceinline__ uint32_t dw(uint32_t pos) const {  // bytes [pos, pos + 4), LE
    const uint32_t x = lead + pos, al = x & ~3u;
    const uint32_t w0 = __builtin_amdgcn_raw_buffer_load_b32(r, al, 0, 0);
    const uint32_t w1 = __builtin_amdgcn_raw_buffer_load_b32(r, al + 4, 0, 0);
    return __builtin_amdgcn_alignbyte(w1, w0, x & 3);
  }
};
__device__ __forceinline__ GKeys gkeys(const uint8_t* keys, uint32_t total) {
  GKeys g;
  g.lead = uint32_t(reinterpret_cast<uintptr_t>(keys) & 15);
  g.r = make_rsrc(keys - g.lead, g.lead + total);
  return g;
}
// LDS key image (unaligned ds_read_b32: the gfx9 unaligned access mode)
struct LKeys {
  const uint8_t* base;
  __device__ __forceinline__ uint32_t dw(uint32_t pos) const {
    return *reinterpret_cast<const uint32_t*>(base + pos);
  }
};

// Lexicographic byte order of keys [a, a + la) and [b, b + lb) (src/key.rs:77-81 via Vec<u8>
// Ord): -1, 0, 1.
template <class KS>
__device__ __forceinline__ int key_cmp(const KS& S, uint32_t a, uint32_t la, uint32_t b, uint32_t lb) {
  const uint32_t m = la < lb ? la : lb;
  for (uint32_t i = 0; i < m; i += 4) {
    uint32_t x = S.dw(a + i), y = S.dw(b + i);
    if (m - i < 4) {
      const uint32_t mk = (1u << (8 * (m - i))) - 1;
      x &= mk;
      y &= mk;
    }
    if (x != y) {
      const uint32_t z = __builtin_ctz(x ^ y) & ~7u;
      return ((x >> z) & 0xFF) < ((y >> z) & 0xFF) ? -1 : 1;
    }
  }
  return la < lb ? -1 : (la > lb ? 1 : 0);
}

// ---------------------------------------------------------------- merge
struct MergeArgs {
  const uint8_t* keys;
  const uint32_t* key_off;
  uint64_t n;               // entries of the input stream
  const uint32_t* run_start;
  uint32_t nrun;
  uint32_t nc_max;          // bound on candidates (= tiles)
  const u32x4* k16;         // n: every input key's first 16 bytes as big-endian words (key16_kernel)
  uint32_t* cand;           // nc_max: sorted candidate -> input index
  u32x4* ck;                // nc_max: first 16 key bytes (big-endian words) per candidate, run-major
  uint32_t* cklen;          // nc_max: its key length
  u32x4* cks;               // nc_max: ck in sorted candidate order
  uint32_t* ckslen;
  uint32_t* bounds;         // (nc_max + 1) x nrun: tile t's first entry in run r
  uint32_t* mrank;          // n: in-tile merged rank of a surviving entry, kNone if dropped
  uint32_t* sp;             // n: survivor prefix (tiles too large for LDS)
  uint32_t* tcnt;           // nc_max: survivors per tile
  uint64_t* tpre;           // nc_max + 1: tile bases inside their scan part (kTScan tiles)
  uint64_t* tpart;          // per scan part: its tiles' survivors
  uint64_t* tbase;          // per scan part + 1: the part's base (the last: all survivors)
  uint32_t* perm;           // n: merged position -> input index
  uint32_t* big;            // nc_max: tiles left to merge_big_kernel (their count in mstats[5])
  uint64_t* mstats;         // [0] merged entries [1] candidates (tiles) [3] error flags [5] big tiles
  uint32_t two;             // LSMBLK_MERGE_TWO_LEVEL: TwoMergeIterator(runs 0..nrun-2, run nrun-1)
  uint32_t two_end;         // two-level, key-range shard: LSMBLK_TWO_END_* (where b's last key lies)
};

// LSMBLK_MERGE_TWO_LEVEL: the reference's compact() input, TwoMergeIterator(a = MergeIterator(upper
// runs), b = the lower level's SstConcatIterator) (src/compact.rs:170-173,188-196,206-215), followed
// through two_merge_iterator.rs:19-93 (tests/test_merge_oracle.py pins this closed form against the
// line-by-line iterator):
//   * the stream ends when b does (is_valid / choose_a, :32-42,60-66): nothing at all when b is
//     empty, and no a-entry whose user key is >= b's last key;
//   * a key held by a only: a's versions (a = MergeIterator: the lowest upper run holding it);
//   * a key held by b only: all of b's versions;
//   * a key held by both: skip_b (:45-50) drops every other b version, starting with the first,
//     and b wins the equal-key choice, so b's 2nd, 4th, ... versions come first, then a's versions.
// Run B = nrun - 1 is b.  Survival and the merged rank inside a tile (equal keys never straddle
// tiles) follow from the same searches as the run-priority merge.

// Run starts and the per-run candidate prefix (ceil(len / kMS) candidates per run) in LDS.
__device__ __forceinline__ void load_runs(const MergeArgs& a, uint32_t* s_rs, uint32_t* s_cb) {
  for (uint32_t i = threadIdx.x; i <= a.nrun; i += blockDim.x) s_rs[i] = a.run_start[i];
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t c = 0;
    for (uint32_t r = 0; r < a.nrun; ++r) {
      s_cb[r] = c;
      c += (s_rs[r + 1] - s_rs[r] + kMS - 1) / kMS;
    }
    s_cb[a.nrun] = c;
  }
  __syncthreads();
}

// largest r < nrun with v[r] <= x (v non-decreasing, v[0] <= x)
__device__ __forceinline__ uint32_t find_run(const uint32_t* v, uint32_t nrun, uint32_t x) {
  uint32_t lo = 0, hi = nrun;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (v[mid] <= x) lo = mid;
    else hi = mid;
  }
  return lo;
}

// First 16 bytes of the key at arena position pos (len bytes) as big-endian words, zero padded:
// five aligned dword loads through the descriptor (none straddles its bound) and alignbytes.
__device__ __forceinline__ u32x4 key16(const GKeys& G, uint32_t pos, uint32_t len) {
  const uint32_t x = G.lead + pos, al = x & ~3u, b = x & 3;
  uint32_t w[5];
#pragma unroll
  for (uint32_t j = 0; j < 5; ++j) w[j] = __builtin_amdgcn_raw_buffer_load_b32(G.r, al + 4 * j, 0, 0);
  uint32_t o[4];
#pragma unroll
  for (uint32_t i = 0; i < 4; ++i) {
    uint32_t v = __builtin_amdgcn_alignbyte(w[i + 1], w[i], b);
    const int32_t keep = int32_t(len) - int32_t(4 * i);  // bytes of this word inside the key
    if (keep < 4) v &= keep <= 0 ? 0u : (1u << (8 * keep)) - 1;
    o[i] = __builtin_bswap32(v);
  }
  return u32x4{o[0], o[1], o[2], o[3]};
}

// Key order on (16-byte prefix, length, global index): the prefixes decide unless equal and
// both keys are longer than 16 bytes (then the tails are compared in global memory).
__device__ __forceinline__ int kcmp16(const MergeArgs& a, const GKeys& G, const u32x4& x, uint32_t xl, uint32_t xg,
                                      const u32x4& y, uint32_t yl, uint32_t yg) {
  // two 64-bit compares, one branch (a branch per word compiled to divergent exec-mask code)
  const uint64_t xh = (uint64_t(x.x) << 32) | x.y, xo = (uint64_t(x.z) << 32) | x.w;
  const uint64_t yh = (uint64_t(y.x) << 32) | y.y, yo = (uint64_t(y.z) << 32) | y.w;
  const bool lt = xh < yh || (xh == yh && xo < yo);
  if (xh != yh || xo != yo) return lt ? -1 : 1;
  if (xl <= 16 || yl <= 16) return xl < yl ? -1 : (xl > yl ? 1 : 0);
  return key_cmp(G, a.key_off[xg] + 16, xl - 16, a.key_off[yg] + 16, yl - 16);
}

// The merge tiles keep each key's first 16 bytes in LDS as two u64 (most significant word first:
// u32x4 {w1, w0, w3, w2} of the big-endian words), so that a compare is two 64-bit compares
// without branches; kcmp16's chain of word compares compiled to a divergent branch per word
// (exec-mask SALU around every step of every binary search, PMC: SALU 5.9e8 against VALU 7.3e8).
__device__ __forceinline__ u32x4 k16_swap(const u32x4& k) { return u32x4{k.y, k.x, k.w, k.z}; }
__device__ __forceinline__ int kcmp16s(const MergeArgs& a, const GKeys& G, const u32x4& x, uint32_t xl, uint32_t xg,
                                       const u32x4& y, uint32_t yl, uint32_t yg) {
  const uint64_t xh = (uint64_t(x.y) << 32) | x.x, xo = (uint64_t(x.w) << 32) | x.z;
  const uint64_t yh = (uint64_t(y.y) << 32) | y.x, yo = (uint64_t(y.w) << 32) | y.z;
  const bool lt = xh < yh || (xh == yh && xo < yo);
  if (xh != yh || xo != yo) return lt ? -1 : 1;
  if (xl <= 16 || yl <= 16) return xl < yl ? -1 : (xl > yl ? 1 : 0);
  return key_cmp(G, a.key_off[xg] + 16, xl - 16, a.key_off[yg] + 16, yl - 16);
}

// Every input key's first 16 bytes, once, in entry order (coalesced: the key arena is read front
// to back): the merge tiles, the bound searches and the rules then read one 16-B word per key in
// the same round trip as its offsets, instead of the offsets and then the key bytes.
// A key over 65 535 bytes is refused (LSMBLK_ERR_SEGMENTS -> LSMBLK_E_INVAL): the merge tiles
// keep u16 key lengths (a longer key's truncated length could rank two distinct keys
// as equal and drop one), and the block format stores key lengths `as u16` anyway
// (src/block/builder.rs:63-64).
__global__ __launch_bounds__(256) void key16_kernel(const uint8_t* keys, const uint32_t* key_off, uint64_t n,
                                                    u32x4* k16, uint64_t* merr) {
  const uint64_t e = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  if (e >= n) return;
  const GKeys G = gkeys(keys, key_off[n]);
  const uint32_t p = key_off[e], kl = key_off[e + 1] - p;
  k16[e] = key16(G, p, kl);
  if (kl > 0xFFFFu) atomicOr(reinterpret_cast<unsigned long long*>(merr), (unsigned long long)LSMBLK_ERR_SEGMENTS);
}

// Every candidate's first 16 key bytes and length, in run-major candidate order (ck, cklen): the
// rank and bound searches below then read one 16-B word per step instead of an offset and then
// the key bytes (two dependent round trips).
__global__ __launch_bounds__(256) void cand_key_kernel(MergeArgs a) {
  __shared__ uint32_t s_rs[kMaxRuns + 1], s_cb[kMaxRuns + 1];
  load_runs(a, s_rs, s_cb);
  const uint32_t c = blockIdx.x * 256 + threadIdx.x;
  if (c >= s_cb[a.nrun] || c >= a.nc_max) return;
  const uint32_t r = find_run(s_cb, a.nrun, c), p = s_rs[r] + (c - s_cb[r]) * kMS;
  if (p >= a.n) return;  // (a bad run table: cand_rank_kernel merges nothing)
  a.ck[c] = a.k16[p];
  a.cklen[c] = a.key_off[p + 1] - a.key_off[p];
}

__global__ __launch_bounds__(256) void cand_rank_kernel(MergeArgs a) {
  __shared__ uint32_t s_rs[kMaxRuns + 1], s_cb[kMaxRuns + 1];
  load_runs(a, s_rs, s_cb);
  bool ok = s_rs[0] == 0 && uint64_t(s_rs[a.nrun]) == a.n;
  for (uint32_t r = 0; r < a.nrun; ++r) ok = ok && s_rs[r] <= s_rs[r + 1];
  const uint32_t NC = ok ? s_cb[a.nrun] : 0u;  // a bad run table merges nothing
  const uint32_t c = blockIdx.x * 256 + threadIdx.x;
  if (c == 0) {
    a.mstats[1] = NC;
    if (!ok) atomicOr(reinterpret_cast<unsigned long long*>(a.mstats + 3), (unsigned long long)LSMBLK_ERR_SEGMENTS);
  }
  if (c >= NC) return;
  const GKeys K = gkeys(a.keys, a.key_off[a.n]);
  const uint32_t r = find_run(s_cb, a.nrun, c), j = c - s_cb[r];
  const uint32_t p = s_rs[r] + j * kMS;
  const u32x4 x = a.ck[c];
  const uint32_t xl = a.cklen[c];
  uint32_t rank = j;
  for (uint32_t r2 = 0; r2 < a.nrun; ++r2) {
    if (r2 == r) continue;
    // candidates of r2 ordered before (x, r, j): key < x, or key == x and r2 < r
    uint32_t lo = 0, hi = s_cb[r2 + 1] - s_cb[r2];
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1, q = s_cb[r2] + mid;
      const int cm = kcmp16(a, K, a.ck[q], a.cklen[q], s_rs[r2] + mid * kMS, x, xl, p);
      if (cm < 0 || (cm == 0 && r2 < r)) lo = mid + 1;
      else hi = mid;
    }
    rank += lo;
  }
  a.cand[rank] = p;
  a.cks[rank] = x;
  a.ckslen[rank] = xl;
}

__global__ __launch_bounds__(256) void bounds_kernel(MergeArgs a) {
  __shared__ uint32_t s_rs[kMaxRuns + 1], s_cb[kMaxRuns + 1];
  load_runs(a, s_rs, s_cb);
  const uint32_t NC = uint32_t(a.mstats[1]);
  const uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  const uint32_t t = uint32_t(i / a.nrun), r = uint32_t(i % a.nrun);
  if (t > a.nc_max || r >= a.nrun) return;
  uint32_t* out = a.bounds + uint64_t(t) * a.nrun + r;  // tile-major: a tile's bounds share a line
  if (t >= NC) {  // (rows past the last tile too: the tile kernels see those tiles empty)
    *out = s_rs[r + 1];
    return;
  }
  const GKeys K = gkeys(a.keys, a.key_off[a.n]);
  const uint32_t x = a.cand[t], xl = a.ckslen[t];
  const u32x4 xk = a.cks[t];
  const uint32_t base = s_rs[r], C = s_cb[r + 1] - s_cb[r];
  uint32_t lo = 0, hi = C;  // first candidate of r with key >= x
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1, q = s_cb[r] + mid;
    if (kcmp16(a, K, a.ck[q], a.cklen[q], base + mid * kMS, xk, xl, x) < 0) lo = mid + 1;
    else hi = mid;
  }
  uint32_t e0 = lo == 0 ? base : base + (lo - 1) * kMS + 1;
  uint32_t e1 = lo < C ? base + lo * kMS : s_rs[r + 1];
  while (e0 < e1) {  // first entry in [e0, e1) with key >= x (else e1)
    const uint32_t mid = (e0 + e1) >> 1;
    if (kcmp16(a, K, a.k16[mid], a.key_off[mid + 1] - a.key_off[mid], mid, xk, xl, x) < 0) e0 = mid + 1;
    else e1 = mid;
  }
  *out = e0;
}

struct TileHdr {
  uint32_t lo[kMaxRuns], tb[kMaxRuns + 1];  // run r's sub-range start; tile index of its first entry
  uint32_t rsp[kMaxRuns];                  // survivors before run r's sub-range
  uint32_t total, nsurv;
  uint32_t wsum[kBigTT / 64];
};
template <uint32_t E>
struct alignas(16) MTileLdsT {
  TileHdr h;
  u32x4 kw[E];          // first 16 key bytes as big-endian words, zero padded, in kcmp16s order
  uint16_t klen[E];        // (key lengths are u16 in the block format)
  uint16_t sp[E + 1];   // survivor prefix over the tile (run-major order)
  uint8_t surv[E];
};
using MTileLds = MTileLdsT<kMTE>;
using MTileBigLds = MTileLdsT<kBigTE>;

// The tile's per-run sub-ranges (wave 0; lane r = run r).
__device__ __forceinline__ void tile_ranges(const MergeArgs& a, TileHdr& H, uint32_t t) {
  const uint32_t l = lane_id();
  uint32_t lo = 0, hi = 0;
  if (l < a.nrun) {
    const uint32_t* row = a.bounds + uint64_t(t) * a.nrun;
    lo = row[l];
    hi = row[a.nrun + l];
    if (hi < lo) hi = lo;  // only with unsorted runs (output then unspecified, flagged by mflag)
  }
  const uint32_t m = hi - lo, mi = wave_incl_scan32(m);
  if (l < a.nrun) {
    H.lo[l] = lo;
    H.tb[l] = mi - m;
  }
  if (l == 63) {
    H.total = mi;
    H.tb[a.nrun] = mi;
  }
}

// Two-level mode: b's last key, where the reference's stream ends.  In a key-range shard
// (lsmblk_compact_merge_batch_ex) the end is that of the WHOLE compaction's b: in this range
// (b's local last key, as for the whole stream), above it (no cut-off here: inf), or below it /
// b empty (nothing of a survives: !nonempty).
struct TwoEnd {
  u32x4 k16;
  uint32_t len, g, pos;
  bool nonempty, inf;
};
__device__ __forceinline__ TwoEnd two_end(const MergeArgs& a, const GKeys& G) {
  TwoEnd t{};
  const uint32_t e0 = a.run_start[a.nrun - 1], e1 = a.run_start[a.nrun];
  t.nonempty = e1 > e0 && a.two_end != LSMBLK_TWO_END_BELOW;
  t.inf = a.two_end == LSMBLK_TWO_END_ABOVE;
  if (a.two_end == LSMBLK_TWO_END_ABOVE) t.nonempty = true;  // b's keys lie beyond this range
  if (t.nonempty && !t.inf) {
    t.g = e1 - 1;
    t.pos = a.key_off[t.g];
    t.len = a.key_off[t.g + 1] - t.pos;
    t.k16 = key16(G, t.pos, t.len);
  }
  return t;
}

// Every tile entry's first 16 key bytes and length into LDS.
template <uint32_t E, uint32_t T>
__device__ __forceinline__ void load_tile_keys(const MergeArgs& a, MTileLdsT<E>& L, const GKeys& G) {
  const TileHdr& H = L.h;
  for (uint32_t u = threadIdx.x; u < H.total; u += T) {
    const uint32_t r = find_run(H.tb, a.nrun, u), g = H.lo[r] + u - H.tb[r];
    L.kw[u] = k16_swap(a.k16[g]);  // (kcmp16s form)
    L.klen[u] = uint16_t(a.key_off[g + 1] - a.key_off[g]);
  }
}

// Survivor prefix over the tile (L.sp, H.nsurv, H.rsp) from L.surv.
template <uint32_t E, uint32_t T>
__device__ __forceinline__ void tile_survivor_prefix(const MergeArgs& a, MTileLdsT<E>& L) {
  TileHdr& H = L.h;
  const uint32_t tid = threadIdx.x, l = lane_id(), w = tid >> 6, nrun = a.nrun, total = H.total;
  uint32_t carry = 0;
  for (uint32_t c0 = 0; c0 < total; c0 += T) {
    const uint32_t u = c0 + tid;
    const uint32_t sv = u < total ? L.surv[u] : 0u;
    const uint32_t inc = wave_incl_scan32(sv);
    if (l == 63) H.wsum[w] = inc;
    __syncthreads();
    uint32_t before = 0, tot = 0;
#pragma unroll
    for (uint32_t x = 0; x < T / 64; ++x) {
      before += x < w ? H.wsum[x] : 0u;
      tot += H.wsum[x];
    }
    if (u < total) L.sp[u] = uint16_t(carry + before + inc - sv);
    carry += tot;
    __syncthreads();
  }
  if (tid == 0) {
    L.sp[total] = uint16_t(carry);
    H.nsurv = carry;
  }
  __syncthreads();
  if (tid < nrun) {
    H.rsp[tid] = L.sp[H.tb[tid]];
  }
  __syncthreads();
}

// LDS fast path: 128 threads per tile; every key's first 16 bytes in LDS.
template <uint32_t E, uint32_t T>
__device__ void merge_tile_lds(const MergeArgs& a, MTileLdsT<E>& L, uint32_t t) {
  TileHdr& H = L.h;
  const uint32_t tid = threadIdx.x, nrun = a.nrun, total = H.total;
  const GKeys G = gkeys(a.keys, a.key_off[a.n]);
  load_tile_keys<E, T>(a, L, G);
  __syncthreads();
  // first index of run r2's sub-range whose key is >= (x, xl) (> with upper)
  auto bound = [&](uint32_t r2, const u32x4& x, uint32_t xl, uint32_t xg, bool upper) -> uint32_t {
    const uint32_t b = H.tb[r2];
    uint32_t lo = 0, hi = H.tb[r2 + 1] - b;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      const int c = kcmp16s(a, G, L.kw[b + mid], L.klen[b + mid], H.lo[r2] + mid, x, xl, xg);
      if (c < 0 || (upper && c == 0)) lo = mid + 1;
      else hi = mid;
    }
    return lo;
  };
  const uint32_t B = nrun - 1;
  TwoEnd te{};
  if (a.two) te = two_end(a, G);
  const u32x4 tek = k16_swap(te.k16);
  // phase A: survival -- no lower-index run holds the key (MergeIterator advances those heads)
  for (uint32_t u = tid; u < total; u += T) {
    const uint32_t r = find_run(H.tb, nrun, u), g = H.lo[r] + u - H.tb[r];
    const u32x4 x = L.kw[u];
    const uint32_t xl = L.klen[u];
    bool held = false;
    for (uint32_t r2 = 0; r2 < r && !held; ++r2) {
      const uint32_t p = bound(r2, x, xl, g, false), b = H.tb[r2];
      held = p < H.tb[r2 + 1] - b && kcmp16s(a, G, L.kw[b + p], L.klen[b + p], H.lo[r2] + p, x, xl, g) == 0;
    }
    uint32_t sv = !held;
    if (a.two) {
      if (r == B) sv = held ? ((u - H.tb[B]) - bound(B, x, xl, g, false)) & 1u : 1u;  // skip_b
      else sv = sv && te.nonempty && (te.inf || kcmp16s(a, G, x, xl, g, tek, te.len, te.g) < 0);
    }
    L.surv[u] = uint8_t(sv);
  }
  __syncthreads();
  tile_survivor_prefix<E, T>(a, L);
  // phase B: merged rank inside the tile = survivors with a smaller key in every other run +
  // survivors before this entry in its own run (its group's earlier versions included)
  for (uint32_t u = tid; u < total; u += T) {
    const uint32_t r = find_run(H.tb, nrun, u), g = H.lo[r] + u - H.tb[r];
    uint32_t rank = kNone;
    if (L.surv[u]) {
      const u32x4 x = L.kw[u];
      const uint32_t xl = L.klen[u];
      rank = L.sp[u] - H.rsp[r];
      for (uint32_t r2 = 0; r2 < nrun; ++r2) {
        if (r2 == r || H.tb[r2 + 1] == H.tb[r2]) continue;
        // two-level: b's surviving versions of an equal key come before a's
        const uint32_t p = bound(r2, x, xl, g, a.two && r2 == B);
        rank += L.sp[H.tb[r2] + p] - H.rsp[r2];
      }
    }
    a.mrank[g] = rank;
  }
  if (tid == 0) a.tcnt[t] = H.nsurv;
}

// Global path (a tile of more than kMTE entries: many versions of one key, or many runs), one
// wave: keys compared in global memory, survival kept in mrank[] and the survivor prefix in
// sp[], handed between lanes through L2 (sc1 stores / loads, drained with vmcnt(0)).
__device__ void merge_tile_global(const MergeArgs& a, TileHdr& H, uint32_t* rsv, uint32_t t) {  // rsv: LDS, kMaxRuns
  const uint32_t l = lane_id(), nrun = a.nrun, total = H.total;
  const GKeys G = gkeys(a.keys, a.key_off[a.n]);
  auto kpos = [&](uint32_t r, uint32_t k, uint32_t& len) -> uint32_t {
    const uint32_t g = H.lo[r] + k, p = a.key_off[g];
    len = a.key_off[g + 1] - p;
    return p;
  };
  auto bound = [&](uint32_t r, uint32_t xp, uint32_t xl, bool upper) -> uint32_t {
    uint32_t lo = 0, hi = H.tb[r + 1] - H.tb[r];
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      uint32_t ml;
      const uint32_t mp = kpos(r, mid, ml);
      const int c = key_cmp(G, mp, ml, xp, xl);
      if (c < 0 || (upper && c == 0)) lo = mid + 1;
      else hi = mid;
    }
    return lo;
  };
  const uint32_t B = nrun - 1;
  TwoEnd te{};
  if (a.two) te = two_end(a, G);
  auto ld = [](const uint32_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  auto stv = [](uint32_t* p, uint32_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  auto drain = [&]() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync();
  };
  for (uint32_t u = l; u < total; u += 64) {  // phase A: survival
    const uint32_t r = find_run(H.tb, nrun, u), k = u - H.tb[r];
    uint32_t xl;
    const uint32_t xp = kpos(r, k, xl);
    bool held = false;
    for (uint32_t r2 = 0; r2 < r && !held; ++r2) {
      const uint32_t p = bound(r2, xp, xl, false);
      if (p < H.tb[r2 + 1] - H.tb[r2]) {
        uint32_t ql;
        const uint32_t qp = kpos(r2, p, ql);
        held = key_cmp(G, qp, ql, xp, xl) == 0;
      }
    }
    uint32_t sv = !held;
    if (a.two) {
      if (r == B) sv = held ? (k - bound(B, xp, xl, false)) & 1u : 1u;  // skip_b
      else sv = sv && te.nonempty && (te.inf || key_cmp(G, xp, xl, te.pos, te.len) < 0);
    }
    stv(a.mrank + H.lo[r] + k, sv);
  }
  drain();
  uint32_t carry = 0;  // survivor prefix
  for (uint32_t c0 = 0; c0 < total; c0 += 64) {
    const uint32_t u = c0 + l;
    uint32_t sv = 0, g = 0;
    if (u < total) {
      const uint32_t r = find_run(H.tb, nrun, u);
      g = H.lo[r] + u - H.tb[r];
      sv = ld(a.mrank + g);
    }
    const uint32_t inc = wave_incl_scan32(sv);
    if (u < total) stv(a.sp + g, carry + inc - sv);
    carry += __builtin_amdgcn_readlane(inc, 63);
  }
  drain();
  auto sp_at = [&](uint32_t u) -> uint32_t {  // prefix at tile index u (u == total: all)
    if (u >= total) return carry;
    const uint32_t r = find_run(H.tb, nrun, u);
    return ld(a.sp + H.lo[r] + u - H.tb[r]);
  };
  if (l < nrun) {
    const uint32_t b0 = sp_at(H.tb[l]), b1 = sp_at(H.tb[l + 1]);
    H.rsp[l] = b0;
    rsv[l] = b1 - b0;
  }
  wave_sync();
  for (uint32_t u = l; u < total; u += 64) {  // phase B: rank
    const uint32_t r = find_run(H.tb, nrun, u), k = u - H.tb[r], g = H.lo[r] + k;
    uint32_t rank = kNone;
    if (ld(a.mrank + g)) {
      uint32_t xl;
      const uint32_t xp = kpos(r, k, xl);
      rank = ld(a.sp + g) - H.rsp[r];
      for (uint32_t r2 = 0; r2 < nrun; ++r2) {
        const uint32_t m2 = H.tb[r2 + 1] - H.tb[r2];
        if (r2 == r || m2 == 0) continue;
        const uint32_t p = bound(r2, xp, xl, a.two && r2 == B);
        rank += p == m2 ? rsv[r2] : ld(a.sp + H.lo[r2] + p) - H.rsp[r2];
      }
    }
    a.mrank[g] = rank;  // each lane reads and rewrites only its own entries' words here
  }
  if (l == 0) a.tcnt[t] = carry;
}

__global__ __launch_bounds__(kMTT) void merge_tile_kernel(MergeArgs a) {
  __shared__ MTileLds L;
  // (tiles past the candidate count are empty: bounds_kernel.  The XCD-aware tile order of
  // rot_double made this kernel slower: 1.94 -> 2.09 ms on config C)
  const uint32_t t = blockIdx.x;
  if (threadIdx.x < 64) tile_ranges(a, L.h, t);
  __syncthreads();
  const uint32_t total = L.h.total;
  if (total == 0) {
    if (threadIdx.x == 0) a.tcnt[t] = 0;
    return;
  }
  if (total <= kMTE) {
    merge_tile_lds<kMTE, kMTT>(a, L, t);
  } else if (threadIdx.x == 0) {  // to merge_big_kernel
    const uint64_t i = atomicAdd(reinterpret_cast<unsigned long long*>(a.mstats + 5), 1ull);
    a.big[i] = t;
  }
}

// The tiles merge_tile_kernel left (over kMTE entries): kBigGrid persistent workgroups over the
// list, LDS tables up to kBigTE entries, the one-wave global path beyond.
__global__ __launch_bounds__(kBigTT) void merge_big_kernel(MergeArgs a) {
  __shared__ MTileBigLds L;
  __shared__ uint32_t rsv[kMaxRuns];  // the global path's per-run survivor counts
  const uint32_t nb = uni(uint32_t(a.mstats[5]));
  for (uint32_t i = blockIdx.x; i < nb; i += gridDim.x) {
    const uint32_t t = a.big[i];
    if (threadIdx.x < 64) tile_ranges(a, L.h, t);
    __syncthreads();
    if (L.h.total <= kBigTE) merge_tile_lds<kBigTE, kBigTT>(a, L, t);
    else if (threadIdx.x < 64) merge_tile_global(a, L.h, rsv, t);
    __syncthreads();
  }
}

// Exclusive scan of the tile survivor counts in two levels (one workgroup over all the tiles
// took 0.25 ms at config C's 254 K tiles): tscan_part_kernel scans kTScan tiles per workgroup
// into tpre[] and writes the part's total; tscan_top_kernel scans the parts into tbase[], the
// bases perm_kernel adds.
constexpr uint32_t kTScan = 2048;  // tiles per part (256 threads x 8)

__global__ __launch_bounds__(256) void tscan_part_kernel(MergeArgs a) {
  constexpr uint32_t kPer = kTScan / 256;
  __shared__ uint32_t ws[4];
  const uint32_t NC = uint32_t(a.mstats[1]);
  const uint64_t i0 = uint64_t(blockIdx.x) * kTScan + threadIdx.x * kPer;
  if (uint64_t(blockIdx.x) * kTScan >= NC) return;  // (uniform)
  uint32_t v[kPer], sum = 0;
#pragma unroll
  for (uint32_t j = 0; j < kPer; ++j) {
    v[j] = i0 + j < NC ? a.tcnt[i0 + j] : 0u;
    sum += v[j];
  }
  const uint32_t inc = wave_incl_scan32(sum), w = wave_id();
  if (lane_id() == 63) ws[w] = inc;
  __syncthreads();
  uint32_t run = inc - sum;
  for (uint32_t x = 0; x < w; ++x) run += ws[x];
#pragma unroll
  for (uint32_t j = 0; j < kPer; ++j) {
    if (i0 + j < NC) a.tpre[i0 + j] = run;
    run += v[j];
  }
  if (threadIdx.x == 0) a.tpart[blockIdx.x] = uint64_t(ws[0]) + ws[1] + ws[2] + ws[3];
}

__global__ __launch_bounds__(1024) void tscan_top_kernel(MergeArgs a) {
  const uint32_t t = threadIdx.x, w = t >> 6;
  const uint32_t NC = uint32_t(a.mstats[1]), np = (NC + kTScan - 1) / kTScan;
  __shared__ uint64_t wsum[16];
  uint64_t carry = 0;
  for (uint32_t r = 0; r < np; r += 1024) {
    const uint32_t i = r + t;
    const uint64_t v = i < np ? a.tpart[i] : 0ull;
    const uint64_t inc = wave_incl_scan<uint64_t>(v);
    if (lane_id() == 63) wsum[w] = inc;
    __syncthreads();
    uint64_t base = carry, tot = carry;
    for (uint32_t x = 0; x < 16; ++x) {
      if (x < w) base += wsum[x];
      tot += wsum[x];
    }
    if (i < np) a.tbase[i] = base + inc - v;
    carry = tot;
    __syncthreads();
  }
  if (t == 0) {
    a.tbase[np] = carry;
    a.mstats[0] = carry;
  }
}

__global__ __launch_bounds__(64) void perm_kernel(MergeArgs a) {
  __shared__ TileHdr H;
  const uint32_t t = blockIdx.x;
  if (t >= uni(uint32_t(a.mstats[1]))) return;
  tile_ranges(a, H, t);
  wave_sync();
  const uint64_t base = a.tpre[t] + a.tbase[t / kTScan];
  const uint32_t cnt = a.tcnt[t];
  for (uint32_t u = lane_id(); u < H.total; u += 64) {
    const uint32_t r = find_run(H.tb, a.nrun, u), g = H.lo[r] + u - H.tb[r];
    const uint32_t k = a.mrank[g];
    if (k < cnt) a.perm[base + k] = g;
  }
}

// ---------------------------------------------------------------- merged-order rules + gather
// The per-entry rules of compact_generate_sst (src/compact.rs:239-276) in the closed form of
// lsmblk_compact_filter_batch (lsmblk_gpu.hip, filt_keep), evaluated over the merged order
// perm[]: an entry needs only itself and its merged predecessor.  mode 0 keeps every merged
// entry (lsmblk_merge_batch).
constexpr uint32_t kGTile = 1024;  // merged entries per workgroup (4 rounds of 256)

struct GatherArgs {
  const uint8_t* keys;
  const uint32_t* key_off;
  const uint8_t* vals;
  const uint32_t* val_off;
  const uint64_t* ts;
  const uint32_t* perm;
  const u32x4* k16;         // n_max: the input keys' first 16 bytes (key16_kernel)
  const uint64_t* nm;       // device: merged entries
  uint64_t n_max;           // bound on merged entries (grid)
  uint32_t rules;           // 0: keep all; 1: compaction rules
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
  uint32_t* keep;           // n_max
  uint64_t* tile_sum;       // 3 per tile
  uint64_t* tile_pre;       // 3 per tile: exclusive prefix inside its scan part (kGScan tiles)
  uint64_t* part_sum;       // 3 per scan part
  uint64_t* part_pre;       // 3 per scan part: the part's base
  uint64_t* stats;          // [0] kept [1] key bytes [2] value bytes [3] error flags
  const uint64_t* merr;     // the merge stage's error flags (bad run table)
  lsmblk_key_range range;   // key-range shard (has_lo / has_hi 0: unbounded)
  uint32_t two;             // two-level merge order: the rules run as the loop (mgroup_kernel)
  uint8_t* ksame;           // two-level: per kept entry, the loop's same_as_last_key (or null)
  uint32_t* kidx;           // per kept entry, its input index (or null)
};

// Byte order of key (x, xl) against a range bound (y, yl) in device memory: -1, 0, 1.
__device__ __forceinline__ int bound_cmp(const uint8_t* x, uint32_t xl, const uint8_t* y, uint32_t yl) {
  const uint32_t m = xl < yl ? xl : yl;
  for (uint32_t t = 0; t < m; ++t)
    if (x[t] != y[t]) return x[t] < y[t] ? -1 : 1;
  return xl < yl ? -1 : (xl > yl ? 1 : 0);
}

// lo <= key < hi.  The bounds are user keys, so all the versions of a key fall on one side.
__device__ __forceinline__ bool in_range(const GatherArgs& a, uint32_t i) {
  if (!a.range.has_lo && !a.range.has_hi) return true;
  const uint32_t k0 = a.key_off[i], kl = a.key_off[i + 1] - k0;
  if (a.range.has_lo && bound_cmp(a.keys + k0, kl, a.range.lo, a.range.lo_len) < 0) return false;
  if (a.range.has_hi && bound_cmp(a.keys + k0, kl, a.range.hi, a.range.hi_len) >= 0) return false;
  return true;
}

__device__ __forceinline__ bool same_key_g(const GatherArgs& a, uint32_t i, uint32_t j) {
  const uint32_t a0 = a.key_off[i], al = a.key_off[i + 1] - a0;
  const uint32_t b0 = a.key_off[j], bl = a.key_off[j + 1] - b0;
  if (al != bl) return false;
  uint32_t x = 0;
  for (; x + 16 <= al; x += 16) {
    const u32x4 p = *reinterpret_cast<const u32x4*>(a.keys + a0 + x);
    const u32x4 q = *reinterpret_cast<const u32x4*>(a.keys + b0 + x);
    if (p.x != q.x || p.y != q.y || p.z != q.z || p.w != q.w) return false;
  }
  for (; x < al; ++x)
    if (a.keys[a0 + x] != a.keys[b0 + x]) return false;
  return true;
}

// Byte order of the keys at arena positions (pa, la) and (pb, lb), x / y their first 16 bytes
// (k16): those decide unless equal with both keys longer (then the tails, in global memory).
__device__ __forceinline__ int key_cmp16(const GKeys& G, const u32x4& x, uint32_t pa, uint32_t la, const u32x4& y,
                                         uint32_t pb, uint32_t lb) {
  const uint64_t xh = (uint64_t(x.x) << 32) | x.y, xo = (uint64_t(x.z) << 32) | x.w;  // (as kcmp16)
  const uint64_t yh = (uint64_t(y.x) << 32) | y.y, yo = (uint64_t(y.z) << 32) | y.w;
  const bool lt = xh < yh || (xh == yh && xo < yo);
  if (xh != yh || xo != yo) return lt ? -1 : 1;
  if (la <= 16 || lb <= 16) return la < lb ? -1 : (la > lb ? 1 : 0);
  return key_cmp(G, pa + 16, la - 16, pb + 16, lb - 16);
}

__device__ __forceinline__ bool prefix_filtered(const GatherArgs& a, uint32_t i) {
  const uint32_t k0 = a.key_off[i], kl = a.key_off[i + 1] - k0;
  for (uint32_t f = 0; f < a.npfx; ++f) {
    const uint32_t f0 = a.pfx_off[f], fl = a.pfx_off[f + 1] - f0;
    if (fl > kl) continue;
    bool m = true;
    for (uint32_t x = 0; x < fl && m; ++x) m = a.pfx[f0 + x] == a.keys[k0 + x];
    if (m) return true;
  }
  return false;
}

// Two-level merge order: a key's versions are not newest first (b's versions come before a's), so
// the closed form of mkeep does not hold.  The thread of a key's first merged entry runs the loop
// of compact_generate_sst (src/compact.rs:234-299) over that key's versions as written: it enters
// every key with same_as_last_key false (keys are never empty), and `last_key` becomes the key when
// an entry is added or dropped as a bottom-level tombstone, not when the prefix filter drops it.
// keep[j] = kept | same_as_last_key << 1 (the rotation's "key != last_key", :279).
__global__ __launch_bounds__(256) void mgroup_kernel(GatherArgs a) {
  const uint64_t N = *a.nm;
  const uint64_t j0 = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  if (j0 >= N) return;
  if (j0 > 0 && a.perm[j0] < a.n_max && a.perm[j0 - 1] < a.n_max && same_key_g(a, a.perm[j0 - 1], a.perm[j0]))
    return;
  bool lk = false, fkbw = true;  // last_key == this key; first_key_below_watermark
  for (uint64_t j = j0; j < N; ++j) {
    const uint32_t i = a.perm[j];
    if (i >= a.n_max || (j > j0 && !same_key_g(a, a.perm[j - 1], i))) break;
    const bool same = lk, below = a.ts[i] <= a.wm, empty = a.val_off[i + 1] == a.val_off[i];
    if (!same) fkbw = true;
    bool kept = false;
    if (a.bottom && !same && below && empty) {  // :244-254
      lk = true;
      fkbw = false;
    } else if (!(below && same && !fkbw)) {     // :256-260
      if (below) fkbw = false;
      if (!(below && prefix_filtered(a, i))) {  // :262-275
        kept = true;
        lk = true;                              // :294-297
      }
    }
    a.keep[j] = (kept ? 1u : 0u) | (same ? 2u : 0u);
  }
}

__global__ __launch_bounds__(256) void mflag_kernel(GatherArgs a) {
  const uint64_t N = *a.nm;
  const GKeys G = gkeys(a.keys, a.key_off[a.n_max]);
  // Every thread loads its own merged entry (input index, key position and length, first 16 key
  // bytes, value length, ts) once and takes its merged predecessor's from the neighbouring thread
  // through LDS (thread 0 loads its predecessor): half the gathers of loading both per thread.
  __shared__ u32x4 s16[256];
  __shared__ uint32_t sidx[256], sk0[256], skl[256];
  __shared__ uint64_t sts[256];
  const uint32_t t = threadIdx.x;
  uint32_t c = 0;
  uint64_t kb = 0, vb = 0;
#pragma unroll 1
  for (uint32_t sub = 0; sub < kGTile / 256; ++sub) {
    const uint64_t j = uint64_t(blockIdx.x) * kGTile + sub * 256 + t;
    const bool live = j < N;
    const uint32_t i = live ? a.perm[j] : kNone;
    const bool iv = live && i < a.n_max;
    uint32_t k0 = 0, kl = 0, vl = 0;
    u32x4 x16{0u, 0u, 0u, 0u};
    uint64_t tsi = 0;
    if (iv) {
      k0 = a.key_off[i];
      kl = a.key_off[i + 1] - k0;
      vl = a.val_off[i + 1] - a.val_off[i];
      x16 = a.k16[i];
      if (a.rules) tsi = a.ts[i];
    }
    __syncthreads();  // (the previous round's neighbour reads are done)
    s16[t] = x16;
    sidx[t] = iv ? i : kNone;
    sk0[t] = k0;
    skl[t] = kl;
    sts[t] = tsi;
    __syncthreads();
    if (!live) continue;
    bool k = false;
    uint32_t same = 0;
    // the merged order must be non-decreasing in the user key: an unsorted input run (which
    // MergeIterator assumes away, merge_iterator.rs:135-138) is reported, never followed.  One
    // compare with the merged predecessor gives the order and the rules' same-key test.
    uint32_t ip = 0, p0 = 0, pl = 0;
    u32x4 p16{0u, 0u, 0u, 0u};
    uint64_t tsp = 0;
    if (t > 0) {
      ip = sidx[t - 1];
      p16 = s16[t - 1];
      p0 = sk0[t - 1];
      pl = skl[t - 1];
      tsp = sts[t - 1];
    } else if (j > 0) {
      ip = a.perm[j - 1];
      if (ip < a.n_max) {
        p0 = a.key_off[ip];
        pl = a.key_off[ip + 1] - p0;
        p16 = a.k16[ip];
        if (a.rules) tsp = a.ts[ip];
      }
    }
    bool ordered = iv && ip < a.n_max;
    int cmp = -1;
    if (ordered && j > 0) {
      cmp = key_cmp16(G, p16, p0, pl, x16, k0, kl);
      ordered = cmp <= 0;
    }
    if (ordered) {
      if (a.two && a.rules) {
        const uint32_t g = a.keep[j];
        k = (g & 1u) && in_range(a, i);
        same = g & 2u;
      } else if (!in_range(a, i)) {
        k = false;
      } else if (!a.rules || tsi > a.wm) {
        k = true;  // (above the watermark every version is kept)
      } else {
        // the rules of the closed form (filt_keep, src/compact.rs:239-276) over the preloaded fields
        const bool start = !(j > 0 && cmp == 0);
        if (!start && tsp <= a.wm) k = false;               // a later version at or below the watermark
        else if (a.bottom && start && vl == 0) k = false;   // :244-254
        else k = !(a.npfx && prefix_filtered(a, i));        // CompactionFilter::Prefix, :264-275
      }
    } else {
      atomicOr(reinterpret_cast<unsigned long long*>(a.stats + 3), (unsigned long long)LSMBLK_ERR_MALFORMED);
    }
    a.keep[j] = (k ? 1u : 0u) | same;
    if (k) {
      c += 1;
      kb += kl;
      vb += vl;
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

// Exclusive scan of the gather tiles' (kept, key bytes, value bytes) in two levels, as the
// merge's tile scan: parts of kGScan tiles (mscan_part_kernel), then the parts' bases and the
// totals (mscan_top_kernel); mwrite adds its part's base.
constexpr uint32_t kGScan = 1024;  // gather tiles per part (256 threads x 4)

__global__ __launch_bounds__(256) void mscan_part_kernel(GatherArgs a) {
  constexpr uint32_t kPer = kGScan / 256;
  __shared__ uint64_t ws[4][3];
  const uint64_t N = *a.nm, ntiles = (N + kGTile - 1) / kGTile;
  const uint64_t i0 = uint64_t(blockIdx.x) * kGScan + threadIdx.x * kPer;
  if (uint64_t(blockIdx.x) * kGScan >= ntiles) return;  // (uniform)
  const uint32_t w = wave_id();
  uint64_t v[kPer][3], sum[3] = {0, 0, 0};
#pragma unroll
  for (uint32_t j = 0; j < kPer; ++j)
#pragma unroll
    for (uint32_t q = 0; q < 3; ++q) {
      v[j][q] = i0 + j < ntiles ? a.tile_sum[3 * (i0 + j) + q] : 0ull;
      sum[q] += v[j][q];
    }
#pragma unroll
  for (uint32_t q = 0; q < 3; ++q) {
    const uint64_t inc = wave_incl_scan<uint64_t>(sum[q]);
    if (lane_id() == 63) ws[w][q] = inc;
    sum[q] = inc - sum[q];  // the thread's exclusive prefix inside its wave
  }
  __syncthreads();
#pragma unroll
  for (uint32_t q = 0; q < 3; ++q) {
    uint64_t run = sum[q];
    for (uint32_t x = 0; x < w; ++x) run += ws[x][q];
#pragma unroll
    for (uint32_t j = 0; j < kPer; ++j) {
      if (i0 + j < ntiles) a.tile_pre[3 * (i0 + j) + q] = run;
      run += v[j][q];
    }
    if (threadIdx.x == 0) a.part_sum[3 * uint64_t(blockIdx.x) + q] = ws[0][q] + ws[1][q] + ws[2][q] + ws[3][q];
  }
}

__global__ __launch_bounds__(1024) void mscan_top_kernel(GatherArgs a) {
  const uint32_t t = threadIdx.x, w = t >> 6;
  const uint64_t N = *a.nm, ntiles = (N + kGTile - 1) / kGTile, np = (ntiles + kGScan - 1) / kGScan;
  __shared__ uint64_t wsum[16][3];
  uint64_t carry[3] = {0, 0, 0};
  for (uint64_t r = 0; r < np; r += 1024) {
    const uint64_t i = r + t;
    uint64_t v[3], inc[3];
#pragma unroll
    for (uint32_t q = 0; q < 3; ++q) {
      v[q] = i < np ? a.part_sum[3 * i + q] : 0ull;
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
      if (i < np) a.part_pre[3 * i + q] = base + inc[q] - v[q];
      carry[q] = tot;
    }
    __syncthreads();
  }
  if (t == 0) {
    const uint64_t tot[3] = {carry[0], carry[1], carry[2]};
#pragma unroll
    for (uint32_t q = 0; q < 3; ++q) a.stats[q] = tot[q];
    uint32_t err = uint32_t(*a.merr);
    if (tot[1] > 0xFFFFFFFFull || tot[2] > 0xFFFFFFFFull) err |= LSMBLK_ERR_OVERFLOW;
    if (tot[0] > a.entry_cap || tot[1] > a.key_cap || tot[2] > a.val_cap) err |= LSMBLK_ERR_CAPACITY;
    if (!err) {
      a.okey_off[tot[0]] = uint32_t(tot[1]);
      a.oval_off[tot[0]] = uint32_t(tot[2]);
    }
    if (err) atomicOr(reinterpret_cast<unsigned long long*>(a.stats + 3), (unsigned long long)err);
  }
}

// Pieces of a lane's 16-B copy loop whose loads are all issued before their stores: a
// load -> store per piece waits out a full memory round trip every 16 bytes.
constexpr uint32_t kCopyB = 8;

// len (>= 16) bytes src -> dst by one lane as 16-B pieces (the last overlapping the one before),
// kCopyB loads in flight at a time.  Dst is global or LDS (generic pointer).
__device__ __forceinline__ void copy16_batched(uint8_t* dst, const uint8_t* src, uint32_t len) {
  const uint32_t np = (len + 15) >> 4;
  for (uint32_t b = 0; b < np; b += kCopyB) {
    u32x4 v[kCopyB];
#pragma unroll
    for (uint32_t i = 0; i < kCopyB; ++i) {
      const uint32_t p = min(16 * (b + i), len - 16);
      if (b + i < np) v[i] = *reinterpret_cast<const u32x4*>(src + p);
    }
#pragma unroll
    for (uint32_t i = 0; i < kCopyB; ++i) {
      const uint32_t p = min(16 * (b + i), len - 16);
      if (b + i < np) *reinterpret_cast<u32x4*>(dst + p) = v[i];
    }
  }
}

// Every lane's run [so, so + len) of sbase -> [dof, dof + len) of dbase (len >= 16 where
// `mine`; any alignment; dbase global or LDS) by the whole wave, packed: the runs' 16-B pieces
// are numbered over the lanes and lane l moves pieces l, l + 64, ..., kCopyB loads in flight,
// so neighbouring lanes read neighbouring pieces of one run.  Called by every lane of the wave.
__device__ __forceinline__ void wave_copy_packed(bool mine, const uint8_t* sbase, uint32_t so, uint8_t* dbase,
                                                 uint32_t dof, uint32_t len) {
  const uint32_t l = lane_id();
  const uint32_t np = mine ? (len + 15) >> 4 : 0u;
  const uint32_t incl = wave_incl_scan32(np);
  const uint32_t total = __builtin_amdgcn_readlane(incl, 63);
  const uint32_t first = incl - np;
  for (uint32_t g0 = 0; g0 < total; g0 += 64 * kCopyB) {
    u32x4 v[kCopyB];
    uint32_t d[kCopyB];
#pragma unroll
    for (uint32_t j = 0; j < kCopyB; ++j) {
      const uint32_t g = g0 + 64 * j + l, gg = min(g, total - 1);
      uint32_t lo = 0;  // owner: the last lane whose first piece number is <= gg
#pragma unroll
      for (uint32_t step = 32; step >= 1; step >>= 1) {
        const uint32_t f = uint32_t(__shfl(first, int((lo + step) & 63), 64));
        if (lo + step < 64 && f <= gg) lo += step;
      }
      const uint32_t o_so = uint32_t(__shfl(so, int(lo), 64)), o_dof = uint32_t(__shfl(dof, int(lo), 64));
      const uint32_t o_len = uint32_t(__shfl(len, int(lo), 64)), o_first = uint32_t(__shfl(first, int(lo), 64));
      const uint32_t off = min(16 * (gg - o_first), o_len - 16);
      d[j] = ~0u;
      if (g < total) {
        v[j] = *reinterpret_cast<const u32x4*>(sbase + o_so + off);
        d[j] = o_dof + off;
      }
    }
#pragma unroll
    for (uint32_t j = 0; j < kCopyB; ++j)
      if (d[j] != ~0u) *reinterpret_cast<u32x4*>(dbase + d[j]) = v[j];
  }
}

// len bytes src -> dst by one lane, any alignment: 16-B unaligned pieces, the last overlapping.
__device__ __forceinline__ void lane_copy(uint8_t* dst, const uint8_t* src, uint32_t len) {
  if (len < 16) {
    for (uint32_t x = 0; x < len; ++x) dst[x] = src[x];
    return;
  }
  copy16_batched(dst, src, len);
}

// len bytes from global src into the LDS image at dst (any alignment): 16-B pieces, the last
// overlapping the one before; shorter runs by overlapping 8/4-byte or single-byte stores.
__device__ __forceinline__ void lds_put(uint8_t* dst, const uint8_t* src, uint32_t len) {
  if (len >= 16) {
    copy16_batched(dst, src, len);
  } else if (len >= 8) {
    *reinterpret_cast<u32x2*>(dst) = *reinterpret_cast<const u32x2*>(src);
    *reinterpret_cast<u32x2*>(dst + len - 8) = *reinterpret_cast<const u32x2*>(src + len - 8);
  } else if (len >= 4) {
    *reinterpret_cast<uint32_t*>(dst) = *reinterpret_cast<const uint32_t*>(src);
    *reinterpret_cast<uint32_t*>(dst + len - 4) = *reinterpret_cast<const uint32_t*>(src + len - 4);
  } else {
    for (uint32_t x = 0; x < len; ++x) dst[x] = src[x];
  }
}

// LDS image [lo, lo + len) -> global bytes at gdst_aligned + lo (lo < 16): aligned 16-B stores,
// only the two edge chunks byte-masked.
__device__ __forceinline__ void flush_img(uint8_t* gdst_aligned, const uint8_t* img, uint32_t lo, uint32_t len) {
  flush_chunks<1>(gdst_aligned, img, lo, len, threadIdx.x, blockDim.x);
}

constexpr uint32_t kGKImg = 6144;   // LDS image of a round's keys
constexpr uint32_t kGVImg = 28672;  // LDS image of a round's values

// Kept entries in merged order -> the output stream.  Per round of 256 merged positions the
// kept keys and values form one contiguous output range each: lanes copy their entry's bytes
// into LDS images of those ranges, which are then flushed with aligned, coalesced 16-B stores
// (rounds whose ranges exceed the images copy lane by lane straight to global memory).
// The tile's four rounds load their entry metadata (keep -> perm -> offsets, ts) up front, so the
// tile waits out those two dependent round trips once instead of once per round: rounds that
// each waited keep -> perm -> offsets -> bytes held the kernel at about half the HBM rate.
// META: the kept entries' offsets, ts, same-key flags (and kidx); BYTES: their key and value
// bytes.  lsmblk_compact_batch runs the two halves apart (META first, then BYTES beside the SST
// rotation, which needs only the metadata); every other caller runs both in one launch.
template <bool META, bool BYTES>
__global__ __launch_bounds__(256) void mwrite_kernel(GatherArgs a) {
  if (a.stats[3]) return;
  const uint64_t N = *a.nm;
  constexpr uint32_t R = kGTile / 256;
  __shared__ uint64_t ws[R][4][3];
  __shared__ __attribute__((aligned(16))) uint8_t kimg[kGKImg + 32], vimg[kGVImg + 32];
  const uint32_t w = wave_id();
  const uint64_t j0 = uint64_t(blockIdx.x) * kGTile;
  if (j0 >= N) return;
  const uint32_t nr = uint32_t(min<uint64_t>(R, (N - j0 + 255) / 256));  // rounds holding entries
  uint32_t kf[R], ix[R], kso[R], kl[R], vso[R], vl[R];
  uint64_t tsv[R];
#pragma unroll
  for (uint32_t r = 0; r < R; ++r) {
    const uint64_t j = j0 + 256 * r + threadIdx.x;
    kf[r] = j < N ? a.keep[j] : 0u;
  }
#pragma unroll
  for (uint32_t r = 0; r < R; ++r) ix[r] = (kf[r] & 1u) ? a.perm[j0 + 256 * r + threadIdx.x] : 0u;
#pragma unroll
  for (uint32_t r = 0; r < R; ++r) {
    const bool k = kf[r] & 1u;
    const uint32_t i = ix[r];
    kso[r] = k ? a.key_off[i] : 0u;
    kl[r] = k ? a.key_off[i + 1] : 0u;
    vso[r] = k ? a.val_off[i] : 0u;
    vl[r] = k ? a.val_off[i + 1] : 0u;
    tsv[r] = k ? a.ts[i] : 0ull;
  }
  uint64_t o[R], ko[R], vo[R];
#pragma unroll
  for (uint32_t r = 0; r < R; ++r) {
    const bool k = kf[r] & 1u;
    kl[r] -= kso[r];
    vl[r] -= vso[r];
    const uint32_t ic = wave_incl_scan32(k ? 1u : 0u);
    const uint64_t ik = wave_incl_scan<uint64_t>(kl[r]), iv = wave_incl_scan<uint64_t>(vl[r]);
    if (lane_id() == 63) ws[r][w][0] = ic, ws[r][w][1] = ik, ws[r][w][2] = iv;
    o[r] = ic - 1;
    ko[r] = ik - kl[r];
    vo[r] = iv - vl[r];
  }
  __syncthreads();
  const uint64_t gp = blockIdx.x / kGScan;
  uint64_t carry[3] = {a.tile_pre[3 * uint64_t(blockIdx.x)] + a.part_pre[3 * gp],
                       a.tile_pre[3 * uint64_t(blockIdx.x) + 1] + a.part_pre[3 * gp + 1],
                       a.tile_pre[3 * uint64_t(blockIdx.x) + 2] + a.part_pre[3 * gp + 2]};
  uint64_t K0[R + 1], V0[R + 1];
#pragma unroll
  for (uint32_t r = 0; r < R; ++r) {
    uint64_t b[3] = {carry[0], carry[1], carry[2]};
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
      if (q < w) b[0] += ws[r][q][0], b[1] += ws[r][q][1], b[2] += ws[r][q][2];
    }
    o[r] += b[0];
    ko[r] += b[1];
    vo[r] += b[2];
    K0[r] = carry[1];
    V0[r] = carry[2];
#pragma unroll
    for (uint32_t q = 0; q < 3; ++q) carry[q] += ws[r][0][q] + ws[r][1][q] + ws[r][2][q] + ws[r][3][q];
    if (META && (kf[r] & 1u)) {
      a.okey_off[o[r]] = uint32_t(ko[r]);
      a.oval_off[o[r]] = uint32_t(vo[r]);
      a.ots[o[r]] = tsv[r];
      if (a.ksame) a.ksame[o[r]] = uint8_t(kf[r] >> 1);
      if (a.kidx) a.kidx[o[r]] = ix[r];
    }
  }
  if (!BYTES) return;
  K0[R] = carry[1];
  V0[R] = carry[2];
  // the copy rounds, not unrolled (each round's copy loop holds 8 x 16 B of loads per lane):
  // round r's values sit in slot 0, the slots shifting down after every round
#pragma unroll 1
  for (uint32_t r = 0; r < nr; ++r) {
    const bool k = kf[0] & 1u;
    const uint32_t kb = uint32_t(K0[0] & 15), vb = uint32_t(V0[0] & 15);
    const bool staged = K0[1] - K0[0] + kb <= kGKImg && V0[1] - V0[0] + vb <= kGVImg;
    if (staged) {
      // runs of 16 B or more by the whole wave, packed; shorter ones lane by lane
      const uint32_t kd = kb + uint32_t(ko[0] - K0[0]), vd = vb + uint32_t(vo[0] - V0[0]);
      if (k && kl[0] < 16) lds_put(kimg + kd, a.keys + kso[0], kl[0]);
      if (k && vl[0] < 16) lds_put(vimg + vd, a.vals + vso[0], vl[0]);
      wave_copy_packed(k && kl[0] >= 16, a.keys, kso[0], kimg, kd, kl[0]);
      wave_copy_packed(k && vl[0] >= 16, a.vals, vso[0], vimg, vd, vl[0]);
      __syncthreads();
      flush_img(a.okeys + (K0[0] - kb), kimg, kb, uint32_t(K0[1] - K0[0]));
      flush_img(a.ovals + (V0[0] - vb), vimg, vb, uint32_t(V0[1] - V0[0]));
      __syncthreads();
    } else if (k) {
      lane_copy(a.okeys + ko[0], a.keys + kso[0], kl[0]);
      lane_copy(a.ovals + vo[0], a.vals + vso[0], vl[0]);
    }
#pragma unroll
    for (uint32_t q = 0; q + 1 < R; ++q) {
      kf[q] = kf[q + 1], kso[q] = kso[q + 1], kl[q] = kl[q + 1], vso[q] = vso[q + 1], vl[q] = vl[q + 1];
      ko[q] = ko[q + 1], vo[q] = vo[q + 1];
    }
#pragma unroll
    for (uint32_t q = 0; q < R; ++q) K0[q] = K0[q + 1], V0[q] = V0[q + 1];
  }
}

__global__ void merge_empty_kernel(uint64_t* mstats, uint32_t* okey_off, uint32_t* oval_off, uint64_t entry_cap,
                                   uint64_t* stats) {
  if (threadIdx.x == 0) {
    mstats[0] = mstats[1] = mstats[3] = mstats[5] = 0;  // (workspace: no stale error word for gate_kernel)
    if (entry_cap + 1 > 0 && okey_off) {
      okey_off[0] = 0;
      oval_off[0] = 0;
    }
    stats[0] = stats[1] = stats[2] = 0;
  }
}

// ---------------------------------------------------------------- SST rotation
// compact_generate_sst starts a new SST before adding entry e when the open SsTableBuilder's
// estimate_size() >= target_sst_size and key(e) differs from the last key (src/compact.rs:278-289).
// estimate_size() is data.len(): the finished blocks plus their 4-byte CRCs
// (src/table/builder.rs:105-123), so it grows only when a block is finished -- while adding the
// first entry of the next block.  With blocks j = [s_j, s_{j+1}) of an SST starting at g and
// D_j = sum over i < j of (size_i + 4), the check at entry e in (s_j, s_{j+1}] sees D_j; the SST
// therefore ends at F(g) = the first key change after s_{j*}, j* = min{ j : D_j >= target }.
// F depends on the greedy packing from g only, so it is computed for EVERY entry g in
// parallel, by pointer doubling over nxt(s) = the greedy end of a block starting at s:
//   rot_adj_kernel     rec = klen + vlen, alcp = LCP with the predecessor (+ unsorted / same-key
//                      bits), as plan_adj_kernel
//   rot_next_kernel    J0[s] = nxt(s), S0[s] = size of block [s, nxt(s)) + 4 (LCP against the
//                      block's first key = running min of alcp for sorted keys, direct
//                      compares after an unsorted pair; BlockBuilder::add's reject rule)
//   rot_double_kernel  J_k = J_{k-1} o J_{k-1}, S_k = S_{k-1} + S_{k-1} o J_{k-1} (until every
//                      chain reaches the target or the end)
//   rot_f_kernel       F(g) by binary lifting over the levels, then the next key change
//   rot_chain_kernel   the SST chain 0, F(0), F(F(0)), ... by doubling F (level k appends
//                      chain elements [2^k, 2^(k+1)) and squares F), for K levels; then
//   rot_walk_kernel    one lane: every 2^K-th chain element through F^(2^K), and
//   rot_fill_kernel    one thread per such anchor: the 2^K - 1 elements after it through F
//   rot_finish_kernel  sst_start[] and the SST count.
// The kept stream's versions of a key must be newest first (as MergeIterator yields SST data);
// then "same as last key" is "same key as the previous kept entry" (DESIGN.md).
constexpr uint32_t kRotSame = 0x40000000u;      // alcp bit: key equals the predecessor's
constexpr uint32_t kRotUnsorted = 0x80000000u;  // alcp bit: predecessor's key is greater
constexpr uint32_t kRotLcp = 0x3FFFFFFFu;
constexpr uint32_t kRotMaxLevels = 32;

struct RotArgs {
  const uint8_t* keys;
  const uint32_t* key_off;
  const uint32_t* val_off;
  const uint64_t* dn;       // device: entries of the stream
  uint64_t n_max;           // grid bound
  uint32_t block_size;
  uint64_t target;
  uint32_t* rec;            // n_max + 1
  uint32_t* alcp;           // n_max + 1
  u32x2* JS;                // levels x (n_max + 1): {J_k[s], S_k[s]} side by side, so a doubling
                            // step gathers both with one 8-B load (two 4-B gathers cost two sectors)
  uint32_t levels;          // levels allocated for J / S
  uint32_t* F0;             // n_max + 1: F (kept for the chain's fill)
  uint32_t* F1;             // n_max + 1 each: the doubling ping-pong F^(2^k)
  uint32_t* F2;
  uint32_t* need;           // kRotMaxLevels: level k still has a chain short of target and end
  uint32_t* chain_end;      // [0] set once the SST chain reached the end
  uint32_t* rerr;           // [0] error flags of the lifting walks (a chain link that does not advance)
  uint32_t poison;          // diagnostics (LSMBLK_DEBUG_ROT_POISON): corrupt the levels before the lifting
  uint32_t* starts;         // sst_cap: SST start entries (the chain), then n
  uint32_t sst_cap;
  uint32_t* nsst;           // device: SST count handed to the encode (0 after an error)
  uint64_t* stats;          // [0] SSTs [3] error flags
  // key-range shard (lsmblk_shard_*): the stream is the range's own m entries, then the halo
  uint64_t m;
  uint32_t shard_last;      // the stream ends where the whole compaction's stream ends
  uint32_t* FL;             // flevels x (n_max + 1): F^(2^k); level 0 is F
  uint32_t flevels;
  uint64_t* sstate;         // kShardWords: the carry step's result
  const uint8_t* ksame;     // two-level merge: same_as_last_key per entry from the rules loop
                            // (null: a key equal to its predecessor's)
  // lsmblk_compact_batch: the kept stream's key bytes are written beside the rotation, so rot_adj
  // reads each kept key in the merge input instead: kidx[e] = its input index, k16 = the input
  // keys' first 16 bytes, akeys / akey_off = the input key arena (kidx null: the kept stream)
  const uint32_t* kidx;
  const u32x4* k16;
  const uint8_t* akeys;
  const uint32_t* akey_off;
  uint64_t an;              // input entries
};

// sstate words
constexpr uint32_t kShP = 0, kShE1 = 1, kShCnt = 2, kShEnd = 3, kShD0 = 4, kShDout = 5, kShErr = 6, kShSegs = 7;
constexpr uint32_t kShardWords = 16;  // [8, 12): the encode's stats

__device__ __forceinline__ uint64_t rot_n(const RotArgs& a) { return uni64(*a.dn); }

// LCP of keys (pp, pl) and (kp, kl) through the descriptor; *less = key p < key k (byte order)
__device__ __forceinline__ uint32_t glcp(const GKeys& K, uint32_t pp, uint32_t pl, uint32_t kp, uint32_t kl,
                                         int* order) {
  const uint32_t m = pl < kl ? pl : kl;
  for (uint32_t i = 0; i < m; i += 4) {
    uint32_t x = K.dw(pp + i), y = K.dw(kp + i);
    if (m - i < 4) {
      const uint32_t mk = (1u << (8 * (m - i))) - 1;
      x &= mk;
      y &= mk;
    }
    if (x != y) {
      const uint32_t z = __builtin_ctz(x ^ y) & ~7u;
      if (order) *order = ((x >> z) & 0xFF) < ((y >> z) & 0xFF) ? -1 : 1;
      return i + (z >> 3);
    }
  }
  if (order) *order = pl < kl ? -1 : (pl > kl ? 1 : 0);
  return m;
}

// LCP of two keys from their first 16 bytes (big-endian words, zero padded) and, past a tie on
// those, the tails at arena positions pp / kp; *order as glcp's (the first key against the second).
__device__ __forceinline__ uint32_t lcp_k16(const GKeys& G, const u32x4& x, uint32_t pp, uint32_t pl, const u32x4& y,
                                          uint32_t kp, uint32_t kl, int* order) {
  const uint32_t m = pl < kl ? pl : kl;
  const uint32_t xs[4] = {x.x, x.y, x.z, x.w}, ys[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
  for (uint32_t w = 0; w < 4; ++w) {
    if (xs[w] != ys[w]) {
      const uint32_t z = 4 * w + (__builtin_clz(xs[w] ^ ys[w]) >> 3);
      if (z < m) {
        const uint32_t sh = 24 - 8 * (z & 3);
        *order = ((xs[w] >> sh) & 0xFF) < ((ys[w] >> sh) & 0xFF) ? -1 : 1;
        return z;
      }
      *order = pl < kl ? -1 : (pl > kl ? 1 : 0);  // (a zero pad against a key byte)
      return m;
    }
  }
  if (m <= 16) {
    *order = pl < kl ? -1 : (pl > kl ? 1 : 0);
    return m;
  }
  return 16 + glcp(G, pp + 16, pl - 16, kp + 16, kl - 16, order);
}

__global__ __launch_bounds__(256) void rot_adj_kernel(RotArgs a) {
  const uint64_t n = rot_n(a);
  const uint32_t t = threadIdx.x;
  const uint64_t e = uint64_t(blockIdx.x) * 256 + t;
  if (a.kidx) {
    // The kept keys through the merge input (see RotArgs).  Every thread loads its own entry's
    // input index, key length and first 16 key bytes once and takes its predecessor's from the
    // neighbouring thread through LDS (thread 0 loads its predecessor): half the gathers of
    // loading both per thread.  The key arena positions are loaded only for a tie on 16 bytes.
    __shared__ u32x4 s16[256];
    __shared__ uint32_t sidx[256], slen[256];
    uint32_t i = 0, kl = 0, vl = 0;
    u32x4 x16{0u, 0u, 0u, 0u};
    if (e < n) {
      const uint32_t kp = a.key_off[e];
      kl = a.key_off[e + 1] - kp;
      vl = a.val_off[e + 1] - a.val_off[e];
      i = a.kidx[e];
      x16 = a.k16[i];
    }
    s16[t] = x16;
    sidx[t] = i;
    slen[t] = kl;
    __syncthreads();
    if (e >= n) return;
    a.rec[e] = kl + vl;
    uint32_t al = 0;
    if (e > 0) {
      uint32_t ip, pl;
      u32x4 p16;
      if (t > 0) {
        ip = sidx[t - 1];
        pl = slen[t - 1];
        p16 = s16[t - 1];
      } else {
        ip = a.kidx[e - 1];
        pl = a.key_off[e] - a.key_off[e - 1];
        p16 = a.k16[ip];
      }
      const GKeys K = gkeys(a.akeys, a.akey_off[a.an]);
      const bool tie = pl > 16 && kl > 16 && p16.x == x16.x && p16.y == x16.y && p16.z == x16.z && p16.w == x16.w;
      int ord = 0;
      const uint32_t lcp = lcp_k16(K, p16, tie ? a.akey_off[ip] : 0u, pl, x16, tie ? a.akey_off[i] : 0u, kl, &ord);
      const bool same = a.ksame ? a.ksame[e] != 0 : ord == 0;
      al = (lcp < kRotLcp ? lcp : kRotLcp) | (ord > 0 ? kRotUnsorted : 0u) | (same ? kRotSame : 0u);
    }
    a.alcp[e] = al;
    return;
  }
  if (e >= n) return;
  const uint32_t kp = a.key_off[e], kl = a.key_off[e + 1] - kp;
  a.rec[e] = kl + (a.val_off[e + 1] - a.val_off[e]);
  uint32_t al = 0;
  if (e > 0) {
    const GKeys K = gkeys(a.keys, a.key_off[n]);
    const uint32_t pp = a.key_off[e - 1], pl = kp - pp;
    int ord = 0;
    const uint32_t lcp = glcp(K, pp, pl, kp, kl, &ord);
    const bool same = a.ksame ? a.ksame[e] != 0 : ord == 0;
    al = (lcp < kRotLcp ? lcp : kRotLcp) | (ord > 0 ? kRotUnsorted : 0u) | (same ? kRotSame : 0u);
  }
  a.alcp[e] = al;
}

// Raise a level flag: one atomic per wave at most, none once the flag reads as set (hundreds
// of thousands of waves OR-ing one word serialise at the memory side, ~12 ns each).
__device__ __forceinline__ void or_need(uint32_t* flag, bool v) {
  if (__ballot(v) && lane_id() == 0 && !__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
    atomicOr(flag, 1u);
}

// The workgroup's starts [s0, s0 + 256) walk at most a block's worth of entries past them
// (each entry after the first grows the block by >= 16 bytes): (rec, alcp) of [s0, s0 + 256 +
// kRotWin) are staged in LDS once, coalesced, instead of every lane re-reading its ~30 successors
// from L2; a walk past the window (blocks over 8 KiB) reads global memory.
constexpr uint32_t kRotWin = 512;
constexpr uint32_t kRotStep = 4;

__global__ __launch_bounds__(256) void rot_next_kernel(RotArgs a) {
  __shared__ uint32_t srec[256 + kRotWin], salcp[256 + kRotWin];
  const uint64_t n = rot_n(a);
  const uint64_t s0 = uint64_t(blockIdx.x) * 256, s = s0 + threadIdx.x;
  for (uint32_t i = threadIdx.x; i < 256 + kRotWin; i += 256) {
    const uint64_t e = s0 + i;
    srec[i] = e < n ? a.rec[e] : 0u;
    salcp[i] = e < n ? a.alcp[e] : 0u;
  }
  __syncthreads();
  bool short_chain = false;
  if (s < n) {
    const uint64_t bs = a.block_size;
    uint64_t before = 2 + uint64_t(srec[threadIdx.x]) + 16;  // entry s always accepted, prefix 0
    uint32_t pmin = kRotLcp;
    bool direct = false, stop = false;
    uint32_t sp = 0, sl = 0;
    GKeys K;
    uint64_t e = s + 1;
    // Fast walk: sorted pairs inside the LDS window, kRotStep entries' (rec, alcp) read ahead of
    // their use.  (A loop reading `in window ? LDS : global` was if-converted into a global load
    // per entry as well, and each entry's LDS read waited for the previous entry's update.)
    const uint64_t wend = min(n, s0 + 256 + kRotWin);
    for (bool slow = false; !stop && !slow && e + kRotStep <= wend;) {
      uint32_t r[kRotStep], al[kRotStep];
#pragma unroll
      for (uint32_t j = 0; j < kRotStep; ++j) {
        r[j] = srec[e - s0 + j];
        al[j] = salcp[e - s0 + j];
      }
#pragma unroll
      for (uint32_t j = 0; j < kRotStep; ++j) {
        if (stop || slow) continue;
        if (before + r[j] + 14 > bs) {
          stop = true;  // BlockBuilder::add rejects (builder.rs:56-60)
        } else if (al[j] & kRotUnsorted) {
          slow = true;  // the general loop compares against the first key from here on
        } else {
          pmin = min(pmin, al[j] & kRotLcp);
          before += uint64_t(r[j]) + 16 - pmin;
          ++e;
        }
      }
    }
    // General walk: the window's last entries, past the window, and direct compares after an
    // unsorted pair.
    for (; !stop && e < n; ++e) {
      const uint64_t x = e - s0;
      const bool in = x < 256 + kRotWin;
      uint32_t r, al;
      if (in) {
        r = srec[x];
        al = salcp[x];
      } else {
        r = a.rec[e];
        al = a.alcp[e];
      }
      if (before + r + 14 > bs) break;  // BlockBuilder::add rejects (builder.rs:56-60)
      uint32_t p;
      if (!direct && (al & kRotUnsorted)) {  // LCP vs the first key directly from here on
        direct = true;
        K = gkeys(a.keys, a.key_off[n]);
        sp = a.key_off[s];
        sl = a.key_off[s + 1] - sp;
      }
      if (!direct) {
        pmin = min(pmin, al & kRotLcp);
        p = pmin;
      } else {
        const uint32_t kp = a.key_off[e];
        p = glcp(K, sp, sl, kp, a.key_off[e + 1] - kp, nullptr);
      }
      before += uint64_t(r) + 16 - p;
    }
    const uint64_t sz = before + 4;
    a.JS[s] = u32x2{uint32_t(e), sz > 0xFFFFFFFFull ? 0xFFFFFFFFu : uint32_t(sz)};
    short_chain = e < n && sz < a.target;
  } else if (s == n) {
    a.JS[s] = u32x2{uint32_t(n), 0u};
  }
  or_need(a.need + 0, short_chain);
}

// kRotPer entries per thread (a block-stride apart, so each round stays coalesced): all their
// loads are in flight together -- one entry per thread left the kernel latency-bound.
constexpr uint32_t kRotPer = 4;

__global__ __launch_bounds__(256) void rot_double_kernel(RotArgs a, uint32_t k) {
  if (!*(volatile uint32_t*)(a.need + k - 1)) return;  // every chain done one level down
  const uint64_t n = rot_n(a);
  // (XCD-aware tile order: the gathers J_{k-1}(s) land a few tiles ahead, on the same XCD, whose
  // L2 then serves both them and that tile's own linear read -- 1.84 -> 1.61 ms on config C; the
  // same order made rot_next and rot_f slower, 0.55 -> 0.62 and 0.54 -> 0.57 ms)
  const uint64_t s0 = uint64_t(xcd_tile(blockIdx.x, gridDim.x)) * 256 * kRotPer + threadIdx.x;
  const uint64_t N1 = a.n_max + 1;
  const u32x2* L0 = a.JS + (k - 1) * N1;
  bool short_chain = false;
  u32x2 v[kRotPer], w[kRotPer];
#pragma unroll
  for (uint32_t i = 0; i < kRotPer; ++i) {
    const uint64_t s = s0 + 256 * i;
    v[i] = s <= n ? L0[s] : u32x2{0u, 0u};
  }
#pragma unroll
  for (uint32_t i = 0; i < kRotPer; ++i) {
    const uint64_t s = s0 + 256 * i;
    w[i] = s <= n ? L0[v[i].x] : u32x2{0u, 0u};
  }
#pragma unroll
  for (uint32_t i = 0; i < kRotPer; ++i) {
    const uint64_t s = s0 + 256 * i;
    if (s <= n) {
      const uint64_t ss = uint64_t(v[i].y) + w[i].y;
      a.JS[k * N1 + s] = u32x2{w[i].x, ss > 0xFFFFFFFFull ? 0xFFFFFFFFu : uint32_t(ss)};
      short_chain = short_chain || (w[i].x < n && ss < a.target);
    }
  }
  or_need(a.need + k, short_chain);
}

// Levels k and k + 1 from level k - 1 in one pass: J_k(s) = J_{k-1}(J_{k-1}(s)) and J_{k+1}(s) =
// J_k(J_k(s)) = J_{k-1}^4(s) -- one linear read and three dependent gathers of level k - 1 (the
// later gathers land a few tiles ahead, mostly in L2) instead of two passes that each read,
// gather and write a whole level.  need[k] / need[k + 1] as two rot_double_kernel passes would set
// them (no short chain at level k means none at k + 1: the rot_top walk never reads past it).
__global__ __launch_bounds__(256) void rot_double2_kernel(RotArgs a, uint32_t k) {
  if (!*(volatile uint32_t*)(a.need + k - 1)) return;  // every chain done one level down
  const uint64_t n = rot_n(a);
  const uint64_t s0 = uint64_t(xcd_tile(blockIdx.x, gridDim.x)) * 256 * kRotPer + threadIdx.x;
  const uint64_t N1 = a.n_max + 1;
  const u32x2* L0 = a.JS + (k - 1) * N1;
  auto sat = [](uint64_t v) { return v > 0xFFFFFFFFull ? 0xFFFFFFFFu : uint32_t(v); };
  bool short1 = false, short2 = false;
  u32x2 v[kRotPer], w[kRotPer], y[kRotPer], z[kRotPer];
#pragma unroll
  for (uint32_t i = 0; i < kRotPer; ++i) {
    const uint64_t s = s0 + 256 * i;
    v[i] = s <= n ? L0[s] : u32x2{0u, 0u};
  }
#pragma unroll
  for (uint32_t i = 0; i < kRotPer; ++i) w[i] = s0 + 256 * i <= n ? L0[v[i].x] : u32x2{0u, 0u};
#pragma unroll
  for (uint32_t i = 0; i < kRotPer; ++i) y[i] = s0 + 256 * i <= n ? L0[w[i].x] : u32x2{0u, 0u};
#pragma unroll
  for (uint32_t i = 0; i < kRotPer; ++i) z[i] = s0 + 256 * i <= n ? L0[y[i].x] : u32x2{0u, 0u};
#pragma unroll
  for (uint32_t i = 0; i < kRotPer; ++i) {
    const uint64_t s = s0 + 256 * i;
    if (s <= n) {
      const uint64_t s1 = uint64_t(v[i].y) + w[i].y;                // S_k(s)
      const uint64_t s2 = s1 + uint64_t(y[i].y) + z[i].y;          // S_k(s) + S_k(J_k(s))
      a.JS[k * N1 + s] = u32x2{w[i].x, sat(s1)};
      a.JS[(k + 1) * N1 + s] = u32x2{z[i].x, sat(s2)};
      short1 = short1 || (w[i].x < n && s1 < a.target);
      short2 = short2 || (z[i].x < n && s2 < a.target);
    }
  }
  or_need(a.need + k, short1);
  or_need(a.need + k + 1, short2);
}

// Highest block-chain level computed (J / S levels 0 .. top).// Highest block-chain level computed (J / S levels 0 .. top).
__device__ __forceinline__ uint32_t rot_top(const RotArgs& a) {
  uint32_t kc = 1;
  while (kc < a.levels && a.need[kc - 1]) ++kc;
  return kc - 1;
}

// Lifting from block start pos with acc bytes of data section: the longest block chain prefix
// whose data stays below the target.  Returns its last block start (acc updated).
// Every chain link advances (J_k(s) > s for s < n): a link that does not -- corrupt or stale
// levels -- ends the walk with LSMBLK_ERR_INTERNAL instead of looping (each walk is then at most
// n steps).
__device__ __forceinline__ uint64_t lift_target(const RotArgs& a, uint64_t pos, uint64_t& acc, uint64_t n,
                                                uint32_t top, uint64_t& err) {
  const uint64_t N1 = a.n_max + 1;
  while (pos < n) {
    const u32x2 v = a.JS[top * N1 + pos];
    if (acc + v.y >= a.target) break;
    if (v.x <= pos) {
      err |= LSMBLK_ERR_INTERNAL;
      break;
    }
    acc += v.y;
    pos = v.x;
  }
  for (int k = int(top) - 1; k >= 0; --k) {
    if (pos < n) {
      const u32x2 v = a.JS[uint64_t(k) * N1 + pos];
      if (acc + v.y < a.target) {
        acc += v.y;
        pos = v.x;
      }
    }
  }
  return pos;
}

// Lifting from block start pos < bound: the last block start below bound in its chain (acc
// updated with the data of the blocks passed).
__device__ __forceinline__ uint64_t lift_before(const RotArgs& a, uint64_t pos, uint64_t& acc, uint64_t bound,
                                                uint32_t top, uint64_t& err) {
  const uint64_t N1 = a.n_max + 1;
  for (;;) {
    const u32x2 v = a.JS[top * N1 + pos];
    if (v.x >= bound) break;
    if (v.x <= pos) {  // (a link that does not advance: see lift_target)
      err |= LSMBLK_ERR_INTERNAL;
      break;
    }
    acc += v.y;
    pos = v.x;
  }
  for (int k = int(top) - 1; k >= 0; --k) {
    const u32x2 v = a.JS[uint64_t(k) * N1 + pos];
    if (v.x < bound) {
      acc += v.y;
      pos = v.x;
    }
  }
  return pos;
}

// The SST end after the block start sj whose entries first see D >= target: the first key
// change after sj (n when none).
__device__ __forceinline__ uint64_t key_change_after(const RotArgs& a, uint64_t sj, uint64_t n) {
  if (sj >= n) return n;
  uint64_t f = sj + 1;
  while (f < n && (a.alcp[f] & kRotSame)) ++f;
  return f;
}

// Two entries per thread, lifted in lockstep (their gathers in flight together): the lifting
// is a chain of ~levels dependent gathers per entry.
__global__ __launch_bounds__(256) void rot_f_kernel(RotArgs a) {
  const uint64_t n = rot_n(a);
  const uint64_t g0 = uint64_t(blockIdx.x) * 512 + threadIdx.x, g1 = g0 + 256;
  const uint32_t top = rot_top(a);
  const uint64_t N1 = a.n_max + 1;
  // lifting: the longest chain prefix from g whose data stays below the target
  uint64_t p0 = g0, p1 = g1, c0 = 0, c1 = 0;
  bool stuck = false;
  for (;;) {  // top level, repeated while it fits (every move advances: at most n moves)
    bool m0 = false, m1 = false;
    u32x2 v0{0u, 0u}, v1{0u, 0u};
    if (p0 < n) v0 = a.JS[top * N1 + p0];
    if (p1 < n) v1 = a.JS[top * N1 + p1];
    if (p0 < n && c0 + v0.y < a.target) {
      stuck = stuck || v0.x <= p0;
      c0 += v0.y, p0 = v0.x, m0 = true;
    }
    if (p1 < n && c1 + v1.y < a.target) {
      stuck = stuck || v1.x <= p1;
      c1 += v1.y, p1 = v1.x, m1 = true;
    }
    if ((!m0 && !m1) || stuck) break;
  }
  if (stuck) atomicOr(a.rerr, LSMBLK_ERR_INTERNAL);  // (a link that does not advance: lift_target)
  for (int k = int(top) - 1; k >= 0; --k) {
    u32x2 v0{0u, 0u}, v1{0u, 0u};
    if (p0 < n) v0 = a.JS[uint64_t(k) * N1 + p0];
    if (p1 < n) v1 = a.JS[uint64_t(k) * N1 + p1];
    if (p0 < n && c0 + v0.y < a.target) c0 += v0.y, p0 = v0.x;
    if (p1 < n && c1 + v1.y < a.target) c1 += v1.y, p1 = v1.x;
  }
  // s_{j*}: the first block start whose entries see D >= target
  if (g0 < n) a.F0[g0] = uint32_t(p0 < n ? key_change_after(a, a.JS[p0].x, n) : n);
  else if (g0 == n) a.F0[g0] = uint32_t(n);
  if (g1 < n) a.F0[g1] = uint32_t(p1 < n ? key_change_after(a, a.JS[p1].x, n) : n);
  else if (g1 == n) a.F0[g1] = uint32_t(n);
}

// Fault injection (LSMBLK_DEBUG_ROT_POISON, diagnostics builds): every level's link of the entries
// in [n/3, 2n/3) made a self-loop of size 0 -- the shape a stale or raced level would have.
__global__ __launch_bounds__(256) void rot_poison_kernel(RotArgs a) {
  const uint64_t n = rot_n(a), N1 = a.n_max + 1;
  const uint64_t s = n / 3 + uint64_t(blockIdx.x) * 256 + threadIdx.x;
  if (s >= 2 * n / 3) return;
  for (uint32_t k = 0; k < a.levels; ++k) a.JS[k * N1 + s] = u32x2{uint32_t(s), 0u};
}

// ---------------------------------------------------------------- key-range shard rotation
// Range r of a compaction split by user key holds the merged stream's entries [m_0, m_1); its
// rotation stream is those m entries followed by the halo (the next entries of the whole stream,
// enough to finish any block that starts before m).  Everything above is independent of the state
// the whole-stream rotation is in when it reaches the range, so it runs on every rank at once;
// only that state -- carry {p, D}: the open SST's next block starts at entry p (relative to the
// range), its data section holds D bytes there -- passes from rank to rank, and each rank turns its
// carry-in into its carry-out with a few dozen dependent loads:
//   E1 = the open SST's end: the first key change after the block start whose entries first see
//        D >= target (lifting from p with acc = D; p itself when D >= target already)
//   SSTs starting in the range: E1, F(E1), ... while < m, counted by lifting over F^(2^k)
//   the last SST (or the carried one) either ends exactly at m (a key change: ranges split at user
//   keys) -> carry-out {0, 0}, or continues: its block chain crosses m at block start b with data
//   D_b -> carry-out {b - m, D_b}; the crossing block is this rank's (it reads the halo).
// The rank's segments [p, E1, F(E1), ..., end) then encode exactly the whole stream's blocks.
__global__ __launch_bounds__(256) void rot_flev_kernel(RotArgs a, uint32_t k) {
  const uint64_t n = rot_n(a);
  const uint64_t s = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  if (s > n) return;
  const uint64_t N1 = a.n_max + 1;
  const uint32_t* F = a.FL + uint64_t(k - 1) * N1;
  a.FL[uint64_t(k) * N1 + s] = F[F[s]];
}

__global__ void shard_carry_kernel(RotArgs a, const uint64_t* cin, uint64_t* cout) {
  if (threadIdx.x) return;
  const uint64_t n = rot_n(a), m = a.m, N1 = a.n_max + 1;
  const uint32_t top = rot_top(a);
  const uint64_t p = cin[0], D0 = cin[1];
  uint64_t err = *a.rerr, E1 = m, cnt = 0, end = m, pout = 0, Dout = 0, segs = 0;
  // the range must end at a key change (all versions of a user key on one rank)
  if (m > 0 && m < n && (a.alcp[m] & kRotSame)) err |= LSMBLK_ERR_SEGMENTS;
  if (p >= m) {  // the crossing block from an earlier rank covers the whole range
    pout = p - m;
    Dout = D0;
    end = m;
  } else {
    uint64_t sj = p;
    if (D0 < a.target) {
      uint64_t acc = D0;
      const uint64_t pos = lift_target(a, p, acc, n, top, err);
      sj = pos < n ? a.JS[pos].x : n;
    }
    E1 = key_change_after(a, sj, n);
    uint64_t x = p, accx = D0, fl = E1;
    if (E1 < m) {  // SSTs start in the range: E1 and its successors below m
      x = E1;
      cnt = 1;
      for (int k = int(a.flevels) - 1; k >= 0; --k) {
        const uint32_t y = a.FL[uint64_t(k) * N1 + x];
        if (y < m) {
          x = y;
          cnt += 1ull << k;
        }
      }
      fl = a.FL[x];
      if (fl < m) err |= LSMBLK_ERR_CAPACITY;  // more SSTs than the levels cover
      accx = 0;
    }
    segs = cnt + 1;
    if (fl == m) {  // the last SST ends where the next range starts (or the stream ends)
      end = m;
    } else {        // it continues: its block chain crosses m
      const uint64_t pos = lift_before(a, x, accx, m, top, err);
      const u32x2 v = a.JS[pos];
      const uint64_t b = v.x;
      if (b >= n && !a.shard_last) err |= LSMBLK_ERR_SEGMENTS;  // the halo is too short
      end = b;
      pout = b - m;
      Dout = b >= n ? 0 : accx + v.y;  // the whole stream ends inside this SST: nothing continues
    }
  }
  uint64_t* w = a.sstate;
  w[kShP] = p;
  w[kShE1] = E1;
  w[kShCnt] = cnt;
  w[kShEnd] = end;
  w[kShD0] = D0;
  w[kShDout] = Dout;
  w[kShErr] = err;
  w[kShSegs] = err ? 0 : segs;
  cout[0] = pout;
  cout[1] = Dout;
}

// Segment table of the range: [p, E1, F(E1), ..., end), then `end` up to seg_cap.
__global__ __launch_bounds__(256) void shard_seg_kernel(RotArgs a, uint32_t* seg, uint32_t seg_cap,
                                                        uint32_t* nseg) {
  const uint64_t* w = a.sstate;
  const uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  uint64_t segs = w[kShSegs];
  if (segs + 1 > seg_cap) segs = 0;
  const uint64_t N1 = a.n_max + 1;
  if (i == 0) {
    *nseg = uint32_t(segs);
    if (w[kShSegs] + 1 > seg_cap) atomicOr(reinterpret_cast<unsigned long long*>(a.sstate + kShErr),
                                           (unsigned long long)LSMBLK_ERR_CAPACITY);
  }
  if (i >= seg_cap) return;
  if (segs == 0) {
    seg[i] = uint32_t(w[kShEnd]);
    return;
  }
  if (i == 0) {
    seg[0] = uint32_t(w[kShP]);
  } else if (i < segs) {  // chain element i - 1 = F^(i-1)(E1)
    uint64_t x = w[kShE1];
    const uint64_t q = i - 1;
    for (uint32_t k = 0; k < a.flevels; ++k)
      if ((q >> k) & 1) x = a.FL[uint64_t(k) * N1 + x];
    seg[i] = uint32_t(x);
  } else {
    seg[i] = uint32_t(w[kShEnd]);
  }
}

__global__ void shard_stats_kernel(uint64_t* stats, const uint64_t* est, const uint64_t* w) {
  if (threadIdx.x) return;
  const uint64_t err = est[3] | w[kShErr];
  const uint64_t segs = w[kShSegs];
  stats[0] = err ? 0 : est[0];
  stats[1] = err ? 0 : est[1];
  stats[2] = err ? 0 : segs;
  stats[3] = err;
  stats[4] = segs && w[kShD0] > 0;
  stats[5] = segs && w[kShDout] > 0;
  stats[6] = w[kShP];
  stats[7] = w[kShEnd];
}

// Level k: chain elements [2^k, 2^(k+1)) from [0, 2^k) through F^(2^k) (= cur), then
// nxt = cur o cur.  Skipped once the chain has reached the end.
__global__ __launch_bounds__(256) void rot_chain_kernel(RotArgs a, uint32_t k, const uint32_t* cur, uint32_t* nxt) {
  if (*(volatile uint32_t*)a.chain_end) return;
  const uint64_t n = rot_n(a);
  const uint64_t s = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  const uint64_t h = 1ull << k;
  if (s < h && h + s < a.sst_cap) {
    const uint32_t c = a.starts[s];
    a.starts[h + s] = c < n ? cur[c] : uint32_t(n);
  }
  if (nxt && s <= n) nxt[s] = cur[cur[s]];
}

// After each level: has the last chain element computed so far reached the end?
__global__ void rot_chain_check_kernel(RotArgs a, uint32_t k) {
  if (threadIdx.x || *(volatile uint32_t*)a.chain_end) return;
  const uint64_t n = rot_n(a);
  const uint64_t last = (2ull << k) - 1;  // elements [0, 2^(k+1)) are computed now
  // the array is full (rot_finish_kernel then decides whether the chain ended) or it ended
  if (last >= a.sst_cap || a.starts[last] >= n) *a.chain_end = k + 1;
}

// The chain past its first 2^K elements (K doubling levels done, the last without its squaring;
// FH = F^(2^(K-1))): chain element i 2^K for every i, by one lane -- a serial walk of
// 2 SSTs / 2^K dependent loads instead of log2(sst_cap) - K + 1 more squarings of F over all n
// entries (~90 us each at config C's 29.5 M; a load of the walk ~0.3 us).  Past the chain's
// end the anchors are n.
__global__ void rot_walk_kernel(RotArgs a, uint32_t K, const uint32_t* FH) {
  if (threadIdx.x || *(volatile uint32_t*)a.chain_end) return;
  const uint64_t n = rot_n(a);
  uint32_t x = a.starts[0];
  for (uint64_t i = 1ull << K; i < a.sst_cap; i += 1ull << K) {
    x = x < n ? FH[x] : uint32_t(n);
    x = x < n ? FH[x] : uint32_t(n);
    a.starts[i] = x;
  }
}

// Thread i: chain elements i 2^K + 1 .. (i + 1) 2^K - 1 from anchor i through F.
__global__ __launch_bounds__(64) void rot_fill_kernel(RotArgs a, uint32_t K) {
  if (*(volatile uint32_t*)a.chain_end) return;
  const uint64_t n = rot_n(a);
  const uint64_t base = (uint64_t(blockIdx.x) * 64 + threadIdx.x) << K;
  if (base >= a.sst_cap) return;
  uint32_t x = a.starts[base];
  for (uint64_t t = base + 1; t < base + (1ull << K) && t < a.sst_cap; ++t) {
    x = x < n ? a.F0[x] : uint32_t(n);
    a.starts[t] = x;
  }
}

// After the fill every slot of starts[] is a chain element (or n past the end).
__global__ void rot_filled_kernel(RotArgs a, uint32_t levels) {
  if (threadIdx.x == 0 && !*(volatile uint32_t*)a.chain_end) *a.chain_end = levels;
}

__global__ __launch_bounds__(256) void rot_finish_kernel(RotArgs a) {
  const uint64_t n = rot_n(a);
  __shared__ uint32_t s_ns;
  if (threadIdx.x == 0) {
    // SST count: the computed chain elements below n (increasing, then n), by binary search
    const uint32_t done = *a.chain_end;
    const uint64_t cap2 = 1ull << done;  // (HIP's min<uint64_t> compiles to f64 compares)
    uint32_t lo = 0, hi = done ? uint32_t(a.sst_cap < cap2 ? a.sst_cap : cap2) : 1u;
    if (n == 0) {
      hi = 0;
    } else {
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a.starts[mid] < n) lo = mid + 1;
        else hi = mid;
      }
    }
    s_ns = lo;
    uint32_t err = *a.rerr;
    if (uint64_t(lo) + 1 > a.sst_cap) err |= LSMBLK_ERR_CAPACITY;  // the chain did not end in the array
    a.stats[0] = lo;
    *a.nsst = err ? 0u : lo;
    if (err) atomicOr(reinterpret_cast<unsigned long long*>(a.stats + 3), (unsigned long long)err);
  }
  __syncthreads();
  for (uint32_t i = s_ns + threadIdx.x; i < a.sst_cap; i += 256) a.starts[i] = uint32_t(n);
}

// ---------------------------------------------------------------- host side
// Carve the context's compaction arena (grown on demand, which synchronizes).
struct Carve {
  uint8_t* base;
  uint64_t off = 0;
  Carve(uint8_t* b, uint64_t o = 0) : base(b), off(o) {}
  template <typename T>
  T* take(uint64_t count) {
    T* p = reinterpret_cast<T*>(base + off);
    off = (off + count * sizeof(T) + 255) & ~uint64_t(255);
    return p;
  }
};

struct MergePlan {
  MergeArgs m;
  uint32_t* keep;
  uint8_t* ksame;    // two-level: same_as_last_key per kept entry
  uint32_t* kidx;    // per kept entry, its input index (the deferred gather, lsmblk_compact_batch)
  uint64_t* gtile;   // 6 per gather tile
  uint64_t gtiles;
  uint64_t bytes;
};

// Workspace layout for a merge of n entries in nrun runs (the carve is replayed with base null
// to measure it).
MergePlan plan_merge(uint8_t* base, uint64_t n, uint32_t nrun) {
  MergePlan P{};
  Carve cv{base};
  const uint32_t nc_max = uint32_t(n / kMS + nrun + 1);
  P.m.nc_max = nc_max;
  P.m.k16 = cv.take<u32x4>(n + 1);
  P.m.cand = cv.take<uint32_t>(nc_max + 1);
  P.m.ck = cv.take<u32x4>(nc_max + 1);
  P.m.cklen = cv.take<uint32_t>(nc_max + 1);
  P.m.cks = cv.take<u32x4>(nc_max + 1);
  P.m.ckslen = cv.take<uint32_t>(nc_max + 1);
  P.m.bounds = cv.take<uint32_t>(uint64_t(nrun) * (nc_max + 1));
  P.m.mrank = cv.take<uint32_t>(n + 1);
  P.m.sp = cv.take<uint32_t>(n + 1);
  P.m.tcnt = cv.take<uint32_t>(nc_max + 1);
  P.m.tpre = cv.take<uint64_t>(nc_max + 2);
  P.m.tpart = cv.take<uint64_t>(nc_max / kTScan + 2);
  P.m.tbase = cv.take<uint64_t>(nc_max / kTScan + 3);
  P.m.perm = cv.take<uint32_t>(n + 1);
  P.m.big = cv.take<uint32_t>(nc_max + 1);
  P.m.mstats = cv.take<uint64_t>(8);
  P.keep = cv.take<uint32_t>(n + 1);
  P.ksame = cv.take<uint8_t>(n + 1);
  P.kidx = cv.take<uint32_t>(n + 1);
  P.gtiles = (n + kGTile - 1) / kGTile + 1;
  P.gtile = cv.take<uint64_t>(6 * P.gtiles + 6 * (P.gtiles / kGScan + 2));
  P.bytes = cv.off;
  return P;
}

int ensure_ws(lsmblk_ctx* c, uint64_t bytes, hipStream_t st) {
  if (bytes <= c->cws_cap) return LSMBLK_OK;
  return grow(st, &c->cws, &c->cws_cap, bytes, 1);
}

// merge + (rules | keep all) + gather into `out`; stats as lsmblk_compact_filter_batch's.
int merge_gather_locked(lsmblk_ctx* c, const lsmblk_kv_stream* in, const uint32_t* run_start, uint32_t nrun,
                        uint32_t rules, uint64_t wm, int bottom, const uint8_t* pfx, const uint32_t* pfx_off,
                        uint32_t npfx, const lsmblk_key_range* range, const lsmblk_kv_stream* out, uint64_t* stats,
                        hipStream_t st, MergePlan* plan_out, uint32_t two, uint32_t two_end = LSMBLK_TWO_END_IN_RANGE,
                        uint8_t* ksame_out = nullptr, GatherArgs* defer = nullptr) {
  const uint64_t n = in->n;
  MergePlan P = plan_merge(nullptr, n, nrun);
  int rc = ensure_ws(c, P.bytes, st);
  if (rc) return rc;
  P = plan_merge(c->cws, n, nrun);
  if (plan_out) *plan_out = P;
  MergeArgs& m = P.m;
  m.keys = in->keys;
  m.key_off = in->key_off;
  m.n = n;
  m.run_start = run_start;
  m.nrun = nrun;
  m.two = two;
  m.two_end = two_end;
  if (hipMemsetAsync(stats, 0, LSMBLK_STATS_WORDS * 8, st) != hipSuccess) return LSMBLK_E_HIP;
  if (n == 0) {
    LSM_LAUNCH(merge_empty_kernel, dim3(1), dim3(64), 0, st, m.mstats, out->key_off, out->val_off,
                       out->entry_cap, stats);
    return hipGetLastError() == hipSuccess ? LSMBLK_OK : LSMBLK_E_HIP;
  }
  if (hipMemsetAsync(m.mstats, 0, 64, st) != hipSuccess) return LSMBLK_E_HIP;
  const uint32_t nc = m.nc_max;
  LSM_LAUNCH(key16_kernel, dim3(uint32_t((n + 255) / 256)), dim3(256), 0, st, m.keys, m.key_off, n,
             const_cast<u32x4*>(m.k16), m.mstats + 3);
  LSM_LAUNCH(cand_key_kernel, dim3((nc + 255) / 256), dim3(256), 0, st, m);
  LSM_LAUNCH(cand_rank_kernel, dim3((nc + 255) / 256), dim3(256), 0, st, m);
  const uint64_t nb = (uint64_t(nc) + 1) * nrun;
  LSM_LAUNCH(bounds_kernel, dim3(uint32_t((nb + 255) / 256)), dim3(256), 0, st, m);
  LSM_LAUNCH(merge_tile_kernel, dim3(nc), dim3(kMTT), 0, st, m);
  LSM_LAUNCH(merge_big_kernel, dim3(std::min(nc, kBigGrid)), dim3(kBigTT), 0, st, m);
  LSM_LAUNCH(tscan_part_kernel, dim3((nc + kTScan - 1) / kTScan), dim3(256), 0, st, m);
  LSM_LAUNCH(tscan_top_kernel, dim3(1), dim3(1024), 0, st, m);
  LSM_LAUNCH(perm_kernel, dim3(nc), dim3(64), 0, st, m);
  if (hipGetLastError() != hipSuccess) return LSMBLK_E_HIP;
  GatherArgs g;
  g.keys = in->keys;
  g.key_off = in->key_off;
  g.vals = in->vals;
  g.val_off = in->val_off;
  g.ts = in->ts;
  g.perm = m.perm;
  g.k16 = m.k16;
  g.nm = m.mstats;
  g.n_max = n;
  g.rules = rules;
  g.wm = wm;
  g.bottom = bottom ? 1u : 0u;
  g.npfx = npfx;
  g.pfx = pfx;
  g.pfx_off = pfx_off;
  g.okeys = out->keys;
  g.okey_off = out->key_off;
  g.ovals = out->vals;
  g.oval_off = out->val_off;
  g.ots = out->ts;
  g.entry_cap = out->entry_cap;
  g.key_cap = out->key_cap;
  g.val_cap = out->val_cap;
  g.keep = P.keep;
  g.tile_sum = P.gtile;
  g.tile_pre = P.gtile + 3 * P.gtiles;
  g.part_sum = P.gtile + 6 * P.gtiles;
  g.part_pre = g.part_sum + 3 * (P.gtiles / kGScan + 2);
  g.stats = stats;
  g.merr = m.mstats + 3;
  g.range = range ? *range : lsmblk_key_range{};
  g.two = two;
  g.ksame = two && rules ? (ksame_out ? ksame_out : P.ksame) : nullptr;
  const uint32_t gt = uint32_t((n + kGTile - 1) / kGTile);
  if (two && rules) LSM_LAUNCH(mgroup_kernel, dim3(uint32_t((n + 255) / 256)), dim3(256), 0, st, g);
  LSM_LAUNCH(mflag_kernel, dim3(gt), dim3(256), 0, st, g);
  LSM_LAUNCH(mscan_part_kernel, dim3(uint32_t((P.gtiles + kGScan - 1) / kGScan)), dim3(256), 0, st, g);
  LSM_LAUNCH(mscan_top_kernel, dim3(1), dim3(1024), 0, st, g);
  if (defer) {  // the metadata now (with kidx), the bytes by the caller (mwrite_bytes)
    g.kidx = P.kidx;
    LSM_LAUNCH_NAMED("mwrite_kernel<true,false>", mwrite_kernel<true, false>, dim3(gt), dim3(256), 0, st, g);
    *defer = g;
  } else {
    g.kidx = nullptr;
    LSM_LAUNCH_NAMED("mwrite_kernel<true,true>", mwrite_kernel<true, true>, dim3(gt), dim3(256), 0, st, g);
  }
  return hipGetLastError() == hipSuccess ? LSMBLK_OK : LSMBLK_E_HIP;
}

// The deferred half of merge_gather_locked: the kept entries' key and value bytes.
int mwrite_bytes(const GatherArgs& g, uint64_t n, hipStream_t st) {
  if (n == 0) return LSMBLK_OK;
  LSM_LAUNCH_NAMED("mwrite_kernel<false,true>", mwrite_kernel<false, true>, dim3(uint32_t((n + kGTile - 1) / kGTile)), dim3(256), 0, st, g);
  return hipGetLastError() == hipSuccess ? LSMBLK_OK : LSMBLK_E_HIP;
}

__global__ void set_u64_kernel(uint64_t* p, uint64_t v) {
  if (threadIdx.x == 0) *p = v;
}

// The kept-entry count the rotation and the encode see: 0 after any merge / rules error.
// The rotation's entry count: the kept entries, or 0 after an error of the rules / gather (fst[3]) or
// of the merge itself (merr = its mstats[3]: an unsorted run is reported there only).  With 0 the
// rotation on the second stream reads nothing -- in particular never the kept keys that the byte
// gather on the caller's stream is still writing.
__global__ void gate_kernel(const uint64_t* fst, const uint64_t* merr, uint64_t* dn) {
  if (threadIdx.x == 0) *dn = (fst[3] | *merr) ? 0ull : fst[0];
}

#ifndef LSMBLK_ROT_HOPS
#define LSMBLK_ROT_HOPS 16
#endif
// Top-level hops a lift makes for an SST of full blocks (0: no cap, every level).
constexpr uint64_t kRotHops = LSMBLK_ROT_HOPS;

uint32_t rot_levels(uint64_t target, uint32_t block_size) {
  // a block and its CRC take >= 23 bytes (4 + 1 + 8 + 2 + 2 + 2 + 4), so an SST reaches the
  // target within ceil(target / 23) blocks: 2^(levels-1) hops cover it
  const uint64_t j = target / 23 + 2;
  uint32_t k = 1;
  while (k < kRotMaxLevels && (1ull << (k - 1)) < j) ++k;
  // Every lift repeats its top level while it fits (rot_f_kernel, lift_target, lift_before), so
  // the levels above the one whose hop covers 1 / kRotHops of an SST of full blocks are not
  // built: each doubling level is a pass over every entry, each extra hop one gather per entry.
  // (Small blocks among them only add hops, never change a result.)
  if (kRotHops && block_size) {
    const uint64_t jb = target / block_size / kRotHops + 1;
    uint32_t c = 1;
    while (c < k && (1ull << (c - 1)) < jb) ++c;
    k = c;
  }
  return k;
}

struct RotPlan {
  RotArgs r;
  uint64_t* dn;     // device n for the rotation
  uint64_t bytes;
};

// flevels > 0: the shard layout (F^(2^k) levels instead of the chain ping-pong, carry state).
RotPlan plan_rot(uint8_t* base, uint64_t off, uint64_t n_max, uint64_t target, uint32_t block_size,
                 uint32_t flevels = 0) {
  RotPlan P{};
  Carve cv{base, off};
  const uint64_t N1 = n_max + 1;
  const uint32_t L = rot_levels(target, block_size);
  P.r.n_max = n_max;
  P.r.target = target;
  P.r.levels = L;
  P.r.rec = cv.take<uint32_t>(N1);
  P.r.alcp = cv.take<uint32_t>(N1);
  P.r.JS = cv.take<u32x2>(N1 * L);
  if (flevels) {
    P.r.flevels = flevels;
    P.r.FL = cv.take<uint32_t>(N1 * flevels);
    P.r.F0 = P.r.FL;
    P.r.F1 = nullptr;
    P.r.sstate = cv.take<uint64_t>(kShardWords);
  } else {
    P.r.F0 = cv.take<uint32_t>(N1);
    P.r.F1 = cv.take<uint32_t>(N1);
    P.r.F2 = cv.take<uint32_t>(N1);
  }
  P.r.need = cv.take<uint32_t>(kRotMaxLevels + 3);
  P.r.chain_end = P.r.need + kRotMaxLevels;
  P.r.nsst = P.r.need + kRotMaxLevels + 1;
  P.r.rerr = P.r.need + kRotMaxLevels + 2;
  P.dn = cv.take<uint64_t>(2);
  P.bytes = cv.off;
  return P;
}

// SST cut points of the stream (keys, key_off, val_off; *dn entries, <= n_max) into starts[]
// The carry-independent part: adjacency, block chains and their doubling levels, F.
int rotation_chains(const RotArgs& r, hipStream_t st) {
  if (hipMemsetAsync(r.need, 0, (kRotMaxLevels + 3) * sizeof(uint32_t), st) != hipSuccess) return LSMBLK_E_HIP;
  const uint32_t g = uint32_t((r.n_max + 1 + 255) / 256);
  LSM_LAUNCH(rot_adj_kernel, dim3(g), dim3(256), 0, st, r);
  LSM_LAUNCH(rot_next_kernel, dim3(g), dim3(256), 0, st, r);
  const uint32_t gd = uint32_t((r.n_max + 1 + 256 * kRotPer - 1) / (256 * kRotPer));
  // two levels per pass while two remain (rot_double2_kernel), then the last one alone
  for (uint32_t k = 1; k < r.levels;) {
    if (k + 1 < r.levels) {
      LSM_LAUNCH(rot_double2_kernel, dim3(gd), dim3(256), 0, st, r, k);
      k += 2;
    } else {
      LSM_LAUNCH(rot_double_kernel, dim3(gd), dim3(256), 0, st, r, k);
      k += 1;
    }
  }
  if (kDiag && r.poison) LSM_LAUNCH(rot_poison_kernel, dim3(uint32_t((r.n_max / 3 + 256) / 256)), dim3(256), 0, st, r);
  LSM_LAUNCH(rot_f_kernel, dim3(uint32_t((r.n_max + 1 + 511) / 512)), dim3(256), 0, st, r);
  return hipGetLastError() == hipSuccess ? LSMBLK_OK : LSMBLK_E_HIP;
}

int rotation_locked(lsmblk_ctx* c, RotArgs r, hipStream_t st) {
  (void)c;
  if (hipMemsetAsync(r.starts, 0, sizeof(uint32_t), st) != hipSuccess) return LSMBLK_E_HIP;
  int rc = rotation_chains(r, st);
  if (rc) return rc;
  const uint32_t g = uint32_t((r.n_max + 1 + 255) / 256);
  // K doubling levels (chain elements [0, 2^K); the last level does not square F), then the
  // walk + fill: K = 3 up to sst_cap 4096 (walk <= 1024 loads), growing with the capacity so the
  // walk stays that short.  Config C (1 803 SSTs, sst_cap 4 096): 12 levels, 0.89 ms ->
  // 4 levels + walk + fill 0.40 ms -> 3 levels (2 squarings) + walk + fill.  The fill follows
  // 2^K - 1 elements through F one after another per thread, so K stays <= kRotFillMax: a larger
  // capacity (sst_cap > 2^17) takes every doubling level instead (ceil(log2 sst_cap) squarings,
  // no walk, no fill) -- never a chain of serial loads that grows with the capacity.
  uint32_t lc = 0;  // ceil(log2(sst_cap))
  while (lc < 32 && (1ull << lc) < r.sst_cap) ++lc;
  constexpr uint32_t kRotFillMax = 8;
  const uint32_t K = lc <= 12 ? 3u : (lc - 9 <= kRotFillMax ? lc - 9 : 32u);  // 32: doubling to the end
  uint32_t* cur = r.F0;
  uint32_t* nxt = r.F1;
  for (uint32_t k = 0; k < 32 && (1ull << k) < r.sst_cap; ++k) {
    if (k == K) {
      LSM_LAUNCH(rot_walk_kernel, dim3(1), dim3(64), 0, st, r, K, cur);
      LSM_LAUNCH(rot_fill_kernel, dim3(uint32_t(((r.sst_cap >> K) + 1 + 63) / 64)), dim3(64), 0, st, r, K);
      LSM_LAUNCH(rot_filled_kernel, dim3(1), dim3(64), 0, st, r, lc);
      break;
    }
    const bool last = k + 1 == K && (2ull << k) < r.sst_cap;  // the walk follows: no squaring
    LSM_LAUNCH(rot_chain_kernel, dim3(last ? uint32_t(((1ull << k) + 255) / 256) : g), dim3(256), 0, st, r,
                       k, cur, last ? nullptr : nxt);
    LSM_LAUNCH(rot_chain_check_kernel, dim3(1), dim3(64), 0, st, r, k);
    if (last) continue;             // cur stays F^(2^k) = F^(2^(K-1)) for the walk
    cur = nxt;                      // F^(2^(k+1))
    nxt = cur == r.F1 ? r.F2 : r.F1;  // F (F0) is kept for the fill
  }
  LSM_LAUNCH(rot_finish_kernel, dim3(1), dim3(256), 0, st, r);
  return hipGetLastError() == hipSuccess ? LSMBLK_OK : LSMBLK_E_HIP;
}

// Final stats of lsmblk_compact_batch from the stage stats.
__global__ void compact_stats_kernel(uint64_t* stats, const uint64_t* fst, const uint64_t* rst, const uint64_t* est,
                                     const uint64_t* mst) {
  if (threadIdx.x) return;
  const uint64_t err = fst[3] | rst[3] | est[3];
  stats[0] = err ? 0 : est[0];
  stats[1] = err ? 0 : est[1];
  stats[2] = rst[0];
  stats[3] = err;
  stats[4] = mst[0];
  stats[5] = fst[0];
  stats[6] = fst[1];
  stats[7] = fst[2];
}

int check_merge_args(lsmblk_ctx* c, const lsmblk_kv_stream* in, const uint32_t* run_start, uint32_t nrun,
                     const lsmblk_kv_stream* out, const uint64_t* stats) {
  if (!c || !in || !run_start || !out || !stats || !in->key_off || !in->val_off) return LSMBLK_E_INVAL;
  if (!out->key_off || !out->val_off) return LSMBLK_E_INVAL;
  if (nrun == 0 || nrun > kMaxRuns || in->n >= 0xFFFFFFF0ull) return LSMBLK_E_INVAL;
  return LSMBLK_OK;
}

uint32_t shard_flevels(uint32_t sst_cap) {
  uint32_t k = 1;
  while (k < 32 && (1ull << k) < uint64_t(sst_cap) + 1) ++k;
  return k;
}

// The rotation arguments of the last lsmblk_shard_rotation_prepare on this context.
RotArgs shard_args(lsmblk_ctx* c, const lsmblk_kv_stream* ext) {
  const RotPlan P = plan_rot(c->rws, 0, c->shard_n, c->shard_target, c->shard_block_size, shard_flevels(c->shard_sst_cap));
  RotArgs r = P.r;
  r.dn = P.dn;
  r.m = c->shard_m;
  r.shard_last = c->shard_flags & LSMBLK_SHARD_LAST;
  r.block_size = c->shard_block_size;
  if (ext) {
    r.keys = ext->keys;
    r.key_off = ext->key_off;
    r.val_off = ext->val_off;
  }
  return r;
}

__global__ void copy_u64_kernel(uint64_t* dst, const uint64_t* src) {
  if (threadIdx.x == 0) *dst = *src;
}

}  // namespace

extern "C" {

uint64_t lsmblk_shard_halo_entries(uint32_t block_size) { return uint64_t(block_size) / 16 + 2; }

int lsmblk_compact_merge_batch(lsmblk_ctx* c, const lsmblk_kv_stream* in, const uint32_t* run_start, uint32_t nrun,
                               const lsmblk_compact_opts* o, const lsmblk_key_range* range,
                               const lsmblk_kv_stream* kept, uint64_t* stats, void* stream) {
  if (o && o->merge_mode != LSMBLK_MERGE_RUNS) return LSMBLK_E_INVAL;  // two-level: the _ex form
  return lsmblk_compact_merge_batch_ex(c, in, run_start, nrun, o, range, LSMBLK_TWO_END_IN_RANGE, kept, nullptr, stats,
                                       stream);
}

int lsmblk_compact_merge_batch_ex(lsmblk_ctx* c, const lsmblk_kv_stream* in, const uint32_t* run_start, uint32_t nrun,
                                  const lsmblk_compact_opts* o, const lsmblk_key_range* range, uint32_t two_end,
                                  const lsmblk_kv_stream* kept, uint8_t* kept_same, uint64_t* stats, void* stream) {
  int rc = check_merge_args(c, in, run_start, nrun, kept, stats);
  if (rc) return rc;
  if (!o || (o->nprefix && (!o->prefixes || !o->prefix_off))) return LSMBLK_E_INVAL;
  if (o->merge_mode != LSMBLK_MERGE_RUNS && o->merge_mode != LSMBLK_MERGE_TWO_LEVEL) return LSMBLK_E_INVAL;
  const uint32_t two = o->merge_mode == LSMBLK_MERGE_TWO_LEVEL;
  if (two_end > LSMBLK_TWO_END_BELOW || (two && !kept_same)) return LSMBLK_E_INVAL;
  if (range && ((range->has_lo && range->lo_len && !range->lo) || (range->has_hi && range->hi_len && !range->hi)))
    return LSMBLK_E_INVAL;
  std::lock_guard<std::mutex> g(c->mu);
  DeviceGuard dg(c->device, c);
  if (!dg.ok) return LSMBLK_E_HIP;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (hipMemsetAsync(stats + 4, 0, 8, st) != hipSuccess) return LSMBLK_E_HIP;
  MergePlan MP{};
  if ((rc = merge_gather_locked(c, in, run_start, nrun, 1, o->watermark, o->bottom_level, o->prefixes, o->prefix_off,
                                o->nprefix, range, kept, stats, st, &MP, two, two_end, two ? kept_same : nullptr)))
    return rc;
  if (in->n) LSM_LAUNCH(copy_u64_kernel, dim3(1), dim3(64), 0, st, stats + 4, MP.m.mstats);
  return hipGetLastError() == hipSuccess ? LSMBLK_OK : LSMBLK_E_HIP;
}

int lsmblk_shard_rotation_prepare(lsmblk_ctx* c, const lsmblk_kv_stream* ext, uint64_t n_own, uint32_t flags,
                                  uint32_t block_size, uint64_t target_sst_size, uint32_t sst_cap, void* stream) {
  return lsmblk_shard_rotation_prepare_ex(c, ext, nullptr, n_own, flags, block_size, target_sst_size, sst_cap, stream);
}

int lsmblk_shard_rotation_prepare_ex(lsmblk_ctx* c, const lsmblk_kv_stream* ext, const uint8_t* ext_same, uint64_t n_own,
                                     uint32_t flags, uint32_t block_size, uint64_t target_sst_size, uint32_t sst_cap,
                                     void* stream) {
  if (!c || !ext || !ext->key_off || !ext->val_off) return LSMBLK_E_INVAL;
  if (block_size == 0 || target_sst_size == 0 || sst_cap == 0 || n_own > ext->n || ext->n >= 0xFFFFFFF0ull)
    return LSMBLK_E_INVAL;
  std::lock_guard<std::mutex> g(c->mu);
  DeviceGuard dg(c->device, c);
  if (!dg.ok) return LSMBLK_E_HIP;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  c->shard_ready = false;
  const uint32_t fl = shard_flevels(sst_cap);
  const RotPlan P0 = plan_rot(nullptr, 0, ext->n, target_sst_size, block_size, fl);
  int rc = grow(st, &c->rws, &c->rws_cap, P0.bytes, 1);
  if (rc) return rc;
  c->shard_n = ext->n;
  c->shard_m = n_own;
  c->shard_target = target_sst_size;
  c->shard_block_size = block_size;
  c->shard_flags = flags;
  c->shard_sst_cap = sst_cap;
  RotArgs r = shard_args(c, ext);
  r.ksame = ext_same;  // two-level: the loop's same_as_last_key (baked into alcp by rot_adj)
  r.poison = c->rot_poison;
  LSM_LAUNCH(set_u64_kernel, dim3(1), dim3(64), 0, st, const_cast<uint64_t*>(r.dn), uint64_t(ext->n));
  if ((rc = rotation_chains(r, st))) return rc;
  const uint32_t gr = uint32_t((ext->n + 1 + 255) / 256);
  for (uint32_t k = 1; k < fl; ++k) LSM_LAUNCH(rot_flev_kernel, dim3(gr), dim3(256), 0, st, r, k);
  if (hipGetLastError() != hipSuccess) return LSMBLK_E_HIP;
  c->shard_ready = true;
  return LSMBLK_OK;
}

int lsmblk_shard_rotation_carry(lsmblk_ctx* c, const uint64_t* carry_in, uint64_t* carry_out, void* stream) {
  if (!c || !carry_in || !carry_out) return LSMBLK_E_INVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->shard_ready) return LSMBLK_E_INVAL;
  DeviceGuard dg(c->device, c);
  if (!dg.ok) return LSMBLK_E_HIP;
  const RotArgs r = shard_args(c, nullptr);
  LSM_LAUNCH(shard_carry_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), r, carry_in,
                     carry_out);
  return hipGetLastError() == hipSuccess ? LSMBLK_OK : LSMBLK_E_HIP;
}

int lsmblk_shard_encode_batch(lsmblk_ctx* c, const lsmblk_kv_stream* ext, uint8_t* out, uint64_t out_cap,
                              uint64_t* blk_off, uint64_t blk_cap, uint32_t* seg_start, uint32_t* seg_blk,
                              uint32_t seg_cap, uint64_t* stats, void* stream) {
  if (!c || !ext || !ext->key_off || !ext->val_off || !out || !blk_off || !seg_start || !seg_blk || !stats)
    return LSMBLK_E_INVAL;
  if (seg_cap < 2 || blk_cap == 0 || (reinterpret_cast<uintptr_t>(out) & 15) != 0) return LSMBLK_E_INVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->shard_ready || ext->n != c->shard_n) return LSMBLK_E_INVAL;
  DeviceGuard dg(c->device, c);
  if (!dg.ok) return LSMBLK_E_HIP;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const RotArgs r = shard_args(c, ext);
  uint64_t* est = r.sstate + 8;
  if (hipMemsetAsync(stats, 0, LSMBLK_COMPACT_STATS_WORDS * 8, st) != hipSuccess) return LSMBLK_E_HIP;
  if (hipMemsetAsync(blk_off, 0, 8, st) != hipSuccess) return LSMBLK_E_HIP;
  LSM_LAUNCH(shard_seg_kernel, dim3((seg_cap + 255) / 256), dim3(256), 0, st, r, seg_start, seg_cap, r.nsst);
  if (hipGetLastError() != hipSuccess) return LSMBLK_E_HIP;
  int rc = lsmblk_impl::encode_locked(c, ext, nullptr, seg_start, r.nsst, seg_cap - 1, c->shard_block_size, out,
                                      out_cap, blk_off, blk_cap, est, st, true);
  if (rc) return rc;
  if ((rc = lsmblk_impl::segment_blocks_locked(c, seg_start, seg_cap - 1, est, seg_blk, st))) return rc;
  LSM_LAUNCH(shard_stats_kernel, dim3(1), dim3(64), 0, st, stats, est, r.sstate);
  return hipGetLastError() == hipSuccess ? LSMBLK_OK : LSMBLK_E_HIP;
}

int lsmblk_merge_batch(lsmblk_ctx* c, const lsmblk_kv_stream* in, const uint32_t* run_start, uint32_t nrun,
                       const lsmblk_kv_stream* out, uint64_t* stats, void* stream) {
  int rc = check_merge_args(c, in, run_start, nrun, out, stats);
  if (rc) return rc;
  std::lock_guard<std::mutex> g(c->mu);
  DeviceGuard dg(c->device, c);
  if (!dg.ok) return LSMBLK_E_HIP;
  return merge_gather_locked(c, in, run_start, nrun, 0, 0, 0, nullptr, nullptr, 0, nullptr, out, stats,
                             reinterpret_cast<hipStream_t>(stream), nullptr, 0);
}

int lsmblk_merge_batch_ex(lsmblk_ctx* c, const lsmblk_kv_stream* in, const uint32_t* run_start, uint32_t nrun,
                          uint32_t merge_mode, const lsmblk_kv_stream* out, uint64_t* stats, void* stream) {
  int rc = check_merge_args(c, in, run_start, nrun, out, stats);
  if (rc) return rc;
  if (merge_mode != LSMBLK_MERGE_RUNS && merge_mode != LSMBLK_MERGE_TWO_LEVEL) return LSMBLK_E_INVAL;
  std::lock_guard<std::mutex> g(c->mu);
  DeviceGuard dg(c->device, c);
  if (!dg.ok) return LSMBLK_E_HIP;
  return merge_gather_locked(c, in, run_start, nrun, 0, 0, 0, nullptr, nullptr, 0, nullptr, out, stats,
                             reinterpret_cast<hipStream_t>(stream), nullptr, merge_mode == LSMBLK_MERGE_TWO_LEVEL);
}

int lsmblk_sst_rotation_batch(lsmblk_ctx* c, const lsmblk_kv_stream* in, uint32_t block_size,
                              uint64_t target_sst_size, uint32_t* sst_start, uint32_t sst_cap, uint64_t* stats,
                              void* stream) {
  if (!c || !in || !sst_start || !stats || !in->key_off || !in->val_off) return LSMBLK_E_INVAL;
  if (block_size == 0 || target_sst_size == 0 || sst_cap == 0 || in->n >= 0xFFFFFFF0ull) return LSMBLK_E_INVAL;
  std::lock_guard<std::mutex> g(c->mu);
  DeviceGuard dg(c->device, c);
  if (!dg.ok) return LSMBLK_E_HIP;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  RotPlan P = plan_rot(nullptr, 0, in->n, target_sst_size, block_size);
  int rc = ensure_ws(c, P.bytes, st);
  if (rc) return rc;
  P = plan_rot(c->cws, 0, in->n, target_sst_size, block_size);
  if (hipMemsetAsync(stats, 0, LSMBLK_STATS_WORDS * 8, st) != hipSuccess) return LSMBLK_E_HIP;
  LSM_LAUNCH(set_u64_kernel, dim3(1), dim3(64), 0, st, P.dn, uint64_t(in->n));
  RotArgs r = P.r;
  r.keys = in->keys;
  r.key_off = in->key_off;
  r.val_off = in->val_off;
  r.dn = P.dn;
  r.block_size = block_size;
  r.starts = sst_start;
  r.sst_cap = sst_cap;
  r.stats = stats;
  r.poison = c->rot_poison;
  return rotation_locked(c, r, st);
}

int lsmblk_compact_batch(lsmblk_ctx* c, const lsmblk_kv_stream* in, const uint32_t* run_start, uint32_t nrun,
                         const lsmblk_compact_opts* o, const lsmblk_kv_stream* kept, uint8_t* out, uint64_t out_cap,
                         uint64_t* blk_off, uint64_t blk_cap, uint32_t* sst_start, uint32_t* sst_blk, uint32_t sst_cap,
                         uint64_t* stats, void* stream) {
  int rc = check_merge_args(c, in, run_start, nrun, kept, stats);
  if (rc) return rc;
  if (!o || !out || !blk_off || !sst_start || !sst_blk || sst_cap < 2 || blk_cap == 0) return LSMBLK_E_INVAL;
  if (o->block_size == 0 || o->target_sst_size == 0 || (o->nprefix && (!o->prefixes || !o->prefix_off)))
    return LSMBLK_E_INVAL;
  if (o->merge_mode != LSMBLK_MERGE_RUNS && o->merge_mode != LSMBLK_MERGE_TWO_LEVEL) return LSMBLK_E_INVAL;
  if ((reinterpret_cast<uintptr_t>(out) & 15) != 0) return LSMBLK_E_INVAL;
  const uint32_t two = o->merge_mode == LSMBLK_MERGE_TWO_LEVEL;
  std::lock_guard<std::mutex> g(c->mu);
  DeviceGuard dg(c->device, c);
  if (!dg.ok) return LSMBLK_E_HIP;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const uint64_t n = in->n;
  // workspace: merge + gather, then rotation, then the stage stats
  MergePlan M = plan_merge(nullptr, n, nrun);
  RotPlan R = plan_rot(nullptr, M.bytes, n, o->target_sst_size, o->block_size);
  const uint64_t stats_off = (R.bytes + 255) & ~uint64_t(255);
  if ((rc = ensure_ws(c, stats_off + 4 * 64, st))) return rc;
  uint64_t* sts = reinterpret_cast<uint64_t*>(c->cws + stats_off);
  uint64_t *fst = sts, *rst = sts + 8, *est = sts + 16;
  if (hipMemsetAsync(sts, 0, 4 * 64, st) != hipSuccess) return LSMBLK_E_HIP;
  if (hipMemsetAsync(stats, 0, LSMBLK_COMPACT_STATS_WORDS * 8, st) != hipSuccess) return LSMBLK_E_HIP;
  if (hipMemsetAsync(blk_off, 0, 8, st) != hipSuccess) return LSMBLK_E_HIP;
  // The rotation needs only the kept entries' metadata (and their keys, read in the merge input
  // through kidx), so the kept stream's key and value bytes are gathered on `st` while the
  // rotation runs on the context's second stream; the encode waits for both.  (Reverted in round 4
  // after a GPU-suite hang; re-landed once that hang's cause was found in grow(), DESIGN.md
  // section 10.)
  MergePlan MP{};
  GatherArgs G{};
  if ((rc = merge_gather_locked(c, in, run_start, nrun, 1, o->watermark, o->bottom_level, o->prefixes, o->prefix_off,
                                o->nprefix, nullptr, kept, fst, st, &MP, two, LSMBLK_TWO_END_IN_RANGE, nullptr, &G)))
    return rc;
  R = plan_rot(c->cws, M.bytes, n, o->target_sst_size, o->block_size);
  LSM_LAUNCH(gate_kernel, dim3(1), dim3(64), 0, st, fst, (const uint64_t*)(MP.m.mstats + 3), R.dn);
  RotArgs r = R.r;
  r.keys = kept->keys;
  r.key_off = kept->key_off;
  r.val_off = kept->val_off;
  r.dn = R.dn;  // kept entries (0 after a merge / rules error)
  r.block_size = o->block_size;
  r.starts = sst_start;
  r.sst_cap = sst_cap;
  r.stats = rst;
  r.ksame = two ? MP.ksame : nullptr;
  r.kidx = MP.kidx;
  r.k16 = MP.m.k16;
  r.akeys = in->keys;
  r.akey_off = in->key_off;
  r.an = n;
  r.poison = c->rot_poison;
  if ((rc = lsmblk_impl::fork_aux(c, st))) return rc;
  rc = rotation_locked(c, r, c->aux);
  if (!rc) rc = mwrite_bytes(G, n, st);
  // joined on every path once forked: after an error the caller's stream still
  // waits for the rotation work already queued on c->aux, which writes sst_start and the workspace
  const int jrc = lsmblk_impl::join_aux(c, st);
  if (rc) return rc;
  if (jrc) return jrc;
  lsmblk_kv_stream ks = *kept;
  ks.n = n;  // bound; the encode reads the kept count from fst[0]
  if ((rc = lsmblk_impl::encode_locked(c, &ks, R.dn, sst_start, r.nsst, sst_cap - 1, o->block_size, out, out_cap,
                                       blk_off, blk_cap, est, st)))
    return rc;
  if ((rc = lsmblk_impl::segment_blocks_locked(c, sst_start, sst_cap - 1, est, sst_blk, st))) return rc;
  LSM_LAUNCH(compact_stats_kernel, dim3(1), dim3(64), 0, st, stats, fst, rst, est, MP.m.mstats);
  return hipGetLastError() == hipSuccess ? LSMBLK_OK : LSMBLK_E_HIP;
}

}  // extern "C"
