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
//   tile_scan_kernel   exclusive scan of per-tile survivor counts -> tile bases
//   perm_kernel        perm[tile base + in-tile rank] = input index
// Then, over the merged order:
//   mflag_kernel / mscan_kernel / mwrite_kernel   the compaction rules (or keep-all for a plain
//                      merge), output offsets, and the gather of the kept entries.
#include "lsmblk_dev.hpp"

namespace {

constexpr uint32_t kMS = 64;        // every kMS-th entry of a run is a merge candidate
constexpr uint32_t kMaxRuns = 64;   // runs per merge (one lane per run in the tile kernels)
constexpr uint32_t kMTE = 512;      // tile entries with LDS tables
constexpr uint32_t kMTK = 8192;     // tile key bytes staged in LDS
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
  uint32_t* cand;           // nc_max: sorted candidate -> input index
  uint32_t* bounds;         // nrun rows of nc_max + 1: tile t's first entry in run r
  uint32_t* mrank;          // n: in-tile merged rank of a surviving entry, kNone if dropped
  uint32_t* sp;             // n: survivor prefix (tiles too large for LDS)
  uint32_t* tcnt;           // nc_max: survivors per tile
  uint64_t* tpre;           // nc_max + 1: tile bases
  uint32_t* perm;           // n: merged position -> input index
  uint64_t* mstats;         // [0] merged entries [1] candidates (tiles) [3] error flags
};

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
  const uint32_t xp = a.key_off[p], xl = a.key_off[p + 1] - xp;
  uint32_t rank = j;
  for (uint32_t r2 = 0; r2 < a.nrun; ++r2) {
    if (r2 == r) continue;
    // candidates of r2 ordered before (x, r, j): key < x, or key == x and r2 < r
    uint32_t lo = 0, hi = s_cb[r2 + 1] - s_cb[r2];
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1, q = s_rs[r2] + mid * kMS;
      const uint32_t qp = a.key_off[q];
      const int cm = key_cmp(K, qp, a.key_off[q + 1] - qp, xp, xl);
      if (cm < 0 || (cm == 0 && r2 < r)) lo = mid + 1;
      else hi = mid;
    }
    rank += lo;
  }
  a.cand[rank] = p;
}

__global__ __launch_bounds__(256) void bounds_kernel(MergeArgs a) {
  __shared__ uint32_t s_rs[kMaxRuns + 1], s_cb[kMaxRuns + 1];
  load_runs(a, s_rs, s_cb);
  const uint32_t NC = uint32_t(a.mstats[1]);
  const uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  const uint32_t t = uint32_t(i / a.nrun), r = uint32_t(i % a.nrun);
  if (t > NC) return;
  uint32_t* row = a.bounds + uint64_t(r) * (a.nc_max + 1);
  if (t == NC) {
    row[t] = s_rs[r + 1];
    return;
  }
  const GKeys K = gkeys(a.keys, a.key_off[a.n]);
  const uint32_t x = a.cand[t], xp = a.key_off[x], xl = a.key_off[x + 1] - xp;
  const uint32_t base = s_rs[r], C = s_cb[r + 1] - s_cb[r];
  uint32_t lo = 0, hi = C;  // first candidate of r with key >= x
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1, q = base + mid * kMS, qp = a.key_off[q];
    if (key_cmp(K, qp, a.key_off[q + 1] - qp, xp, xl) < 0) lo = mid + 1;
    else hi = mid;
  }
  uint32_t e0 = lo == 0 ? base : base + (lo - 1) * kMS + 1;
  uint32_t e1 = lo < C ? base + lo * kMS : s_rs[r + 1];
  while (e0 < e1) {  // first entry in [e0, e1) with key >= x (else e1)
    const uint32_t mid = (e0 + e1) >> 1, qp = a.key_off[mid];
    if (key_cmp(K, qp, a.key_off[mid + 1] - qp, xp, xl) < 0) e0 = mid + 1;
    else e1 = mid;
  }
  row[t] = e0;
}

struct alignas(16) MTileLds {
  uint32_t lo[kMaxRuns], tb[kMaxRuns + 1], kb[kMaxRuns + 1], kbeg[kMaxRuns];
  uint32_t rsp[kMaxRuns], rsv[kMaxRuns];  // survivors before run r's sub-range / inside it
  uint32_t total, nsurv;
  uint32_t koff[kMTE];
  uint32_t sp[kMTE + 1];
  uint16_t klen[kMTE];
  uint8_t surv[kMTE];
  uint8_t kimg[kMTK + 16];
};

// The tile's per-run sub-ranges into LDS: lane r holds run r's [lo, hi).  Each run's key bytes
// are staged as the 16-B aligned arena chunks covering them (aligned buffer loads never
// straddle the descriptor bound, which would zero a whole unaligned load): kbeg[r] = the
// aligned descriptor offset of run r's first chunk, kb[r] = its LDS offset.
__device__ __forceinline__ void tile_ranges(const MergeArgs& a, MTileLds& L, uint32_t t, uint32_t glead) {
  const uint32_t l = lane_id();
  uint32_t lo = 0, hi = 0, A = 0, B = 0;
  if (l < a.nrun) {
    const uint32_t* row = a.bounds + uint64_t(l) * (a.nc_max + 1);
    lo = row[t];
    hi = row[t + 1];
    if (hi < lo) hi = lo;  // only with unsorted runs (output then unspecified, flagged by mflag)
    if (hi > lo) {
      A = (glead + a.key_off[lo]) & ~15u;
      B = (glead + a.key_off[hi] + 15) & ~15u;
    }
  }
  const uint32_t m = hi - lo, kbytes = B - A;
  const uint32_t mi = wave_incl_scan32(m), ki = wave_incl_scan32(kbytes);
  if (l < a.nrun) {
    L.lo[l] = lo;
    L.tb[l] = mi - m;
    L.kb[l] = ki - kbytes;
    L.kbeg[l] = A;
  }
  if (l == 63) {
    L.total = mi;
    L.tb[a.nrun] = mi;
    L.kb[a.nrun] = ki;
  }
  wave_sync();
}

// One wave per tile.  LDS mode: keys staged, tables in LDS.  Global mode (a tile of more than
// kMTE entries or kMTK key bytes: many versions of one key, or many runs): keys read through
// the descriptor, survival kept in mrank[] and the survivor prefix in sp[], both handed between
// lanes through L2 (sc1 stores / loads, drained with vmcnt(0)).
template <bool kLds>
__device__ void merge_tile(const MergeArgs& a, MTileLds& L, uint32_t t) {
  const uint32_t l = lane_id(), nrun = a.nrun, total = L.total;
  const GKeys G = gkeys(a.keys, a.key_off[a.n]);
  const LKeys LK{L.kimg};
  if constexpr (kLds) {
    // stage every run's key bytes (16-B unaligned buffer loads -> unaligned LDS stores); a run's
    // last piece may spill into the next run's bytes, which the next run then rewrites
    for (uint32_t r = 0; r < nrun; ++r) {
      const uint32_t kb = L.kb[r], nb = L.kb[r + 1] - kb, src = L.kbeg[r];
      for (uint32_t o = 16 * l; o < nb; o += 1024) {
        const u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(G.r, src + o, 0, 0);
        *reinterpret_cast<u32x4*>(L.kimg + kb + o) = q;
      }
    }
    for (uint32_t u = l; u < total; u += 64) {
      const uint32_t r = find_run(L.tb, nrun, u), g = L.lo[r] + u - L.tb[r];
      const uint32_t k0 = a.key_off[g];
      L.koff[u] = L.kb[r] + G.lead + k0 - L.kbeg[r];
      L.klen[u] = uint16_t(a.key_off[g + 1] - k0);
    }
    wave_sync();
  }
  // key of tile entry (run r, index k of its sub-range)
  auto kpos = [&](uint32_t r, uint32_t k, uint32_t& len) -> uint32_t {
    if constexpr (kLds) {
      const uint32_t u = L.tb[r] + k;
      len = L.klen[u];
      return L.koff[u];
    } else {
      const uint32_t g = L.lo[r] + k, p = a.key_off[g];
      len = a.key_off[g + 1] - p;
      return p;
    }
  };
  auto cmp = [&](uint32_t ap, uint32_t al, uint32_t bp, uint32_t bl) -> int {
    if constexpr (kLds) return key_cmp(LK, ap, al, bp, bl);
    else return key_cmp(G, ap, al, bp, bl);
  };
  // first index of run r's sub-range whose key is >= x
  auto lower = [&](uint32_t r, uint32_t xp, uint32_t xl) -> uint32_t {
    uint32_t lo = 0, hi = L.tb[r + 1] - L.tb[r];
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      uint32_t ml;
      const uint32_t mp = kpos(r, mid, ml);
      if (cmp(mp, ml, xp, xl) < 0) lo = mid + 1;
      else hi = mid;
    }
    return lo;
  };
  auto set_surv = [&](uint32_t u, uint32_t g, uint32_t v) {
    if constexpr (kLds) L.surv[u] = uint8_t(v);
    else __hip_atomic_store(a.mrank + g, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  auto get_surv = [&](uint32_t u, uint32_t g) -> uint32_t {
    if constexpr (kLds) return L.surv[u];
    else return __hip_atomic_load(a.mrank + g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  auto set_sp = [&](uint32_t u, uint32_t g, uint32_t v) {
    if constexpr (kLds) L.sp[u] = v;
    else __hip_atomic_store(a.sp + g, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  auto get_sp = [&](uint32_t u, uint32_t g) -> uint32_t {
    if constexpr (kLds) return L.sp[u];
    else return __hip_atomic_load(a.sp + g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  auto drain = [&]() {
    if constexpr (!kLds) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync();
  };
  // phase A: survival -- no lower-index run holds the key (MergeIterator advances those heads)
  for (uint32_t u = l; u < total; u += 64) {
    const uint32_t r = find_run(L.tb, nrun, u), k = u - L.tb[r], g = L.lo[r] + k;
    uint32_t xl;
    const uint32_t xp = kpos(r, k, xl);
    uint32_t s = 1;
    for (uint32_t r2 = 0; r2 < r && s; ++r2) {
      const uint32_t p = lower(r2, xp, xl);
      if (p < L.tb[r2 + 1] - L.tb[r2]) {
        uint32_t ql;
        const uint32_t qp = kpos(r2, p, ql);
        if (cmp(qp, ql, xp, xl) == 0) s = 0;
      }
    }
    set_surv(u, g, s);
  }
  drain();
  // survivor prefix over the tile (run-major order), then per-run bases and counts
  uint32_t carry = 0;
  for (uint32_t c0 = 0; c0 < total; c0 += 64) {
    const uint32_t u = c0 + l;
    uint32_t s = 0, g = 0;
    if (u < total) {
      const uint32_t r = find_run(L.tb, nrun, u);
      g = L.lo[r] + u - L.tb[r];
      s = get_surv(u, g);
    }
    const uint32_t inc = wave_incl_scan32(s);
    if (u < total) set_sp(u, g, carry + inc - s);
    carry += __builtin_amdgcn_readlane(inc, 63);
  }
  drain();
  if (l < nrun) {
    const uint32_t u0 = L.tb[l], u1 = L.tb[l + 1];
    const uint32_t b0 = u0 < total ? get_sp(u0, L.lo[l]) : carry;
    const uint32_t b1 = u1 < total ? get_sp(u1, L.lo[find_run(L.tb, nrun, u1)] + u1 - L.tb[find_run(L.tb, nrun, u1)])
                                   : carry;
    L.rsp[l] = b0;
    L.rsv[l] = u1 > u0 ? b1 - b0 : 0u;
  }
  if (l == 0) L.nsurv = carry;
  wave_sync();
  // phase B: merged rank inside the tile = survivors with a smaller key in every other run +
  // survivors before this entry in its own run (its group's earlier versions included)
  for (uint32_t u = l; u < total; u += 64) {
    const uint32_t r = find_run(L.tb, nrun, u), k = u - L.tb[r], g = L.lo[r] + k;
    uint32_t rank = kNone;
    if (get_surv(u, g)) {
      uint32_t xl;
      const uint32_t xp = kpos(r, k, xl);
      rank = get_sp(u, g) - L.rsp[r];
      for (uint32_t r2 = 0; r2 < nrun; ++r2) {
        if (r2 == r) continue;
        const uint32_t m2 = L.tb[r2 + 1] - L.tb[r2];
        if (m2 == 0) continue;
        const uint32_t p = lower(r2, xp, xl);
        rank += p == m2 ? L.rsv[r2] : get_sp(L.tb[r2] + p, L.lo[r2] + p) - L.rsp[r2];
      }
    }
    a.mrank[g] = rank;  // each lane reads and rewrites only its own entries' words here
  }
  if (l == 0) a.tcnt[t] = L.nsurv;
}

__global__ __launch_bounds__(64) void merge_tile_kernel(MergeArgs a) {
  __shared__ MTileLds L;
  const uint32_t t = blockIdx.x;
  if (t >= uni(uint32_t(a.mstats[1]))) return;
  tile_ranges(a, L, t, uint32_t(reinterpret_cast<uintptr_t>(a.keys) & 15));
  if (L.total == 0) {
    if (lane_id() == 0) a.tcnt[t] = 0;
    return;
  }
  if (L.total <= kMTE && L.kb[a.nrun] <= kMTK) merge_tile<true>(a, L, t);
  else merge_tile<false>(a, L, t);
}

// One workgroup: exclusive scan of the tile survivor counts (coalesced rounds of 1024 tiles).
__global__ __launch_bounds__(1024) void tile_scan_kernel(MergeArgs a) {
  const uint32_t t = threadIdx.x, w = t >> 6;
  const uint32_t NC = uint32_t(a.mstats[1]);
  __shared__ uint64_t wsum[16];
  uint64_t carry = 0;
  for (uint32_t r = 0; r < NC; r += 1024) {
    const uint32_t i = r + t;
    const uint64_t v = i < NC ? a.tcnt[i] : 0;
    const uint64_t inc = wave_incl_scan<uint64_t>(v);
    if (lane_id() == 63) wsum[w] = inc;
    __syncthreads();
    uint64_t base = carry, tot = carry;
    for (uint32_t x = 0; x < 16; ++x) {
      if (x < w) base += wsum[x];
      tot += wsum[x];
    }
    if (i < NC) a.tpre[i] = base + inc - v;
    carry = tot;
    __syncthreads();
  }
  if (t == 0) {
    a.tpre[NC] = carry;
    a.mstats[0] = carry;
  }
}

__global__ __launch_bounds__(64) void perm_kernel(MergeArgs a) {
  __shared__ MTileLds L;
  const uint32_t t = blockIdx.x;
  if (t >= uni(uint32_t(a.mstats[1]))) return;
  tile_ranges(a, L, t, uint32_t(reinterpret_cast<uintptr_t>(a.keys) & 15));
  const uint64_t base = a.tpre[t];
  for (uint32_t u = lane_id(); u < L.total; u += 64) {
    const uint32_t r = find_run(L.tb, a.nrun, u), g = L.lo[r] + u - L.tb[r];
    const uint32_t k = a.mrank[g];
    if (k < a.tcnt[t]) a.perm[base + k] = g;
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
  uint64_t* tile_pre;       // 3 per tile
  uint64_t* stats;          // [0] kept [1] key bytes [2] value bytes [3] error flags
  const uint64_t* merr;     // the merge stage's error flags (bad run table)
};

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

// The merged order must be non-decreasing in the user key: an unsorted input run (which
// MergeIterator assumes away, merge_iterator.rs:135-138) is reported, never followed.
__device__ __forceinline__ bool merged_in_order(const GatherArgs& a, uint64_t j) {
  const uint32_t i = a.perm[j];
  if (i >= a.n_max) return false;
  if (j == 0) return true;
  const uint32_t ip = a.perm[j - 1];
  if (ip >= a.n_max) return false;
  const GKeys K = gkeys(a.keys, a.key_off[a.n_max]);
  const uint32_t p0 = a.key_off[ip], p1 = a.key_off[i];
  return key_cmp(K, p0, a.key_off[ip + 1] - p0, p1, a.key_off[i + 1] - p1) <= 0;
}

__device__ __forceinline__ bool mkeep(const GatherArgs& a, uint64_t j) {
  if (!a.rules) return true;
  const uint32_t i = a.perm[j];
  const uint64_t t = a.ts[i];
  if (t > a.wm) return true;
  bool start = true;
  if (j > 0) {
    const uint32_t ip = a.perm[j - 1];
    start = !same_key_g(a, ip, i);
    if (!start && a.ts[ip] <= a.wm) return false;  // a later version at or below the watermark
  }
  if (a.bottom && start && a.val_off[i + 1] == a.val_off[i]) return false;  // :244-254
  const uint32_t k0 = a.key_off[i], kl = a.key_off[i + 1] - k0;
  for (uint32_t f = 0; f < a.npfx; ++f) {  // CompactionFilter::Prefix, :264-275
    const uint32_t f0 = a.pfx_off[f], fl = a.pfx_off[f + 1] - f0;
    if (fl > kl) continue;
    bool m = true;
    for (uint32_t x = 0; x < fl && m; ++x) m = a.pfx[f0 + x] == a.keys[k0 + x];
    if (m) return false;
  }
  return true;
}

__global__ __launch_bounds__(256) void mflag_kernel(GatherArgs a) {
  const uint64_t N = *a.nm;
  uint32_t c = 0;
  uint64_t kb = 0, vb = 0;
#pragma unroll
  for (uint32_t sub = 0; sub < kGTile / 256; ++sub) {
    const uint64_t j = uint64_t(blockIdx.x) * kGTile + sub * 256 + threadIdx.x;
    if (j < N) {
      bool k = false;
      if (merged_in_order(a, j)) k = mkeep(a, j);
      else atomicOr(reinterpret_cast<unsigned long long*>(a.stats + 3), (unsigned long long)LSMBLK_ERR_MALFORMED);
      a.keep[j] = k;
      if (k) {
        const uint32_t i = a.perm[j];
        c += 1;
        kb += a.key_off[i + 1] - a.key_off[i];
        vb += a.val_off[i + 1] - a.val_off[i];
      }
    }
  }
  __shared__ uint64_t ws[4][3];
  const uint32_t w = threadIdx.x >> 6;
  const uint32_t sc = wave_sum32(c);
  const uint64_t sk = wave_sum<uint64_t>(kb), sv = wave_sum<uint64_t>(vb);
  if (lane_id() == 0) ws[w][0] = sc, ws[w][1] = sk, ws[w][2] = sv;
  __syncthreads();
  if (threadIdx.x < 3) {
    const uint32_t q = threadIdx.x;
    a.tile_sum[3 * uint64_t(blockIdx.x) + q] = ws[0][q] + ws[1][q] + ws[2][q] + ws[3][q];
  }
}

__global__ __launch_bounds__(1024) void mscan_kernel(GatherArgs a) {
  const uint32_t t = threadIdx.x, w = t >> 6;
  const uint64_t N = *a.nm, ntiles = (N + kGTile - 1) / kGTile;
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

// len bytes src -> dst by one lane, any alignment: 16-B unaligned pieces, the last overlapping.
__device__ __forceinline__ void lane_copy(uint8_t* dst, const uint8_t* src, uint32_t len) {
  if (len < 16) {
    for (uint32_t x = 0; x < len; ++x) dst[x] = src[x];
    return;
  }
  for (uint32_t o = 0;; o += 16) {
    const uint32_t p = o + 16 <= len ? o : len - 16;
    *reinterpret_cast<u32x4*>(dst + p) = *reinterpret_cast<const u32x4*>(src + p);
    if (p == len - 16) break;
  }
}

__global__ __launch_bounds__(256) void mwrite_kernel(GatherArgs a) {
  if (a.stats[3]) return;
  const uint64_t N = *a.nm;
  __shared__ uint64_t ws[4][3];
  const uint32_t w = threadIdx.x >> 6;
  uint64_t carry[3] = {a.tile_pre[3 * uint64_t(blockIdx.x)], a.tile_pre[3 * uint64_t(blockIdx.x) + 1],
                       a.tile_pre[3 * uint64_t(blockIdx.x) + 2]};
  for (uint32_t sub = 0; sub < kGTile / 256; ++sub) {
    const uint64_t j = uint64_t(blockIdx.x) * kGTile + sub * 256 + threadIdx.x;
    const bool k = j < N && a.keep[j];
    const uint32_t i = k ? a.perm[j] : 0u;
    const uint32_t kl = k ? a.key_off[i + 1] - a.key_off[i] : 0u;
    const uint32_t vl = k ? a.val_off[i + 1] - a.val_off[i] : 0u;
    const uint32_t ic = wave_incl_scan32(k ? 1u : 0u);
    const uint64_t ik = wave_incl_scan<uint64_t>(kl), iv = wave_incl_scan<uint64_t>(vl);
    if (lane_id() == 63) ws[w][0] = ic, ws[w][1] = ik, ws[w][2] = iv;
    __syncthreads();
    uint64_t o = carry[0] + ic - 1, ko = carry[1] + ik - kl, vo = carry[2] + iv - vl;
    for (uint32_t q = 0; q < w; ++q) o += ws[q][0], ko += ws[q][1], vo += ws[q][2];
#pragma unroll
    for (uint32_t q = 0; q < 3; ++q) carry[q] += ws[0][q] + ws[1][q] + ws[2][q] + ws[3][q];
    __syncthreads();
    if (k) {
      a.okey_off[o] = uint32_t(ko);
      a.oval_off[o] = uint32_t(vo);
      a.ots[o] = a.ts[i];
      lane_copy(a.okeys + ko, a.keys + a.key_off[i], kl);
      lane_copy(a.ovals + vo, a.vals + a.val_off[i], vl);
    }
  }
}

__global__ void merge_empty_kernel(uint64_t* mstats, uint32_t* okey_off, uint32_t* oval_off, uint64_t entry_cap,
                                   uint64_t* stats) {
  if (threadIdx.x == 0) {
    mstats[0] = 0;
    mstats[1] = 0;
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
//                      chain elements [2^k, 2^(k+1)) and squares F)
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
  uint32_t* J;              // levels x (n_max + 1)
  uint32_t* S;              // levels x (n_max + 1)
  uint32_t levels;          // levels allocated for J / S
  uint32_t* F0;             // n_max + 1: F, then the doubling ping-pong
  uint32_t* F1;
  uint32_t* need;           // kRotMaxLevels: level k still has a chain short of target and end
  uint32_t* chain_end;      // [0] set once the SST chain reached the end
  uint32_t* starts;         // sst_cap: SST start entries (the chain), then n
  uint32_t sst_cap;
  uint32_t* nsst;           // device: SST count handed to the encode (0 after an error)
  uint64_t* stats;          // [0] SSTs [3] error flags
};

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

__global__ __launch_bounds__(256) void rot_adj_kernel(RotArgs a) {
  const uint64_t n = rot_n(a);
  const uint64_t e = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  if (e >= n) return;
  const uint32_t kp = a.key_off[e], kl = a.key_off[e + 1] - kp;
  a.rec[e] = kl + (a.val_off[e + 1] - a.val_off[e]);
  uint32_t al = 0;
  if (e > 0) {
    const GKeys K = gkeys(a.keys, a.key_off[n]);
    const uint32_t pp = a.key_off[e - 1], pl = kp - pp;
    int ord = 0;
    const uint32_t lcp = glcp(K, pp, pl, kp, kl, &ord);
    al = (lcp < kRotLcp ? lcp : kRotLcp) | (ord > 0 ? kRotUnsorted : 0u) | (ord == 0 ? kRotSame : 0u);
  }
  a.alcp[e] = al;
}

__device__ __forceinline__ void or_need(uint32_t* flag, bool v) {
  if (__ballot(v) && lane_id() == 0) atomicOr(flag, 1u);
}

__global__ __launch_bounds__(256) void rot_next_kernel(RotArgs a) {
  const uint64_t n = rot_n(a);
  const uint64_t s = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  bool short_chain = false;
  if (s < n) {
    const uint64_t bs = a.block_size;
    uint64_t before = 2 + uint64_t(a.rec[s]) + 16;  // entry s always accepted, prefix 0
    uint32_t pmin = kRotLcp;
    bool direct = false;
    uint32_t sp = 0, sl = 0;
    GKeys K;
    uint64_t e = s + 1;
    for (; e < n; ++e) {
      const uint32_t r = a.rec[e], al = a.alcp[e];
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
    a.J[s] = uint32_t(e);
    a.S[s] = sz > 0xFFFFFFFFull ? 0xFFFFFFFFu : uint32_t(sz);
    short_chain = e < n && sz < a.target;
  } else if (s == n) {
    a.J[s] = uint32_t(n);
    a.S[s] = 0;
  }
  or_need(a.need + 0, short_chain);
}

__global__ __launch_bounds__(256) void rot_double_kernel(RotArgs a, uint32_t k) {
  if (!*(volatile uint32_t*)(a.need + k - 1)) return;  // every chain done one level down
  const uint64_t n = rot_n(a);
  const uint64_t s = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  const uint64_t N1 = a.n_max + 1;
  bool short_chain = false;
  if (s <= n) {
    const uint32_t* J0 = a.J + (k - 1) * N1;
    const uint32_t* S0 = a.S + (k - 1) * N1;
    const uint32_t j = J0[s];
    const uint32_t jj = J0[j];
    const uint64_t ss = uint64_t(S0[s]) + S0[j];
    a.J[k * N1 + s] = jj;
    a.S[k * N1 + s] = ss > 0xFFFFFFFFull ? 0xFFFFFFFFu : uint32_t(ss);
    short_chain = jj < n && ss < a.target;
  }
  or_need(a.need + k, short_chain);
}

__global__ __launch_bounds__(256) void rot_f_kernel(RotArgs a) {
  const uint64_t n = rot_n(a);
  const uint64_t g = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  if (g > n) return;
  if (g == n) {
    a.F0[g] = uint32_t(n);
    return;
  }
  const uint64_t N1 = a.n_max + 1;
  uint32_t kc = 1;  // levels computed: 0 .. kc-1
  while (kc < a.levels && a.need[kc - 1]) ++kc;
  uint64_t pos = g, acc = 0;
  const uint32_t top = kc - 1;
  // lifting: the longest chain prefix from g whose data stays below the target
  while (pos < n && acc + a.S[top * N1 + pos] < a.target) {
    acc += a.S[top * N1 + pos];
    pos = a.J[top * N1 + pos];
  }
  for (int k = int(top) - 1; k >= 0; --k) {
    if (pos < n && acc + a.S[uint64_t(k) * N1 + pos] < a.target) {
      acc += a.S[uint64_t(k) * N1 + pos];
      pos = a.J[uint64_t(k) * N1 + pos];
    }
  }
  uint64_t f = n;
  if (pos < n) {
    const uint64_t sj = a.J[pos];  // s_{j*}: the first block start whose entries see D >= target
    if (sj < n) {
      f = sj + 1;
      while (f < n && (a.alcp[f] & kRotSame)) ++f;  // the first key change after it
    }
  }
  a.F0[g] = uint32_t(f);
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
  if (s <= n) nxt[s] = cur[cur[s]];
}

// After each level: has the last chain element computed so far reached the end?
__global__ void rot_chain_check_kernel(RotArgs a, uint32_t k) {
  if (threadIdx.x || *(volatile uint32_t*)a.chain_end) return;
  const uint64_t n = rot_n(a);
  const uint64_t last = (2ull << k) - 1;  // elements [0, 2^(k+1)) are computed now
  // the array is full (rot_finish_kernel then decides whether the chain ended) or it ended
  if (last >= a.sst_cap || a.starts[last] >= n) *a.chain_end = k + 1;
}

__global__ __launch_bounds__(256) void rot_finish_kernel(RotArgs a) {
  const uint64_t n = rot_n(a);
  __shared__ uint32_t s_ns;
  if (threadIdx.x == 0) {
    // SST count: the computed chain elements below n (increasing, then n), by binary search
    const uint32_t done = *a.chain_end;
    uint32_t lo = 0, hi = done ? uint32_t(min<uint64_t>(a.sst_cap, 1ull << done)) : 1u;
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
    uint32_t err = 0;
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
  P.m.cand = cv.take<uint32_t>(nc_max + 1);
  P.m.bounds = cv.take<uint32_t>(uint64_t(nrun) * (nc_max + 1));
  P.m.mrank = cv.take<uint32_t>(n + 1);
  P.m.sp = cv.take<uint32_t>(n + 1);
  P.m.tcnt = cv.take<uint32_t>(nc_max + 1);
  P.m.tpre = cv.take<uint64_t>(nc_max + 2);
  P.m.perm = cv.take<uint32_t>(n + 1);
  P.m.mstats = cv.take<uint64_t>(8);
  P.keep = cv.take<uint32_t>(n + 1);
  P.gtiles = (n + kGTile - 1) / kGTile + 1;
  P.gtile = cv.take<uint64_t>(6 * P.gtiles);
  P.bytes = cv.off;
  return P;
}

int ensure_ws(lsmblk_ctx* c, uint64_t bytes) {
  if (bytes <= c->cws_cap) return LSMBLK_OK;
  return grow(&c->cws, &c->cws_cap, bytes, 1);
}

// merge + (rules | keep all) + gather into `out`; stats as lsmblk_compact_filter_batch's.
int merge_gather_locked(lsmblk_ctx* c, const lsmblk_kv_stream* in, const uint32_t* run_start, uint32_t nrun,
                        uint32_t rules, uint64_t wm, int bottom, const uint8_t* pfx, const uint32_t* pfx_off,
                        uint32_t npfx, const lsmblk_kv_stream* out, uint64_t* stats, hipStream_t st,
                        MergePlan* plan_out) {
  const uint64_t n = in->n;
  MergePlan P = plan_merge(nullptr, n, nrun);
  int rc = ensure_ws(c, P.bytes);
  if (rc) return rc;
  P = plan_merge(c->cws, n, nrun);
  if (plan_out) *plan_out = P;
  MergeArgs& m = P.m;
  m.keys = in->keys;
  m.key_off = in->key_off;
  m.n = n;
  m.run_start = run_start;
  m.nrun = nrun;
  if (hipMemsetAsync(stats, 0, LSMBLK_STATS_WORDS * 8, st) != hipSuccess) return LSMBLK_E_HIP;
  if (n == 0) {
    hipLaunchKernelGGL(merge_empty_kernel, dim3(1), dim3(64), 0, st, m.mstats, out->key_off, out->val_off,
                       out->entry_cap, stats);
    return hipGetLastError() == hipSuccess ? LSMBLK_OK : LSMBLK_E_HIP;
  }
  if (hipMemsetAsync(m.mstats, 0, 64, st) != hipSuccess) return LSMBLK_E_HIP;
  const uint32_t nc = m.nc_max;
  hipLaunchKernelGGL(cand_rank_kernel, dim3((nc + 255) / 256), dim3(256), 0, st, m);
  const uint64_t nb = (uint64_t(nc) + 1) * nrun;
  hipLaunchKernelGGL(bounds_kernel, dim3(uint32_t((nb + 255) / 256)), dim3(256), 0, st, m);
  hipLaunchKernelGGL(merge_tile_kernel, dim3(nc), dim3(64), 0, st, m);
  hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(1024), 0, st, m);
  hipLaunchKernelGGL(perm_kernel, dim3(nc), dim3(64), 0, st, m);
  if (hipGetLastError() != hipSuccess) return LSMBLK_E_HIP;
  GatherArgs g;
  g.keys = in->keys;
  g.key_off = in->key_off;
  g.vals = in->vals;
  g.val_off = in->val_off;
  g.ts = in->ts;
  g.perm = m.perm;
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
  g.stats = stats;
  g.merr = m.mstats + 3;
  const uint32_t gt = uint32_t((n + kGTile - 1) / kGTile);
  hipLaunchKernelGGL(mflag_kernel, dim3(gt), dim3(256), 0, st, g);
  hipLaunchKernelGGL(mscan_kernel, dim3(1), dim3(1024), 0, st, g);
  hipLaunchKernelGGL(mwrite_kernel, dim3(gt), dim3(256), 0, st, g);
  return hipGetLastError() == hipSuccess ? LSMBLK_OK : LSMBLK_E_HIP;
}

__global__ void set_u64_kernel(uint64_t* p, uint64_t v) {
  if (threadIdx.x == 0) *p = v;
}

// The kept-entry count the rotation and the encode see: 0 after any merge / rules error.
__global__ void gate_kernel(const uint64_t* fst, uint64_t* dn) {
  if (threadIdx.x == 0) *dn = fst[3] ? 0ull : fst[0];
}

uint32_t rot_levels(uint64_t target) {
  // a block and its CRC take >= 23 bytes (4 + 1 + 8 + 2 + 2 + 2 + 4), so an SST reaches the
  // target within ceil(target / 23) blocks: 2^(levels-1) hops cover it
  const uint64_t j = target / 23 + 2;
  uint32_t k = 1;
  while (k < kRotMaxLevels && (1ull << (k - 1)) < j) ++k;
  return k;
}

struct RotPlan {
  RotArgs r;
  uint64_t* dn;     // device n for the rotation
  uint64_t bytes;
};

RotPlan plan_rot(uint8_t* base, uint64_t off, uint64_t n_max, uint64_t target) {
  RotPlan P{};
  Carve cv{base, off};
  const uint64_t N1 = n_max + 1;
  const uint32_t L = rot_levels(target);
  P.r.n_max = n_max;
  P.r.target = target;
  P.r.levels = L;
  P.r.rec = cv.take<uint32_t>(N1);
  P.r.alcp = cv.take<uint32_t>(N1);
  P.r.J = cv.take<uint32_t>(N1 * L);
  P.r.S = cv.take<uint32_t>(N1 * L);
  P.r.F0 = cv.take<uint32_t>(N1);
  P.r.F1 = cv.take<uint32_t>(N1);
  P.r.need = cv.take<uint32_t>(kRotMaxLevels + 2);
  P.r.chain_end = P.r.need + kRotMaxLevels;
  P.r.nsst = P.r.need + kRotMaxLevels + 1;
  P.dn = cv.take<uint64_t>(2);
  P.bytes = cv.off;
  return P;
}

// SST cut points of the stream (keys, key_off, val_off; *dn entries, <= n_max) into starts[]
int rotation_locked(lsmblk_ctx* c, RotArgs r, hipStream_t st) {
  (void)c;
  if (hipMemsetAsync(r.need, 0, (kRotMaxLevels + 2) * sizeof(uint32_t), st) != hipSuccess) return LSMBLK_E_HIP;
  if (hipMemsetAsync(r.starts, 0, sizeof(uint32_t), st) != hipSuccess) return LSMBLK_E_HIP;
  const uint32_t g = uint32_t((r.n_max + 1 + 255) / 256);
  hipLaunchKernelGGL(rot_adj_kernel, dim3(g), dim3(256), 0, st, r);
  hipLaunchKernelGGL(rot_next_kernel, dim3(g), dim3(256), 0, st, r);
  for (uint32_t k = 1; k < r.levels; ++k) hipLaunchKernelGGL(rot_double_kernel, dim3(g), dim3(256), 0, st, r, k);
  hipLaunchKernelGGL(rot_f_kernel, dim3(g), dim3(256), 0, st, r);
  uint32_t* cur = r.F0;
  uint32_t* nxt = r.F1;
  for (uint32_t k = 0; k < 32 && (1ull << k) < r.sst_cap; ++k) {
    hipLaunchKernelGGL(rot_chain_kernel, dim3(g), dim3(256), 0, st, r, k, cur, nxt);
    hipLaunchKernelGGL(rot_chain_check_kernel, dim3(1), dim3(64), 0, st, r, k);
    uint32_t* t = cur;
    cur = nxt;
    nxt = t;
  }
  hipLaunchKernelGGL(rot_finish_kernel, dim3(1), dim3(256), 0, st, r);
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

}  // namespace

extern "C" {

int lsmblk_merge_batch(lsmblk_ctx* c, const lsmblk_kv_stream* in, const uint32_t* run_start, uint32_t nrun,
                       const lsmblk_kv_stream* out, uint64_t* stats, void* stream) {
  int rc = check_merge_args(c, in, run_start, nrun, out, stats);
  if (rc) return rc;
  std::lock_guard<std::mutex> g(c->mu);
  DeviceGuard dg(c->device);
  if (!dg.ok) return LSMBLK_E_HIP;
  return merge_gather_locked(c, in, run_start, nrun, 0, 0, 0, nullptr, nullptr, 0, out, stats,
                             reinterpret_cast<hipStream_t>(stream), nullptr);
}

int lsmblk_sst_rotation_batch(lsmblk_ctx* c, const lsmblk_kv_stream* in, uint32_t block_size,
                              uint64_t target_sst_size, uint32_t* sst_start, uint32_t sst_cap, uint64_t* stats,
                              void* stream) {
  if (!c || !in || !sst_start || !stats || !in->key_off || !in->val_off) return LSMBLK_E_INVAL;
  if (block_size == 0 || target_sst_size == 0 || sst_cap == 0 || in->n >= 0xFFFFFFF0ull) return LSMBLK_E_INVAL;
  std::lock_guard<std::mutex> g(c->mu);
  DeviceGuard dg(c->device);
  if (!dg.ok) return LSMBLK_E_HIP;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  RotPlan P = plan_rot(nullptr, 0, in->n, target_sst_size);
  int rc = ensure_ws(c, P.bytes);
  if (rc) return rc;
  P = plan_rot(c->cws, 0, in->n, target_sst_size);
  if (hipMemsetAsync(stats, 0, LSMBLK_STATS_WORDS * 8, st) != hipSuccess) return LSMBLK_E_HIP;
  hipLaunchKernelGGL(set_u64_kernel, dim3(1), dim3(64), 0, st, P.dn, uint64_t(in->n));
  RotArgs r = P.r;
  r.keys = in->keys;
  r.key_off = in->key_off;
  r.val_off = in->val_off;
  r.dn = P.dn;
  r.block_size = block_size;
  r.starts = sst_start;
  r.sst_cap = sst_cap;
  r.stats = stats;
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
  if ((reinterpret_cast<uintptr_t>(out) & 15) != 0) return LSMBLK_E_INVAL;
  std::lock_guard<std::mutex> g(c->mu);
  DeviceGuard dg(c->device);
  if (!dg.ok) return LSMBLK_E_HIP;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const uint64_t n = in->n;
  // workspace: merge + gather, then rotation, then the stage stats
  MergePlan M = plan_merge(nullptr, n, nrun);
  RotPlan R = plan_rot(nullptr, M.bytes, n, o->target_sst_size);
  const uint64_t stats_off = (R.bytes + 255) & ~uint64_t(255);
  if ((rc = ensure_ws(c, stats_off + 4 * 64))) return rc;
  uint64_t* sts = reinterpret_cast<uint64_t*>(c->cws + stats_off);
  uint64_t *fst = sts, *rst = sts + 8, *est = sts + 16;
  if (hipMemsetAsync(sts, 0, 4 * 64, st) != hipSuccess) return LSMBLK_E_HIP;
  if (hipMemsetAsync(stats, 0, LSMBLK_COMPACT_STATS_WORDS * 8, st) != hipSuccess) return LSMBLK_E_HIP;
  if (hipMemsetAsync(blk_off, 0, 8, st) != hipSuccess) return LSMBLK_E_HIP;
  MergePlan MP{};
  if ((rc = merge_gather_locked(c, in, run_start, nrun, 1, o->watermark, o->bottom_level, o->prefixes, o->prefix_off,
                                o->nprefix, kept, fst, st, &MP)))
    return rc;
  R = plan_rot(c->cws, M.bytes, n, o->target_sst_size);
  hipLaunchKernelGGL(gate_kernel, dim3(1), dim3(64), 0, st, fst, R.dn);
  RotArgs r = R.r;
  r.keys = kept->keys;
  r.key_off = kept->key_off;
  r.val_off = kept->val_off;
  r.dn = R.dn;  // kept entries (0 after a merge / rules error)
  r.block_size = o->block_size;
  r.starts = sst_start;
  r.sst_cap = sst_cap;
  r.stats = rst;
  if ((rc = rotation_locked(c, r, st))) return rc;
  lsmblk_kv_stream ks = *kept;
  ks.n = n;  // bound; the encode reads the kept count from fst[0]
  if ((rc = lsmblk_impl::encode_locked(c, &ks, R.dn, sst_start, r.nsst, sst_cap - 1, o->block_size, out, out_cap,
                                       blk_off, blk_cap, est, st)))
    return rc;
  if ((rc = lsmblk_impl::segment_blocks_locked(c, sst_start, sst_cap - 1, est, sst_blk, st))) return rc;
  hipLaunchKernelGGL(compact_stats_kernel, dim3(1), dim3(64), 0, st, stats, fst, rst, est, MP.m.mstats);
  return hipGetLastError() == hipSuccess ? LSMBLK_OK : LSMBLK_E_HIP;
}

}  // extern "C"
