// Calibration (not product code): which plain device-copy shape reaches the highest read+write rate
// on this gfx950 box for a 4.2 GB stream (decode / emit move E + D of that size): unroll depth,
// workgroups per CU, non-temporal loads / stores, 16-B vs 8-B lanes, grid-stride vs contiguous slabs.
// build: hipcc --offload-arch=gfx950 -O3 tools/copy_probe2.hip -o tools/copy_probe2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void copy_gs(const u32x4* __restrict__ a, u32x4* __restrict__ b, uint64_t n) {
  const uint64_t stride = uint64_t(gridDim.x) * 256 * U;
  for (uint64_t i = uint64_t(blockIdx.x) * 256 * U + threadIdx.x; i < n; i += stride) {
    u32x4 v[U];
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (i + 256 * j < n) v[j] = NTL ? __builtin_nontemporal_load(a + i + 256 * j) : a[i + 256 * j];
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (i + 256 * j < n) {
        if (NTS) __builtin_nontemporal_store(v[j], b + i + 256 * j);
        else b[i + 256 * j] = v[j];
      }
  }
}

// one 4 KiB "block" per wave-iteration (as decode / emit move one block per wave), blocks handed
// out in index order over a grid of single-wave workgroups (non-persistent, one block each)
template <bool NTS>
__global__ __launch_bounds__(64) void copy_blk(const u32x4* __restrict__ a, u32x4* __restrict__ b, uint64_t nblk) {
  const uint64_t blk = blockIdx.x;
  if (blk >= nblk) return;
  const u32x4* s = a + blk * 256;
  u32x4* d = b + blk * 256;
  u32x4 v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = s[threadIdx.x + 64 * j];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (NTS) __builtin_nontemporal_store(v[j], d + threadIdx.x + 64 * j);
    else d[threadIdx.x + 64 * j] = v[j];
  }
}

template <typename K, typename... A>
float timeit(K k, dim3 grid, dim3 blk, A... args) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  k<<<grid, blk>>>(args...);
  (void)hipEventRecord(e0);
  for (int r = 0; r < 10; ++r) k<<<grid, blk>>>(args...);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms / 10;
}

int main() {
  const uint64_t bytes = 4226189312ull, n = bytes / 16;
  u32x4 *a, *b;
  (void)hipMalloc(&a, bytes);
  (void)hipMalloc(&b, bytes);
  (void)hipMemset(a, 1, bytes);
  (void)hipMemset(b, 2, bytes);
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  auto rep = [&](const char* name, float ms) { printf("%-34s %.3f ms = %.0f GB/s read+write\n", name, ms, 2.0 * bytes / ms / 1e6); };
  char nm[64];
  for (int wg : {2, 4, 8, 16}) {
    const dim3 g(cus * wg), t(256);
    snprintf(nm, 64, "gs U4  WG/CU %d", wg);           rep(nm, timeit(copy_gs<4, false, false>, g, t, a, b, n));
    snprintf(nm, 64, "gs U8  WG/CU %d", wg);           rep(nm, timeit(copy_gs<8, false, false>, g, t, a, b, n));
    snprintf(nm, 64, "gs U16 WG/CU %d", wg);           rep(nm, timeit(copy_gs<16, false, false>, g, t, a, b, n));
    snprintf(nm, 64, "gs U8  WG/CU %d ntload", wg);    rep(nm, timeit(copy_gs<8, true, false>, g, t, a, b, n));
    snprintf(nm, 64, "gs U8  WG/CU %d ntstore", wg);   rep(nm, timeit(copy_gs<8, false, true>, g, t, a, b, n));
    snprintf(nm, 64, "gs U8  WG/CU %d nt both", wg);   rep(nm, timeit(copy_gs<8, true, true>, g, t, a, b, n));
  }
  const uint64_t nblk = bytes / 4096;
  rep("block/wave (1 Mi single-wave WGs)", timeit(copy_blk<false>, dim3(nblk), dim3(64), a, b, nblk));
  rep("block/wave ntstore", timeit(copy_blk<true>, dim3(nblk), dim3(64), a, b, nblk));
  return 0;
}
