// Calibration (not product code): does the ORDER in which persistent waves take 4 KiB blocks set
// the copy rate?  emit_kernel is a persistent grid whose waves take blocks w, w + NW, w + 2 NW, ...
// (one block ahead prefetched) and runs at about the grid-stride copy rate (5.2 TB/s), while one
// single-wave workgroup per block reached 5.7 (copy_probe2).  Variants, 4.2 GB read + written:
//   blk1   one block per single-wave workgroup (1 Mi workgroups)
//   blk4   one block per wave, 4-wave workgroups
//   pw     persistent waves, block stride NW, no prefetch
//   pwpf   persistent waves, block stride NW, next block's loads issued before this block's stores
//   slab   persistent waves, each a contiguous slab of blocks
//   blkk K one single-wave workgroup per K consecutive blocks, one block ahead prefetched
//   pwx    persistent waves, consecutive blocks on consecutive workgroups (XCDs)
// build: hipcc --offload-arch=gfx950 -O3 tools/copy_probe3.hip -o tools/copy_probe3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kB = 256;  // 16-B pieces per 4 KiB block

__device__ __forceinline__ uint32_t lane() { return threadIdx.x & 63; }

__global__ __launch_bounds__(64) void blk1(const u32x4* __restrict__ a, u32x4* __restrict__ b, uint64_t nblk) {
  const uint64_t blk = blockIdx.x;
  if (blk >= nblk) return;
  u32x4 v[4];
  for (int j = 0; j < 4; ++j) v[j] = a[blk * kB + lane() + 64 * j];
  for (int j = 0; j < 4; ++j) __builtin_nontemporal_store(v[j], b + blk * kB + lane() + 64 * j);
}

__global__ __launch_bounds__(256) void blk4(const u32x4* __restrict__ a, u32x4* __restrict__ b, uint64_t nblk) {
  const uint64_t blk = uint64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (blk >= nblk) return;
  u32x4 v[4];
  for (int j = 0; j < 4; ++j) v[j] = a[blk * kB + lane() + 64 * j];
  for (int j = 0; j < 4; ++j) __builtin_nontemporal_store(v[j], b + blk * kB + lane() + 64 * j);
}

template <bool PF>
__global__ __launch_bounds__(256) void pw(const u32x4* __restrict__ a, u32x4* __restrict__ b, uint64_t nblk) {
  const uint64_t nw = uint64_t(gridDim.x) * 4;
  uint64_t blk = uint64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (blk >= nblk) return;
  u32x4 v[4];
  for (int j = 0; j < 4; ++j) v[j] = a[blk * kB + lane() + 64 * j];
  for (;;) {
    const uint64_t nx = blk + nw;
    u32x4 w[4];
    if (PF && nx < nblk)
      for (int j = 0; j < 4; ++j) w[j] = a[nx * kB + lane() + 64 * j];
    for (int j = 0; j < 4; ++j) __builtin_nontemporal_store(v[j], b + blk * kB + lane() + 64 * j);
    if (nx >= nblk) break;
    if (PF) {
      for (int j = 0; j < 4; ++j) v[j] = w[j];
    } else {
      for (int j = 0; j < 4; ++j) v[j] = a[nx * kB + lane() + 64 * j];
    }
    blk = nx;
  }
}

__global__ __launch_bounds__(256) void slab(const u32x4* __restrict__ a, u32x4* __restrict__ b, uint64_t nblk) {
  const uint64_t nw = uint64_t(gridDim.x) * 4, w = uint64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const uint64_t per = (nblk + nw - 1) / nw, b0 = w * per, b1 = b0 + per < nblk ? b0 + per : nblk;
  for (uint64_t blk = b0; blk < b1; ++blk) {
    u32x4 v[4];
    for (int j = 0; j < 4; ++j) v[j] = a[blk * kB + lane() + 64 * j];
    for (int j = 0; j < 4; ++j) __builtin_nontemporal_store(v[j], b + blk * kB + lane() + 64 * j);
  }
}

// persistent, consecutive blocks on consecutive workgroups (so on consecutive XCDs, as in
// dispatch order): wave wv of workgroup g takes blocks g + G wv + k NW
template <bool PF>
__global__ __launch_bounds__(256) void pwx(const u32x4* __restrict__ a, u32x4* __restrict__ b, uint64_t nblk) {
  const uint64_t G = gridDim.x, nw = G * 4;
  uint64_t blk = uint64_t(blockIdx.x) + G * (threadIdx.x >> 6);
  if (blk >= nblk) return;
  u32x4 v[4];
  for (int j = 0; j < 4; ++j) v[j] = a[blk * kB + lane() + 64 * j];
  for (;;) {
    const uint64_t nx = blk + nw;
    u32x4 w[4];
    if (PF && nx < nblk)
      for (int j = 0; j < 4; ++j) w[j] = a[nx * kB + lane() + 64 * j];
    for (int j = 0; j < 4; ++j) __builtin_nontemporal_store(v[j], b + blk * kB + lane() + 64 * j);
    if (nx >= nblk) break;
    if (PF) {
      for (int j = 0; j < 4; ++j) v[j] = w[j];
    } else {
      for (int j = 0; j < 4; ++j) v[j] = a[nx * kB + lane() + 64 * j];
    }
    blk = nx;
  }
}

// one single-wave workgroup per K consecutive blocks, the next block's loads issued before this
// block's stores (emit's prefetch, but in dispatch order)
template <int K>
__global__ __launch_bounds__(64) void blkk(const u32x4* __restrict__ a, u32x4* __restrict__ b, uint64_t nblk) {
  uint64_t blk = uint64_t(blockIdx.x) * K;
  if (blk >= nblk) return;
  const uint64_t end = blk + K < nblk ? blk + K : nblk;
  u32x4 v[4];
  for (int j = 0; j < 4; ++j) v[j] = a[blk * kB + lane() + 64 * j];
  for (;;) {
    const uint64_t nx = blk + 1;
    u32x4 w[4];
    if (nx < end)
      for (int j = 0; j < 4; ++j) w[j] = a[nx * kB + lane() + 64 * j];
    for (int j = 0; j < 4; ++j) __builtin_nontemporal_store(v[j], b + blk * kB + lane() + 64 * j);
    if (nx >= end) break;
    for (int j = 0; j < 4; ++j) v[j] = w[j];
    blk = nx;
  }
}

template <class K, class... A>
float timeit(K k, dim3 g, dim3 t, A... args) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  k<<<g, t>>>(args...);
  (void)hipEventRecord(e0);
  for (int r = 0; r < 10; ++r) k<<<g, t>>>(args...);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms / 10;
}

int main() {
  const uint64_t nblk = 1031542, bytes = nblk * 4096;
  u32x4 *a = nullptr, *b = nullptr;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) return 1;
  (void)hipMemset(a, 1, bytes);
  (void)hipMemset(b, 0, bytes);
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  auto rep = [&](const char* name, float ms) { printf("%-28s %.3f ms = %.0f GB/s read+write\n", name, ms, 2.0 * bytes / ms / 1e6); };
  for (int rep_i = 0; rep_i < 2; ++rep_i) {
    rep("blk1", timeit(blk1, dim3(uint32_t(nblk)), dim3(64), a, b, nblk));
    rep("blk4", timeit(blk4, dim3(uint32_t((nblk + 3) / 4)), dim3(256), a, b, nblk));
    rep("blkk 2", timeit(blkk<2>, dim3(uint32_t((nblk + 1) / 2)), dim3(64), a, b, nblk));
    rep("blkk 4", timeit(blkk<4>, dim3(uint32_t((nblk + 3) / 4)), dim3(64), a, b, nblk));
    rep("blkk 8", timeit(blkk<8>, dim3(uint32_t((nblk + 7) / 8)), dim3(64), a, b, nblk));
    rep("blkk 32", timeit(blkk<32>, dim3(uint32_t((nblk + 31) / 32)), dim3(64), a, b, nblk));
    for (int wg : {3, 4, 8}) {
      char nm[64];
      snprintf(nm, 64, "pw   WG/CU %d", wg);   rep(nm, timeit(pw<false>, dim3(cus * wg), dim3(256), a, b, nblk));
      snprintf(nm, 64, "pwpf WG/CU %d", wg);   rep(nm, timeit(pw<true>, dim3(cus * wg), dim3(256), a, b, nblk));
      snprintf(nm, 64, "slab WG/CU %d", wg);   rep(nm, timeit(slab, dim3(cus * wg), dim3(256), a, b, nblk));
      snprintf(nm, 64, "pwx  WG/CU %d", wg);   rep(nm, timeit(pwx<false>, dim3(cus * wg), dim3(256), a, b, nblk));
      snprintf(nm, 64, "pwxpf WG/CU %d", wg);  rep(nm, timeit(pwx<true>, dim3(cus * wg), dim3(256), a, b, nblk));
    }
  }
  return 0;
}
