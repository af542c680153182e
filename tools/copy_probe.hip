// Calibration (not product code): the best plain device copy / read this probe finds for 4.2 GB
// on gfx950, to put decode / emit (read one stream, write another) beside an achievable bound.
// build: hipcc --offload-arch=gfx950 -O3 tools/copy_probe.hip -o tools/copy_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <utility>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_k(const u32x4* __restrict__ a, u32x4* __restrict__ b, uint64_t n) {
  const uint64_t stride = uint64_t(gridDim.x) * 256 * U;
  for (uint64_t i = uint64_t(blockIdx.x) * 256 * U + threadIdx.x; i < n; i += stride) {
    u32x4 v[U];
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (i + 256 * j < n) v[j] = NT ? __builtin_nontemporal_load(a + i + 256 * j) : a[i + 256 * j];
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (i + 256 * j < n) {
        if (NT) __builtin_nontemporal_store(v[j], b + i + 256 * j);
        else b[i + 256 * j] = v[j];
      }
  }
}

// The same copy at byte offsets (so, dof) through buffer descriptors (as the product's large-block
// run copies do): unaligned 16-B loads and stores.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
template <int U>
__global__ __launch_bounds__(256) void copy_u(const uint8_t* a, uint8_t* b, uint32_t n16, uint32_t so, uint32_t dof,
                                              uint32_t bytes) {
  const __amdgpu_buffer_rsrc_t RA = rsrc(a, bytes + 64), RB = rsrc(b, bytes + 64);
  const uint32_t stride = gridDim.x * 256 * U;
  for (uint32_t i = blockIdx.x * 256 * U + threadIdx.x; i < n16; i += stride) {
    u32x4 v[U];
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (i + 256 * j < n16)
        v[j] = __builtin_amdgcn_raw_buffer_load_b128(RA, so + 16 * (i + 256 * j), 0, 0);
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (i + 256 * j < n16)
        __builtin_amdgcn_raw_buffer_store_b128(v[j], RB, dof + 16 * (i + 256 * j), 0, 0);
  }
}

template <int U>
__global__ __launch_bounds__(256) void read_k(const u32x4* __restrict__ a, uint64_t n, uint32_t* out) {
  const uint64_t stride = uint64_t(gridDim.x) * 256 * U;
  uint32_t acc = 0;
  for (uint64_t i = uint64_t(blockIdx.x) * 256 * U + threadIdx.x; i < n; i += stride) {
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (i + 256 * j < n) {
        const u32x4 v = __builtin_nontemporal_load(a + i + 256 * j);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
      }
  }
  if (acc == 0x9E3779B9u) out[0] = acc;
}

int main() {
  const uint64_t bytes = 4226189312ull, n = bytes / 16;
  u32x4 *a, *b;
  uint32_t* o;
  (void)hipMalloc(&a, bytes);
  (void)hipMalloc(&b, bytes);
  (void)hipMalloc(&o, 64);
  (void)hipMemset(a, 1, bytes);
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int wg : {4, 8, 16}) {
    const uint32_t grid = uint32_t(cus * wg);
    float ms = 0;
    for (int nt = 0; nt < 2; ++nt) {
      auto k = nt ? copy_k<4, true> : copy_k<4, false>;
      k<<<grid, 256>>>(a, b, n);
      (void)hipEventRecord(e0);
      for (int r = 0; r < 10; ++r) k<<<grid, 256>>>(a, b, n);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      (void)hipEventElapsedTime(&ms, e0, e1);
      ms /= 10;
      printf("copy%s WG/CU %2d: %.3f ms = %.0f GB/s read+write\n", nt ? "(nt)" : "    ", wg, ms, 2.0 * bytes / ms / 1e6);
    }
    read_k<4><<<grid, 256>>>(a, n, o);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 10; ++r) read_k<4><<<grid, 256>>>(a, n, o);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 10;
    printf("read  WG/CU %2d: %.3f ms = %.0f GB/s\n", wg, ms, 1.0 * bytes / ms / 1e6);
  }
  // unaligned 16-B copies (1 GiB, byte offsets so / dof): what misalignment costs each side
  const uint32_t ub = 1u << 30;
  for (auto [so, dof] : {std::pair<uint32_t, uint32_t>{0, 0}, {3, 0}, {0, 7}, {3, 7}, {5, 5}}) {
    float ms = 0;
    const uint32_t grid = uint32_t(cus * 8);
    copy_u<4><<<grid, 256>>>(reinterpret_cast<uint8_t*>(a), reinterpret_cast<uint8_t*>(b), ub / 16, so, dof, ub);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 10; ++r)
      copy_u<4><<<grid, 256>>>(reinterpret_cast<uint8_t*>(a), reinterpret_cast<uint8_t*>(b), ub / 16, so, dof, ub);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 10;
    printf("copy_u src+%u dst+%u: %.3f ms = %.0f GB/s read+write\n", so, dof, ms, 2.0 * ub / ms / 1e6);
  }
  return 0;
}
