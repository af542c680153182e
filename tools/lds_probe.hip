// LDS read-rate probe (timing experiment, not product code): cycles per ds_read_b32
// wave-instruction per CU for several lane -> address patterns, with 4..20 waves per CU.
// build: hipcc --offload-arch=gfx950 -O3 tools/lds_probe.hip -o tools/lds_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int kIters = 4096;

template <int MODE>
__global__ __launch_bounds__(256) void probe(uint32_t* out, uint32_t seed) {
  __shared__ uint32_t tab[2048];
  for (int i = threadIdx.x; i < 2048; i += 256) tab[i] = i * 2654435761u;
  __syncthreads();
  const uint32_t l = threadIdx.x & 63;
  uint32_t x = seed ^ (l * 0x9E3779B9u) ^ (blockIdx.x * 0x85EBCA6Bu);
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  x ^= x >> 16;
  uint32_t ad[8];  // byte addresses, fixed per lane: the probe times the LDS, not the VALU
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    uint32_t a;
    if (MODE == 0) a = 16 * k + ((x >> (4 * k)) & 15);                       // nibble tables
    else if (MODE == 1) a = 64 * k + l;                                        // lane-linear
    else if (MODE == 2) a = 16 * k;                                            // broadcast
    else if (MODE == 3) a = 256 * (k & 3) + ((x >> (8 * (k & 3))) & 255) + 1024 * (k >> 2);  // byte tables
    else a = (17 * l + k) & 2047;                                              // stride-17 windows
    ad[k] = 4 * a + uint32_t(reinterpret_cast<uintptr_t>(tab));
  }
  uint32_t acc = 0;
  for (int it = 0; it < kIters; ++it) {
    uint32_t v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) asm volatile("ds_read_b32 %0, %1" : "=v"(v[k]) : "v"(ad[k]));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += v[k];
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

template <int MODE>
float run(int wgs_per_cu, int cus) {
  uint32_t* d;
  (void)hipMalloc(&d, 1 << 20);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  probe<MODE><<<wgs_per_cu * cus, 256>>>(d, 1);
  (void)hipEventRecord(a);
  probe<MODE><<<wgs_per_cu * cus, 256>>>(d, 2);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipFree(d);
  return ms;
}

int main() {
  int cus = 0, clk = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);  // kHz
  const char* names[] = {"nibble", "linear", "bcast", "byte", "stride17"};
  for (int wg : {1, 2, 3, 5}) {
    for (int mode = 0; mode < 5; ++mode) {
      float ms = mode == 0 ? run<0>(wg, cus) : mode == 1 ? run<1>(wg, cus) : mode == 2 ? run<2>(wg, cus)
               : mode == 3 ? run<3>(wg, cus) : run<4>(wg, cus);
      const double instr_per_cu = double(wg) * 4 * kIters * 8;
      const double cyc = ms * 1e-3 * clk * 1e3;
      printf("waves/CU %2d %-8s %.3f ms  %.2f cycles per ds_read_b32 per CU\n", 4 * wg, names[mode], ms, cyc / instr_per_cu);
    }
  }
  return 0;
}
