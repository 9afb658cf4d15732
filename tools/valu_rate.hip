// valu_rate.hip — issue rate of the VALU instructions the GF kernels are made
// of (v_perm_b32, v_bitop3_b32 xor3, v_xor_b32, v_and_b32, shifts), measured
// on the whole chip: every SIMD runs W waves of 8 independent chains of N
// instructions; rate = wave-instructions / (SIMDs x cycles).  A rate of 0.5
// per cycle per SIMD = one wave64 instruction every 2 cycles (SIMD-32 peak).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/valu_rate tools/valu_rate.hip
//   tools/valu_rate
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int kChains = 8;
constexpr int kIters = 4096;

template <int OP>
__global__ void __launch_bounds__(256) chain(uint32_t* out, uint32_t seed) {
  uint32_t v[kChains], t0 = seed ^ threadIdx.x, t1 = seed * 3u + blockIdx.x;
#pragma unroll
  for (int c = 0; c < kChains; ++c) v[c] = seed + c * 0x01010101u + threadIdx.x;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int c = 0; c < kChains; ++c) {
      if (OP == 0) v[c] = __builtin_amdgcn_perm(t0, t1, v[c] & 0x07070707u);  // perm + and
      if (OP == 1) v[c] = __builtin_amdgcn_perm(t0, t1, v[c]);                // perm only
      if (OP == 2) {
        uint32_t r;
        asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(v[c]), "v"(t0), "v"(t1));
        v[c] = r;
      }
      if (OP == 3) v[c] = v[c] ^ t0;
      if (OP == 4) v[c] = (v[c] >> 3) + t1;
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < kChains; ++c) s ^= v[c];
  if (s == 0x12345678u) out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OP>
double run(int cus, int waves_per_simd, const char* name, double ops_per_iter) {
  uint32_t* out;
  (void)hipMalloc(&out, 64 << 20);
  const int blocks = cus * waves_per_simd;  // 256 threads = 4 waves = one per SIMD
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(chain<OP>, dim3(blocks), dim3(256), 0, 0, out, 1u);
  (void)hipDeviceSynchronize();
  float best = 1e9f;
  for (int r = 0; r < 5; ++r) {
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(chain<OP>, dim3(blocks), dim3(256), 0, 0, out, 1u);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  int clk_khz = 0;
  (void)hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
  const double wave_instr = (double)blocks * 4 * kIters * kChains * ops_per_iter;
  const double simds = (double)cus * 4;
  const double cycles = best * 1e-3 * clk_khz * 1e3;
  const double rate = wave_instr / simds / cycles;
  printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"clock_mhz\": %d, "
         "\"wave_instr_per_simd_cycle\": %.3f}\n",
         name, waves_per_simd, best, clk_khz / 1000, rate);
  (void)hipFree(out);
  return rate;
}

int main() {
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  for (int w : {1, 2, 4, 8}) {
    run<0>(cus, w, "v_and + v_perm", 2);
    run<1>(cus, w, "v_perm", 1);
    run<2>(cus, w, "v_bitop3 (xor3)", 1);
    run<3>(cus, w, "v_xor", 1);
    run<4>(cus, w, "v_lshrrev + v_add", 2);
  }
  return 0;
}
