// What a 16-byte-per-lane vector load costs beside MFMAs, by form: 8 waves
// per CU (one 512-thread workgroup, 2 per SIMD) in barrier lock-step, each
// iteration 32 v_mfma_f32_16x16x32_bf16 per wave in 4 groups of 8, and after
// each group one load of 1 KB per wave from an L2-resident buffer:
//   mode 0: no loads; 1: global_load_lds_dwordx4 into an LDS ring;
//   2: global_load_dwordx4 into VGPRs (inline asm, two register sets);
//   3: both (2 glds + 2 register loads per iteration).
// Prints s_memtime cycles per iteration (mean over workgroups).  GPU box:
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench/bin/issue_ubench tools/ubench/issue_ubench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void glds16(const void* gsrc, void* ldst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gsrc,
                                   (__attribute__((address_space(3))) void*)ldst, 16, 0, 0);
}

template <int MODE>
__global__ __launch_bounds__(512, 1) void issue_k(const uint16_t* __restrict__ src, int iters, int span,
                                                  float* __restrict__ out, unsigned long long* __restrict__ cyc) {
  __shared__ __attribute__((aligned(16))) uint16_t ring[4 * 8 * 512];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  f32x4 acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = (f32x4)(float)(tid + i);
  bf16x8 a, b;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(0.001f * (lane + i));
    b[i] = (__bf16)(0.002f * (wave + i));
  }
  u32x4 rA[4], rB[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) rA[g] = rB[g] = (u32x4)0u;
  const int base = (blockIdx.x * 8 + wave) * 64 + lane;
  // one iteration into register set R (the set loaded two iterations ago)
  auto body = [&](int it, u32x4(&R)[4]) {
    if constexpr (MODE != 0) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    if constexpr (MODE >= 2) asm volatile("" : "+v"(R[0]), "+v"(R[1]), "+v"(R[2]), "+v"(R[3]));
    asm volatile("s_barrier" ::: "memory");
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[k], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      const uint16_t* p = src + (size_t)(((it * 4 + g) * 512 * 64 + base * 8) % span);
      const bool lds = MODE == 1 || (MODE == 3 && (g & 1) == 0);
      const bool reg = MODE == 2 || (MODE == 3 && (g & 1) == 1);
      if (lds) glds16(p, ring + ((it & 3) * 8 + wave) * 512);
      if (reg) asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(R[g]) : "v"(p) : "memory");
    }
  };
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; it += 2) {
    body(it, rA);
    body(it + 1, rB);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  s += (float)(rA[0][0] ^ rA[1][1] ^ rB[2][2] ^ rB[3][3]) * 1e-30f;
  out[blockIdx.x * 512 + tid] = s;
  if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  const int G = 256, iters = 2000;
  const int span = 1 << 20;  // elements: 2 MB, L2-resident after the first pass
  uint16_t* src;
  float* out;
  unsigned long long* cyc;
  (void)hipMalloc(&src, (size_t)span * 2 + 65536);
  (void)hipMemset(src, 0x3c, (size_t)span * 2 + 65536);
  (void)hipMalloc(&out, G * 512 * 4);
  (void)hipMalloc(&cyc, G * 8);
  std::vector<unsigned long long> h(G);
  const char* names[4] = {"MFMA only", "+ 4 glds / wave / iter", "+ 4 global_load_dwordx4 / wave / iter",
                          "+ 2 glds + 2 global_load_dwordx4"};
  for (int rep = 0; rep < 2; ++rep)
    for (int mode = 0; mode < 4; ++mode) {
      for (int w = 0; w < 2; ++w) {
        switch (mode) {
          case 0: issue_k<0><<<G, 512>>>(src, iters, span, out, cyc); break;
          case 1: issue_k<1><<<G, 512>>>(src, iters, span, out, cyc); break;
          case 2: issue_k<2><<<G, 512>>>(src, iters, span, out, cyc); break;
          default: issue_k<3><<<G, 512>>>(src, iters, span, out, cyc); break;
        }
      }
      (void)hipDeviceSynchronize();
      (void)hipMemcpy(h.data(), cyc, G * 8, hipMemcpyDeviceToHost);
      double m = 0;
      for (int i = 0; i < G; ++i) m += (double)h[i];
      m /= G;
      printf("mode %d %-42s %7.0f cycles / iteration (MFMA floor 1024 per SIMD)\n", mode, names[mode], m / iters);
    }
  return 0;
}
