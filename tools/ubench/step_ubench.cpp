// Micro-benchmark of one conv tap step's skeleton on gfx950: per step each of
// 8 waves (2 per SIMD) issues NR ds_read_b128 and NM 16x16x32 bf16 MFMAs,
// then (optionally) a workgroup barrier.  Prints cycles per step (s_memtime
// is the 100 MHz constant clock on gfx950: converted with the measured ratio
// against the kernel wall time).  Build + run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/step_ubench tools/ubench/step_ubench.cpp && /tmp/step_ubench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

template <int PTW, int CTW, int MODE, int WAVES, int WGS = 1>
__global__ __launch_bounds__(WAVES * 64, WGS) void step_kernel(float* out, int steps, long long* cyc) {
  // MODE bit0: LDS reads, bit1: barrier each step, bit2: pipelined reads (next-step frags),
  // bit3: pipelined + forced interleave (1 read per MFMA group), bit4: pipelined + all
  // reads first, bit5: conflict-free B addresses
  constexpr int LDSN = 65536 / WGS;
  __shared__ __attribute__((aligned(16))) unsigned short lds[LDSN];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < LDSN; i += blockDim.x) lds[i] = (unsigned short)(i * 7);
  __syncthreads();
  int pb[PTW];
#pragma unroll
  for (int p = 0; p < PTW; ++p)
    pb[p] = (MODE & 32) ? ((lane >> 4) * 16 + p * 64 + (lane & 15)) * 16 : ((lane >> 4) * 392 + p * 16 + (lane & 15)) * 16 + (wave & 3) * 1024;
  int wb[CTW];
#pragma unroll
  for (int c = 0; c < CTW; ++c) wb[c] = LDSN * 2 - 32768 + ((lane >> 4) * 128 + c * 16 + (lane & 15)) * 16;
  f32x4 acc[PTW][CTW];
#pragma unroll
  for (int p = 0; p < PTW; ++p)
#pragma unroll
    for (int c = 0; c < CTW; ++c) acc[p][c] = (f32x4)0.f;
  u16x8 fa[CTW], fb[PTW];
#pragma unroll
  for (int c = 0; c < CTW; ++c) fa[c] = *(const u16x8*)((const char*)lds + wb[c]);
#pragma unroll
  for (int p = 0; p < PTW; ++p) fb[p] = *(const u16x8*)((const char*)lds + pb[p]);
  long long t0 = clock64();
  for (int s = 0; s < steps; ++s) {
    const int off = (s % 9) * 16;
    if constexpr (MODE & 4) {
      u16x8 na[CTW];
#pragma unroll
      for (int c = 0; c < CTW; ++c) na[c] = *(const u16x8*)((const char*)lds + wb[c] + off);
#pragma unroll
      for (int p = 0; p < PTW; ++p) {
#pragma unroll
        for (int c = 0; c < CTW; ++c)
          acc[p][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa[c]),
                                                               __builtin_bit_cast(bf16x8, fb[p]), acc[p][c], 0, 0, 0);
        fb[p] = *(const u16x8*)((const char*)lds + pb[p] + off);
      }
#pragma unroll
      for (int c = 0; c < CTW; ++c) fa[c] = na[c];
      if constexpr (MODE & 8) {
        __builtin_amdgcn_sched_group_barrier(0x100, CTW, 0);
#pragma unroll
        for (int p = 0; p < PTW; ++p) {
          __builtin_amdgcn_sched_group_barrier(0x008, CTW, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
      }
      if constexpr (MODE & 16) {
        __builtin_amdgcn_sched_group_barrier(0x100, CTW + PTW, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, CTW * PTW, 0);
      }
    } else {
      if constexpr (MODE & 1) {
#pragma unroll
        for (int c = 0; c < CTW; ++c) fa[c] = *(const u16x8*)((const char*)lds + wb[c] + off);
      }
#pragma unroll
      for (int p = 0; p < PTW; ++p) {
        u16x8 b = fb[p];
        if constexpr (MODE & 1) b = *(const u16x8*)((const char*)lds + pb[p] + off);
#pragma unroll
        for (int c = 0; c < CTW; ++c)
          acc[p][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa[c]),
                                                               __builtin_bit_cast(bf16x8, b), acc[p][c], 0, 0, 0);
      }
    }
    if constexpr (MODE & 2) {
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
  }
  long long t1 = clock64();
  float s = 0.f;
#pragma unroll
  for (int p = 0; p < PTW; ++p)
#pragma unroll
    for (int c = 0; c < CTW; ++c) s += acc[p][c][0] + acc[p][c][1] + acc[p][c][2] + acc[p][c][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x < 256) cyc[blockIdx.x] = t1 - t0;
}

template <int PTW, int CTW, int MODE, int WAVES, int WGS = 1>
void run(const char* name, float* out, long long* cyc) {
  const int steps = 2000;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  step_kernel<PTW, CTW, MODE, WAVES, WGS><<<256 * WGS, WAVES * 64>>>(out, 10, cyc);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  step_kernel<PTW, CTW, MODE, WAVES, WGS><<<256 * WGS, WAVES * 64>>>(out, steps, cyc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<long long> h(256);
  hipMemcpy(h.data(), cyc, 256 * 8, hipMemcpyDeviceToHost);
  double avg = 0;
  for (auto v : h) avg += v;
  avg /= 256;
  const double ns_per_step = ms * 1e6 / steps;
  const int mfma_per_simd = PTW * CTW * (WAVES / 4) * WGS;
  printf("%-34s ns/step %7.1f  (=%6.0f cyc @2.4GHz; MFMA floor %5d cyc, %.0f%%)  memtime/step %.1f\n", name,
         ns_per_step, ns_per_step * 2.4, mfma_per_simd * 16, 100.0 * mfma_per_simd * 16 / (ns_per_step * 2.4),
         avg / steps);
}

int main() {
  float* out;
  long long* cyc;
  hipMalloc(&out, 256 * 1024 * 4);
  hipMalloc(&cyc, 256 * 8);
  run<13, 2, 0, 8>("8w 13x2 mfma only", out, cyc);
  run<13, 2, 3, 8>("8w 13x2 mfma+lds+barrier", out, cyc);
  run<13, 2, 6 + 8, 8>("8w 13x2 pipe interleave", out, cyc);
  run<13, 2, 0, 4, 2>("2x4w 13x2 mfma only", out, cyc);
  run<13, 2, 3, 4, 2>("2x4w 13x2 mfma+lds+barrier", out, cyc);
  run<13, 2, 6 + 8, 4, 2>("2x4w 13x2 pipe interleave", out, cyc);
  run<7, 4, 3, 4, 2>("2x4w 7x4 mfma+lds+barrier", out, cyc);
  run<7, 4, 6 + 8, 4, 2>("2x4w 7x4 pipe interleave", out, cyc);
  run<4, 4, 3, 4, 2>("2x4w 4x4 mfma+lds+barrier", out, cyc);
  run<4, 4, 6 + 8, 4, 2>("2x4w 4x4 pipe interleave", out, cyc);
  return 0;
}
