// Does s_barrier on gfx950 wait for the workgroup's outstanding vector memory
// operations?  Each wave issues loads (or stores) to cold HBM lines, stamps
// s_memtime, runs `s_waitcnt lgkmcnt(0); s_barrier`, stamps again; the wave
// then waits for its loads (vmcnt(0)) and stamps a third time.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ unsigned long long st[64][8][3];

template <int MODE>  // 0 = nothing outstanding, 1 = loads outstanding, 2 = stores outstanding
__global__ __launch_bounds__(512) void kern(const unsigned* __restrict__ src, unsigned* __restrict__ dst, unsigned* out, int stride) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  unsigned v = 0;
  const size_t base = ((size_t)blockIdx.x * 512 + tid) * stride;
  if (MODE == 1) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v += __builtin_nontemporal_load(src + base + j * 16);
  }
  if (MODE == 2) {
#pragma unroll
    for (int j = 0; j < 4; ++j) dst[base + j * 16] = tid + j;
  }
  unsigned long long t0, t1, t2;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t2)::"memory");
  if (blockIdx.x < 64 && lane == 0) {
    st[blockIdx.x][wave][0] = t0;
    st[blockIdx.x][wave][1] = t1;
    st[blockIdx.x][wave][2] = t2;
  }
  if (v == 0xdeadbeef) out[0] = v;
}

int main() {
  const int blocks = 1024, stride = 256;  // 1 KB apart: every load a distinct cold line
  const size_t n = (size_t)blocks * 512 * stride + 64;
  unsigned *src, *dst, *out;
  hipMalloc(&src, n * 4);
  hipMalloc(&dst, n * 4);
  hipMalloc(&out, 64);
  hipMemset(src, 1, n * 4);
  auto run = [&](auto k, const char* name) {
    for (int rep = 0; rep < 3; ++rep) {
      hipMemset(dst, 0, n * 4);  // also evicts src from L2/MALL mostly
      hipLaunchKernelGGL(k, dim3(blocks), dim3(512), 0, 0, src, dst, out, stride);
      hipDeviceSynchronize();
    }
    std::vector<unsigned long long> h(64 * 8 * 3);
    hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(st), h.size() * 8);
    double bar = 0, wait = 0;
    for (int b = 0; b < 64; ++b) {
      unsigned long long mx = 0;
      for (int w = 0; w < 8; ++w) mx = std::max(mx, h[(b * 8 + w) * 3]);
      for (int w = 0; w < 8; ++w) {
        bar += (double)(h[(b * 8 + w) * 3 + 1] - mx);
        wait += (double)(h[(b * 8 + w) * 3 + 2] - h[(b * 8 + w) * 3 + 1]);
      }
    }
    printf("%-18s barrier after last arrival %8.1f ticks, vmcnt(0) after barrier %8.1f ticks\n", name, bar / 512, wait / 512);
  };
  run(kern<0>, "nothing pending");
  run(kern<1>, "loads pending");
  run(kern<2>, "stores pending");
  return 0;
}
