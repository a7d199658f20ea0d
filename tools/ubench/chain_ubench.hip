// What does a dependent step cost at the few-crop tail's scale?  (a) a chain
// of N dependent trivial kernels in one hipGraph (each reads the previous
// one's 58 x 1024 fp32 rows and writes its own, one 64-thread workgroup per
// row, as resid_layernorm does); (b) one cooperative kernel doing the same N
// steps with a grid barrier between them (device-scope release / acquire:
// the cross-XCD visibility a kernel boundary also provides).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      printf("%s failed: %s\n", #x, hipGetErrorString(e_));                   \
      return 1;                                                               \
    }                                                                         \
  } while (0)

constexpr int ROWS = 58, COLS = 1024;

__global__ __launch_bounds__(64) void step_kernel(const float* __restrict__ x, float* __restrict__ y) {
  const int r = blockIdx.x, l = threadIdx.x;
#pragma unroll
  for (int i = 0; i < COLS / 64; ++i) y[r * COLS + i * 64 + l] = x[r * COLS + i * 64 + l] * 0.5f + 1.0f;
}

// grid barrier: one arrival counter per barrier instance (no reset races)
__device__ __forceinline__ void grid_barrier(unsigned* ctr, unsigned nblocks) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE);  // device scope by default on global memory
    while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < nblocks) __builtin_amdgcn_s_sleep(1);
  }
  __syncthreads();
}

__global__ __launch_bounds__(64) void coop_kernel(float* a, float* b, unsigned* ctrs, int nsteps) {
  const int r = blockIdx.x % ROWS, l = threadIdx.x;
  for (int s = 0; s < nsteps; ++s) {
    const float* x = (s & 1) ? b : a;
    float* y = (s & 1) ? a : b;
    if (blockIdx.x < ROWS) {
#pragma unroll
      for (int i = 0; i < COLS / 64; ++i) y[r * COLS + i * 64 + l] = x[r * COLS + i * 64 + l] * 0.5f + 1.0f;
    }
    grid_barrier(ctrs + s, gridDim.x);
  }
}

int main() {
  const int N = 48;
  float *a, *b;
  unsigned* ctrs;
  CK(hipMalloc(&a, ROWS * COLS * 4));
  CK(hipMalloc(&b, ROWS * COLS * 4));
  CK(hipMalloc(&ctrs, N * 4 * 64));
  CK(hipMemset(a, 0, ROWS * COLS * 4));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  // (a) graph of N dependent kernels
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  for (int s = 0; s < N; ++s) step_kernel<<<ROWS, 64, 0, st>>>((s & 1) ? b : a, (s & 1) ? a : b);
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 20; ++w) CK(hipGraphLaunch(ge, st));
  CK(hipEventRecord(e0, st));
  const int R = 50;
  for (int i = 0; i < R; ++i) CK(hipGraphLaunch(ge, st));
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("(a) graph of %d dependent kernels: %.2f us per graph, %.2f us per step\n", N, ms * 1e3 / R, ms * 1e3 / R / N);
  // (b) cooperative kernel with N grid barriers, grid = ROWS or 256 workgroups
  for (int grid : {ROWS, 256}) {
    int nsteps = N;
    void* args[] = {&a, &b, &ctrs, &nsteps};
    float tot = 0;
    for (int i = 0; i < 20 + R; ++i) {
      CK(hipMemsetAsync(ctrs, 0, N * 4 * 64, st));
      CK(hipEventRecord(e0, st));
      CK(hipLaunchCooperativeKernel((const void*)coop_kernel, dim3(grid), dim3(64), args, 0, st));
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (i >= 20) tot += ms;
    }
    printf("(b) cooperative kernel, %d workgroups, %d grid barriers: %.2f us per kernel, %.2f us per step\n", grid, N,
           tot * 1e3 / R, tot * 1e3 / R / N);
  }
  return 0;
}
