// VERDICT r05 item 3 asked whether LayerNorm folded into the next GEMM's
// prologue pays at few crops (the reference's one-video call: 29 crops = 58
// token rows).  The residual row is produced by the previous GEMM as four
// fp32 split-K partial slabs plus the fp32 residual stream (5 x 58 x 1024
// fp32 = 1.16 MB, L2 / Infinity-Cache resident).  Each of the QKV GEMM's
// column-tile workgroups would have to sum and normalise all 58 rows before
// its first MFMA.  This times, in one hipGraph of 200 repetitions each:
//  (a) ln_rows: today's resid_layernorm shape -- one 256-thread workgroup per
//      row sums the 5 slabs, normalises and writes the 16-bit row (58 WGs);
//  (b) ln_prologue: the fused prologue alone -- G workgroups (the QKV GEMM's
//      96 column tiles, or 48) each read all 58 x 5 rows and normalise them
//      into LDS (the GEMM body that would follow is omitted; four waves, two
//      rows per wave in flight, wave reductions);
// each after a producer kernel that rewrites the slabs (so they are fresh
// in L2 / MALL as after the real split-K GEMM).  Time per launch from
// rocprofv3 --kernel-trace (the producer's own time excluded).
//
//   hipcc -O3 --offload-arch=gfx950 -o ln_prologue_ubench ln_prologue_ubench.hip
//   rocprofv3 --kernel-trace --stats -d out -o run -- ./ln_prologue_ubench
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      printf("%s failed: %s\n", #x, hipGetErrorString(e_));                   \
      return 1;                                                               \
    }                                                                         \
  } while (0)

constexpr int ROWS = 58, COLS = 1024, SLABS = 5;

__global__ __launch_bounds__(256) void produce(float* __restrict__ s, float v) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < SLABS * ROWS * COLS) s[i] = v + (float)(i & 1023) * 1e-3f;
}

__device__ __forceinline__ float block_sum(float v, float* red) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
  return t;
}

// (a) one workgroup per row
__global__ __launch_bounds__(256) void ln_rows(const float* __restrict__ s, const float* __restrict__ gam,
                                               const float* __restrict__ bet, _Float16* __restrict__ y) {
  __shared__ float red[4];
  const int r = blockIdx.x;
  float v[4], sum = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = i * 256 + threadIdx.x;
    float a = 0.f;
#pragma unroll
    for (int k = 0; k < SLABS; ++k) a += s[(k * ROWS + r) * COLS + c];
    v[i] = a;
    sum += a;
  }
  const float mean = block_sum(sum, red) * (1.f / COLS);
  float sq = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) sq += (v[i] - mean) * (v[i] - mean);
  const float rstd = rsqrtf(block_sum(sq, red) * (1.f / COLS) + 1e-5f);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = i * 256 + threadIdx.x;
    y[r * COLS + c] = (_Float16)((v[i] - mean) * rstd * gam[c] + bet[c]);
  }
}

// (b) every workgroup normalises all rows into LDS (the fused GEMM prologue):
// wave w takes rows w, w + 4, ..., two at a time, each lane 16 consecutive
// columns (5 slabs x 4 float4 loads per row, all in flight together), mean
// and variance by wave reductions -- no workgroup barrier until the end
__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__global__ __launch_bounds__(256) void ln_prologue(const float* __restrict__ s, const float* __restrict__ gam,
                                                   const float* __restrict__ bet, _Float16* __restrict__ sink) {
  __shared__ _Float16 a[ROWS * COLS];  // 116 KB: the GEMM's A operand
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int r0 = wave; r0 < ROWS; r0 += 8) {
    float v[2][16];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = min(r0 + 4 * h, ROWS - 1);
#pragma unroll
      for (int i = 0; i < 16; ++i) v[h][i] = 0.f;
#pragma unroll
      for (int k = 0; k < SLABS; ++k)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float4 t = *(const float4*)(s + (k * ROWS + r) * COLS + lane * 16 + 4 * i);
          v[h][4 * i] += t.x;
          v[h][4 * i + 1] += t.y;
          v[h][4 * i + 2] += t.z;
          v[h][4 * i + 3] += t.w;
        }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = r0 + 4 * h;
      if (r >= ROWS) break;
      float sum = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) sum += v[h][i];
      const float mean = wsum(sum) * (1.f / COLS);
      float sq = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) sq += (v[h][i] - mean) * (v[h][i] - mean);
      const float rstd = rsqrtf(wsum(sq) * (1.f / COLS) + 1e-5f);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int c = lane * 16 + i;
        a[r * COLS + c] = (_Float16)((v[h][i] - mean) * rstd * gam[c] + bet[c]);
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) sink[blockIdx.x] = a[(blockIdx.x * 131) % (ROWS * COLS)];
}

int main() {
  float *s, *gam, *bet;
  _Float16 *y, *sink;
  CK(hipMalloc(&s, SLABS * ROWS * COLS * 4));
  CK(hipMalloc(&gam, COLS * 4));
  CK(hipMalloc(&bet, COLS * 4));
  CK(hipMalloc(&y, ROWS * COLS * 2));
  CK(hipMalloc(&sink, 1024 * 2));
  CK(hipMemset(gam, 0, COLS * 4));
  CK(hipMemset(bet, 0, COLS * 4));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const int pgrid = (SLABS * ROWS * COLS + 255) / 256;
  const int reps = 200;
  for (int arm = 0; arm < 3; ++arm) {
    const int G = arm == 1 ? 96 : 48;
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int r = 0; r < reps; ++r) {
      produce<<<pgrid, 256, 0, st>>>(s, (float)r);
      if (arm == 0) ln_rows<<<ROWS, 256, 0, st>>>(s, gam, bet, y);
      else ln_prologue<<<G, 256, 0, st>>>(s, gam, bet, sink);
    }
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, st));  // warm-up
    CK(hipStreamSynchronize(st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, st));
    CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(e1, st));
    CK(hipStreamSynchronize(st));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("arm %s: %d x (producer + consumer) in %.3f ms = %.2f us per pair\n",
           arm == 0 ? "ln_rows (58 WGs, today's separate LayerNorm)"
                    : (arm == 1 ? "ln_prologue (96 WGs: the QKV GEMM's column tiles)" : "ln_prologue (48 WGs)"),
           reps, ms, ms * 1e3f / reps);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  return 0;
}
