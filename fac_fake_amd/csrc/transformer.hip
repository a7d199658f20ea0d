// Patch embedding, transformer encoder and head of CViT
// (CViT-main/model/cvit.py:5-78 and :150-179) on gfx950.
//
// Token layout: the residual stream is fp32 [2B][1024], row 2b = CLS token of
// crop b, row 2b+1 = its single patch token (num_patches = (7//7)^2 = 1,
// cvit.py:150).  Linear layers run as 16-bit x 16-bit MFMA GEMMs
// (C = A[M][K] * W[N][K]^T) with fp32 accumulation and fused epilogues:
// bias, exact-erf GELU, ReLU, fp32 residual add, or split-K fp32 partials.
#include "common.hpp"

namespace fac {

enum GemmEpi : int {
  EPI_F32 = 0,        // out f32 = acc + bias
  EPI_F32_RELU = 1,   // out f32 = relu(acc + bias)
  EPI_T_GELU = 2,     // out T = gelu(acc + bias)
  EPI_RESID = 3,      // out f32 += acc + bias   (Residual, cvit.py:10-11)
  EPI_PARTIAL = 4,    // out f32 [z][M][N] = acc (split-K slab)
  EPI_T = 5,          // out T = acc + bias
};

// Async global -> LDS copy of 16 bytes per lane (global_load_lds_dwordx4).
__device__ __forceinline__ void glds16(const void* gsrc, void* ldst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gsrc,
                                   (__attribute__((address_space(3))) void*)ldst, 16, 0, 0);
}

// C[M][N] = A[M][K] . W[N][K]^T on a BM x BN output tile (BM = 32 or 64, BN =
// 128, or 32 / 64 for the few-row calls: more workgroups streaming W),
// BK = 64, 4 waves in a WM x (4/WM) grid, each wave FM x FN MFMA 16x16x32
// tiles.  Both operand tiles go global -> LDS by global_load_lds into an
// NS-slot ring: tile kt lives in slot kt % NS and is issued NS-1 steps ahead
// (GPW glds per wave per tile, counted in vmcnt; wait + barrier in one asm
// statement so no LDS access can sit between them).  These GEMMs have
// M = 2B = 512 rows and K = 1024..2048: they are latency-bound, and the ring
// depth is what hides the HBM/L2 latency.  LDS rows are 128 B (64 k); the
// 16-byte chunk c of row r sits at position c ^ ((r >> 1) & 7), applied on
// the glds SOURCE address (the LDS side of a glds is lane-linear) and on the
// fragment read: conflict-free for the ds_read_b128 lane groups.
// blockIdx.z selects a K range of Kper (split-K; Kper % 64 == 0).
// Every output's K sum runs in the same order (k-tiles of 64 in sequence, two
// MFMA k-steps each) for every BM / BN / WM / NS, so the tile variant never
// changes a result bit: a crop's logits stay independent of its batch.
template <class T, int EPI, int BM, int WM, int NS, int BN = 128>
__global__ __launch_bounds__(256, NS <= 3 ? 2 : 1) void gemm_nt(const uint16_t* __restrict__ A, int lda,
                                                                const uint16_t* __restrict__ Wt, int ldw,
                                                                const float* __restrict__ bias,
                                                                void* __restrict__ out_, int ldo, int M, int N,
                                                                int Kper) {
  constexpr int BK = 64, WN = 4 / WM;
  constexpr int FM = BM / WM / 16, FN = BN / WN / 16;
  constexpr int SLOT = (BM + BN) * BK;    // elements
  constexpr int GPW = (BM + BN) / 8 / 4;  // glds per wave per tile (8 rows per instruction)
  static_assert((BM + BN) % 32 == 0 && FM >= 1 && FN >= 1 && NS >= 3 && FM * WM * 16 == BM && FN * WN * 16 == BN,
                "gemm tile");
  __shared__ __attribute__((aligned(16))) uint16_t smem[NS * SLOT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
  const int k0 = blockIdx.z * Kper;
  const int nkt = Kper / BK;

  // this lane's glds sources: instruction i of this wave covers tile rows
  // 8*(4i + wave) .. +7 (rows < BM: A, else W), lane -> (row, position)
  const uint16_t* gsrc[GPW];
#pragma unroll
  for (int i = 0; i < GPW; ++i) {
    const int row = 8 * (4 * i + wave) + (lane >> 3), pos = lane & 7;
    const int c = pos ^ ((row >> 1) & 7);
    if (row < BM) {
      const int m = m0 + row < M ? m0 + row : M - 1;  // rows past M: any valid row, never stored
      gsrc[i] = A + (size_t)m * lda + k0 + c * 8;
    } else {
      gsrc[i] = Wt + (size_t)(n0 + row - BM) * ldw + k0 + c * 8;
    }
  }
  // tiles past the end are dummy re-reads of tile 0 into slots never read again
  auto issue = [&](int kt) {
    const int slot = kt % NS, t = kt < nkt ? kt : 0;
#pragma unroll
    for (int i = 0; i < GPW; ++i) glds16(gsrc[i] + t * BK, smem + slot * SLOT + 8 * (4 * i + wave) * BK);
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4)0.f;

#pragma unroll
  for (int t = 0; t < NS - 1; ++t) issue(t);
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"((NS - 2) * GPW) : "memory");
  for (int kt = 0; kt < nkt; ++kt) {
    issue(kt + NS - 1);  // into the slot consumed at kt-1 (all waves passed its barrier)
    const uint16_t* sa = smem + (kt % NS) * SLOT;
    const uint16_t* sb = sa + BM * BK;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      const int c = ks * 4 + (lane >> 4);
      u16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int r = wm * (BM / WM) + i * 16 + (lane & 15);
        af[i] = *(const u16x8*)(sa + r * BK + ((c ^ ((r >> 1) & 7)) << 3));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int r = wn * (BN / WN) + j * 16 + (lane & 15);
        bfr[j] = *(const u16x8*)(sb + r * BK + ((c ^ ((r >> 1) & 7)) << 3));
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = T::mfma(af[i], bfr[j], acc[i][j]);
    }
    // retire tile kt+1 (tiles kt+2 .. kt+NS-1 stay in flight)
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"((NS - 2) * GPW) : "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the dummy tiles

  // all bias values in flight at once (one wait, not a round trip per tile column)
  float bvs[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j)
    bvs[j] = (EPI == EPI_PARTIAL || bias == nullptr) ? 0.f : bias[n0 + wn * (BN / WN) + j * 16 + (lane & 15)];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = n0 + wn * (BN / WN) + j * 16 + (lane & 15);
    const float bv = bvs[j];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * (BM / WM) + i * 16 + (lane >> 4) * 4 + r;
        if (m >= M) continue;
        const float v = acc[i][j][r] + bv;
        if constexpr (EPI == EPI_F32) {
          ((float*)out_)[(size_t)m * ldo + n] = v;
        } else if constexpr (EPI == EPI_F32_RELU) {
          ((float*)out_)[(size_t)m * ldo + n] = fmaxf(v, 0.f);
        } else if constexpr (EPI == EPI_T_GELU) {
          const float g = 0.5f * v * (1.0f + erff(v * 0.70710678118654752440f));
          ((uint16_t*)out_)[(size_t)m * ldo + n] = T::from_f32(g);
        } else if constexpr (EPI == EPI_RESID) {
          ((float*)out_)[(size_t)m * ldo + n] += v;
        } else if constexpr (EPI == EPI_PARTIAL) {
          ((float*)out_)[((size_t)blockIdx.z * M + m) * ldo + n] = v;
        } else {
          ((uint16_t*)out_)[(size_t)m * ldo + n] = T::from_f32(v);
        }
      }
  }
}

// LayerNorm(1024, eps 1e-5 unless given) of one row held by one wave (16 floats
// per lane: columns i*256 + 4*lane + j) -> 16-bit (PreNorm, cvit.py:13-20).
template <class T>
__device__ __forceinline__ void ln_row_store(const f32x4 (&v)[4], const float* __restrict__ g,
                                             const float* __restrict__ bta, uint16_t* __restrict__ yr, int lane,
                                             float eps = 1e-5f) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) s += v[i][0] + v[i][1] + v[i][2] + v[i][3];
  const float mean = wave_sum(s) * (1.0f / 1024.0f);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float d = v[i][j] - mean;
      q += d * d;
    }
  const float rstd = 1.0f / sqrtf(wave_sum(q) * (1.0f / 1024.0f) + eps);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = i * 256 + lane * 4;
    const f32x4 gg = *(const f32x4*)(g + c), bb = *(const f32x4*)(bta + c);
    u16x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = T::from_f32((v[i][j] - mean) * rstd * gg[j] + bb[j]);
    *(u16x4*)(yr + c) = o;
  }
}

// Sum of the S split-K partial slabs of row `row` (slab s at (s*R + row)),
// columns i*256 + 4*lane .. +3, added in split order (deterministic).  S is
// a template argument so all S loads of a column group are in flight at once.
template <int S>
__device__ __forceinline__ f32x4 slab_sum(const float* __restrict__ slab, size_t R, int row, int c) {
  f32x4 p = *(const f32x4*)(slab + (size_t)row * 1024 + c);
#pragma unroll
  for (int k = 1; k < S; ++k) p += *(const f32x4*)(slab + ((size_t)k * R + row) * 1024 + c);
  return p;
}

// Token rows of the residual stream + layer 0's PreNorm, one wave per row
// (cvit.py:171-175 patch_to_embedding, cat(cls, y), += pos_embedding[0:B]
// with pos indexed by the crop's batch slot p_b; then cvit.py:19-20):
//   x[2b]   = cls + pos[p_b]
//   x[2b+1] = (sum_s slab[s][b]) + bias + pos[p_b]
//   y[r]    = LayerNorm_0(x[r]) -> 16-bit
template <class T, int S>
__global__ __launch_bounds__(64) void embed_finalize_ln(const float* __restrict__ slab, int B,
                                                        const float* __restrict__ bias,
                                                        const float* __restrict__ cls,
                                                        const float* __restrict__ pos,
                                                        const int32_t* __restrict__ pidx, float* __restrict__ x,
                                                        const float* __restrict__ g, const float* __restrict__ bta,
                                                        uint16_t* __restrict__ y, int* __restrict__ err, int seq) {
  const int r = blockIdx.x, b = r >> 1, lane = threadIdx.x;
  int p = pidx[b];
  if (p < 0 || p >= 32) {
    // the flag names the forward (its call number on the context, >= 1)
    if (lane == 0 && (r & 1) == 0 && err) __hip_atomic_store(err, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    p = p < 0 ? 0 : 31;
  }
  f32x4 v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = i * 256 + lane * 4;
    const f32x4 pe = *(const f32x4*)(pos + p * 1024 + c);
    if (r & 1) v[i] = (slab_sum<S>(slab, B, b, c) + *(const f32x4*)(bias + c)) + pe;
    else v[i] = *(const f32x4*)(cls + c) + pe;
    *(f32x4*)(x + (size_t)r * 1024 + c) = v[i];
  }
  ln_row_store<T>(v, g, bta, y + (size_t)r * 1024, lane);
}

// LayerNorm(1024, eps 1e-5) (PreNorm, cvit.py:13-20): one wave per row,
// fp32 statistics, 16-bit output feeding the next GEMM.
template <class T>
__global__ __launch_bounds__(64) void layernorm_rows(const float* __restrict__ x, const float* __restrict__ g,
                                                     const float* __restrict__ bta, uint16_t* __restrict__ y,
                                                     int R) {
  const int row = blockIdx.x, lane = threadIdx.x;
  const float* xr = x + (size_t)row * 1024;
  f32x4 v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = *(const f32x4*)(xr + i * 256 + lane * 4);
  ln_row_store<T>(v, g, bta, y + (size_t)row * 1024, lane);
}

// Residual add of a split-K projection + the next PreNorm LayerNorm, fused:
//   x[r] += (sum_s slab[s][r]) + bias      (Residual, cvit.py:10-11)
//   y[r]  = LayerNorm(x[r]) * g + b -> 16-bit (PreNorm, cvit.py:19-20)
// One 64-thread workgroup per row (R = 2B = 512 workgroups).
template <class T, int S>
__global__ __launch_bounds__(64) void resid_layernorm(float* __restrict__ x, const float* __restrict__ slab,
                                                      const float* __restrict__ bias, const float* __restrict__ g,
                                                      const float* __restrict__ bta, uint16_t* __restrict__ y,
                                                      int R, float eps) {
  const int row = blockIdx.x, lane = threadIdx.x;
  float* xr = x + (size_t)row * 1024;
  f32x4 v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = i * 256 + lane * 4;
    v[i] = (slab_sum<S>(slab, R, row, c) + *(const f32x4*)(bias + c)) + *(const f32x4*)(xr + c);
    *(f32x4*)(xr + c) = v[i];
  }
  ln_row_store<T>(v, g, bta, y + (size_t)row * 1024, lane, eps);
}

// After the last layer only the CLS rows matter (cvit.py:177): finish their
// residual add from the FF2 split-K partials and convert to 16-bit for the head.
template <class T, int S>
__global__ __launch_bounds__(256) void resid_cls(const float* __restrict__ x, const float* __restrict__ slab,
                                                 const float* __restrict__ bias, uint16_t* __restrict__ c, int B) {
  const int i = blockIdx.x * 256 + threadIdx.x;  // over B*256 float4 groups
  if (i >= B * 256) return;
  const int b = i >> 8, col = (i & 255) * 4, row = 2 * b, R = 2 * B;
  const f32x4 v = (slab_sum<S>(slab, R, row, col) + *(const f32x4*)(bias + col)) + *(const f32x4*)(x + (size_t)row * 1024 + col);
  u16x4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = T::from_f32(v[j]);
  *(u16x4*)(c + (size_t)b * 1024 + col) = o;
}

// CLS rows of the fp32 residual stream -> 16-bit [B][1024] (cvit.py:177).
template <class T>
__global__ __launch_bounds__(256) void gather_cls(const float* __restrict__ x, uint16_t* __restrict__ c, int B) {
  const int i = blockIdx.x * 256 + threadIdx.x;  // over B*256 float4 groups
  if (i >= B * 256) return;
  const int b = i >> 8, q = i & 255;
  const f32x4 v = *(const f32x4*)(x + (size_t)(2 * b) * 1024 + q * 4);
  u16x4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = T::from_f32(v[j]);
  *(u16x4*)(c + (size_t)b * 1024 + q * 4) = o;
}

// Attention core for n = 2 tokens, 8 heads x 128 (cvit.py:43-60):
// dots = q.k^T * dim^-0.5 (dim = 1024, so 1/32), softmax over keys, out = attn.v.
// One wave per (crop, head); qkv is fp32 [2B][3072] laid out '(qkv h d)'.
// attn_pair: the wave's lane holds dims lane and lane + 64 of head h of crop
// b; o0 / o1 = the outputs of its two tokens (rows 2b, 2b+1) at those dims.
__device__ __forceinline__ void attn_pair(const float* __restrict__ qkv, int b, int h, int lane, float scale,
                                          float (&o0)[2], float (&o1)[2]) {
  const float* r0 = qkv + (size_t)(2 * b) * 3072 + h * 128;
  const float* r1 = r0 + 3072;
  float q0[2], q1[2], k0[2], k1[2], v0[2], v1[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int d = lane + 64 * i;
    q0[i] = r0[d];
    k0[i] = r0[1024 + d];
    v0[i] = r0[2048 + d];
    q1[i] = r1[d];
    k1[i] = r1[1024 + d];
    v1[i] = r1[2048 + d];
  }
  float s00 = 0.f, s01 = 0.f, s10 = 0.f, s11 = 0.f;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    s00 += q0[i] * k0[i];
    s01 += q0[i] * k1[i];
    s10 += q1[i] * k0[i];
    s11 += q1[i] * k1[i];
  }
  s00 = wave_sum(s00) * scale;
  s01 = wave_sum(s01) * scale;
  s10 = wave_sum(s10) * scale;
  s11 = wave_sum(s11) * scale;
  const float m0 = fmaxf(s00, s01), m1 = fmaxf(s10, s11);
  const float e00 = expf(s00 - m0), e01 = expf(s01 - m0);
  const float e10 = expf(s10 - m1), e11 = expf(s11 - m1);
  const float a00 = e00 / (e00 + e01), a01 = e01 / (e00 + e01);
  const float a10 = e10 / (e10 + e11), a11 = e11 / (e10 + e11);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    o0[i] = a00 * v0[i] + a01 * v1[i];
    o1[i] = a10 * v0[i] + a11 * v1[i];
  }
}

template <class T>
__global__ __launch_bounds__(256) void attention2(const float* __restrict__ qkv, uint16_t* __restrict__ o,
                                                  int B, float scale) {
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (wid >= B * 8) return;
  const int b = wid >> 3, h = wid & 7;
  float o0[2], o1[2];
  attn_pair(qkv, b, h, lane, scale, o0, o1);
  uint16_t* p0 = o + (size_t)(2 * b) * 1024 + h * 128;
  uint16_t* p1 = p0 + 1024;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int d = lane + 64 * i;
    p0[d] = T::from_f32(o0[i]);
    p1[d] = T::from_f32(o1[i]);
  }
}

// (Round 5, measured and not kept: attention + to_out as one launch for
// few rows, each workgroup computing the attention outputs of its own K
// range into an LDS A panel before the GEMM -- bit-identical, but 17.9 us
// against 4.9 + 5.1 for the two launches at B = 29: 32 column tiles each
// redo the 58 (crop, head) pairs of their K range, 15 per wave in series.)

// Final Linear(2048 -> 2) + per-logit sigmoid (cvit.py:164, pred_sig in
// cvit_prediction.py:258-259); fp32 weights and activations.  One wave per crop.
__global__ __launch_bounds__(256) void head_out(const float* __restrict__ hid, const float* __restrict__ w2,
                                                const float* __restrict__ b2, float* __restrict__ logits,
                                                float* __restrict__ probs, int B) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (b >= B) return;
  const float* hr = hid + (size_t)b * 2048;
  float s0 = 0.f, s1 = 0.f;
  for (int k = lane * 4; k < 2048; k += 256) {
    const f32x4 h = *(const f32x4*)(hr + k);
    const f32x4 a = *(const f32x4*)(w2 + k);
    const f32x4 c = *(const f32x4*)(w2 + 2048 + k);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s0 += h[j] * a[j];
      s1 += h[j] * c[j];
    }
  }
  s0 = wave_sum(s0) + b2[0];
  s1 = wave_sum(s1) + b2[1];
  if (lane == 0) {
    logits[2 * b] = s0;
    logits[2 * b + 1] = s1;
    if (probs) {
      probs[2 * b] = 1.0f / (1.0f + expf(-s0));
      probs[2 * b + 1] = 1.0f / (1.0f + expf(-s1));
    }
  }
}

// Video-level score (pre_process_prediction, cvit_prediction.py:266-281) over
// n per-crop logit pairs: p = sigmoid(logits); if n > 2: f = mean p0,
// r = mean p1, score = f if f > r else |1 - r|; else 0.5.  The sigmoids run
// in parallel; the two sums stay sequential fp32 in crop order (the
// reference's Python sum() over 0-d tensors), done by one lane from LDS.
__global__ __launch_bounds__(1024) void video_score(const float* __restrict__ logits, int n,
                                                    float* __restrict__ score) {
  constexpr int CAP = 4096;  // crops per LDS pass
  __shared__ float sp[2 * CAP];
  float f = 0.f, r = 0.f;
  for (int base = 0; base < n; base += CAP) {
    const int m = n - base < CAP ? n - base : CAP;
    __syncthreads();
    for (int i = threadIdx.x; i < 2 * m; i += blockDim.x) sp[i] = 1.0f / (1.0f + expf(-logits[2 * base + i]));
    __syncthreads();
    if (threadIdx.x == 0)
      for (int i = 0; i < m; ++i) {
        f += sp[2 * i];
        r += sp[2 * i + 1];
      }
  }
  if (threadIdx.x != 0) return;
  if (n <= 2) {
    *score = 0.5f;
    return;
  }
  f = f / (float)n;
  r = r / (float)n;
  *score = f > r ? f : fabsf(1.0f - r);
}

// Segmented video_score: one workgroup per video v over logits rows
// [seg[v], seg[v+1]), the same sigmoid (expf) and the same sequential fp32
// sums in crop order as video_score, so each video's score is bit-identical
// to video_score on its own rows (several videos' crops scored in one batch,
// cvit_prediction.py:73-83 run video by video in the reference).
__global__ __launch_bounds__(256) void video_score_seg(const float* __restrict__ logits,
                                                       const int* __restrict__ seg, int nv,
                                                       float* __restrict__ score) {
  constexpr int CAP = 1024;
  __shared__ float sp[2 * CAP];
  const int v = blockIdx.x;
  if (v >= nv) return;
  const int lo = seg[v], n = seg[v + 1] - lo;
  float f = 0.f, r = 0.f;
  for (int base = 0; base < n; base += CAP) {
    const int m = n - base < CAP ? n - base : CAP;
    __syncthreads();
    for (int i = threadIdx.x; i < 2 * m; i += blockDim.x)
      sp[i] = 1.0f / (1.0f + expf(-logits[2 * (size_t)(lo + base) + i]));
    __syncthreads();
    if (threadIdx.x == 0)
      for (int i = 0; i < m; ++i) {
        f += sp[2 * i];
        r += sp[2 * i + 1];
      }
  }
  if (threadIdx.x != 0) return;
  if (n <= 2) {
    score[v] = 0.5f;
    return;
  }
  f = f / (float)n;
  r = r / (float)n;
  score[v] = f > r ? f : fabsf(1.0f - r);
}

}  // namespace fac

namespace fac {

// Tile variants (BM x BN, WM, ring NS): 0 = 64x128 ring 3 (2 WG/CU), 1 =
// 64x128 ring 6, 2 = 32x128 ring 3 (2 WG/CU), 3 = 32x128 ring 7; for few rows
// (the reference's one-video call: M = 2B <= 58), 4 = 64x32 ring 3, 5 = 64x32
// ring 6, 6 = 32x64 ring 3.  (Round 5: 64x32 with rings of 9 and 12 slots --
// up to 11 of a K = 1024 call's 16 k-tiles in flight -- gave the B = 29
// forward nothing: 0.733 vs 0.743 ms.)
constexpr int kGemmVariants = 7;
constexpr int gemm_bm(int v) { return v == 2 || v == 3 || v == 6 ? 32 : 64; }
constexpr int gemm_bn(int v) { return v == 4 || v == 5 ? 32 : (v == 6 ? 64 : 128); }

template <class T, int EPI>
static void launch_gemm_v(int variant, dim3 grid, const uint16_t* A, int lda, const uint16_t* W, int ldw,
                          const float* bias, void* out, int ldo, int M, int N, int Kper, hipStream_t st) {
  switch (variant) {
    case 0: gemm_nt<T, EPI, 64, 2, 3><<<grid, 256, 0, st>>>(A, lda, W, ldw, bias, out, ldo, M, N, Kper); break;
    case 1: gemm_nt<T, EPI, 64, 2, 6><<<grid, 256, 0, st>>>(A, lda, W, ldw, bias, out, ldo, M, N, Kper); break;
    case 2: gemm_nt<T, EPI, 32, 1, 3><<<grid, 256, 0, st>>>(A, lda, W, ldw, bias, out, ldo, M, N, Kper); break;
    case 3: gemm_nt<T, EPI, 32, 1, 7><<<grid, 256, 0, st>>>(A, lda, W, ldw, bias, out, ldo, M, N, Kper); break;
    case 4: gemm_nt<T, EPI, 64, 2, 3, 32><<<grid, 256, 0, st>>>(A, lda, W, ldw, bias, out, ldo, M, N, Kper); break;
    case 5: gemm_nt<T, EPI, 64, 2, 6, 32><<<grid, 256, 0, st>>>(A, lda, W, ldw, bias, out, ldo, M, N, Kper); break;
    default: gemm_nt<T, EPI, 32, 1, 3, 64><<<grid, 256, 0, st>>>(A, lda, W, ldw, bias, out, ldo, M, N, Kper); break;
  }
}

template <class T>
static hipError_t launch_gemm_t(int epi, const uint16_t* A, int lda, const uint16_t* W, int ldw, const float* bias,
                                void* out, int ldo, int M, int N, int K, int splits, int variant, hipStream_t st) {
  const int bm = gemm_bm(variant);
  dim3 grid(N / gemm_bn(variant), (M + bm - 1) / bm, splits);
  const int Kper = K / splits;
  switch (epi) {
    case EPI_F32: launch_gemm_v<T, EPI_F32>(variant, grid, A, lda, W, ldw, bias, out, ldo, M, N, Kper, st); break;
    case EPI_F32_RELU: launch_gemm_v<T, EPI_F32_RELU>(variant, grid, A, lda, W, ldw, bias, out, ldo, M, N, Kper, st); break;
    case EPI_T_GELU: launch_gemm_v<T, EPI_T_GELU>(variant, grid, A, lda, W, ldw, bias, out, ldo, M, N, Kper, st); break;
    case EPI_RESID: launch_gemm_v<T, EPI_RESID>(variant, grid, A, lda, W, ldw, bias, out, ldo, M, N, Kper, st); break;
    case EPI_PARTIAL: launch_gemm_v<T, EPI_PARTIAL>(variant, grid, A, lda, W, ldw, bias, out, ldo, M, N, Kper, st); break;
    default: launch_gemm_v<T, EPI_T>(variant, grid, A, lda, W, ldw, bias, out, ldo, M, N, Kper, st); break;
  }
  return hipGetLastError();
}

// Few-row calls (M = 2B rows up to 64: the reference's <= 29-crop video
// call) default to a narrow tile, so several times more workgroups stream the
// weights (set_gemm_small; bit-identical to the wide tiles).
static int kSmallM = 64, kSmallVariant = 5;
void set_gemm_small(int max_m, int variant) {
  kSmallM = max_m;
  kSmallVariant = variant;
}

// variant < 0: pick by shape.  Alone (tools/gemm_sweep.py, bf16, B = 256) the
// 32x128 / ring-3 tile (2 WG/CU) wins the encoder GEMMs at M = 512 rows
// (K = 1024..2048: QKV 11.1 us, FF1 11.5, FF2/4 7.1, head 8.7 vs 13-18 us for
// 64x128); the long-K patch GEMM (K = 25088, split 14) and every GEMM with
// more than 1024 rows take 64x128 / ring 3 (ResVitKan's 3072-crop encoder,
// M = 6144: +1.2 %, profiles/r06_tail_gemm_ab.txt).  variant -2: the encoder
// that runs beside the next batch's conv stack (the software pipeline,
// fac_forward_nhwc_u8_pipelined), where what counts is the CU time its
// workgroups take from the convs: the 64x128 tile at every M > kSmallM (half
// the workgroups, each A row read once per 128 columns instead of per 32
// rows x 128; headline +0.2 to +1.7 %, same-box alternations, same file).
hipError_t launch_gemm(int dtype, int epi, const uint16_t* A, int lda, const uint16_t* W, int ldw, const float* bias,
                       void* out, int ldo, int M, int N, int K, int splits, hipStream_t st, int variant) {
  if (N % 128 != 0 || splits < 1 || K % (64 * splits) != 0 || M <= 0 || epi < 0 || epi > EPI_T)
    return hipErrorInvalidValue;
  if (variant < 0)
    variant = M <= kSmallM ? kSmallVariant : ((variant == -2 || M > 1024 || (K / splits >= 1024 && K >= 8192)) ? 0 : 2);
  if (variant >= kGemmVariants) return hipErrorInvalidValue;
  if (dtype == 0) return launch_gemm_t<BF16>(epi, A, lda, W, ldw, bias, out, ldo, M, N, K, splits, variant, st);
  return launch_gemm_t<F16>(epi, A, lda, W, ldw, bias, out, ldo, M, N, K, splits, variant, st);
}

template <class T>
static hipError_t embed_ln_t(const float* slab, int S, int B, const float* bias, const float* cls, const float* pos,
                             const int32_t* pidx, float* x, const float* g, const float* bt, uint16_t* y, int* err,
                             int seq, hipStream_t st) {
  switch (S) {
    case 7: embed_finalize_ln<T, 7><<<2 * B, 64, 0, st>>>(slab, B, bias, cls, pos, pidx, x, g, bt, y, err, seq); break;
    case 14: embed_finalize_ln<T, 14><<<2 * B, 64, 0, st>>>(slab, B, bias, cls, pos, pidx, x, g, bt, y, err, seq); break;
    case 28: embed_finalize_ln<T, 28><<<2 * B, 64, 0, st>>>(slab, B, bias, cls, pos, pidx, x, g, bt, y, err, seq); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_embed_finalize_ln(int dtype, const float* slab, int S, int B, const float* bias, const float* cls,
                                    const float* pos, const int32_t* pidx, float* x, const float* g, const float* bt,
                                    uint16_t* y, int* err, int seq, hipStream_t st) {
  if (dtype == 0) return embed_ln_t<BF16>(slab, S, B, bias, cls, pos, pidx, x, g, bt, y, err, seq, st);
  return embed_ln_t<F16>(slab, S, B, bias, cls, pos, pidx, x, g, bt, y, err, seq, st);
}

hipError_t launch_layernorm(int dtype, const float* x, const float* g, const float* b, uint16_t* y, int R,
                            hipStream_t st) {
  if (dtype == 0) layernorm_rows<BF16><<<R, 64, 0, st>>>(x, g, b, y, R);
  else layernorm_rows<F16><<<R, 64, 0, st>>>(x, g, b, y, R);
  return hipGetLastError();
}

template <class T>
static hipError_t resid_ln_t(float* x, const float* slab, int S, const float* bias, const float* g, const float* b,
                             uint16_t* y, int R, hipStream_t st, float eps) {
  switch (S) {
    case 1: resid_layernorm<T, 1><<<R, 64, 0, st>>>(x, slab, bias, g, b, y, R, eps); break;
    case 2: resid_layernorm<T, 2><<<R, 64, 0, st>>>(x, slab, bias, g, b, y, R, eps); break;
    case 4: resid_layernorm<T, 4><<<R, 64, 0, st>>>(x, slab, bias, g, b, y, R, eps); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_resid_layernorm(int dtype, float* x, const float* slab, int S, const float* bias, const float* g,
                                  const float* b, uint16_t* y, int R, hipStream_t st, float eps) {
  if (dtype == 0) return resid_ln_t<BF16>(x, slab, S, bias, g, b, y, R, st, eps);
  return resid_ln_t<F16>(x, slab, S, bias, g, b, y, R, st, eps);
}

template <class T>
static hipError_t resid_cls_t(const float* x, const float* slab, int S, const float* bias, uint16_t* c, int B,
                              hipStream_t st) {
  dim3 grid(B);
  switch (S) {
    case 1: resid_cls<T, 1><<<grid, 256, 0, st>>>(x, slab, bias, c, B); break;
    case 2: resid_cls<T, 2><<<grid, 256, 0, st>>>(x, slab, bias, c, B); break;
    case 4: resid_cls<T, 4><<<grid, 256, 0, st>>>(x, slab, bias, c, B); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_resid_cls(int dtype, const float* x, const float* slab, int S, const float* bias, uint16_t* c, int B,
                            hipStream_t st) {
  if (dtype == 0) return resid_cls_t<BF16>(x, slab, S, bias, c, B, st);
  return resid_cls_t<F16>(x, slab, S, bias, c, B, st);
}

hipError_t launch_gather_cls(int dtype, const float* x, uint16_t* c, int B, hipStream_t st) {
  dim3 grid(B);
  if (dtype == 0) gather_cls<BF16><<<grid, 256, 0, st>>>(x, c, B);
  else gather_cls<F16><<<grid, 256, 0, st>>>(x, c, B);
  return hipGetLastError();
}

hipError_t launch_attention2(int dtype, const float* qkv, uint16_t* o, int B, float scale, hipStream_t st) {
  dim3 grid((B * 8 + 3) / 4);
  if (dtype == 0) attention2<BF16><<<grid, 256, 0, st>>>(qkv, o, B, scale);
  else attention2<F16><<<grid, 256, 0, st>>>(qkv, o, B, scale);
  return hipGetLastError();
}

hipError_t launch_head_out(const float* hid, const float* w2, const float* b2, float* logits, float* probs, int B,
                           hipStream_t st) {
  head_out<<<(B + 3) / 4, 256, 0, st>>>(hid, w2, b2, logits, probs, B);
  return hipGetLastError();
}

hipError_t launch_video_score(const float* logits, int n, float* score, hipStream_t st) {
  video_score<<<1, 1024, 0, st>>>(logits, n, score);
  return hipGetLastError();
}

hipError_t launch_video_score_seg(const float* logits, const int* seg, int nv, float* score, hipStream_t st) {
  video_score_seg<<<nv, 256, 0, st>>>(logits, seg, nv, score);
  return hipGetLastError();
}

}  // namespace fac
