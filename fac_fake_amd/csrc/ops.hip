// Layer-level kernels for the §8f model families (include/fac_ops.h):
//   * convnd_igemm: N-d convolution + folded BN (+ ReLU, + residual) as an
//     implicit GEMM on MFMA — the ResNet-50 stem of ResVitKan
//     (CViT-main/ResVitKan/ResVitKan.py:124-240) and S3D's Conv3d layers
//     (sx_exp_deepfakedetect-master/S3D/model.py:50-82);
//   * pool_nd: max / average pooling, channels-last;
//   * pack_input: 3-channel image staging (uint8 or fp32 planar -> 16-bit);
//   * KANLinear (CViT-main/ResVitKan/kan.py:90-132, 189-206) in fp32.
//
// convnd_igemm: rows = output positions, columns = output channels,
// k = (tap, 8-channel piece).  A 128 x BN output tile per 256-thread
// workgroup (4 waves, 2 x 2, each 64 x BN/2 = 4 x BN/32 MFMA tiles), K in
// steps of 32 (4 pieces of 8 channels).  The A tile is gathered on the fly
// (im2col-free): every thread owns one GEMM row and two of its four pieces,
// tracks its pieces' (channel piece, tap) incrementally (no divisions in the
// K loop) and copies 16 bytes per piece, zero outside the input (padding) or
// beyond the real K (a zero page).  Both operands go global -> LDS by
// global_load_lds into a 4-slot ring of [piece][row] images (16-byte
// entries: the 16 lanes of a ds_read_b128 group read 16 consecutive entries,
// conflict-free), issued three K steps ahead with counted vmcnt waits, the
// wait and the barrier in one asm statement (as in conv.hip).  The
// epilogue stages the fp32 tile in LDS and writes 16-byte channel vectors
// (bias, ReLU, residual, ReLU, convert), so a row's BN channels leave in one
// contiguous burst.
#include <algorithm>
#include <climits>
#include <type_traits>
#include <cstdlib>

#include "common.hpp"
#include "fac_cvit.h"
#include "fac_ops.h"

namespace fac {

struct ConvP {
  const uint16_t* in;
  const uint16_t* w;
  const float* bias;
  const uint16_t* res;
  void* out;
  int D, H, W, C8;
  int Do, Ho, Wo, Cout;
  int KD, KH, KW;
  int SD, SH, SW, PD, PH, PW;
  int Kp, ksteps, ktot8;
  int ldo, c_off, ldr, r_off, flags;
  int vec_out, vec_res;
  int M;
  void* out1;  // column segments of fac_conv_nd_split (split1 = split2 = INT_MAX: one output)
  void* out2;
  int ldo1, ldo2, split1, split2;
  int ny;  // column tiles when the grid is flat (gridDim.y == 1, ny > 1), else 0
};

// (channel piece, tap) of one K piece, advanced in place by 4 pieces
struct Trk {
  int c8, tx, ty, tz, kp;
};

__device__ __forceinline__ void trk_norm(Trk& t, int C8, int KH, int KW) {
  while (t.c8 >= C8) {
    t.c8 -= C8;
    if (++t.tx == KW) {
      t.tx = 0;
      if (++t.ty == KH) {
        t.ty = 0;
        ++t.tz;
      }
    }
  }
}

// 16 zero bytes: the glds source of padding / out-of-range K pieces
__device__ const uint16_t g_zero16[64] = {0};
// write-only target of stores that must issue but whose values nobody reads
// (convnd_pt's padding channels, bneck_pw2's rows past M): 16 bytes per lane
__device__ uint16_t g_sink[64 * 8];

// Async global -> LDS copy of 16 bytes per lane (global_load_lds_dwordx4):
// the wave's 64 pieces land contiguously at the wave-uniform LDS address.
__device__ __forceinline__ void glds16(const void* gsrc, void* ldst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gsrc,
                                   (__attribute__((address_space(3))) void*)ldst, 16, 0, 0);
}

#ifdef ND_STAMPS
// diagnostic build only (tools/ubench/nd_ubench.hip): s_memtime stamps of
// every wave of the first workgroups, per K step, into a buffer of their own
__device__ unsigned long long nd_st[8][40][8][4];
__device__ unsigned long long nd_ev[8][8][4];  // per wave: entry, prologue done, loop done, end
#define ND_STAMP(k)                                                                          \
  do {                                                                                       \
    __builtin_amdgcn_sched_barrier(0);                                                       \
    unsigned long long t_;                                                                   \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");               \
    __builtin_amdgcn_sched_barrier(0);                                                       \
    if (blockIdx.x < 8 && lane == 0 && s < 40) nd_st[blockIdx.x][s][wave][(k)] = t_;         \
  } while (0)
#define ND_EV(k)                                                                             \
  do {                                                                                       \
    __builtin_amdgcn_sched_barrier(0);                                                       \
    unsigned long long t_;                                                                   \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");               \
    __builtin_amdgcn_sched_barrier(0);                                                       \
    if (blockIdx.x < 8 && (threadIdx.x & 63) == 0) nd_ev[blockIdx.x][threadIdx.x >> 6][(k)] = t_; \
  } while (0)
#else
#define ND_STAMP(k) \
  do {              \
  } while (0)
#define ND_EV(k) \
  do {           \
  } while (0)
#endif

// UT (uniform tap): cin % 64 == 0, so every K step (64 channels) lies in one
// tap and the tap / channel offset of a step is the same for every lane: the
// gather is one precomputed row offset + a wave-uniform step offset per A
// piece, validity by three unsigned compares, and no per-lane (channel piece,
// tap) tracking or per-piece branches (the generic path's VALU work was ~8.5
// instructions per MFMA on the ResNet-50 layers in a round-3 SQ_INSTS_VALU pass).
//
// IL (interleaved issue): the next stage's glds pieces are issued
// one at a time between the step's MFMA groups instead of all at the step
// start.  A CU's TA takes ~1.3k cycles for the 48 KB of a 256 x 128 stage,
// and issued in one block by all 8 waves at once (lock-step after the
// barrier) that time added to the ~1.1k cycles of the MFMAs (s_memtime
// stamps, tools/ubench/nd_ubench.hip); interleaved, one wave's stalled glds
// issue overlaps the other SIMD wave's MFMAs.
template <class T, int BM, int BN, int WM, int WN, int OCC, int NS, bool UT = false, bool IL = false>
__global__ __launch_bounds__(WM * WN * 64, OCC) void convnd_igemm(ConvP p) {
  constexpr int NW = WM * WN, NT = NW * 64;  // waves, threads
  constexpr int BK = 64;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int RT = WTM / 16, CT = WTN / 16;
  constexpr int SLOT_A = BM * BK, SLOT = (BM + BN) * BK;  // u16 elements per ring slot
  constexpr int NA = BM / 8 / NW, NB = BN / 8 / NW;       // glds per wave per stage (8 rows each)
  static_assert(NA * 8 * NW == BM && NB * 8 * NW == BN, "tile rows per wave");
  constexpr int PER = NA + NB;
  constexpr int SPITCH = BN + 4;              // fp32 staging row pitch
  constexpr int OPER = NS * SLOT;
  constexpr int STG = BM * SPITCH * 2;        // u16 elements of the fp32 staging tile
  constexpr int SMEM = OPER > STG ? OPER : STG;
  __shared__ __attribute__((aligned(16))) uint16_t smem[SMEM];

  ND_EV(0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  int bx = blockIdx.x, by = blockIdx.y;
  if ((gridDim.x & 7) == 0) bx = (bx & 7) * (gridDim.x >> 3) + (bx >> 3);  // XCD-contiguous tiles
  if (p.ny) {
    // flat grid: the ny column tiles of one row tile are consecutive on one
    // XCD, so they share the row tile's A gather through that XCD's L2
    by = bx % p.ny;
    bx /= p.ny;
  }
  const int m0 = bx * BM, n0 = by * BN;

  // LDS images: rows of 64 k (128 B), the 16-byte piece j of row r at position
  // j ^ ((r >> 1) & 7) (conflict-free ds_read_b128, as in transformer.hip's
  // gemm_nt).  glds instruction i of this wave fills rows 8*(NW i + wave) + lane/8,
  // position lane % 8, so it copies piece j = (lane % 8) ^ ((row >> 1) & 7) —
  // the same j for all of this lane's instructions, and 8 lanes cover one
  // row's 128 contiguous bytes of K (coalesced when a K step stays in one tap).
  const int pos = lane & 7, rsub = lane >> 3;
  static_assert(NW % 2 == 0, "4*NW*i must vanish mod 8");
  const int j = pos ^ ((4 * wave + (lane >> 4)) & 7);
  // per A instruction: the output position of its row
  const uint16_t* rbase[NA];
  int riz[NA], riy[NA], rix[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int m = m0 + 8 * (NW * i + wave) + rsub;
    const int mm = m < p.M ? m : 0;
    const int ox = mm % p.Wo, t1 = mm / p.Wo;
    const int oy = t1 % p.Ho, t2 = t1 / p.Ho;
    const int oz = t2 % p.Do, n = t2 / p.Do;
    riz[i] = m < p.M ? oz * p.SD - p.PD : -(1 << 29);  // rows past M: always out of range -> zeros
    riy[i] = oy * p.SH - p.PH;
    rix[i] = ox * p.SW - p.PW;
    rbase[i] = p.in + (size_t)n * p.D * p.H * p.W * p.C8 * 8;
  }
  // this lane's K piece (channel piece, tap), advanced 8 pieces per stage
  Trk t{j, 0, 0, 0, j};
  if constexpr (!UT) trk_norm(t, p.C8, p.KH, p.KW);
  const uint16_t* wsrc[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) wsrc[i] = p.w + (size_t)(n0 + 8 * (NW * i + wave) + rsub) * p.Kp + j * 8;
  // UT: element offset of each A row's tap-(0,0,0) input pixel (+ this lane's
  // piece), and the wave-uniform step state: channel offset c0, tap (uz,uy,ux)
  long long roff[UT ? NA : 1];
  if constexpr (UT) {
#pragma unroll
    for (int i = 0; i < NA; ++i)
      roff[i] = (rbase[i] - p.in) + (((long long)riz[i] * p.H + riy[i]) * p.W + rix[i]) * (p.C8 * 8) + j * 8;
  }
  int uc = 0, uz = 0, uy = 0, ux = 0;
  const long long rowstride = (long long)p.W * p.C8 * 8, planestride = rowstride * p.H;

  // glds piece q (A pieces 0..NA-1, then B) of stage st at the step state
  // (UT: the wave-uniform (uz, uy, ux, uc); else this lane's tracked piece t)
  auto ut_piece = [&](int st, int q) {
    uint16_t* slot = smem + (st % NS) * SLOT;
    if constexpr (!UT) {
      if (q < NA) {
        const bool real = st < p.ksteps && t.kp < p.ktot8;
        const int iz = riz[q] + t.tz, iy = riy[q] + t.ty, ix = rix[q] + t.tx;
        const bool ok = real && (unsigned)iz < (unsigned)p.D && (unsigned)iy < (unsigned)p.H &&
                        (unsigned)ix < (unsigned)p.W;
        const uint16_t* src = ok ? rbase[q] + (((size_t)iz * p.H + iy) * p.W + ix) * p.C8 * 8 + t.c8 * 8 : g_zero16;
        glds16(src, slot + (NW * q + wave) * 64 * 8);
      } else {
        glds16(st < p.ksteps ? wsrc[q - NA] + (size_t)st * BK : g_zero16, slot + SLOT_A + (NW * (q - NA) + wave) * 64 * 8);
      }
      return;
    }
    const bool real = st < p.ksteps;
    if (q < NA) {
      const long long toff = uz * planestride + uy * rowstride + (long long)ux * p.C8 * 8 + uc;
      const bool ok = real & ((unsigned)(riz[q] + uz) < (unsigned)p.D) & ((unsigned)(riy[q] + uy) < (unsigned)p.H) &
                      ((unsigned)(rix[q] + ux) < (unsigned)p.W);
      const uint16_t* src = ok ? p.in + (roff[q] + toff) : g_zero16;
      glds16(src, slot + (NW * q + wave) * 64 * 8);
    } else {
      glds16(real ? wsrc[q - NA] + (size_t)st * BK : g_zero16, slot + SLOT_A + (NW * (q - NA) + wave) * 64 * 8);
    }
  };
  auto ut_advance = [&] {
    if constexpr (!UT) {
      t.kp += 8;
      t.c8 += 8;
      trk_norm(t, p.C8, p.KH, p.KW);
      return;
    }
    uc += 64;
    if (uc == p.C8 * 8) {
      uc = 0;
      if (++ux == p.KW) {
        ux = 0;
        if (++uy == p.KH) {
          uy = 0;
          ++uz;
        }
      }
    }
  };
  // stage st -> ring slot st % NS; stages past the end copy zeros into slots never read
  auto issue = [&](int st) {
    uint16_t* slot = smem + (st % NS) * SLOT;
    if constexpr (UT) {
#pragma unroll
      for (int q = 0; q < PER; ++q) ut_piece(st, q);
      ut_advance();
      return;
    }
    const bool real = st < p.ksteps && t.kp < p.ktot8;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int iz = riz[i] + t.tz, iy = riy[i] + t.ty, ix = rix[i] + t.tx;
      const bool ok = real && (unsigned)iz < (unsigned)p.D && (unsigned)iy < (unsigned)p.H &&
                      (unsigned)ix < (unsigned)p.W;
      const uint16_t* src = ok ? rbase[i] + (((size_t)iz * p.H + iy) * p.W + ix) * p.C8 * 8 + t.c8 * 8 : g_zero16;
      glds16(src, slot + (NW * i + wave) * 64 * 8);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i)
      glds16(st < p.ksteps ? wsrc[i] + (size_t)st * BK : g_zero16, slot + SLOT_A + (NW * i + wave) * 64 * 8);
    t.kp += 8;
    t.c8 += 8;
    trk_norm(t, p.C8, p.KH, p.KW);
  };

  f32x4 acc[RT][CT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) acc[rt][ct] = (f32x4)0.f;

#pragma unroll
  for (int st = 0; st < NS - 1; ++st) issue(st);
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"((NS - 2) * PER) : "memory");
  ND_EV(1);
  for (int s = 0; s < p.ksteps; ++s) {
    ND_STAMP(0);
    const uint16_t* a = smem + (s % NS) * SLOT;
    const uint16_t* b = a + SLOT_A;
    if constexpr (IL) {
      // stage s+NS-1 into the slot consumed at step s-1 (every wave passed its
      // barrier), one piece after each of the first QPK MFMA groups of a K half
      constexpr int KH = BK / 32, QPK = (PER + KH - 1) / KH;
      static_assert(QPK <= RT, "a glds piece per MFMA group at most");
      const int st = s + NS - 1;
#pragma unroll
      for (int ks = 0; ks < KH; ++ks) {
        const int c = ks * 4 + (lane >> 4);
        u16x8 fb[CT], fa[RT];
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
          const int r = wn * WTN + ct * 16 + (lane & 15);
          fb[ct] = *(const u16x8*)(b + r * BK + ((c ^ ((r >> 1) & 7)) << 3));
        }
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          const int r = wm * WTM + rt * 16 + (lane & 15);
          fa[rt] = *(const u16x8*)(a + r * BK + ((c ^ ((r >> 1) & 7)) << 3));
        }
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int ct = 0; ct < CT; ++ct) acc[rt][ct] = T::mfma(fa[rt], fb[ct], acc[rt][ct]);
          __builtin_amdgcn_sched_barrier(0);
          if (rt < QPK && ks * QPK + rt < PER) ut_piece(st, ks * QPK + rt);
        }
      }
      ut_advance();
      ND_STAMP(1);
    } else {
    issue(s + NS - 1);  // into the slot consumed at step s-1 (every wave passed its barrier)
    ND_STAMP(1);
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      const int c = ks * 4 + (lane >> 4);
      u16x8 fb[CT];
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const int r = wn * WTN + ct * 16 + (lane & 15);
        fb[ct] = *(const u16x8*)(b + r * BK + ((c ^ ((r >> 1) & 7)) << 3));
      }
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const int r = wm * WTM + rt * 16 + (lane & 15);
        const u16x8 fa = *(const u16x8*)(a + r * BK + ((c ^ ((r >> 1) & 7)) << 3));
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) acc[rt][ct] = T::mfma(fa, fb[ct], acc[rt][ct]);
      }
    }
    }
    // retire stage s+1 (stage s+2 stays in flight)
#ifdef ND_STAMPS
    ND_STAMP(2);
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)" ::"n"((NS - 2) * PER) : "memory");
    ND_STAMP(3);
    asm volatile("s_barrier" ::: "memory");
#else
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"((NS - 2) * PER) : "memory");
#endif
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");  // dummy stages landed: LDS is free
  ND_EV(2);

  // ---- epilogue: bias (+ReLU) in registers -> fp32 LDS tile -> 8-channel
  // vectors.  The residual's 16-byte vectors are loaded first, so their
  // latency overlaps the staging.
  constexpr int QPR = BN / 8;                 // 8-channel pieces per row
  constexpr int QPT = BM * QPR / NT;          // pieces per thread
  const bool resid = p.flags & FAC_CONV_RESID;
  // all bias values first (one wait for the lot, not one round trip per
  // channel tile), then the residual vectors
  float bvs[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) bvs[ct] = p.bias ? p.bias[n0 + wn * WTN + ct * 16 + (lane & 15)] : 0.f;
  u16x8 rv[QPT];
#pragma unroll
  for (int i = 0; i < QPT; ++i) {
    const int q = tid + i * NT, row = q / QPR, cp = q - row * QPR;
    const int mo = m0 + row, c = n0 + cp * 8;
    rv[i] = (u16x8)0;
    if (resid && p.vec_res && mo < p.M && c + 8 <= p.Cout)
      rv[i] = *(const u16x8*)(p.res + (size_t)mo * p.ldr + p.r_off + c);
  }
  float* stg = (float*)smem;
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int col = wn * WTN + ct * 16 + (lane & 15);
    const float bv = bvs[ct];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[rt][ct][r] + bv;
        if (p.flags & FAC_CONV_RELU) v = relu(v);
        stg[(wm * WTM + rt * 16 + (lane >> 4) * 4 + r) * SPITCH + col] = v;
      }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < QPT; ++i) {
    const int q = tid + i * NT, row = q / QPR, cp = q - row * QPR;
    const int mo = m0 + row, c = n0 + cp * 8;
    if (mo >= p.M || c >= p.Cout) continue;
    const int nc = min(8, p.Cout - c);
    const f32x4 lo = *(const f32x4*)(stg + row * SPITCH + cp * 8);
    const f32x4 hi = *(const f32x4*)(stg + row * SPITCH + cp * 8 + 4);
    float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    if (resid) {
      if (p.vec_res && nc == 8) {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] += T::to_f32(rv[i][k]);
      } else {
        const uint16_t* r = p.res + (size_t)mo * p.ldr + p.r_off + c;
        for (int k = 0; k < nc; ++k) v[k] += T::to_f32(r[k]);
      }
    }
    if (p.flags & FAC_CONV_RELU2) {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = relu(v[k]);
    }
    if (p.flags & FAC_CONV_OUT_F32) {
      float* o = (float*)p.out + (size_t)mo * p.ldo + p.c_off + c;
      for (int k = 0; k < nc; ++k) o[k] = v[k];
    } else {
      // column segments (fac_conv_nd_split): [0, split1) -> out (ldo, c_off),
      // [split1, split2) -> out1 (ldo1), [split2, cout) -> out2 (ldo2)
      uint16_t* o;
      if (c >= p.split2) o = (uint16_t*)p.out2 + (size_t)mo * p.ldo2 + (c - p.split2);
      else if (c >= p.split1) o = (uint16_t*)p.out1 + (size_t)mo * p.ldo1 + (c - p.split1);
      else o = (uint16_t*)p.out + (size_t)mo * p.ldo + p.c_off + c;
      if (p.vec_out && nc == 8) {
        const u16x4 a = T::pack4((f32x4){v[0], v[1], v[2], v[3]});
        const u16x4 b = T::pack4((f32x4){v[4], v[5], v[6], v[7]});
        *(u16x8*)o = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
      } else {
        for (int k = 0; k < nc; ++k) o[k] = T::from_f32(v[k]);
      }
    }
  }
#ifdef ND_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  ND_EV(3);
}

// ---- pooling: one thread per (output position, 8-channel piece)
template <class T>
__global__ __launch_bounds__(256) void pool_nd(fac_pool_desc p, int total) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= total) return;
  const int C8 = p.c / 8;
  const int c8 = t % C8, mo = t / C8;
  const int ox = mo % p.ow, t1 = mo / p.ow;
  const int oy = t1 % p.oh, t2 = t1 / p.oh;
  const int oz = t2 % p.od, n = t2 / p.od;
  const uint16_t* inb = (const uint16_t*)p.in + (size_t)n * p.d * p.h * p.w * p.c + c8 * 8;
  float a[8];
  const bool mx = p.mode == 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = mx ? -__builtin_inff() : 0.f;
  for (int kz = 0; kz < p.kd; ++kz) {
    const int iz = oz * p.sd - p.pd + kz;
    if ((unsigned)iz >= (unsigned)p.d) continue;
    for (int ky = 0; ky < p.kh; ++ky) {
      const int iy = oy * p.sh - p.ph + ky;
      if ((unsigned)iy >= (unsigned)p.h) continue;
      for (int kx = 0; kx < p.kw; ++kx) {
        const int ix = ox * p.sw - p.pw + kx;
        if ((unsigned)ix >= (unsigned)p.w) continue;
        const u16x8 v = *(const u16x8*)(inb + (((size_t)iz * p.h + iy) * p.w + ix) * p.c);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float f = T::to_f32(v[i]);
          a[i] = mx ? fmaxf(a[i], f) : a[i] + f;
        }
      }
    }
  }
  if (!mx) {
    const float inv = (float)(p.kd * p.kh * p.kw);  // count_include_pad=True
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = a[i] / inv;
  }
  const u16x4 lo = T::pack4((f32x4){a[0], a[1], a[2], a[3]});
  const u16x4 hi = T::pack4((f32x4){a[4], a[5], a[6], a[7]});
  *(u16x8*)((uint16_t*)p.out + (size_t)mo * p.ldo + p.c_off + c8 * 8) = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

// ---- pool_max_win (round 4): max pooling with a compile-time window
// (S3D's (1,3,3)/(1,2,2), (3,3,3)/2 and (2,2,2)/2, ResNet's 3x3/2), one
// thread per (output position, 8-channel piece) as pool_nd, but branch-free:
// taps outside the input re-read the nearest tap inside it (in floor mode
// every window holds one, and a max over a repeat is unchanged), so all
// KD*KH*KW loads issue together; pool_nd's per-tap bounds checks made each
// load an exec-masked branch with its own wait.
template <class T, int KD, int KH, int KW>
__global__ __launch_bounds__(256) void pool_max_win(fac_pool_desc p, int total) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= total) return;
  const int C8 = p.c / 8;
  const int c8 = t % C8, mo = t / C8;
  const int ox = mo % p.ow, t1 = mo / p.ow;
  const int oy = t1 % p.oh, t2 = t1 / p.oh;
  const int oz = t2 % p.od, n = t2 / p.od;
  const uint16_t* inb = (const uint16_t*)p.in + (size_t)n * p.d * p.h * p.w * p.c + c8 * 8;
  int iz[KD], iy[KH], ix[KW];
#pragma unroll
  for (int k = 0; k < KD; ++k) iz[k] = min(max(oz * p.sd - p.pd + k, 0), p.d - 1);
#pragma unroll
  for (int k = 0; k < KH; ++k) iy[k] = min(max(oy * p.sh - p.ph + k, 0), p.h - 1);
#pragma unroll
  for (int k = 0; k < KW; ++k) ix[k] = min(max(ox * p.sw - p.pw + k, 0), p.w - 1);
  u16x8 v[KD * KH * KW];
#pragma unroll
  for (int a = 0; a < KD; ++a)
#pragma unroll
    for (int b = 0; b < KH; ++b)
#pragma unroll
      for (int c = 0; c < KW; ++c)
        v[(a * KH + b) * KW + c] = *(const u16x8*)(inb + (((size_t)iz[a] * p.h + iy[b]) * p.w + ix[c]) * p.c);
  float m[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) m[i] = -__builtin_inff();
#pragma unroll
  for (int k = 0; k < KD * KH * KW; ++k)
#pragma unroll
    for (int i = 0; i < 8; ++i) m[i] = fmaxf(m[i], T::to_f32(v[k][i]));
  const u16x4 lo = T::pack4((f32x4){m[0], m[1], m[2], m[3]});
  const u16x4 hi = T::pack4((f32x4){m[4], m[5], m[6], m[7]});
  *(u16x8*)((uint16_t*)p.out + (size_t)mo * p.ldo + p.c_off + c8 * 8) = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

// ---- 3x3x3 / stride-1 / pad-1 max pooling (S3D's Inception branch3,
// model.py:84-342: MaxPool3d(3, 1, 1) before the 1x1x1 conv): one thread per
// (clip, position, 8-channel piece) walks the frames, taking each frame's
// 3x3 spatial max once (9 reads, the neighbours' rows shared in L1/L2) and
// the frame max over a sliding window of three, so the map is read from HBM
// about once and written once — one pass instead of the separable version's
// three, bit-identical (a max selects one of its inputs either way).
// zg: output frames per thread (all of them by default).  Round 3 tried
// 1 / 2 / 4 of S3D's 8 frames per thread for more parallelism: the whole
// S3D step got 9 / 4 / 1 % slower (same box, tools/archive/pool_ab.sh): the frame
// walk's reuse of the frame maxima, not latency, is what counts.
template <class T>
__global__ __launch_bounds__(256) void maxpool3_s1(fac_pool_desc p, int total, int zg) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= total) return;
  const int C8 = p.c / 8;
  const int c8 = t % C8, t1 = t / C8;
  const int x = t1 % p.w, t2 = t1 / p.w;
  const int y = t2 % p.h, t3 = t2 / p.h;
  const int ngr = (p.d + zg - 1) / zg;
  const int zgi = t3 % ngr, n = t3 / ngr;
  const int z0 = zgi * zg, z1 = min(p.d, z0 + zg);
  const size_t fs = (size_t)p.h * p.w * p.c;
  const uint16_t* inb = (const uint16_t*)p.in + (size_t)n * p.d * fs + c8 * 8;
  // neighbours outside the map re-read the centre row / column (a max over
  // a repeat): branch-free, so the nine loads issue together instead of one
  // exec-masked load (and its wait) at a time
  const int rows[3] = {y > 0 ? y - 1 : y, y, y + 1 < p.h ? y + 1 : y};
  const int cols[3] = {x > 0 ? x - 1 : x, x, x + 1 < p.w ? x + 1 : x};
  auto frame_max = [&](int z, float (&m)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) m[i] = -__builtin_inff();
    const uint16_t* f = inb + (size_t)z * fs;
    u16x8 v[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) v[k] = *(const u16x8*)(f + ((size_t)rows[k / 3] * p.w + cols[k % 3]) * p.c);
#pragma unroll
    for (int k = 0; k < 9; ++k)
#pragma unroll
      for (int i = 0; i < 8; ++i) m[i] = fmaxf(m[i], T::to_f32(v[k][i]));
  };
  float pm[8], cm[8], nm[8];
  if (z0 > 0) {
    frame_max(z0 - 1, pm);
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) pm[i] = -__builtin_inff();
  }
  frame_max(z0, cm);
  uint16_t* ob = (uint16_t*)p.out + ((size_t)n * p.d * p.h * p.w + (size_t)y * p.w + x) * p.ldo + p.c_off + c8 * 8;
  for (int z = z0; z < z1; ++z) {
    if (z + 1 < p.d) {
      frame_max(z + 1, nm);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) nm[i] = -__builtin_inff();
    }
    float a[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      a[i] = fmaxf(fmaxf(pm[i], cm[i]), nm[i]);
      pm[i] = cm[i];
      cm[i] = nm[i];
    }
    const u16x4 lo = T::pack4((f32x4){a[0], a[1], a[2], a[3]});
    const u16x4 hi = T::pack4((f32x4){a[4], a[5], a[6], a[7]});
    *(u16x8*)(ob + (size_t)z * p.h * p.w * p.ldo) = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  }
}

// ---- maxpool3_roll (round 4): the same MaxPool3d(3, 1, 1) for 7-wide maps
// (S3D's 4x7x7 Inception blocks), with three loads per output instead of
// nine: 61.5-65.8 -> 33.6-35.2 us per call at 384 clips, bf16
// (tools/archive/pool_roll_ab.py; on the 8x14x14 maps the W = 14 instance was no
// faster than maxpool3_s1 at 2 waves per SIMD: 200 / 300 vs 225 / 287 us).  One thread per (clip,
// frame group, row y, 8-channel piece) walks a whole row of W positions
// (compile time, fully unrolled) through the frames: per input frame the
// three rows y-1..y+1 of each column are max-ed (3 loads per column), the
// row's frame maxima F(x) = max over the 3 columns are rolled along x, and
// the frame window along z: A = max(F(z-1), F(z)) and F(z) are kept packed
// (16-bit, exact: a max selects one of its inputs) for the whole row, so
// out(z) = max(A, F(z+1)).  Bit-identical to maxpool3_s1 up to the sign of
// a zero (IEEE max of +0 and -0).  zg: output frames per thread.
template <class T>
__device__ __forceinline__ void max8(float (&m)[8], const u16x8 v) {
#pragma unroll
  for (int i = 0; i < 8; ++i) m[i] = fmaxf(m[i], T::to_f32(v[i]));
}
template <class T>
__device__ __forceinline__ u16x8 pack8(const float (&a)[8]) {
  const u16x4 lo = T::pack4((f32x4){a[0], a[1], a[2], a[3]});
  const u16x4 hi = T::pack4((f32x4){a[4], a[5], a[6], a[7]});
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

template <class T, int W>
__global__ __launch_bounds__(256, W > 8 ? 2 : 3) void maxpool3_roll(fac_pool_desc p, int total, int zg) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= total) return;
  const int C = p.c, C8 = C / 8;
  const int c8 = t % C8, t1 = t / C8;
  const int y = t1 % p.h, t2 = t1 / p.h;
  const int ngr = (p.d + zg - 1) / zg;
  const int zgi = t2 % ngr, n = t2 / ngr;
  const int z0 = zgi * zg, z1 = min(p.d, z0 + zg);
  const size_t rs = (size_t)W * C, fs = (size_t)p.h * rs;
  // rows y-1 / y+1 outside the map re-read row y (a max over a repeat)
  const int ym = y > 0 ? y - 1 : y, yp = y + 1 < p.h ? y + 1 : y;
  const uint16_t* inb = (const uint16_t*)p.in + (size_t)n * p.d * fs + c8 * 8;
  // the row's frame maxima F(z, x), x = 0..W-1 in order, each handed to
  // use(x, F) as soon as its three columns are in
  auto frame = [&](int z, auto&& use) {
    const uint16_t* f = inb + (size_t)z * fs;
    float cm[8], cc[8], cn[8];  // column maxima x-2, x-1, x (rolled)
#pragma unroll
    for (int i = 0; i < 8; ++i) cm[i] = cc[i] = cn[i] = -__builtin_inff();
#pragma unroll
    for (int x = 0; x <= W; ++x) {
      if (x < W) {
        const u16x8 a = *(const u16x8*)(f + (size_t)ym * rs + (size_t)x * C);
        const u16x8 b = *(const u16x8*)(f + (size_t)y * rs + (size_t)x * C);
        const u16x8 c = *(const u16x8*)(f + (size_t)yp * rs + (size_t)x * C);
#pragma unroll
        for (int i = 0; i < 8; ++i) cn[i] = fmaxf(fmaxf(T::to_f32(a[i]), T::to_f32(b[i])), T::to_f32(c[i]));
      }
      if (x > 0) {
        float m[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          m[i] = cc[i];
          if (x > 1) m[i] = fmaxf(m[i], cm[i]);
          if (x < W) m[i] = fmaxf(m[i], cn[i]);
        }
        use(x - 1, m);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        cm[i] = cc[i];
        cc[i] = cn[i];
      }
    }
  };
  // A(x) = max(F(z-1, x), F(z, x)) and F(z, x), packed 16-bit (exact: a max
  // selects one of its inputs)
  u16x8 A[W], Fc[W];
  frame(z0, [&](int x, const float (&m)[8]) { Fc[x] = A[x] = pack8<T>(m); });
  if (z0 > 0)
    frame(z0 - 1, [&](int x, const float (&m)[8]) {
      float a[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = m[i];
      max8<T>(a, Fc[x]);
      A[x] = pack8<T>(a);
    });
  uint16_t* ob = (uint16_t*)p.out + ((size_t)n * p.d * p.h + (size_t)y) * W * p.ldo + p.c_off + c8 * 8;
  const size_t ofs = (size_t)p.h * W * p.ldo;
  for (int z = z0; z < z1; ++z) {
    uint16_t* o = ob + (size_t)z * ofs;
    if (z + 1 < p.d) {
      frame(z + 1, [&](int x, const float (&m)[8]) {
        float a[8], b[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          a[i] = fmaxf(T::to_f32(A[x][i]), m[i]);
          b[i] = fmaxf(T::to_f32(Fc[x][i]), m[i]);
        }
        *(u16x8*)(o + (size_t)x * p.ldo) = pack8<T>(a);
        A[x] = pack8<T>(b);
        Fc[x] = pack8<T>(m);
      });
    } else {
#pragma unroll
      for (int x = 0; x < W; ++x) *(u16x8*)(o + (size_t)x * p.ldo) = A[x];
    }
  }
}

// ---- maxpool3_lds14 (round 4): MaxPool3d(3, 1, 1) on 14 x 14 maps (S3D's
// Mixed_3b / 3c branch3 at 112^2 clips).  maxpool3_s1 reads each input nine
// times through L1, which the ~20 resident waves of a CU thrash (0.25 of the
// HBM rate).  Here one workgroup per (clip, 64-channel slice) walks the
// frames: each frame's 14 x 14 x 64 slice is read from HBM once into an LDS
// image with a -inf border (16 x 16 cells of 8 x 16 bytes, double-buffered,
// the next frame prefetched into registers behind the current one's
// arithmetic), every position's 3 x 3 frame maximum comes from LDS, and the
// window over the frames is rolled in registers (A = max(F(z-1), F(z)),
// F(z), packed 16-bit: a max selects one of its inputs).  Bit-identical to
// maxpool3_s1 up to the sign of a zero.
template <class T>
__global__ __launch_bounds__(256) void maxpool3_lds14(fac_pool_desc p) {
  constexpr int S = 14, B = 16, NIT = (S * S * 8 + 255) / 256;  // 1568 items (position, piece): 7 per thread
  __shared__ __attribute__((aligned(16))) uint16_t img[2][B * B * 8 * 8];
  const int tid = threadIdx.x;
  const int nsl = p.c / 64, n = blockIdx.x / nsl, cs = blockIdx.x - n * nsl;
  // the -inf border of both images (the interior is rewritten every frame)
  const uint16_t ninf = T::from_f32(-__builtin_inff());
  for (int q = tid; q < 2 * B * B * 8; q += 256) {
    const int b = q / (B * B * 8), r = q - b * (B * B * 8), cell = r / 8, hy = cell / B, hx = cell - hy * B;
    if (hy == 0 || hy == B - 1 || hx == 0 || hx == B - 1) {
      u16x8 v;
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = ninf;
      *(u16x8*)(img[b] + r * 8) = v;
    }
  }
  const size_t fs = (size_t)S * S * p.c;
  const uint16_t* inb = (const uint16_t*)p.in + (size_t)n * p.d * fs + cs * 64;
  int gof[NIT], lof[NIT];  // per item: global element offset in a frame, LDS element offset of its centre
  bool val[NIT];
#pragma unroll
  for (int j = 0; j < NIT; ++j) {
    const int q = tid + 256 * j, px = q / 8, c8 = q - px * 8, y = px / S, x = px - y * S;
    val[j] = q < S * S * 8;
    gof[j] = val[j] ? px * p.c + c8 * 8 : 0;
    lof[j] = (((y + 1) * B + x + 1) * 8 + c8) * 8;
  }
  u16x8 pre[NIT];
  auto load = [&](int z) {
#pragma unroll
    for (int j = 0; j < NIT; ++j) pre[j] = *(const u16x8*)(inb + (size_t)z * fs + gof[j]);
  };
  auto put = [&](int b) {
#pragma unroll
    for (int j = 0; j < NIT; ++j)
      if (val[j]) *(u16x8*)(img[b] + lof[j]) = pre[j];
  };
  // F(z) of item j from image b: the 3 x 3 max around its centre
  auto fmax9 = [&](int b, int j, float (&m)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) m[i] = -__builtin_inff();
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
      for (int dx = -1; dx <= 1; ++dx) max8<T>(m, *(const u16x8*)(img[b] + lof[j] + (dy * B + dx) * 64));
  };
  u16x8 A[NIT], Fc[NIT];
  load(0);
  put(0);
  __syncthreads();
  if (p.d > 1) load(1);
#pragma unroll
  for (int j = 0; j < NIT; ++j) {
    float m[8];
    fmax9(0, j, m);
    Fc[j] = A[j] = pack8<T>(m);
  }
  uint16_t* ob = (uint16_t*)p.out + (size_t)n * p.d * S * S * p.ldo + p.c_off + cs * 64;
  for (int z = 0; z < p.d; ++z) {
    uint16_t* o = ob + (size_t)z * S * S * p.ldo;
    if (z + 1 < p.d) {
      const int b = (z + 1) & 1;
      put(b);
      __syncthreads();
      if (z + 2 < p.d) load(z + 2);
#pragma unroll
      for (int j = 0; j < NIT; ++j) {
        if (!val[j]) continue;
        float m[8], a[8], c[8];
        fmax9(b, j, m);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          a[i] = fmaxf(T::to_f32(A[j][i]), m[i]);
          c[i] = fmaxf(T::to_f32(Fc[j][i]), m[i]);
        }
        const int q = tid + 256 * j, px = q / 8, c8 = q - px * 8;
        *(u16x8*)(o + (size_t)px * p.ldo + c8 * 8) = pack8<T>(a);
        A[j] = pack8<T>(c);
        Fc[j] = pack8<T>(m);
      }
    } else {
#pragma unroll
      for (int j = 0; j < NIT; ++j) {
        if (!val[j]) continue;
        const int q = tid + 256 * j, px = q / 8, c8 = q - px * 8;
        *(u16x8*)(o + (size_t)px * p.ldo + c8 * 8) = A[j];
      }
    }
  }
}

// ---- maxpool3_pw (round 6): S3D's Inception branch3 -- MaxPool3d(3, 1, 1)
// then BasicConv3d(cin, cout, 1) + BN + ReLU (model.py:84-342, e.g.
// :100-103) -- as one launch, so the pooled map (as large as the block
// input) is never written to HBM and read back.  A unit is (clip, G
// consecutive frames) of an S x S map; per 64-channel chunk of the input:
//  1. every (position, 16-byte piece) of the unit takes the max over its
//     frames z-1..z+1 (three global loads, clamped to the clip: a max over a
//     repeat) into an LDS image (double-buffered, one barrier per chunk);
//  2. each wave then forms its MFMA B fragments directly: a 16-lane row of
//     a fragment holds whole image rows (16 / S of them, lane = x), so the
//     max over y-1..y+1 is three LDS reads and the max over x-1..x+1 two DPP
//     row shifts (neighbours outside the row: the lane itself);
//  3. the fragments feed the 1x1 conv's MFMAs straight from registers
//     (weights [n][k] read as A fragments from global / L1, transposed as in
//     conv_pw: each lane ends with 8 consecutive channels of one position).
// Maxima are exact (a max selects one of its inputs), taken on the 16-bit
// patterns: fp16 with v_pk_max_f16, bf16 as int16 keys (x ^ 0x7fff for
// negative x, monotonic in the float order) with v_pk_max_i16.  Outputs are
// what fac_pool_nd then the 1x1 conv produce, up to fp32 summation order and
// the sign of a zero.
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <class T>
__device__ __forceinline__ uint32_t mp_key(uint32_t v) {  // an involution
  if constexpr (T::id == 0) {
    const s16x2 s = __builtin_bit_cast(s16x2, v);
    return __builtin_bit_cast(uint32_t, s ^ ((s >> (s16x2)15) & (s16x2)0x7fff));
  } else {
    return v;
  }
}
template <class T>
__device__ __forceinline__ uint32_t mp_max(uint32_t a, uint32_t b) {
  if constexpr (T::id == 0)
    return __builtin_bit_cast(uint32_t,
                              __builtin_elementwise_max(__builtin_bit_cast(s16x2, a), __builtin_bit_cast(s16x2, b)));
  else
    return __builtin_bit_cast(uint32_t,
                              __builtin_elementwise_max(__builtin_bit_cast(f16x2, a), __builtin_bit_cast(f16x2, b)));
}
template <class T>
__device__ __forceinline__ u32x4 mp_max4(u32x4 a, u32x4 b) {
  u32x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = mp_max<T>(a[i], b[i]);
  return r;
}

// S: map side; G: frames per unit (divides the clip's frames); NCT: output
// channels per workgroup / 32 (blockIdx.y walks the column blocks)
template <class T, int S, int G, int NCT>
__global__ __launch_bounds__(256, 2) void maxpool3_pw(const uint16_t* __restrict__ in, const uint16_t* __restrict__ w,
                                                      const float* __restrict__ bias, uint16_t* __restrict__ out,
                                                      int nunits, int D, int C, int kp, int ldo, int c_off,
                                                      int relu_on) {
  constexpr int P = G * S * S;              // positions per unit
  constexpr int RPT = 16 / S;               // image rows per 16-lane fragment row
  constexpr int NR = G * S;                 // image rows per unit
  constexpr int NT = (NR + RPT - 1) / RPT;  // MFMA position tiles per unit
  constexpr int RTW = (NT + 3) / 4;         // per wave
  constexpr int NIT = (P * 8 + 255) / 256;  // phase-1 items per thread
  constexpr int TMS = P * 64;               // elements per LDS image
  constexpr int CT = 2 * NCT;               // 16-channel MFMA tiles
  __shared__ __attribute__((aligned(16))) uint16_t tm[2 * TMS];
  __shared__ __attribute__((aligned(16))) uint16_t wl[2][2 * CT * 512];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  // units dealt to XCDs in contiguous ranges (block b runs on XCD b % 8), so
  // the frames a unit shares with its neighbours are re-read from one L2
  const int per = (int)(gridDim.x >> 3);
  const int u = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
  if (u >= nunits) return;
  const int n0 = blockIdx.y * 32 * NCT;
  const int ngr = D / G, clip = u / ngr, z0 = (u - clip * ngr) * G;
  const int fs = S * S * C;
  const uint16_t* xb = in + (size_t)clip * D * fs;

  // phase 1 geometry: item q = (position p, piece c8): the element offset of
  // its centre frame, and packed: LDS slot | c8 << 16 (8: no item) | frame
  // z-1 in the clip << 20 | frame z+1 in the clip << 21
  int qoff[NIT], qinf[NIT];
#pragma unroll
  for (int j = 0; j < NIT; ++j) {
    // (a non-item, q >= P * 8, points at its unit's first position: the
    // branch-free loads below still read it, so it must be in the clip)
    const int q = tid + 256 * j, item = q < P * 8, p = item ? q >> 3 : 0, c8 = q & 7;
    const int zz = p / (S * S), pos = p - zz * S * S, z = z0 + zz;
    qoff[j] = z * fs + pos * C + (item ? c8 * 8 : 0);
    qinf[j] = (p * 8 + (c8 ^ ((p >> 1) & 7))) * 8 | (item ? c8 : 8) << 16 | (z > 0) << 20 | (z + 1 < D) << 21;
  }
  // phase 2 geometry: this lane's image row within a fragment row and column
  const int lr = r16 < RPT * S ? r16 / S : RPT - 1, x = r16 < RPT * S ? r16 - lr * S : S - 1;
  const bool xl = x == 0, xr = x == S - 1;
  // weight fragments: row r16 of channel tile ct = channel
  // 32 (ct >> 1) + 8 (r16 >> 2) + 4 (ct & 1) + (r16 & 3) (conv_pw's order);
  // a chunk's 2 x CT fragments (k-step s, tile ct) are copied to LDS by
  // global_load_lds, fragment f = s * CT + ct by wave f % 4, each a 1 KB
  // lane-ordered image [g][r16][8] (one conflict-free ds_read_b128 per use),
  // double-buffered: issued with the chunk's pixel loads, so a chunk costs
  // one memory round trip and no VGPRs hold weights across it
  constexpr int WFW = (2 * CT + 3) / 4;  // fragments per wave per chunk
  const uint16_t* wsrc[WFW];
#pragma unroll
  for (int i = 0; i < WFW; ++i) {
    const int f = wave + 4 * i, ct = f % CT, s = f / CT;
    wsrc[i] = w + (size_t)(n0 + 32 * (ct >> 1) + 8 * (r16 >> 2) + 4 * (ct & 1) + (r16 & 3)) * kp + s * 32 + g * 8;
  }

  f32x4 acc[RTW][CT];
#pragma unroll
  for (int i = 0; i < RTW; ++i)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) acc[i][ct] = (f32x4)0.f;

  const int nch = kp / 64;
  // chunk kc's pixel loads (pieces past C: zero, which the zero weight rows
  // of k_pad multiply) and its weight fragments (glds); a chunk's loads are
  // issued before the previous chunk's fragments and MFMAs, so each
  // workgroup keeps one chunk in flight while it computes
  u32x4 v[NIT][3];
  // Branch-free: pieces past C (and non-items) load the chunk's first piece
  // of the position, a valid address, and phase 1 zeroes them.
  auto load = [&](int kc) __attribute__((always_inline)) {
    const int kb = kc * 64, nval = min(8, (C - kb) >> 3);
#pragma unroll
    for (int j = 0; j < NIT; ++j) {
      const int c8 = (qinf[j] >> 16) & 15;
      const uint16_t* c = xb + qoff[j] + kb - (c8 < nval ? 0 : (c8 & 7) * 8);
      v[j][0] = *(const u32x4*)(c - ((qinf[j] >> 20) & 1) * fs);
      v[j][1] = *(const u32x4*)c;
      v[j][2] = *(const u32x4*)(c + ((qinf[j] >> 21) & 1) * fs);
    }
#pragma unroll
    for (int i = 0; i < WFW; ++i)
      if (wave + 4 * i < 2 * CT) glds16(wsrc[i] + kb, wl[kc & 1] + (wave + 4 * i) * 512);
  };
  load(0);
  for (int kc = 0; kc < nch; ++kc) {
    uint16_t* const img = tm + (kc & 1) * TMS;
    const uint16_t* const wimg = wl[kc & 1];
    // 1. frame maxima into the image.  (The empty asm pins the maxima here:
    // computed right behind the prefetch, they would wait for its loads.)
#pragma unroll
    for (int j = 0; j < NIT; ++j) asm volatile("" : "+v"(v[j][0]), "+v"(v[j][1]), "+v"(v[j][2]));
    const int nval = min(8, (C - kc * 64) >> 3);
#pragma unroll
    for (int j = 0; j < NIT; ++j) {
      const int c8 = (qinf[j] >> 16) & 15;
      if (c8 >= 8) continue;
      u32x4 m;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        m[i] = mp_max<T>(mp_max<T>(mp_key<T>(v[j][0][i]), mp_key<T>(v[j][1][i])), mp_key<T>(v[j][2][i]));
      *(u32x4*)(img + (qinf[j] & 0xffff)) = c8 < nval ? m : (u32x4)0u;
    }
    __syncthreads();  // (its vmcnt(0) also lands the weight fragments)
    if (kc + 1 < nch) load(kc + 1);  // its image / weight buffers were last read two chunks ago
    // 2 + 3. row and column maxima into B fragments, MFMAs
#pragma unroll
    for (int i = 0; i < RTW; ++i) {
      const int t = wave + 4 * i;
      if (t >= NT) break;
      const int rho = min(t * RPT + lr, NR - 1), y = rho % S, p = rho * S + x;
      const int pu = y > 0 ? p - S : p, pd = y + 1 < S ? p + S : p;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int c8 = s * 4 + g;
        const u32x4 a = *(const u32x4*)(img + (pu * 8 + (c8 ^ ((pu >> 1) & 7))) * 8);
        const u32x4 b = *(const u32x4*)(img + (p * 8 + (c8 ^ ((p >> 1) & 7))) * 8);
        const u32x4 c = *(const u32x4*)(img + (pd * 8 + (c8 ^ ((pd >> 1) & 7))) * 8);
        const u32x4 vm = mp_max4<T>(mp_max4<T>(a, b), c);
        u32x4 f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t ve = vm[e];
          uint32_t l = (uint32_t)__builtin_amdgcn_update_dpp((int)ve, (int)ve, 0x111, 0xf, 0xf, false);  // row_shr:1
          uint32_t r = (uint32_t)__builtin_amdgcn_update_dpp((int)ve, (int)ve, 0x101, 0xf, 0xf, false);  // row_shl:1
          l = xl ? ve : l;
          r = xr ? ve : r;
          f[e] = mp_key<T>(mp_max<T>(mp_max<T>(l, ve), r));
        }
        const u16x8 pf = __builtin_bit_cast(u16x8, f);
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
          acc[i][ct] = T::mfma(*(const u16x8*)(wimg + (s * CT + ct) * 512 + lane * 8), pf, acc[i][ct]);
      }
    }
  }
  // epilogue: bias + ReLU, 16-byte stores of channels n0 + 32 h + 8 g .. + 7
  float bv[CT][4];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int j = 0; j < 4; ++j) bv[ct][j] = bias ? bias[n0 + 32 * (ct >> 1) + 8 * g + 4 * (ct & 1) + j] : 0.f;
  if (r16 >= RPT * S) return;
#pragma unroll
  for (int i = 0; i < RTW; ++i) {
    const int t = wave + 4 * i, rho = t * RPT + lr;
    if (t >= NT || rho >= NR) break;
    uint16_t* o = out + (size_t)(u * P + rho * S + x) * ldo + c_off + n0 + 8 * g;
#pragma unroll
    for (int h = 0; h < NCT; ++h) {
      u16x4 q[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        f32x4 vv;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float z = acc[i][2 * h + e][j] + bv[2 * h + e][j];
          vv[j] = relu_on ? relu(z) : z;
        }
        q[e] = T::pack4(vv);
      }
      *(u16x8*)(o + 32 * h) = __builtin_shufflevector(q[0], q[1], 0, 1, 2, 3, 4, 5, 6, 7);
    }
  }
}

// ---- maxpool2s_pw (round 6): S3D's base.1 + base.2 -- MaxPool3d((1,3,3),
// (1,2,2), (0,1,1)) then BasicConv3d(64, 64, 1) + BN + ReLU (model.py:19-20)
// -- as one launch, so the pooled map is never written and read back (the
// pool read 4.9 GB and wrote 1.2 GB at 1536 clips, the 1x1 read that 1.2 GB
// again).  A unit is (clip, frame, RB pooled rows of a WO-wide map, i.e. the
// 2 RB + 1 input rows under them):
//  1. each (pooled row, input column, 16-byte piece) takes the max over its
//     three input rows 2py-1 .. 2py+1 (three global loads, clamped: a max over
//     a repeat) into an LDS image, piece c8 of column x at c8 ^ ((x >> 1) & 7);
//  2. each wave forms its MFMA B fragments from the image: the max over input
//     columns 2px-1 .. 2px+1 (three LDS reads, clamped), lane = pooled
//     position;
//  3. the 64 -> 64 conv's MFMAs from registers (weights glds'd to LDS as
//     conv_pw's lane-ordered fragments), bias + ReLU, 16-byte stores.
// Exact maxima on 16-bit patterns as in maxpool3_pw (mp_key / mp_max).
template <class T, int WO, int RB>
__global__ __launch_bounds__(256, 3) void maxpool2s_pw(const uint16_t* __restrict__ in, const uint16_t* __restrict__ w,
                                                       const float* __restrict__ bias, uint16_t* __restrict__ out,
                                                       int nunits, int H, int Ho, int ldo, int c_off, int relu_on) {
  constexpr int W = 2 * WO, C = 64, P = RB * WO;  // input row width, channels, pooled positions per unit
  constexpr int NT = (P + 15) / 16, RTW = (NT + 3) / 4;
  constexpr int NIT = (RB * W * 8 + 255) / 256;
  constexpr int CT = 4;  // 64 output channels as 16-channel MFMA tiles
  __shared__ __attribute__((aligned(16))) uint16_t img[RB * W * 64];
  __shared__ __attribute__((aligned(16))) uint16_t wl[2 * CT * 512];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int per = (int)(gridDim.x >> 3);
  const int u = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);  // contiguous units per XCD
  if (u >= nunits) return;
  const int nb = (Ho + RB - 1) / RB, fz = u / nb, py0 = (u - fz * nb) * RB;  // fz = clip * D + frame
  const uint16_t* xb = in + (size_t)fz * H * W * C;
  // weights: fragment f = s * CT + ct by wave f % 4 (conv_pw's channel order)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int f = wave + 4 * i, ct = f % CT, s = f / CT;
    glds16(w + (size_t)(32 * (ct >> 1) + 8 * (r16 >> 2) + 4 * (ct & 1) + (r16 & 3)) * 64 + s * 32 + g * 8,
           wl + f * 512);
  }
  // 1. row maxima: item (pooled row r, input column x, piece c8)
  u32x4 v[NIT][3];
  int slot[NIT];
#pragma unroll
  for (int j = 0; j < NIT; ++j) {
    const int q = tid + 256 * j, c8 = q & 7, x = (q >> 3) % W, r = (q >> 3) / W;
    const int py = min(py0 + r, Ho - 1), y1 = 2 * py;
    const int y0 = max(y1 - 1, 0), y2 = min(y1 + 1, H - 1);
    const uint16_t* c = xb + (size_t)x * C + c8 * 8;
    v[j][0] = *(const u32x4*)(c + (size_t)y0 * W * C);
    v[j][1] = *(const u32x4*)(c + (size_t)y1 * W * C);
    v[j][2] = *(const u32x4*)(c + (size_t)y2 * W * C);
    slot[j] = ((r * W + x) * 8 + (c8 ^ ((x >> 1) & 7))) * 8;
  }
  // every item is real (no branch here: a guarded use let the compiler sink
  // the loads of the guarded items behind the first maxima, a round trip each)
  static_assert(NIT * 256 == RB * W * 8, "whole items per thread");
  __builtin_amdgcn_sched_barrier(0);  // all 3 NIT loads issued before the first maximum
#pragma unroll
  for (int j = 0; j < NIT; ++j) {
    u32x4 m;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      m[i] = mp_max<T>(mp_max<T>(mp_key<T>(v[j][0][i]), mp_key<T>(v[j][1][i])), mp_key<T>(v[j][2][i]));
    *(u32x4*)(img + slot[j]) = m;
  }
  __syncthreads();
  // 2 + 3. column maxima into B fragments, MFMAs
  f32x4 acc[RTW][CT];
#pragma unroll
  for (int i = 0; i < RTW; ++i)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) acc[i][ct] = (f32x4)0.f;
#pragma unroll
  for (int i = 0; i < RTW; ++i) {
    const int t = wave + 4 * i;
    if (t >= NT) break;
    const int p = min(t * 16 + r16, P - 1), r = p / WO, px = p - r * WO;
    const int x1 = 2 * px, x0 = max(x1 - 1, 0), x2 = min(x1 + 1, W - 1);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c8 = s * 4 + g;
      const u32x4 a = *(const u32x4*)(img + ((r * W + x0) * 8 + (c8 ^ ((x0 >> 1) & 7))) * 8);
      const u32x4 b = *(const u32x4*)(img + ((r * W + x1) * 8 + (c8 ^ ((x1 >> 1) & 7))) * 8);
      const u32x4 c = *(const u32x4*)(img + ((r * W + x2) * 8 + (c8 ^ ((x2 >> 1) & 7))) * 8);
      const u32x4 vm = mp_max4<T>(mp_max4<T>(a, b), c);
      u32x4 f;
#pragma unroll
      for (int e = 0; e < 4; ++e) f[e] = mp_key<T>(vm[e]);
      const u16x8 pf = __builtin_bit_cast(u16x8, f);
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) acc[i][ct] = T::mfma(*(const u16x8*)(wl + (s * CT + ct) * 512 + lane * 8), pf, acc[i][ct]);
    }
  }
  // epilogue: bias + ReLU, 16-byte stores of channels 32 h + 8 g .. + 7
  float bv[CT][4];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int j = 0; j < 4; ++j) bv[ct][j] = bias ? bias[32 * (ct >> 1) + 8 * g + 4 * (ct & 1) + j] : 0.f;
#pragma unroll
  for (int i = 0; i < RTW; ++i) {
    const int t = wave + 4 * i, p = t * 16 + r16, r = p / WO, px = p - r * WO;
    if (t >= NT) break;
    if (p >= P || py0 + r >= Ho) continue;
    uint16_t* o = out + ((size_t)fz * Ho * WO + (size_t)(py0 + r) * WO + px) * ldo + c_off + 8 * g;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      u16x4 q[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        f32x4 vv;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float z = acc[i][2 * h + e][j] + bv[2 * h + e][j];
          vv[j] = relu_on ? relu(z) : z;
        }
        q[e] = T::pack4(vv);
      }
      *(u16x8*)(o + 32 * h) = __builtin_shufflevector(q[0], q[1], 0, 1, 2, 3, 4, 5, 6, 7);
    }
  }
}

// ---- sep_tiny (round 6): Mixed_3b's branch2 SepConv3d(16, 32, 3) on 8 x 14
// x 14 maps (model.py:84-110: the (1,3,3) conv 16 -> 32 + BN + ReLU, then the
// (3,1,1) conv 32 -> 32 + BN + ReLU) in one launch.  Through the generic
// implicit GEMM these 16- / 32-channel layers ran at ~0.1 of peak with 230 MB
// of traffic in 0.4 ms (two launches of latency-bound 16-channel gathers and
// the 32-channel map through HBM).  Here one 512-thread workgroup per CU
// walks clips: a clip's whole 8 x 196 x 16 input (50 KB) lands in LDS by
// global_load_lds, the spatial conv writes its 8 x 196 x 32 map to LDS (100
// KB), the temporal conv reads it and stores straight into the block
// output's channel slot; the next clip's input streams in behind the
// temporal phase.  Both convs are transposed MFMAs (rows = channels in
// conv_pw's order, so a lane ends with 8 consecutive channels of a
// position), with the weights in VGPRs; taps outside the frame / clip read
// zero.  K orders as fac_conv_nd's packing: spatial k = tap * 16 + c (k_pad
// 192: 5 steps of two taps), temporal k = dz * 32 + c.
template <class T>
__global__ __launch_bounds__(512, 1) void sep_tiny(const uint16_t* __restrict__ in, const uint16_t* __restrict__ ws,
                                                   const float* __restrict__ bs, int kps, const uint16_t* __restrict__ wt,
                                                   const float* __restrict__ bt, int kpt, uint16_t* __restrict__ out,
                                                   int nclips, int ldo, int c_off, int relu_s, int relu_t) {
  constexpr int S = 14, P = S * S, D = 8, NP = D * P, NT = NP / 16;  // positions per clip, 98 tiles
  constexpr int XEL = NP * 16, MEL = NP * 32;                          // elements: input (16 ch), map (32 ch)
  constexpr int XPL = (NP * 2 + 511) / 512;                           // glds pieces per lane per clip (6.1 -> 7)
  __shared__ __attribute__((aligned(16))) uint16_t smem[XEL + MEL];
  uint16_t* const xs = smem;        // [position][2 pieces]
  uint16_t* const ms = smem + XEL;  // [position][4 pieces], piece g at g ^ ((p >> 2) & 3)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  // weights as A fragments: row r16 of channel tile ct = channel 8 (r16 >> 2) + 4 ct + (r16 & 3)
  const int wrow = 8 * (r16 >> 2) + (r16 & 3);
  u16x8 wsf[5][2], wtf[3][2];
#pragma unroll
  for (int s = 0; s < 5; ++s)
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) wsf[s][ct] = *(const u16x8*)(ws + (size_t)(wrow + 4 * ct) * kps + s * 32 + g * 8);
#pragma unroll
  for (int s = 0; s < 3; ++s)
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) wtf[s][ct] = *(const u16x8*)(wt + (size_t)(wrow + 4 * ct) * kpt + s * 32 + g * 8);
  float bsv[2][4], btv[2][4];
#pragma unroll
  for (int ct = 0; ct < 2; ++ct)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bsv[ct][j] = bs ? bs[8 * g + 4 * ct + j] : 0.f;
      btv[ct][j] = bt ? bt[8 * g + 4 * ct + j] : 0.f;
    }
  // a clip's input: unit q = position q >> 1, half q & 1 (16 consecutive bytes
  // of the dense 16-channel row); units past the clip re-read its last one
  auto issue = [&](int clip) {
    const uint16_t* src = in + (size_t)min(clip, nclips - 1) * NP * 16;
#pragma unroll
    for (int i = 0; i < XPL; ++i) {
      const int q = min((i * 8 + wave) * 64 + lane, NP * 2 - 1);
      if ((i * 8 + wave) * 64 < NP * 2) glds16(src + q * 8, xs + (i * 8 + wave) * 64 * 8);
    }
  };
  int clip = blockIdx.x;
  if (clip < nclips) issue(clip);
  for (; clip < nclips; clip += gridDim.x) {
    __syncthreads();  // (vmcnt(0): this clip's input landed; the previous clip's map reads are done)
    // spatial (1,3,3): B fragment of k-step s, lane group g = tap 2 s + (g >> 1), channel half g & 1
    for (int t = wave; t < NT; t += 8) {
      const int p = t * 16 + r16, z = p / P, pos = p - z * P, y = pos / S, x = pos - y * S;
      f32x4 acc[2] = {(f32x4)0.f, (f32x4)0.f};
#pragma unroll
      for (int s = 0; s < 5; ++s) {
        const int tap = 2 * s + (g >> 1), dy = tap / 3 - 1, dx = tap % 3 - 1;
        const int yy = y + dy, xx = x + dx;
        u16x8 b = (u16x8)0;
        if (tap < 9 && (unsigned)yy < (unsigned)S && (unsigned)xx < (unsigned)S)
          b = *(const u16x8*)(xs + ((z * P + yy * S + xx) * 2 + (g & 1)) * 8);
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) acc[ct] = T::mfma(wsf[s][ct], b, acc[ct]);
      }
      f32x4 v[2];
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float q = acc[ct][j] + bsv[ct][j];
          v[ct][j] = relu_s ? relu(q) : q;
        }
      const u16x4 lo = T::pack4(v[0]), hi = T::pack4(v[1]);
      *(u16x8*)(ms + (p * 4 + (g ^ ((p >> 2) & 3))) * 8) = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    }
    __syncthreads();  // the map is complete; the input image is free
    if (clip + (int)gridDim.x < nclips) issue(clip + gridDim.x);
    // temporal (3,1,1): k-step s = frame z + s - 1, lane group g = channels 8 g .. 8 g + 7
    for (int t = wave; t < NT; t += 8) {
      const int p = t * 16 + r16, z = p / P;
      f32x4 acc[2] = {(f32x4)0.f, (f32x4)0.f};
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const int zz = z + s - 1, pp = p + (s - 1) * P;
        u16x8 b = (u16x8)0;
        if ((unsigned)zz < (unsigned)D) b = *(const u16x8*)(ms + (pp * 4 + (g ^ ((pp >> 2) & 3))) * 8);
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) acc[ct] = T::mfma(wtf[s][ct], b, acc[ct]);
      }
      f32x4 v[2];
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float q = acc[ct][j] + btv[ct][j];
          v[ct][j] = relu_t ? relu(q) : q;
        }
      const u16x4 lo = T::pack4(v[0]), hi = T::pack4(v[1]);
      *(u16x8*)(out + ((size_t)clip * NP + p) * ldo + c_off + 8 * g) = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    }
  }
}

// ---- sep_mid (round 6): Mixed_3c's branch2 SepConv3d(32, 96, 3) on 8 x 14 x
// 14 maps (model.py:84-110), the (1,3,3) conv 32 -> 96 and the (3,1,1) conv
// 96 -> 96, each + BN + ReLU, in one launch.  The 96-channel map of a whole
// clip (301 KB) does not fit LDS, so a unit is (clip, 2 image rows): its 8
// frames x 4 input rows (the band and its halo, 28 KB) land by
// global_load_lds, the spatial conv writes the band's 8 x 28 x 96 map to LDS
// (43 KB), and the temporal conv (which needs no spatial halo) reads it.  Six
// waves: wave w computes output channels 32 (w % 3) .. + 31 of position tiles
// w / 3, w / 3 + 2, ..., with its 18 + 18 weight fragments in VGPRs (the
// layers' own packing: spatial k = tap * 32 + c, temporal k = dz * 128 + c
// over the middle channels zero-padded to 128, of which the 96 real ones are
// read).  Two workgroups per CU.
template <class T>
__global__ __launch_bounds__(384, 2) void sep_mid(const uint16_t* __restrict__ in, const uint16_t* __restrict__ ws,
                                                  const float* __restrict__ bs, int kps, const uint16_t* __restrict__ wt,
                                                  const float* __restrict__ bt, int kpt, uint16_t* __restrict__ out,
                                                  int nunits, int ldo, int c_off, int relu_s, int relu_t) {
  constexpr int S = 14, D = 8, RB = 2, NB = S / RB;  // map side, frames, rows per band, bands per clip
  constexpr int PIN = D * (RB + 2) * S;              // input positions per unit (band + halo rows)
  constexpr int P = D * RB * S, NT = P / 16;         // output positions per unit, 14 tiles
  constexpr int XEL = PIN * 32, MEL = P * 96;        // elements: input (32 ch), map (96 ch)
  constexpr int XU = PIN * 4;                         // 16-byte input units, 28 wave instructions
  static_assert(XU % 64 == 0 && P % 16 == 0, "unit shape");
  __shared__ __attribute__((aligned(16))) uint16_t smem[XEL + MEL];
  uint16_t* const xs = smem;        // [pos_in][4 pieces], piece j at j ^ ((pos_in >> 2) & 3)
  uint16_t* const ms = smem + XEL;  // [pos][12 pieces], piece j at 4 (j >> 2) + ((j & 3) ^ ((pos >> 2) & 3))
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int cp = wave % 3, wr = wave / 3;  // channel pair (32 channels), tile row
  const int wrow = 32 * cp + 8 * (r16 >> 2) + (r16 & 3);
  u16x8 wsf[9][2], wtf[9][2];
#pragma unroll
  for (int s = 0; s < 9; ++s)
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
      wsf[s][ct] = *(const u16x8*)(ws + (size_t)(wrow + 4 * ct) * kps + s * 32 + g * 8);
      wtf[s][ct] = *(const u16x8*)(wt + (size_t)(wrow + 4 * ct) * kpt + (s / 3) * 128 + (s % 3) * 32 + g * 8);
    }
  float bsv[2][4], btv[2][4];
#pragma unroll
  for (int ct = 0; ct < 2; ++ct)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bsv[ct][j] = bs ? bs[32 * cp + 8 * g + 4 * ct + j] : 0.f;
      btv[ct][j] = bt ? bt[32 * cp + 8 * g + 4 * ct + j] : 0.f;
    }
  for (int u = blockIdx.x; u < nunits; u += gridDim.x) {
    const int clip = u / NB, y0 = (u - clip * NB) * RB;
    __syncthreads();  // the previous unit's readers are done with both images
    for (int q0 = wave * 64; q0 < XU; q0 += 6 * 64) {
      const int q = q0 + lane, pin = q >> 2, j = (q & 3) ^ ((pin >> 2) & 3);
      const int z = pin / ((RB + 2) * S), rem = pin - z * (RB + 2) * S, r = rem / S, x = rem - r * S;
      const int y = y0 - 1 + r;
      glds16((unsigned)y < (unsigned)S ? in + ((((size_t)clip * D + z) * S + y) * S + x) * 32 + j * 8 : g_zero16,
             xs + q0 * 8);
    }
    __syncthreads();  // (vmcnt(0)) the band's input landed
    // spatial (1,3,3): k-step s = tap, lane group g = channels 8 g .. 8 g + 7
    for (int t = wr; t < NT; t += 2) {
      const int p = t * 16 + r16, z = p / (RB * S), rem = p - z * RB * S, ry = rem / S, x = rem - ry * S;
      f32x4 acc[2] = {(f32x4)0.f, (f32x4)0.f};
#pragma unroll
      for (int s = 0; s < 9; ++s) {
        const int dy = s / 3 - 1, dx = s % 3 - 1, xx = x + dx;
        const int pin = (z * (RB + 2) + ry + 1 + dy) * S + xx;
        u16x8 b = (u16x8)0;
        if ((unsigned)xx < (unsigned)S) b = *(const u16x8*)(xs + (pin * 4 + (g ^ ((pin >> 2) & 3))) * 8);
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) acc[ct] = T::mfma(wsf[s][ct], b, acc[ct]);
      }
      f32x4 v[2];
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float q = acc[ct][j] + bsv[ct][j];
          v[ct][j] = relu_s ? relu(q) : q;
        }
      const u16x4 lo = T::pack4(v[0]), hi = T::pack4(v[1]);
      *(u16x8*)(ms + (p * 12 + 4 * cp + (g ^ ((p >> 2) & 3))) * 8) = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    }
    __syncthreads();  // the band's map is complete
    // temporal (3,1,1): k-step s = (frame offset s / 3, channel block s % 3)
    for (int t = wr; t < NT; t += 2) {
      const int p = t * 16 + r16, z = p / (RB * S), rem = p - z * RB * S;
      f32x4 acc[2] = {(f32x4)0.f, (f32x4)0.f};
#pragma unroll
      for (int s = 0; s < 9; ++s) {
        const int zz = z + s / 3 - 1, pp = p + (s / 3 - 1) * RB * S;
        u16x8 b = (u16x8)0;
        if ((unsigned)zz < (unsigned)D) b = *(const u16x8*)(ms + (pp * 12 + 4 * (s % 3) + (g ^ ((pp >> 2) & 3))) * 8);
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) acc[ct] = T::mfma(wtf[s][ct], b, acc[ct]);
      }
      f32x4 v[2];
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float q = acc[ct][j] + btv[ct][j];
          v[ct][j] = relu_t ? relu(q) : q;
        }
      const u16x4 lo = T::pack4(v[0]), hi = T::pack4(v[1]);
      const int ry = rem / S, x = rem - ry * S;
      *(u16x8*)(out + ((((size_t)clip * D + z) * S + y0 + ry) * S + x) * ldo + c_off + 32 * cp + 8 * g) =
          __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    }
  }
}

// ---- input staging
template <class T, bool U8>
__global__ __launch_bounds__(256) void pack_input(const void* src, int n_img, int S, float div, float m0, float m1,
                                                  float m2, float s0, float s1, float s2, uint16_t* out, int c_pad) {
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  if (t >= (long long)n_img * S) return;
  const int n = (int)(t / S), s = (int)(t - (long long)n * S);
  float x[3];
  if constexpr (U8) {
    const uint8_t* p = (const uint8_t*)src + (size_t)t * 3;
    x[0] = (float)p[0];
    x[1] = (float)p[1];
    x[2] = (float)p[2];
  } else {
    const float* p = (const float*)src + (size_t)n * 3 * S + s;
    x[0] = p[0];
    x[1] = p[(size_t)S];
    x[2] = p[(size_t)2 * S];
  }
  const float mean[3] = {m0, m1, m2}, sd[3] = {s0, s1, s2};
  uint16_t* o = out + (size_t)t * c_pad;
  u16x8 v = (u16x8)0;
#pragma unroll
  for (int c = 0; c < 3; ++c) v[c] = T::from_f32((x[c] / div - mean[c]) / sd[c]);
  *(u16x8*)o = v;
  for (int c = 8; c < c_pad; c += 8) *(u16x8*)(o + c) = (u16x8)0;
}

// Space-to-depth staging for a stride-2 first conv: image pixel (y, x) goes
// to s2d pixel (y/2 + pb, x/2 + pb), channel ((y%2)*2 + x%2)*4 + c (c < 3;
// channel 3 of each pixel and the pb / pa border are zero), so a KxK stride-2
// conv becomes a stride-1 conv over 2x2-pixel cells with 16 contiguous
// channels per cell (fac_pack_input_s2d).  One thread per s2d cell.
template <class T, bool U8>
__global__ __launch_bounds__(256) void pack_input_s2d(const void* src, int n_img, int frames, int H, int W, int pb,
                                                      int pa, float div, float m0, float m1, float m2, float s0,
                                                      float s1, float s2, uint16_t* out) {
  const int Ho = H / 2 + pb + pa, Wo = W / 2 + pb + pa;
  // 32-bit index math (the launcher checks n_img * Ho * Wo < 2^31): a 64-bit
  // division per cell cost as much as the loads
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= n_img * Ho * Wo) return;
  const int nY = t / Wo, X = t - nY * Wo, n = nY / Ho, Y = nY - n * Ho;
  const float mean[3] = {m0, m1, m2}, sd[3] = {s0, s1, s2};
  u16x8 lo = (u16x8)0, hi = (u16x8)0;
  const int y0 = 2 * (Y - pb), x0 = 2 * (X - pb);
  // branch-free: out-of-image pixels load pixel 0 and are zeroed, so the 12
  // loads issue together (one exec-masked branch per pixel made each wait)
  float v[4][3];
  bool ok[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const int y = y0 + (d >> 1), x = x0 + (d & 1);
    ok[d] = !(y < 0 || y >= H || x < 0 || x >= W || Y < pb || X < pb || Y >= Ho - pa || X >= Wo - pa);
    const int yy = ok[d] ? y : 0, xx = ok[d] ? x : 0;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      if constexpr (U8) {
        v[d][c] = (float)((const uint8_t*)src)[(((size_t)n * H + yy) * W + xx) * 3 + c];
      } else {  // planar [clip][3][frames][H][W]: image n = clip * frames + frame
        const int b = n / frames, f = n - b * frames;
        v[d][c] = ((const float*)src)[((((size_t)b * 3 + c) * frames + f) * H + yy) * W + xx];
      }
    }
  }
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    if (!ok[d]) continue;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const uint16_t h = T::from_f32((v[d][c] / div - mean[c]) / sd[c]);
      if (d < 2) lo[d * 4 + c] = h; else hi[(d - 2) * 4 + c] = h;
    }
  }
  uint16_t* o = out + (size_t)t * 16;
  *(u16x8*)o = lo;
  *(u16x8*)(o + 8) = hi;
}

// ---- KANLinear
// Cox-de Boor recursion of kan.py:90-132 for one input value, in the
// reference's operation order (no contraction: the file is compiled with
// -ffp-contract=off semantics via the explicit _rn intrinsics).
template <int NK>
__device__ __forceinline__ void kan_bases(float x, const float* g, float* b) {
  constexpr int NB0 = NK - 1;
#pragma unroll
  for (int j = 0; j < NB0; ++j) b[j] = (x >= g[j] && x < g[j + 1]) ? 1.f : 0.f;
#pragma unroll
  for (int k = 1; k <= 3; ++k) {
#pragma unroll
    for (int j = 0; j < NB0 - k; ++j) {
      const float l = __fmul_rn(__fdiv_rn(__fsub_rn(x, g[j]), __fsub_rn(g[j + k], g[j])), b[j]);
      const float r = __fmul_rn(__fdiv_rn(__fsub_rn(g[j + k + 1], x), __fsub_rn(g[j + k + 1], g[j + 1])), b[j + 1]);
      b[j] = __fadd_rn(l, r);
    }
  }
}

constexpr int kKanNK = 12;             // grid_size 5 + 2*order 3 + 1 knots
constexpr int kKanF = 1 + kKanNK - 4;  // silu + 8 bases per input
constexpr int kKanRows = 32, kKanIn = 32;

// grid (in-chunks, row-chunks): features of 32 rows x 32 inputs into LDS,
// then every (row, out) pair of the chunk accumulates its 32 x 9 products
// into a partial slab [in-chunk][row][out] (summed in chunk order after).
// Weights are k-major wcat[in][9][out], so the 64 threads of a row group read
// 64 consecutive outputs' weights of one k (coalesced) and each feature is an
// LDS broadcast; a thread keeps 8 rows of one output in registers.
__global__ __launch_bounds__(256) void kan_partial(const float* __restrict__ x, int rows, int in_f, int out_f,
                                                   const float* __restrict__ grid, const float* __restrict__ wcat,
                                                   float* __restrict__ part) {
  __shared__ float feat[kKanRows][kKanIn * kKanF + 1];
  const int ic = blockIdx.x, r0 = blockIdx.y * kKanRows, i0 = ic * kKanIn;
  const int ni = min(kKanIn, in_f - i0), nr = min(kKanRows, rows - r0);
  for (int t = threadIdx.x; t < kKanRows * kKanIn; t += 256) {
    const int r = t / kKanIn, i = t - r * kKanIn;
    float* f = &feat[r][i * kKanF];
    if (r < nr && i < ni) {
      const float v = x[(size_t)(r0 + r) * in_f + i0 + i];
      f[0] = v / (1.f + expf(-v));  // SiLU
      float g[kKanNK], b[kKanNK - 1];
#pragma unroll
      for (int k = 0; k < kKanNK; ++k) g[k] = grid[(size_t)(i0 + i) * kKanNK + k];
      kan_bases<kKanNK>(v, g, b);
#pragma unroll
      for (int k = 0; k < kKanF - 1; ++k) f[1 + k] = b[k];
    } else {
#pragma unroll
      for (int k = 0; k < kKanF; ++k) f[k] = 0.f;
    }
  }
  __syncthreads();
  const int K = ni * kKanF;
  const int ol = threadIdx.x & 63, rg = threadIdx.x >> 6;  // 4 row groups of 8 rows
  const float* w0 = wcat + (size_t)i0 * kKanF * out_f;
  for (int ob = 0; ob < out_f; ob += 64) {
    const int o = ob + ol;
    if (o >= out_f) continue;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < K; ++k) {
      const float w = w0[(size_t)k * out_f + o];
#pragma unroll
      for (int r = 0; r < 8; ++r) acc[r] = fmaf(feat[rg * 8 + r][k], w, acc[r]);
    }
#pragma unroll
    for (int r = 0; r < 8; ++r)
      if (rg * 8 + r < nr) part[((size_t)ic * rows + r0 + rg * 8 + r) * out_f + o] = acc[r];
  }
}

__global__ __launch_bounds__(256) void kan_reduce(const float* __restrict__ part, int chunks, int n, float* __restrict__ y) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= n) return;
  float s = 0.f;
  for (int c = 0; c < chunks; ++c) s += part[(size_t)c * n + t];
  y[t] = s;
}

// GGCA (Global Grouped Coordinate Attention) of the CViT RepBn8 variant,
// CViT-main/model/cvit_GGCA_ADD_DEConv_RepBn8.py:144-207, fused with the
// caller's x = x * GGCA(x) (:436-437).  One workgroup per (image, channel
// group); the group's H x W x CG features go to LDS in fp32, then
//   h-pools [H][CG] (mean / max over x), w-pools [W][CG] (mean / max over y),
//   shared_conv: 1x1 CG->CR, BatchNorm(eval, eps 1e-5), ReLU, 1x1 CR->CG on
//   each of the 2H + 2W pooled vectors,
//   att_h = sigmoid(z(h_avg) + z(h_max)), att_w likewise,
//   out = x * ((x * att_h) * att_w)   (the reference's multiplication order)
// all in fp32, 16-bit output (the patch-embedding GEMM's A operand).
// Byte work: 49 x 512 x 2 B in and out per crop — negligible next to the convs.
template <class T>
__global__ __launch_bounds__(256) void ggca_k(const uint16_t* __restrict__ x, int H, int W, int C, int groups,
                                              const float* __restrict__ w1, const float* __restrict__ b1,
                                              const float* __restrict__ bn4, const float* __restrict__ w2,
                                              const float* __restrict__ b2, uint16_t* __restrict__ out) {
  constexpr int MAXP = 16 * 16, MAXCG = 256, MAXV = 64, MAXCR = 16;
  __shared__ float xs[MAXP * MAXCG / 4];      // H*W*CG <= 16384 floats (64 KB)
  __shared__ float pv[MAXV * MAXCG / 2];      // (2H + 2W) pooled vectors x CG
  __shared__ float hid[MAXV * MAXCR];
  const int img = blockIdx.x / groups, gr = blockIdx.x - img * groups;
  const int CG = C / groups, CR = CG / 16, P = H * W, NV = 2 * H + 2 * W;
  const int tid = threadIdx.x;
  const uint16_t* xb = x + (size_t)img * P * C + gr * CG;
  for (int i = tid; i < P * CG; i += 256) {
    const int pix = i / CG, c = i - pix * CG;
    xs[i] = T::to_f32(xb[(size_t)pix * C + c]);
  }
  __syncthreads();
  // pooled vectors: v = 0..H-1 h_avg, H..2H-1 h_max, 2H..2H+W-1 w_avg, 2H+W.. w_max
  for (int i = tid; i < NV * CG; i += 256) {
    const int v = i / CG, c = i - v * CG;
    float acc;
    if (v < 2 * H) {
      const int y = v < H ? v : v - H;
      acc = xs[(y * W) * CG + c];
      for (int xx = 1; xx < W; ++xx) {
        const float e = xs[(y * W + xx) * CG + c];
        acc = v < H ? acc + e : fmaxf(acc, e);
      }
      if (v < H) acc = acc / (float)W;
    } else {
      const int u = v - 2 * H, xx = u < W ? u : u - W;
      acc = xs[xx * CG + c];
      for (int y = 1; y < H; ++y) {
        const float e = xs[(y * W + xx) * CG + c];
        acc = u < W ? acc + e : fmaxf(acc, e);
      }
      if (u < W) acc = acc / (float)H;
    }
    pv[i] = acc;
  }
  __syncthreads();
  for (int i = tid; i < NV * CR; i += 256) {  // 1x1 CG -> CR, BN (eval), ReLU
    const int v = i / CR, r = i - v * CR;
    float a = 0.f;
    for (int c = 0; c < CG; ++c) a += w1[r * CG + c] * pv[v * CG + c];
    a += b1[r];
    const float inv = 1.0f / sqrtf(bn4[CR + r] + 1e-5f);
    a = (a - bn4[r]) * inv * bn4[2 * CR + r] + bn4[3 * CR + r];
    hid[i] = fmaxf(a, 0.f);
  }
  __syncthreads();
  for (int i = tid; i < NV * CG; i += 256) {  // 1x1 CR -> CG
    const int v = i / CG, c = i - v * CG;
    float a = 0.f;
    for (int r = 0; r < CR; ++r) a += w2[c * CR + r] * hid[v * CR + r];
    pv[i] = a + b2[c];
  }
  __syncthreads();
  uint16_t* ob = out + (size_t)img * P * C + gr * CG;
  for (int i = tid; i < P * CG; i += 256) {
    const int pix = i / CG, c = i - pix * CG;
    const int y = pix / W, xx = pix - y * W;
    const float ah = 1.0f / (1.0f + expf(-(pv[y * CG + c] + pv[(H + y) * CG + c])));
    const float aw = 1.0f / (1.0f + expf(-(pv[(2 * H + xx) * CG + c] + pv[(2 * H + W + xx) * CG + c])));
    const float v = xs[i];
    ob[(size_t)pix * C + c] = T::from_f32(v * ((v * ah) * aw));
  }
}

__global__ __launch_bounds__(256) void sigmoid_k(const float* __restrict__ x, float* __restrict__ y, int n) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t < n) y[t] = 1.f / (1.f + expf(-x[t]));
}


// ---- conv_s2d4: the 4x4 / stride-1 conv over 16-channel space-to-depth cells
// that the 7x7/2 first convs become (fac_pack_input_s2d): ResNet-50's conv1
// (ResVitKan.py:187, 3 -> 64) and S3D's (1,7,7)/(1,2,2) spatial half of
// base.0 (model.py:18), both + folded BN + ReLU, cout 64.  Through the
// generic implicit GEMM this layer is its costliest (K = 256 in 4 short
// k-steps per 128-row tile, every tile re-reading the 32 KB weight and
// paying a prologue and an LDS-staged epilogue).  Here a workgroup keeps the
// whole weight in LDS and walks output boxes of 8 x 28 positions: per box
// the (11 x 31)-cell halo (2 x 16-byte channel pieces per cell) is copied to
// LDS once and all 16 taps read it.  MFMAs run transposed (C^T = W . X^T:
// rows = channels), so each lane ends with 8 consecutive channels of one
// position (channel-permuted tiles, below) and the epilogue stores 16 bytes
// straight from registers.
// k-step s covers taps 2s, 2s+1 (ty = s/2, tx = 2(s%2) + g/2) x 16 channels:
// lane group g reads channel piece g%2 of tap 2s + g/2, i.e. k = 32s + 8g + e,
// the natural fac_conv_nd weight order.
// F32IN (round 4): `in` is S3D's raw fp32 clip batch
// [clip][3][frames][H][W] and the cells are made while staging each box's
// halo -- fac_pack_input_s2d's 16-bit cell image (1.12 GB per 384-clip
// forward written and read back) never exists.  A lane's pieces are fetched
// as three 8-byte float pairs (one per colour plane; a piece is one pixel row
// of a cell: 2 pixels x 3 channels + 2 zeros) into registers one box ahead,
// and converted + written to the other halo buffer after this box's MFMAs
// and stores; plain loads only, so the compiler's vmcnt waits are exact.
// IN: 0 = fac_pack_input_s2d cells, 1 = the fp32 clip (F32IN above), 2 = a
// uint8 clip (decoded video frames, the same 0..255 values a quarter of the
// bytes: one 2-byte pixel pair per colour plane, widened at the cell write).
template <class T, int IN = 0>
__global__ __launch_bounds__(256, 2) void conv_s2d4(const void* __restrict__ in_, const uint16_t* __restrict__ w,
                                                    const float* __restrict__ bias, uint16_t* __restrict__ out,
                                                    int nbox, int Hc, int Wc, int Ho, int Wo, int kp, int relu_on,
                                                    int frames = 1, int H = 0, int W = 0, int pb = 0) {
  const uint16_t* __restrict__ in = (const uint16_t*)in_;
  constexpr int TH = 8, TW = 28, HH = TH + 3, HWD = TW + 3, RPX = 32;  // halo rows, cols, row pitch (cells)
  constexpr int HSL = 2 * HH * RPX;                                       // 16-byte halo slots
  constexpr int HPW = (HSL + 255) / 256;                                  // glds per wave
  constexpr int WEL = 64 * 256;                                           // weight elements
  constexpr int HEL = HPW * 256 * 8;                                     // halo buffer elements
  constexpr int NPC_ = 2 * HH * HWD, PPL_ = (NPC_ + 255) / 256;
  // IN == 2: the raw pixel pairs of two boxes staged in LDS (see load_raw)
  constexpr int RSZ = IN == 2 ? 2 * PPL_ * 3 * 256 * 2 : 0;  // (one dword slot per lane and piece)
  __shared__ __attribute__((aligned(16))) uint16_t smem[WEL + 2 * HEL + RSZ];
  uint16_t* const sw = smem;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int wm = wave >> 1, wn = wave & 1;

  // weights [s][ct][g][r16][8]: the A fragment of (k-step s, channel tile ct)
  // is one contiguous, conflict-free 1 KB read.  Row i of the wave's tile ct
  // (tiles 2wn, 2wn+1) computes channel 32 wn + 8 (i >> 2) + 4 ct + (i & 3), so
  // lane group g ends with channels 32wn + 8g .. +7 of its position: one
  // 16-byte store, 64 contiguous bytes per position per store instruction
  for (int c = tid; c < 64 * 32; c += 256) {
    const int n = c >> 5, k8 = c & 31;
    const int ct = 2 * (n >> 5) + ((n >> 2) & 1), i = 4 * ((n >> 3) & 3) + (n & 3);
    *(u16x8*)(sw + ((((k8 >> 2) * 4 + ct) * 4 + (k8 & 3)) * 16 + i) * 8) =
        *(const u16x8*)(w + (size_t)n * kp + k8 * 8);
  }
  float bv[2][4];
#pragma unroll
  for (int ct = 0; ct < 2; ++ct)
#pragma unroll
    for (int j = 0; j < 4; ++j) bv[ct][j] = bias ? bias[32 * wn + 8 * g + 4 * ct + j] : 0.f;
  // this lane's halo slot offsets (16-byte units) for pixel tile i at tap (0, g/2)
  int bo[7];
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    const int m = (wm * 7 + i) * 16 + r16, py = m / TW, px = m - (m / TW) * TW;
    bo[i] = ((g & 1) * HH + py) * RPX + px + (g >> 1);
  }
  const int bpr = Wo / TW, bpi = (Ho / TH) * bpr;
  // Round 3: the halo is double-buffered (the next box's streams in while this
  // one computes), and the wait for a box's halo counts the previous box's 7
  // output stores per lane as younger operations: vmcnt counts loads and
  // stores in issue order, so `__syncthreads()` / `vmcnt(0)` per box also
  // waited for the previous box's stores to reach HBM.
  auto issue = [&](int bx, uint16_t* halo) {
    const int img = bx / bpi, rr = bx - img * bpi;
    const int y0 = (rr / bpr) * TH, x0 = (rr - (rr / bpr) * bpr) * TW;
#pragma unroll
    for (int i = 0; i < HPW; ++i) {
      const int sl = (i * 4 + wave) * 64 + lane;
      const int pc = sl / (HH * RPX), rem = sl - pc * (HH * RPX), hy = rem / RPX, hx = rem - (rem / RPX) * RPX;
      const uint16_t* src = g_zero16;
      if (pc < 2 && hx < HWD) src = in + (((size_t)img * Hc + y0 + hy) * Wc + x0 + hx) * 16 + pc * 8;
      glds16(src, halo + (i * 4 + wave) * 64 * 8);
    }
  };
  // F32IN: this lane's cell pieces p = tid + 256 j of the dense 2 x 11 x 31
  // halo (piece 0 / 1 = the cell's top / bottom pixel row), as raw float pairs
  constexpr int NPC = 2 * HH * HWD, PPL = (NPC + 255) / 256;
  constexpr bool F32IN = IN != 0;  // the cells are made from a raw clip while staging
  using RawT = typename std::conditional<IN == 2, uint16_t, float2>::type;
  // two register sets of raw pieces (box j in set j & 1, the box loop
  // unrolled by two so the set index is a constant): the pieces of the box
  // after next are loaded BEFORE this box's stores, so the wait for them
  // (one box later) never includes a box's stores -- two boxes of output
  // stores stay in flight instead of one (round 5: the layer was bound by
  // its stores' latency, ~3 TB/s of writes)
  // (the in-image mask is applied when the cells are written, one box later:
  // a select at the load would make the wave wait for the load right there)
  // IN == 2: the pixel pairs go global -> LDS by 2-byte global_load_lds
  // into a per-box staging area (set SET), lane-linear in dword slots (the
  // LDS side of a sub-dword LDS-DMA load is M0 + 4 * lane), each thread
  // reading back only its own pieces; the waits for them are hand-counted (the
  // pieces and the output stores in issue order: LLVM falls back to
  // vmcnt(0) for a register load consumed behind stores, i.e. it would wait
  // for the box's stores)
  RawT raw[2][F32IN && IN != 2 ? PPL : 1][3];
  uint32_t* const rstage = (uint32_t*)(smem + WEL + 2 * HEL);
  unsigned rok[2] = {0u, 0u};
  auto load_raw = [&](auto setc, int bx) {
    constexpr int SET = decltype(setc)::value;
    rok[SET] = 0u;
    const int img = bx / bpi, rr = bx - img * bpi;
    const int y0 = (rr / bpr) * TH, x0 = (rr - (rr / bpr) * bpr) * TW;
    const int clip = img / frames, f = img - clip * frames;
    const size_t cbase = (size_t)clip * 3 * frames * H * W + (size_t)f * H * W;
#pragma unroll
    for (int j = 0; j < PPL; ++j) {
      const int p = tid + 256 * j;
      const int pc = p / (HH * HWD), rem = p - pc * (HH * HWD), hy = rem / HWD, hx = rem - (rem / HWD) * HWD;
      const int Y = y0 + hy, X = x0 + hx, y = 2 * (Y - pb) + pc, x = 2 * (X - pb);
      const bool ok = p < NPC && Y >= pb && X >= pb && y < H && x < W;
      const size_t off = ok ? (size_t)y * W + x : 0;  // branch-free: masked pieces read pixel 0 and are zeroed
      rok[SET] |= ok ? 1u << j : 0u;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        if constexpr (IN == 2)
          __builtin_amdgcn_global_load_lds(
              (const __attribute__((address_space(1))) void*)((const uint8_t*)in_ + cbase + (size_t)c * frames * H * W + off),
              (__attribute__((address_space(3))) void*)(rstage + ((SET * PPL + j) * 3 + c) * 256 + wave * 64), 2, 0, 0);
        else
          raw[SET][j][c] = *(const float2*)((const float*)in_ + cbase + (size_t)c * frames * H * W + off);
      }
    }
  };
  auto store_cells = [&](auto setc, uint16_t* halo) {
    constexpr int SET = decltype(setc)::value;
#pragma unroll
    for (int j = 0; j < PPL; ++j) {
      const int p = tid + 256 * j;
      if (p < NPC) {
        const int pc = p / (HH * HWD), rem = p - pc * (HH * HWD), hy = rem / HWD, hx = rem - (rem / HWD) * HWD;
        float2 rf[3];
        const bool ok = (rok[SET] >> j) & 1u;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          if constexpr (IN == 2) {
            const uint32_t pr = rstage[((SET * PPL + j) * 3 + c) * 256 + tid] & 0xffffu;
            rf[c] = make_float2((float)(pr & 0xff), (float)(pr >> 8));  // little-endian pixel pair
          } else
            rf[c] = raw[SET][j][c];
          if (!ok) rf[c] = make_float2(0.f, 0.f);
        }
        u16x8 v;
        v[0] = T::from_f32(rf[0].x);
        v[1] = T::from_f32(rf[1].x);
        v[2] = T::from_f32(rf[2].x);
        v[3] = 0;
        v[4] = T::from_f32(rf[0].y);
        v[5] = T::from_f32(rf[1].y);
        v[6] = T::from_f32(rf[2].y);
        v[7] = 0;
        *(u16x8*)(halo + ((pc * HH + hy) * RPX + hx) * 8) = v;
      }
    }
  };
  __syncthreads();  // weights in
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  if constexpr (IN == 2) {
    // every box iteration issues one set of pieces (a dummy re-read of box
    // 0 past the end), so the counted waits below are uniform
    if (blockIdx.x < nbox) {
      load_raw(S0{}, blockIdx.x);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      store_cells(S0{}, smem + WEL);
      load_raw(S1{}, blockIdx.x + (int)gridDim.x < nbox ? blockIdx.x + gridDim.x : 0);
    }
  } else if constexpr (F32IN) {
    if (blockIdx.x < nbox) {
      load_raw(S0{}, blockIdx.x);
      store_cells(S0{}, smem + WEL);
      if (blockIdx.x + (int)gridDim.x < nbox) load_raw(S1{}, blockIdx.x + gridDim.x);
    }
  } else {
    if (blockIdx.x < nbox) issue(blockIdx.x, smem + WEL);
  }
  // box iteration `it` (parity P = it & 1: its cells came from raw set P,
  // the next box's from set P^1; the box after next loads into set P)
  auto box = [&](auto pc, int bx, int it) {
    constexpr int P = decltype(pc)::value;
    using SP = std::integral_constant<int, P>;
    using SQ = std::integral_constant<int, P ^ 1>;
    const int img = bx / bpi, rr = bx - img * bpi;
    const int y0 = (rr / bpr) * TH, x0 = (rr - (rr / bpr) * bpr) * TW;
    uint16_t* const halo = smem + WEL + (it & 1) * HEL;
    const bool more = bx + (int)gridDim.x < nbox;
    if constexpr (F32IN) {
      // this box's cells are written (the previous iteration / the prologue)
      // and every wave is done with the other buffer
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    } else {
      // every wave is done with the other buffer (the previous box): refill it
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (more) issue(bx + gridDim.x, smem + WEL + ((it + 1) & 1) * HEL);
      // this box's halo landed; younger: the next box's pieces (if any) and,
      // after the first box, the previous box's 7 stores
      if (it == 0) {
        if (more) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(HPW) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      } else {
        if (more) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(HPW + 7) : "memory");
        else asm volatile("s_waitcnt vmcnt(7)\n\ts_barrier" ::: "memory");
      }
    }
    f32x4 acc[7][2];
#pragma unroll
    for (int i = 0; i < 7; ++i) acc[i][0] = acc[i][1] = (f32x4)0.f;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      u16x8 wf[2];
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) wf[ct] = *(const u16x8*)(sw + (((s * 4 + 2 * wn + ct) * 4 + g) * 16 + r16) * 8);
      const int so = (s >> 1) * RPX + (s & 1) * 2;
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        const u16x8 pf = *(const u16x8*)(halo + (bo[i] + so) * 8);
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) acc[i][ct] = T::mfma(wf[ct], pf, acc[i][ct]);
      }
    }
    if constexpr (IN == 2)
      load_raw(SP{}, bx + 2 * (int)gridDim.x < nbox ? bx + 2 * gridDim.x : 0);
    else if constexpr (F32IN) {
      if (bx + 2 * (int)gridDim.x < nbox) load_raw(SP{}, bx + 2 * gridDim.x);
    }
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      const int m = (wm * 7 + i) * 16 + r16, py = m / TW, px = m - (m / TW) * TW;
      uint16_t* o = out + (((size_t)img * Ho + y0 + py) * Wo + x0 + px) * 64 + 32 * wn + 8 * g;
      u16x4 q[2];
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        f32x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = relu_on ? relu(acc[i][ct][j] + bv[ct][j]) : acc[i][ct][j] + bv[ct][j];
        q[ct] = T::pack4(v);
      }
      *(u16x8*)o = __builtin_shufflevector(q[0], q[1], 0, 1, 2, 3, 4, 5, 6, 7);
    }
    if constexpr (IN == 2) {
      // the next box's pieces (set P^1) landed: younger are the previous
      // box's 7 stores (none before the first box), this iteration's 3 PPL
      // pieces and this box's 7 stores
      if (it == 0)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * PPL + 7) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * PPL + 14) : "memory");
      if (more) store_cells(SQ{}, smem + WEL + ((it + 1) & 1) * HEL);
    } else if constexpr (F32IN) {
      // the next box's cells into the other buffer (its pieces were fetched
      // one box ago, before the previous box's stores, which stay in flight
      // with this box's)
      if (more) store_cells(SQ{}, smem + WEL + ((it + 1) & 1) * HEL);
    }
  };
  int it = 0;
  for (int bx = blockIdx.x; bx < nbox; bx += 2 * gridDim.x, it += 2) {
    box(S0{}, bx, it);
    if (bx + (int)gridDim.x < nbox) box(S1{}, bx + gridDim.x, it + 1);
  }
}

// ---- s3d_base0 (round 5): S3D's base.0 -- SepConv3d(3,
// 64, k 7, s 2, p 3) = the (1,7,7)/(1,2,2) spatial conv + BN + ReLU, then the
// (7,1,1)/(2,1,1) temporal conv + BN + ReLU (model.py:18,63-82) -- in ONE
// launch from the uint8 clip.  conv_s2d4 -> conv_tk2<2,7,2> wrote the
// 16-frame half-resolution map ([n][16][56][56][64], 6.4 MB per clip) and
// read it back: 9.9 GB of HBM per 1536-clip step between the two halves.
// Here a workgroup takes a unit = (clip, 2 x 8 output positions) through
// both halves with the 16-frame map of its 16 positions in LDS:
//  A. spatial: wave w computes frames 2w, 2w+1 -- conv_s2d4's 4x4 conv over
//     16-channel space-to-depth cells, its weight layout, k-step order and
//     transposed MFMAs (rows = channels), so the same sums -- from the
//     unit's cell image (16 frames x 2 pixel rows x 5 x 11 cells);
//  B. bias + ReLU -> 16-bit S image [chunk][frame][position][32 channels]
//     (conv_tk2's slice layout and swizzle);
//  C. temporal: wave (fp, h) computes output frames 2fp, 2fp+1 x channels
//     32h .. 32h+31 exactly as conv_tk2<2,7,2> does (chunk outer, tap inner,
//     zero-padded taps skipped), writes the next unit's cells behind those
//     MFMAs (its pixel pairs were loaded a unit earlier) and stores 16 bytes
//     per lane from registers.
// Bit-identical to the two launches (test_s3d_base0_fused_equals_two_launches).
// LDS: spatial weights 32 KB, temporal weights 56 KB, S image 32 KB, cell
// image 30 KB: one 512-thread workgroup per CU, persistent over units.
#ifdef B0_STAMPS
// tools/ubench/b0_ubench.hip: s_memtime of wave w of workgroup x in its k-th
// unit at: 0 unit start, 1 after barrier A, 2 spatial MFMAs done (+ the pixel
// loads issued), 3 = 2, 4 S frames written, 5 after barrier C, 6 temporal
// MFMAs + next cells done, 7 stored
__device__ unsigned long long b0_st[8][16][8][8];
#define B0_STAMP(k)                                                                               \
  do {                                                                                            \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    unsigned long long t_;                                                                        \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                    \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    const int k_ = (u - (int)blockIdx.x) / (int)gridDim.x;                                        \
    if (blockIdx.x < 8 && lane == 0 && k_ < 16) b0_st[blockIdx.x][k_][wave][(k)] = t_;            \
  } while (0)
#else
#define B0_STAMP(k) \
  do {              \
  } while (0)
#endif

template <class T>
__global__ __launch_bounds__(512, 1) void s3d_base0(const uint8_t* __restrict__ clip,
                                                    const uint16_t* __restrict__ wsp, const float* __restrict__ bsp,
                                                    int kps, const uint16_t* __restrict__ wtm,
                                                    const float* __restrict__ btm, int kpt,
                                                    uint16_t* __restrict__ out, int nunits, int H, int W, int pb,
                                                    int relu_s, int relu_t) {
  constexpr int T_IN = 16, T_OUT = 8, HO = 56, WO = 56;   // frames in / out, half-resolution map
  constexpr int BH = 2, BW = 8;                            // output box (16 positions = one MFMA column tile)
  // cell rows / cols of a box; row pitch RPX and pixel-row plane pitch PP
  // (16-byte slots) chosen by simulating the ds_read_b128 lane groups of the
  // spatial fragment reads over the 8 k-steps: 2-way at most (conflict-free
  // needs 176 slots per frame, 15 KB more than the LDS has left)
  constexpr int CH = BH + 3, CW = BW + 3, RPX = 11, PP = 56;
  constexpr int FSL = 2 * PP;                              // cell slots per frame (2 pixel rows per cell)
  constexpr int NPC = T_IN * 2 * CH * CW, PPL = (NPC + 511) / 512;  // cell pieces per unit / per thread
  constexpr int KD = 7, SD = 2, PD = 3, NF = SD + KD;      // temporal conv
  constexpr int WS_EL = 64 * 256, WT_EL = KD * 2 * 2048, S_EL = 2 * T_IN * 16 * 32, C_EL = T_IN * FSL * 8;
  __shared__ __attribute__((aligned(16))) uint16_t smem[WS_EL + WT_EL + S_EL + C_EL];
  __shared__ float bias_s[64], bias_t[64];
  uint16_t* const sws = smem;
  uint16_t* const swt = smem + WS_EL;
  uint16_t* const simg = swt + WT_EL;
  uint16_t* const cells = simg + S_EL;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  constexpr int BPR = WO / BW, BPC = (HO / BH) * BPR;      // boxes per row / per clip

  // weights: both in conv_s2d4's / conv_tk2's fragment layout
  // [k-step][ct][g][r16][8] (row i of tile ct = channel 32 (ct >> 1) + 8 (i >> 2) + 4 (ct & 1) + (i & 3))
  for (int c = tid; c < 64 * 32; c += 512) {
    const int n = c >> 5, k8 = c & 31;
    const int ct = 2 * (n >> 5) + ((n >> 2) & 1), i = 4 * ((n >> 3) & 3) + (n & 3);
    *(u16x8*)(sws + ((((k8 >> 2) * 4 + ct) * 4 + (k8 & 3)) * 16 + i) * 8) = *(const u16x8*)(wsp + (size_t)n * kps + k8 * 8);
  }
  for (int c = tid; c < 64 * KD * 2 * 4; c += 512) {
    const int n = c / (KD * 2 * 4), k8 = c - n * (KD * 2 * 4);
    const int ct = 2 * (n >> 5) + ((n >> 2) & 1), i = 4 * ((n >> 3) & 3) + (n & 3);
    *(u16x8*)(swt + ((((k8 >> 2) * 4 + ct) * 4 + (k8 & 3)) * 16 + i) * 8) = *(const u16x8*)(wtm + (size_t)n * kpt + k8 * 8);
  }
  if (tid < 64) {
    bias_s[tid] = bsp ? bsp[tid] : 0.f;
    bias_t[tid] = btm ? btm[tid] : 0.f;
  }

  // the pixel pairs of a unit's cell pieces: piece p = tid + 512 j ->
  // (frame f, pixel row pc of the cell, cell row hy, cell column hx); per
  // colour plane one 2-byte pixel pair (x, x+1) of pixel row y
  // Each pixel pair comes in the aligned dword that holds it (w % 4 == 0, x
  // even: never past the row), the pair's half recorded in rsh: no ALU touches
  // a loaded value before the cells are written (the compiler would wait for
  // the load there)
  // Two register sets, the unit loop unrolled by two so the set is a
  // constant: a unit's pixels are loaded two units ahead (one unit of HBM
  // latency cover instead of one spatial phase).
  uint32_t raw[2][PPL][3];
  unsigned rok[2] = {0u, 0u}, rsh[2] = {0u, 0u};
  // unit-independent piece geometry, once: hy | hx << 4 | pc << 8 | f << 9,
  // bit 13 = a piece at all (p < NPC); and its cell slot
  int pgeo[PPL], pslot[PPL];
#pragma unroll
  for (int j = 0; j < PPL; ++j) {
    const int p = tid + 512 * j;
    const int f = p / (2 * CH * CW), r1 = p - f * (2 * CH * CW);
    const int pc = r1 / (CH * CW), r2 = r1 - pc * (CH * CW), hy = r2 / CW, hx = r2 - hy * CW;
    pgeo[j] = p < NPC ? hy | (hx << 4) | (pc << 8) | (f << 9) | (1 << 13) : 0;
    pslot[j] = f * FSL + pc * PP + hy * RPX + hx;
  }
  auto load_raw = [&](auto setc, int u) {
    constexpr int SET = decltype(setc)::value;
    const int n = u / BPC, b = u - n * BPC;
    const int y0 = (b / BPR) * BH, x0 = (b - (b / BPR) * BPR) * BW;
    rok[SET] = 0u;
    rsh[SET] = 0u;
    const size_t cb = (size_t)(n * 3) * T_IN * H * W;
#pragma unroll
    for (int j = 0; j < PPL; ++j) {
      const int gq = pgeo[j];
      const int hy = gq & 15, hx = (gq >> 4) & 15, pc = (gq >> 8) & 1, f = (gq >> 9) & 15;
      const int Y = y0 + hy, X = x0 + hx, y = 2 * (Y - pb) + pc, x = 2 * (X - pb);
      const bool ok = (gq >> 13) && Y >= pb && X >= pb && y < H && x < W;
      const size_t off = ok ? cb + (size_t)(f * H + y) * W + x : 0;
      rok[SET] |= ok ? 1u << j : 0u;
      rsh[SET] |= ((unsigned)(off >> 1) & 1u) << j;
#pragma unroll
      for (int c = 0; c < 3; ++c)
        raw[SET][j][c] = *(const uint32_t*)(clip + (((size_t)c * T_IN * H * W + off) & ~(size_t)3));
    }
  };
  auto store_cells = [&](auto setc) {
    constexpr int SET = decltype(setc)::value;
#pragma unroll
    for (int j = 0; j < PPL; ++j) {
      if (pgeo[j] >> 13) {
        const bool ok = (rok[SET] >> j) & 1u;
        const unsigned sh = ((rsh[SET] >> j) & 1u) * 16u;
        u16x8 v;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const unsigned pr = raw[SET][j][c] >> sh;
          const float lo = ok ? (float)(pr & 0xff) : 0.f, hi = ok ? (float)((pr >> 8) & 0xff) : 0.f;
          v[c] = T::from_f32(lo);
          v[4 + c] = T::from_f32(hi);
        }
        v[3] = 0;
        v[7] = 0;
        *(u16x8*)(cells + pslot[j] * 8) = v;
      }
    }
  };

  // spatial fragment offsets: lane (g, r16) = position (py, px) of the box,
  // piece g & 1 of the cell at tap column offset g >> 1 (conv_s2d4)
  const int py = r16 >> 3, px = r16 & 7;
  const int cbo = (g & 1) * PP + py * RPX + px + (g >> 1);
  // S image: chunk c, frame d, position r16, channel piece q at ((c * 16 + d) * 16 + r16) * 32 + ((q ^ ((r16 >> 1) & 2)) << 3)
  const int rdoff = r16 * 32 + ((g ^ ((r16 >> 1) & 2)) << 3);
  const int fp = wave & 3, hh = wave >> 2;
  const int d0 = 2 * fp * SD - PD;
  const uint16_t* const wl = swt + (hh * 2 * 4 + g) * 128 + r16 * 8;

  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  const int G = gridDim.x;
  if ((int)blockIdx.x < nunits) {
    load_raw(S0{}, blockIdx.x);
    store_cells(S0{});
    load_raw(S1{}, (int)blockIdx.x + G < nunits ? blockIdx.x + G : 0);
  }
  // unit iteration of parity P: its cells came from set P; the next unit's
  // are written from set P^1 (loaded one unit ago), and the unit after next
  // loads into set P
  auto unit = [&](auto pc, int u) {
    constexpr int P = decltype(pc)::value;
    using SP = std::integral_constant<int, P>;
    using SQ = std::integral_constant<int, P ^ 1>;
    const int un = u + G;
    B0_STAMP(0);
    // A: cells of u written, the S image free.  The three phase barriers
    // order LDS only (no global data passes between waves): lgkmcnt +
    // s_barrier, not __syncthreads, whose fence would also wait for the
    // pixel loads just issued and the previous unit's output stores
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    B0_STAMP(1);
    // ---- A: spatial conv of frames 2w, 2w+1
    f32x4 sacc[2][4];
#pragma unroll
    for (int fi = 0; fi < 2; ++fi)
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) sacc[fi][ct] = (f32x4)0.f;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      u16x8 wf[4];
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) wf[ct] = *(const u16x8*)(sws + (((s * 4 + ct) * 4 + g) * 16 + r16) * 8);
      const int so = (s >> 1) * RPX + (s & 1) * 2;
#pragma unroll
      for (int fi = 0; fi < 2; ++fi) {
        const u16x8 pf = *(const u16x8*)(cells + ((2 * wave + fi) * FSL + cbo + so) * 8);
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) sacc[fi][ct] = T::mfma(wf[ct], pf, sacc[fi][ct]);
      }
    }
    // the pixels of the unit after next, issued behind the spatial MFMAs (past
    // the end: a dummy load of unit 0, so the compiler's wait counts are the
    // same on every path)
    load_raw(SP{}, u + 2 * G < nunits ? u + 2 * G : 0);
    B0_STAMP(2);
    // ---- B: this wave's frames of the S image (bias + ReLU, 16-bit), right
    // behind its own MFMAs: the previous unit's temporal reads of S ended
    // before barrier A, and the cells it no longer reads are rewritten only
    // after barrier C
    B0_STAMP(3);
#pragma unroll
    for (int fi = 0; fi < 2; ++fi) {
      const int d = 2 * wave + fi;
#pragma unroll
      for (int c = 0; c < 2; ++c) {  // chunk c = channels 32c .. 32c+31 = tiles 2c, 2c+1
        u16x4 q[2];
#pragma unroll
        for (int cc = 0; cc < 2; ++cc) {
          f32x4 v;
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const float x = sacc[fi][2 * c + cc][jj] + bias_s[32 * c + 8 * g + 4 * cc + jj];
            v[jj] = relu_s ? relu(x) : x;
          }
          q[cc] = T::pack4(v);
        }
        *(u16x8*)(simg + (c * T_IN + d) * 512 + rdoff) = __builtin_shufflevector(q[0], q[1], 0, 1, 2, 3, 4, 5, 6, 7);
      }
    }
    B0_STAMP(4);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // C: the S image is complete
    B0_STAMP(5);
    // ---- C: temporal conv, conv_tk2<2, 7, 2>'s arithmetic
    f32x4 acc[2][2];
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[j][0] = acc[j][1] = (f32x4)0.f;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const uint16_t* cur = simg + c * T_IN * 512 + rdoff;
      u16x8 pxf[NF], wf[KD][2];
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        const int d = d0 + f;
        pxf[f] = (unsigned)d < (unsigned)T_IN ? *(const u16x8*)(cur + d * 512) : (u16x8)0;
      }
#pragma unroll
      for (int t = 0; t < KD; ++t)
#pragma unroll
        for (int cc = 0; cc < 2; ++cc) wf[t][cc] = *(const u16x8*)(wl + (t * 2 + c) * 2048 + cc * 512);
#pragma unroll
      for (int t = 0; t < KD; ++t)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int f = j * SD + t;
          if ((unsigned)(d0 + f) < (unsigned)T_IN) {
#pragma unroll
            for (int cc = 0; cc < 2; ++cc) acc[j][cc] = T::mfma(wf[t][cc], pxf[f], acc[j][cc]);
          }
        }
    }
    // the next unit's cells (the cell image is free since barrier B), here
    // behind the temporal MFMAs rather than in phase B, where nothing hid
    // them: its pixels (set P^1, loaded one unit ago) have landed -- at most
    // this unit's PPL x 3 loads and the previous unit's 2 output stores are
    // younger (an intrinsic, not asm, so the compiler's own wait bookkeeping
    // sees it and adds no vmcnt(0) of its own)
    static_assert(3 * PPL + 2 < 16, "vmcnt immediate");
    __builtin_amdgcn_s_waitcnt(0x0F70 | (3 * PPL + 2));
    if (un < nunits) store_cells(SQ{});
    B0_STAMP(6);
    const int n = u / BPC, b = u - n * BPC;
    const int oy = (b / BPR) * BH + py, ox = (b - (b / BPR) * BPR) * BW + px;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      uint16_t* o = out + (((size_t)n * T_OUT + 2 * fp + j) * (HO * WO) + oy * WO + ox) * 64 + hh * 32 + 8 * g;
      u16x4 q2[2];
#pragma unroll
      for (int cc = 0; cc < 2; ++cc) {
        f32x4 v;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const float x = acc[j][cc][qq] + bias_t[hh * 32 + 8 * g + 4 * cc + qq];
          v[qq] = relu_t ? relu(x) : x;
        }
        q2[cc] = T::pack4(v);
      }
      *(u16x8*)o = __builtin_shufflevector(q2[0], q2[1], 0, 1, 2, 3, 4, 5, 6, 7);
    }
    B0_STAMP(7);
  };
  for (int u = blockIdx.x; u < nunits; u += 2 * G) {
    unit(S0{}, u);
    if (u + G < nunits) unit(S1{}, u + G);
  }
}

// ---- conv_s2d4_mp: conv_s2d4 (+ bias + ReLU) with the MaxPool2d(3, 2, 1)
// that follows it in ResNet-50 (ResVitKan.py:187's torchvision resnet50:
// conv1 -> bn1 -> relu -> maxpool) fused in, so the 112^2 conv output never
// goes through HBM (4x the pooled bytes written, then read back by
// fac_pool_nd).  A box is 4 x 14 pooled outputs = conv rows 2py0-1 .. 2py0+7
// and columns 2px0-1 .. 2px0+27.  A workgroup walks whole column strips of an
// image top to bottom, so conv row 2py0-1 is the previous box's last row,
// kept in registers (at the top edge it is pool padding): each box computes
// the 8 rows 2py0 .. 2py0+7 only.  MFMA tile (r, h) = conv row r of those,
// columns 16h .. 16h+15 (the three past column 28 recompute column 28 and are
// dropped; 1.14x the MFMAs of the conv alone): wave (wm = h, wn) holds its 8
// channels of one column for all rows, so the vertical 3-max of the pool is
// fmaxf in registers; the vertically pooled rows (16-bit: a max of rounded
// values is the rounded max, rounding being monotone) go through a 4 x
// 32-column LDS stage for the horizontal 3-max and leave as 16-byte stores.
// Pool padding (conv row / column -1 at the image's top / left edge) counts
// as 0, which never wins over a ReLU output, i.e. is ignored as MaxPool2d
// ignores it -- hence relu is required.
template <class T>
__global__ __launch_bounds__(256, 2) void conv_s2d4_mp(const uint16_t* __restrict__ in, const uint16_t* __restrict__ w,
                                                       const float* __restrict__ bias, uint16_t* __restrict__ out,
                                                       int nstrip, int Hc, int Wc, int Hp, int Wp, int kp) {
  constexpr int PH = 4, PW = 14;                     // pooled outputs per box
  constexpr int CR = 2 * PH, CC = 2 * PW + 1;        // conv rows computed / columns needed per box (8 x 29)
  constexpr int HH = CR + 3, RPX = 32;               // halo rows, row pitch (cells: columns 0 .. CC + 2)
  constexpr int HSL = 2 * HH * RPX;                  // 16-byte halo slots
  constexpr int HPW = (HSL + 255) / 256;             // glds per wave
  constexpr int WEL = 64 * 256;                      // weight elements
  constexpr int HEL = HPW * 256 * 8;                 // halo buffer elements
  constexpr int VP = 64 + 8;                         // stage pitch per column (elements)
  constexpr int VEL = PH * 32 * VP;                  // vertically pooled stage [py][column][64]
  static_assert(CC - 1 + 3 < RPX, "halo geometry");
  __shared__ __attribute__((aligned(16))) uint16_t smem[WEL + 2 * HEL + VEL];
  uint16_t* const sw = smem;
  uint16_t* const vst = smem + WEL + 2 * HEL;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int wm = wave >> 1, wn = wave & 1;  // wm: column half of the box

  // weights as conv_s2d4 (channel-permuted rows: lane group g ends with
  // channels 32wn + 8g .. +7 of its column)
  for (int c = tid; c < 64 * 32; c += 256) {
    const int n = c >> 5, k8 = c & 31;
    const int ct = 2 * (n >> 5) + ((n >> 2) & 1), i = 4 * ((n >> 3) & 3) + (n & 3);
    *(u16x8*)(sw + ((((k8 >> 2) * 4 + ct) * 4 + (k8 & 3)) * 16 + i) * 8) =
        *(const u16x8*)(w + (size_t)n * kp + k8 * 8);
  }
  float bv[2][4];
#pragma unroll
  for (int ct = 0; ct < 2; ++ct)
#pragma unroll
    for (int j = 0; j < 4; ++j) bv[ct][j] = bias ? bias[32 * wn + 8 * g + 4 * ct + j] : 0.f;
  const int col = 16 * wm + r16, colc = col < CC ? col : CC - 1;
  int bo[CR];  // halo slot of tile r at tap (0, g/2)
#pragma unroll
  for (int r = 0; r < CR; ++r) bo[r] = ((g & 1) * HH + r) * RPX + colc + (g >> 1);
  const int bpr = Wp / PW, nby = Hp / PH;
  // k-th box of this workgroup: strip blockIdx.x + (k / nby) * gridDim.x, box row k % nby
  auto box_of = [&](int k, int& img, int& py0, int& px0) {
    const int s = blockIdx.x + (k / nby) * (int)gridDim.x;
    img = s / bpr;
    px0 = (s - img * bpr) * PW;
    py0 = (k - (k / nby) * nby) * PH;
    return s < nstrip;
  };
  auto issue = [&](int k, uint16_t* halo) {
    int img, py0, px0;
    box_of(k, img, py0, px0);
    const int cy0 = 2 * py0, cx0 = 2 * px0 - 1;  // cell (= conv) row of box row 0, column of column 0
#pragma unroll
    for (int i = 0; i < HPW; ++i) {
      const int sl = (i * 4 + wave) * 64 + lane;
      const int pc = sl / (HH * RPX), rem = sl - pc * (HH * RPX), hy = rem / RPX, hx = rem - (rem / RPX) * RPX;
      const int y = cy0 + hy, x = cx0 + hx;
      const uint16_t* src = g_zero16;
      if (pc < 2 && (unsigned)y < (unsigned)Hc && (unsigned)x < (unsigned)Wc)
        src = in + (((size_t)img * Hc + y) * Wc + x) * 16 + pc * 8;
      glds16(src, halo + (i * 4 + wave) * 64 * 8);
    }
  };
  // stores per thread of a box's horizontal pass: waves whose threads all
  // have a second item issue 2, the rest 1 (counted in the halo wait below)
  constexpr int NIT = PH * PW * 8;
  static_assert(NIT > 256 && NIT <= 512 && (NIT - 256) % 64 == 0, "two store rounds, wave-uniform");
  const bool two = tid + 256 < NIT;
  float carry[2][4];  // the previous box's last conv row (ReLU'd) of this lane's column
  __syncthreads();  // weights in
  {
    int i0, y0, x0;
    if (box_of(0, i0, y0, x0)) issue(0, smem + WEL);
  }
  int img, py0, px0;
  for (int k = 0; box_of(k, img, py0, px0); ++k) {
    uint16_t* const halo = smem + WEL + (k & 1) * HEL;
    int i1, y1, x1;
    const bool more = box_of(k + 1, i1, y1, x1);
    // every wave is done with the other halo buffer and with the stage
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (more) issue(k + 1, smem + WEL + ((k + 1) & 1) * HEL);
    // this box's halo landed; younger: the next box's pieces (if any) and,
    // after the first box, the previous box's 1 or 2 stores
    if (k == 0) {
      if (more) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(HPW) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    } else if (two) {
      if (more) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(HPW + 2) : "memory");
      else asm volatile("s_waitcnt vmcnt(2)\n\ts_barrier" ::: "memory");
    } else {
      if (more) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(HPW + 1) : "memory");
      else asm volatile("s_waitcnt vmcnt(1)\n\ts_barrier" ::: "memory");
    }
    f32x4 acc[CR][2];
#pragma unroll
    for (int r = 0; r < CR; ++r) acc[r][0] = acc[r][1] = (f32x4)0.f;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      u16x8 wf[2];
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) wf[ct] = *(const u16x8*)(sw + (((s * 4 + 2 * wn + ct) * 4 + g) * 16 + r16) * 8);
      const int so = (s >> 1) * RPX + (s & 1) * 2;
#pragma unroll
      for (int r = 0; r < CR; ++r) {
        const u16x8 pf = *(const u16x8*)(halo + (bo[r] + so) * 8);
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) acc[r][ct] = T::mfma(wf[ct], pf, acc[r][ct]);
      }
    }
    // vertical 3-max over conv rows 2py0-1+2py .. +2: the carried row first
    if (py0 == 0) {
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int j = 0; j < 4; ++j) carry[ct][j] = 0.f;  // pool padding
    }
#pragma unroll
    for (int py = 0; py < PH; ++py) {
      u16x4 q[2];
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        f32x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float b = relu(acc[2 * py][ct][j] + bv[ct][j]);
          const float c = relu(acc[2 * py + 1][ct][j] + bv[ct][j]);
          v[j] = fmaxf(fmaxf(carry[ct][j], b), c);
          carry[ct][j] = c;
        }
        q[ct] = T::pack4(v);
      }
      *(u16x8*)(vst + (py * 32 + col) * VP + 32 * wn + 8 * g) = __builtin_shufflevector(q[0], q[1], 0, 1, 2, 3, 4, 5, 6, 7);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    // horizontal 3-max (column 0 is conv column -1 at the left edge) + store
    const bool left = px0 == 0;
    for (int it = tid; it < NIT; it += 256) {
      const int q8 = it & 7, pj = it >> 3, py = pj / PW, j = pj - py * PW;
      const uint16_t* v = vst + (py * 32 + 2 * j) * VP + q8 * 8;
      const u16x8 a = *(const u16x8*)v, b = *(const u16x8*)(v + VP), c = *(const u16x8*)(v + 2 * VP);
      const bool skip_a = left && j == 0;
      f32x4 lo, hi;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        lo[e] = fmaxf(fmaxf(skip_a ? 0.f : T::to_f32(a[e]), T::to_f32(b[e])), T::to_f32(c[e]));
        hi[e] = fmaxf(fmaxf(skip_a ? 0.f : T::to_f32(a[e + 4]), T::to_f32(b[e + 4])), T::to_f32(c[e + 4]));
      }
      const u16x4 l4 = T::pack4(lo), h4 = T::pack4(hi);
      *(u16x8*)(out + (((size_t)img * Hp + py0 + py) * Wp + px0 + j) * 64 + q8 * 8) =
          __builtin_shufflevector(l4, h4, 0, 1, 2, 3, 4, 5, 6, 7);
    }
  }
}

// ---- bneck_pw2: a ResNet-50 layer1 bottleneck's conv3 (1x1, 64 -> 256,
// + bn3 + ReLU + identity residual + ReLU, ResVitKan.py:146-152) and the
// NEXT block's conv1 (1x1, 256 -> N1 + bn1 + ReLU) in one persistent launch:
// a workgroup computes all 256 conv3 channels of a 64-row tile, stores them
// (the next block's residual) and keeps them in LDS as the next conv1's K,
// so the 256-channel map is not read back from HBM by a second launch.
// Both GEMMs run transposed (rows = channels) with conv_pw's channel
// permutation, so every lane stores 16 bytes (8 channels of one position)
// straight from registers; the epilogue arithmetic is conv_pw's, and the
// 16-bit conv3 outputs are exactly what the separate conv1 would read.
// The next tile's A rows and residual block are loaded into registers while
// the current tile computes.
// Rows past M (a partial last tile) load row M-1 and store into g_sink, so
// every load and store is unconditional: the compiler's wait for the next
// tile's registers then counts this tile's stores instead of draining them.

template <class T, int N1>
__global__ __launch_bounds__(512, 1) void bneck_pw2(const uint16_t* __restrict__ a, const uint16_t* __restrict__ w3,
                                                    const float* __restrict__ b3, const uint16_t* __restrict__ res,
                                                    const uint16_t* __restrict__ w1, const float* __restrict__ b1,
                                                    uint16_t* __restrict__ xo, uint16_t* __restrict__ ho, int M,
                                                    int kp3, int kp1, int ldr, int r_off) {
  constexpr int BM = 64, K3 = 64, C3 = 256, PPW = N1 / 64;  // rows per tile, conv3 K / N, conv1 channel pairs per wave
  constexpr int W3EL = C3 * K3, W1EL = N1 * C3, AEL = BM * K3, XEL = BM * C3;
  static_assert(N1 == 64 || N1 == 128, "conv1 width");
  __shared__ __attribute__((aligned(16))) uint16_t smem[W3EL + W1EL + AEL + XEL];
  uint16_t* const s3 = smem;
  uint16_t* const s1 = smem + W3EL;
  uint16_t* const sa = s1 + W1EL;   // A tile: rows of 8 pieces, piece p at p ^ (row & 7)
  uint16_t* const sx = sa + AEL;    // conv3 tile: rows of 32 pieces, piece q at q ^ (row & 15)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;

  // W3 fragments [w][s][ct][g][r16][8]: row i of (wave w, tile ct) = channel
  // 32w + 8(i>>2) + 4ct + (i&3); W1 fragments [P][s][h][g][r16][8] likewise
  for (int c = tid; c < C3 * 8; c += 512) {
    const int n = c >> 3, k8 = c & 7, nn = n & 31;
    const int ct = (nn >> 2) & 1, i = 4 * ((nn >> 3) & 3) + (nn & 3);
    *(u16x8*)(s3 + (((((n >> 5) * 2 + (k8 >> 2)) * 2 + ct) * 4 + (k8 & 3)) * 16 + i) * 8) =
        *(const u16x8*)(w3 + (size_t)n * kp3 + k8 * 8);
  }
  for (int c = tid; c < N1 * 32; c += 512) {
    const int n = c >> 5, k8 = c & 31, nn = n & 31;
    const int h = (nn >> 2) & 1, i = 4 * ((nn >> 3) & 3) + (nn & 3);
    *(u16x8*)(s1 + (((((n >> 5) * 8 + (k8 >> 2)) * 2 + h) * 4 + (k8 & 3)) * 16 + i) * 8) =
        *(const u16x8*)(w1 + (size_t)n * kp1 + k8 * 8);
  }
  float bv3[2][4], bv1[PPW][2][4];
  const int pt2 = wave >> 1;  // conv1: this wave's position tile, channel pairs (wave & 1) * PPW + pp
#pragma unroll
  for (int ct = 0; ct < 2; ++ct)
#pragma unroll
    for (int j = 0; j < 4; ++j) bv3[ct][j] = b3[32 * wave + 8 * g + 4 * ct + j];
#pragma unroll
  for (int pp = 0; pp < PPW; ++pp)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < 4; ++j) bv1[pp][h][j] = b1[32 * ((wave & 1) * PPW + pp) + 8 * g + 4 * h + j];

  const int ntiles = (M + BM - 1) / BM;
  const int arow = tid >> 3, apc = tid & 7;  // this thread's A piece of a tile
  u16x8 an = (u16x8)0, rn[4], rc[4];
  auto load = [&](int t) {
    const int m0 = t * BM;
    an = *(const u16x8*)(a + (size_t)min(m0 + arow, M - 1) * K3 + apc * 8);
#pragma unroll
    for (int pt = 0; pt < 4; ++pt) {
      const int m = min(m0 + pt * 16 + r16, M - 1);
      rn[pt] = *(const u16x8*)(res + (size_t)m * ldr + r_off + 32 * wave + 8 * g);
    }
  };
  int t = blockIdx.x;
  if (t < ntiles) load(t);
  __syncthreads();  // weights in
  for (; t < ntiles; t += gridDim.x) {
    const int m0 = t * BM;
    // A tile into LDS (every wave finished the previous tile's conv3 reads of
    // it before the previous tile's second barrier), next tile's loads out
    *(u16x8*)(sa + (arow * 8 + (apc ^ (arow & 7))) * 8) = an;
#pragma unroll
    for (int pt = 0; pt < 4; ++pt) rc[pt] = rn[pt];
    if (t + (int)gridDim.x < ntiles) load(t + gridDim.x);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    // conv3: channels 32 wave + (2 tiles) x the tile's 64 positions (4 tiles)
    f32x4 acc[4][2];
#pragma unroll
    for (int pt = 0; pt < 4; ++pt) acc[pt][0] = acc[pt][1] = (f32x4)0.f;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      u16x8 wf[2];
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) wf[ct] = *(const u16x8*)(s3 + ((((wave * 2 + s) * 2 + ct) * 4 + g) * 16 + r16) * 8);
#pragma unroll
      for (int pt = 0; pt < 4; ++pt) {
        const int r = pt * 16 + r16;
        const u16x8 pf = *(const u16x8*)(sa + (r * 8 + ((s * 4 + g) ^ (r & 7))) * 8);
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) acc[pt][ct] = T::mfma(wf[ct], pf, acc[pt][ct]);
      }
    }
    // relu(conv3 + b3) + residual, relu -> 16-bit: to HBM and to the LDS tile
#pragma unroll
    for (int pt = 0; pt < 4; ++pt) {
      const int r = pt * 16 + r16, m = m0 + r;
      u16x4 q[2];
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        f32x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = relu(relu(acc[pt][ct][j] + bv3[ct][j]) + T::to_f32(rc[pt][4 * ct + j]));
        q[ct] = T::pack4(v);
      }
      const u16x8 o = __builtin_shufflevector(q[0], q[1], 0, 1, 2, 3, 4, 5, 6, 7);
      *(u16x8*)(sx + (r * 32 + ((4 * wave + g) ^ r16)) * 8) = o;
      *(u16x8*)(m < M ? xo + (size_t)m * C3 + 32 * wave + 8 * g : g_sink + lane * 8) = o;
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    // conv1: channel pairs (wave & 1) * PPW + pp, position tile pt2, K = 256
    f32x4 acc1[PPW][2];
#pragma unroll
    for (int pp = 0; pp < PPW; ++pp) acc1[pp][0] = acc1[pp][1] = (f32x4)0.f;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int r = pt2 * 16 + r16;
      const u16x8 pf = *(const u16x8*)(sx + (r * 32 + ((s * 4 + g) ^ r16)) * 8);
#pragma unroll
      for (int pp = 0; pp < PPW; ++pp) {
        const int P = (wave & 1) * PPW + pp;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const u16x8 wf = *(const u16x8*)(s1 + ((((P * 8 + s) * 2 + h) * 4 + g) * 16 + r16) * 8);
          acc1[pp][h] = T::mfma(wf, pf, acc1[pp][h]);
        }
      }
    }
    const int m = m0 + pt2 * 16 + r16;
    {
#pragma unroll
      for (int pp = 0; pp < PPW; ++pp) {
        u16x4 q[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          f32x4 v;
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = relu(acc1[pp][h][j] + bv1[pp][h][j]);
          q[h] = T::pack4(v);
        }
        *(u16x8*)(m < M ? ho + (size_t)m * N1 + 32 * ((wave & 1) * PPW + pp) + 8 * g : g_sink + lane * 8) =
            __builtin_shufflevector(q[0], q[1], 0, 1, 2, 3, 4, 5, 6, 7);
      }
    }
  }
}

// ---- bneck_pw2_l2: bneck_pw2 for ResNet-50 layer2 (conv3 1x1 128 -> 512 +
// bn3 + ReLU + identity residual + ReLU, next conv1 1x1 512 -> 128 + bn1 +
// ReLU).  The two weights (128 KB each) cannot both stay in LDS beside the
// tiles, so each wave keeps its 64 conv3 output channels' weights in VGPRs
// (16 fragments) and only the conv1 weight lives in LDS; tiles are 16 rows.
// conv3 runs transposed with conv_pw's channel permutation (16-byte stores),
// conv1 transposed over plain 16-channel tiles, one per wave (8-byte stores).
template <class T>
__global__ __launch_bounds__(512, 1) void bneck_pw2_l2(const uint16_t* __restrict__ a, const uint16_t* __restrict__ w3,
                                                       const float* __restrict__ b3, const uint16_t* __restrict__ res,
                                                       const uint16_t* __restrict__ w1, const float* __restrict__ b1,
                                                       uint16_t* __restrict__ xo, uint16_t* __restrict__ ho, int M,
                                                       int kp3, int kp1, int ldr, int r_off) {
  constexpr int BM = 16, K3 = 128, C3 = 512, N1 = 128;
  constexpr int W1EL = N1 * C3, AEL = BM * K3, XEL = BM * C3;
  __shared__ __attribute__((aligned(16))) uint16_t smem[W1EL + AEL + XEL];
  uint16_t* const s1 = smem;
  uint16_t* const sa = s1 + W1EL;  // A tile: rows of 16 pieces, piece p at p ^ row
  uint16_t* const sx = sa + AEL;   // conv3 tile: rows of 64 pieces, piece q at q ^ row
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;

  // conv3 weights of this wave's channels 64 wave + [0, 64) in registers:
  // fragment (k-step s, tile ct), row i = channel 64 wave + 32 (ct >> 1) +
  // 8 (i >> 2) + 4 (ct & 1) + (i & 3); lane (g, r16) holds row r16, k 32 s + 8 g
  u16x8 wr[4][4];
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      const int n = 64 * wave + 32 * (ct >> 1) + 8 * (r16 >> 2) + 4 * (ct & 1) + (r16 & 3);
      wr[s][ct] = *(const u16x8*)(w3 + (size_t)n * kp3 + 32 * s + 8 * g);
    }
  // conv1 weights in LDS, fragments [tile t][s][g][r16][8] (row i of tile t = channel 16 t + i)
  for (int c = tid; c < N1 * (C3 / 8); c += 512) {
    const int n = c >> 6, k8 = c & 63;
    *(u16x8*)(s1 + ((((n >> 4) * 16 + (k8 >> 2)) * 4 + (k8 & 3)) * 16 + (n & 15)) * 8) =
        *(const u16x8*)(w1 + (size_t)n * kp1 + k8 * 8);
  }
  float bv3[4][4], bv1[4];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int j = 0; j < 4; ++j) bv3[ct][j] = b3[64 * wave + 32 * (ct >> 1) + 8 * g + 4 * (ct & 1) + j];
#pragma unroll
  for (int j = 0; j < 4; ++j) bv1[j] = b1[16 * wave + 4 * g + j];

  const int ntiles = (M + BM - 1) / BM;
  const int arow = tid >> 5, ah = tid & 31;  // this thread's 8-byte half-piece of a tile's A rows
  u16x4 an;
  u16x8 rn[2], rc[2];
  auto load = [&](int t) {
    const int m0 = t * BM;
    an = *(const u16x4*)(a + (size_t)min(m0 + arow, M - 1) * K3 + ah * 4);
    const int m = min(m0 + r16, M - 1);
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) rn[pp] = *(const u16x8*)(res + (size_t)m * ldr + r_off + 64 * wave + 32 * pp + 8 * g);
  };
  int t = blockIdx.x;
  if (t < ntiles) load(t);
  __syncthreads();  // conv1 weights in
  for (; t < ntiles; t += gridDim.x) {
    const int m0 = t * BM;
    *(u16x4*)(sa + (arow * 16 + ((ah >> 1) ^ arow)) * 8 + (ah & 1) * 4) = an;
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) rc[pp] = rn[pp];
    if (t + (int)gridDim.x < ntiles) load(t + gridDim.x);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    // conv3: this wave's 64 channels x the tile's 16 positions
    f32x4 acc[4];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) acc[ct] = (f32x4)0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const u16x8 pf = *(const u16x8*)(sa + (r16 * 16 + ((s * 4 + g) ^ r16)) * 8);
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) acc[ct] = T::mfma(wr[s][ct], pf, acc[ct]);
    }
    const int m = m0 + r16;
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {
      u16x4 q[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        f32x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          v[j] = relu(relu(acc[2 * pp + h][j] + bv3[2 * pp + h][j]) + T::to_f32(rc[pp][4 * h + j]));
        q[h] = T::pack4(v);
      }
      const u16x8 o = __builtin_shufflevector(q[0], q[1], 0, 1, 2, 3, 4, 5, 6, 7);
      *(u16x8*)(sx + (r16 * 64 + ((8 * wave + 4 * pp + g) ^ r16)) * 8) = o;
      *(u16x8*)(m < M ? xo + (size_t)m * C3 + 64 * wave + 32 * pp + 8 * g : g_sink + lane * 8) = o;
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    // conv1: channels 16 wave .. +15 x the 16 positions, K = 512
    f32x4 acc1 = (f32x4)0.f;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const u16x8 pf = *(const u16x8*)(sx + (r16 * 64 + ((s * 4 + g) ^ r16)) * 8);
      const u16x8 wf = *(const u16x8*)(s1 + (((wave * 16 + s) * 4 + g) * 16 + r16) * 8);
      acc1 = T::mfma(wf, pf, acc1);
    }
    f32x4 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = relu(acc1[j] + bv1[j]);
    *(u16x4*)(m < M ? ho + (size_t)m * N1 + 16 * wave + 4 * g : g_sink + lane * 8) = T::pack4(v);
  }
}

// ---- conv_pw: stride-1 1x1 convs with K = Cin in {64, 128, 256} — ResNet-50's
// bottleneck expansions (conv3 64 -> 256 / 128 -> 512 + residual + ReLU,
// ResVitKan.py:187's torchvision resnet50 layer1/layer2), their downsample
// 1x1s, layer1's 64 -> 64 reductions, the K = 256 reductions and layer3's
// 256 -> 1024 expansions.  Through the generic implicit GEMM these are
// HBM-bound with one to four K steps per tile, so every
// workgroup is a serial load -> MFMA -> LDS-staged store chain and the chip
// holds too few bytes in flight.  Here a persistent workgroup keeps its
// 64-column weight block in LDS and walks row tiles of 64 * RT positions:
// the next tile's rows stream into the other LDS buffer (glds) while this
// tile computes and stores, and so does its residual block (RES; read into
// registers before the barrier that frees the buffer).  MFMAs transposed (rows = channels) as in conv_s2d4: each lane ends
// with 4 channels of one position and stores 8 bytes from registers.
// A rows (K / 8 16-byte pieces) keep piece p at p ^ (row & 7).
template <class T, int KC, int RT, bool RES>
__global__ __launch_bounds__(256, 3) void conv_pw(const uint16_t* __restrict__ in, const uint16_t* __restrict__ w,
                                                  const float* __restrict__ bias, const uint16_t* __restrict__ res,
                                                  uint16_t* __restrict__ out, int M, int kp, int ldo, int c_off,
                                                  int ldr, int r_off, int flags) {
  constexpr int K = KC * 32, PPR = K / 8, BM = 64 * RT;
  constexpr int WEL = 64 * K, AEL = BM * K;
  constexpr int PER = BM * PPR / 256;  // glds per lane per tile
  constexpr int REL = RES ? BM * 64 : 0, RPER = RES ? BM / 32 : 0;  // residual tile elements, glds
  static_assert(PER * 256 == BM * PPR, "tile pieces");
  __shared__ __attribute__((aligned(16))) uint16_t smem[WEL + 2 * AEL + 2 * REL];
  uint16_t* const sw = smem;
  uint16_t* const sa = smem + WEL;
  uint16_t* const sr = sa + 2 * AEL;  // residual tiles, rows of 8 pieces, piece p at p ^ (row & 7)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int n0 = blockIdx.y * 64;
  const bool relu_on = flags & FAC_CONV_RELU, relu2 = flags & FAC_CONV_RELU2;

  // weights [s][ct][g][r16][8]: one contiguous 1 KB fragment per (k-step,
  // channel tile).  Row i of channel tile ct computes channel pw_ch(ct, i) =
  // 32 (ct >> 1) + 8 (i >> 2) + 4 (ct & 1) + (i & 3), so lane group g ends
  // with channels 8g .. 8g+7 (tiles 0, 1) and 32+8g .. 32+8g+7 (tiles 2, 3)
  // of its position: two 16-byte stores, and each store instruction writes
  // 64 contiguous bytes per position (4-channel, 8-byte lanes gave 32-byte
  // segments)
  for (int c = tid; c < 64 * PPR; c += 256) {
    const int n = c / PPR, k8 = c - n * PPR;
    const int ct = 2 * (n >> 5) + ((n >> 2) & 1), i = 4 * ((n >> 3) & 3) + (n & 3);
    *(u16x8*)(sw + ((((k8 >> 2) * 4 + ct) * 4 + (k8 & 3)) * 16 + i) * 8) =
        *(const u16x8*)(w + (size_t)(n0 + n) * kp + k8 * 8);
  }
  float bv[4][4];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int j = 0; j < 4; ++j) bv[ct][j] = bias ? bias[n0 + 32 * (ct >> 1) + 8 * g + 4 * (ct & 1) + j] : 0.f;
  // this lane's glds slots: row and (logical) piece, fixed across tiles
  int arow[PER], aoff[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int q = (i * 4 + wave) * 64 + lane, r = q / PPR, pp = q - r * PPR;
    arow[i] = r;
    aoff[i] = (pp ^ (r & 7)) * 8;
  }
  // a tile's A rows, then (RES) its 64-column residual block, into buffer buf
  auto issue = [&](int tile, int buf) {
    const int m0 = tile * BM;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int m = m0 + arow[i];
      glds16(m < M ? in + (size_t)m * K + aoff[i] : g_zero16, sa + buf * AEL + (i * 4 + wave) * 64 * 8);
    }
#pragma unroll
    for (int i = 0; i < RPER; ++i) {
      const int q = (i * 4 + wave) * 64 + lane, r = q >> 3, m = m0 + r;
      glds16(m < M ? res + (size_t)m * ldr + r_off + n0 + (((q & 7) ^ (r & 7)) << 3) : g_zero16,
             sr + buf * REL + (i * 4 + wave) * 64 * 8);
    }
  };
  __syncthreads();  // weights in
  const int ntiles = (M + BM - 1) / BM;
  int t = blockIdx.x;
  if (t < ntiles) issue(t, 0);
  for (int it = 0; t < ntiles; ++it, t += gridDim.x) {
    const int buf = it & 1;
    const int mrow = t * BM + wave * RT * 16 + r16;  // this lane's position in row tile 0
    if (t + (int)gridDim.x < ntiles) {
      issue(t + gridDim.x, buf ^ 1);  // its buffer's readers passed the previous tile's barrier
      // this tile's pieces landed.  Younger than them: the next tile's pieces
      // and (after the first tile) the previous tile's 2*RT output stores --
      // vmcnt counts loads and stores in issue order, so a count of only the
      // next tile's pieces also waited for those stores' HBM round trip.  The
      // previous tile is never the partial last one (that is a workgroup's
      // final tile), so every lane issued all of its stores.
      if (it == 0) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(PER + RPER) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(PER + RPER + 2 * RT) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    }
    // residual vectors to registers before the barrier that frees the buffer:
    // channels 8g .. 8g+7 (piece g) and 32+8g .. (piece 4+g) of the lane's position
    u16x8 rv[RT][2];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int r = (wave * RT + rt) * 16 + r16;
        rv[rt][hh] = RES ? *(const u16x8*)(sr + buf * REL + r * 64 + (((hh * 4 + g) ^ (r & 7)) << 3)) : (u16x8)0;
      }
    const uint16_t* a = sa + buf * AEL;
    f32x4 acc[RT][4];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) acc[rt][ct] = (f32x4)0.f;
#pragma unroll
    for (int s = 0; s < KC; ++s) {
      u16x8 wf[4];
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) wf[ct] = *(const u16x8*)(sw + (((s * 4 + ct) * 4 + g) * 16 + r16) * 8);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const int r = (wave * RT + rt) * 16 + r16;
        const u16x8 pf = *(const u16x8*)(a + (r * PPR + ((s * 4 + g) ^ (r & 7))) * 8);
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) acc[rt][ct] = T::mfma(wf[ct], pf, acc[rt][ct]);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // buffers free for the tile after next
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const int m = mrow + rt * 16;
      if (m >= M) continue;
      uint16_t* o = out + (size_t)m * ldo + c_off + n0 + 8 * g;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        u16x4 q[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int ct = 2 * hh + e;
          f32x4 v;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float x = acc[rt][ct][j] + bv[ct][j];
            if (relu_on) x = relu(x);
            if constexpr (RES) x += T::to_f32(rv[rt][hh][4 * e + j]);
            if (relu2) x = relu(x);
            v[j] = x;
          }
          q[e] = T::pack4(v);
        }
        *(u16x8*)(o + hh * 32) = __builtin_shufflevector(q[0], q[1], 0, 1, 2, 3, 4, 5, 6, 7);
      }
    }
  }
}

// ---- pw_res (round 6): ResNet-50's bottleneck conv3 with its identity --
// relu(relu(conv1x1(x) + b3) + x_in) (ResVitKan.py:146-152, torchvision's
// Bottleneck) -- for layer2's 128 -> 512 and layer3's 256 -> 1024.  These
// move 2.25 KB / 4.5 KB of HBM per position (input row, residual and output
// rows) for 0.13 / 0.5 MFLOP: HBM-bound, but convnd_pt ran them at 3.9 /
// 3.4 TB/s against the 5.9 TB/s torch's own add of the same residual and
// output streams reaches on the same box (tools/res_ceiling.py): its K steps
// stream 256-wide weight slices through LDS for a 2-4-step K.  Here one
// 512-thread workgroup per CU keeps its BN x K weight block resident in LDS
// (64 KB, loaded once) and walks BM-row tiles of one column block; the next
// tile's input rows AND its BM x BN residual block go global -> LDS
// (global_load_lds, double-buffered) while this tile computes, so each tile
// waits only for bytes issued a whole tile earlier.  MFMAs transposed (rows =
// channels, conv_pw's channel order): a lane ends with 8 consecutive
// channels of a position, read its residual with one ds_read_b128 and stores
// 16 bytes.  LDS rows keep 16-byte piece p at p ^ (row & 15) (conflict-free
// for the fragment and residual reads: 16 rows of one piece column hit 16
// distinct bank groups).  LDS: weights 64 KB + 2 x input tile + 2 x residual
// tile = 160 KB for both instances.
// DUAL (layer1's first block, K = 64): no identity; a second 1x1 GEMM -- the
// stride-1 downsample conv + bn over the block input x2 -- accumulates onto
// relu(acc + b3) + b_ds (the reference's order, ResVitKan.py:146-152), both
// weight blocks resident (2 x 32 KB), both inputs' tiles streamed (replaces
// convnd_pt DUAL there, which ran this 7.4 GB / 0.63 TFLOP launch at 3.5 TB/s).
// PLAIN (MODE 2: S3D's merged Inception heads at 14 x 14, K = 192 / 256): no
// identity, relu?(acc + b) into up to three column segments (out / out1 /
// out2, fac_conv_nd_split); channels past cout (the zero-padded block tail)
// store to the sink.
template <class T, int KC, int BN, int BM, int MODE = 0>
__global__ __launch_bounds__(512, 1) void pw_res(const uint16_t* __restrict__ in, const uint16_t* __restrict__ w,
                                                 const float* __restrict__ bias, const uint16_t* __restrict__ res,
                                                 uint16_t* __restrict__ out, int M, int kp, int ldo, int c_off, int ldr,
                                                 int r_off, int ny, int relu1, int relu2,
                                                 const uint16_t* __restrict__ in2, const uint16_t* __restrict__ w2,
                                                 const float* __restrict__ bias2, int cout, uint16_t* __restrict__ out1,
                                                 int ldo1, int split1, uint16_t* __restrict__ out2, int ldo2, int split2) {
  constexpr bool DUAL = MODE == 1, RESM = MODE == 0;
  constexpr int K = KC * 32, PPR = K / 8, RPR = BN / 8;  // 16-byte pieces per input / residual row
  constexpr int NW = 8, WN = BN / 64, WM = NW / WN, WPOS = BM / WM, PT = WPOS / 16;
  constexpr int NG = DUAL ? 2 : 1;                                // GEMMs (weight blocks, input tiles)
  constexpr int WEL = BN * K, AEL = BM * K, REL = RESM ? BM * BN : 0;  // elements
  constexpr int APL = BM * PPR / 512, RPL = RESM ? BM * RPR / 512 : 0;  // glds pieces per lane per tile and GEMM
  constexpr int SL = 2 * PT;                                            // 16-byte stores per lane per tile
  constexpr int SWA = PPR % 16 == 0 ? 15 : 7;                           // input-row piece swizzle mask (stays in the row)
  static_assert(PT >= 1 && WPOS % 16 == 0 && APL * 512 == BM * PPR && (!RESM || RPL * 512 == BM * RPR), "tile shape");
  static_assert(PPR % 8 == 0 && (!RESM || RPR >= 16), "piece swizzles");
  static_assert(2 * (NG * WEL + 2 * NG * AEL + 2 * REL) <= 163840, "LDS");
  __shared__ __attribute__((aligned(16))) uint16_t smem[NG * WEL + 2 * NG * AEL + 2 * REL];
  uint16_t* const sw = smem;                 // [gemm][fragment]
  uint16_t* const sa = smem + NG * WEL;      // [buf][gemm][BM][K]
  uint16_t* const sr = sa + 2 * NG * AEL;    // [buf][BM][BN]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int wn = wave % WN, wm = wave / WN;
  const int G = gridDim.x;
  int b = blockIdx.x;
  if ((G & 7) == 0) b = (b & 7) * (G >> 3) + (b >> 3);  // consecutive b on one XCD: a row tile's column blocks share its L2
  const int cb = b % ny, rstep = G / ny, n0 = cb * BN;
  const int nrt = (M + BM - 1) / BM;

  // the column block's weights, fragment (wn', k-step s, channel tile ct) as
  // a lane-ordered 1 KB image [g][r16][8]: row r16 of tile ct = channel
  // 32 (ct >> 1) + 8 (r16 >> 2) + 4 (ct & 1) + (r16 & 3) of group wn'
#pragma unroll
  for (int gi = 0; gi < NG; ++gi) {
    const uint16_t* wg = gi ? w2 : w;
    for (int f = wave; f < WN * KC * 4; f += NW) {
      const int ct = f & 3, s = (f >> 2) % KC, wq = f / (4 * KC);
      const int n = n0 + wq * 64 + 32 * (ct >> 1) + 8 * (r16 >> 2) + 4 * (ct & 1) + (r16 & 3);
      *(u16x8*)(sw + gi * WEL + f * 512 + lane * 8) = *(const u16x8*)(wg + (size_t)n * kp + s * 32 + g * 8);
    }
  }
  float bv[2][8], bv2[2][8];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int n = n0 + wn * 64 + 32 * h + 8 * g + j;
      bv[h][j] = bias ? bias[n] : 0.f;
      bv2[h][j] = DUAL && bias2 ? bias2[n] : 0.f;
    }
  // glds geometry: wave instruction i fills 64 consecutive 16-byte LDS units
  // q = (i NW + wave) 64 + lane of a tile image: row q / PR, slot q % PR,
  // holding the row's piece slot ^ (row & mask)
  int arow[APL], aoff[APL], rrow[RPL > 0 ? RPL : 1], roff[RPL > 0 ? RPL : 1];
#pragma unroll
  for (int i = 0; i < APL; ++i) {
    const int q = (i * NW + wave) * 64 + lane, r = q / PPR, j = q - r * PPR;
    arow[i] = r;
    aoff[i] = (j ^ (r & SWA)) * 8;
  }
#pragma unroll
  for (int i = 0; i < RPL; ++i) {
    const int q = (i * NW + wave) * 64 + lane, r = q / RPR, j = q - r * RPR;
    rrow[i] = r;
    roff[i] = r_off + n0 + (j ^ (r & 15)) * 8;
  }
  // a tile's input rows (and residual block) into buffer buf.  Rows past M
  // re-read row M - 1 (their outputs go to the sink) and tiles past the end
  // re-read tile 0 into a buffer never read: every lane always issues the
  // same pieces per tile from valid rows, branch-free, so the vmcnt counts
  // below hold
  auto issue = [&](int tile, int buf) {
    const int m0 = tile < nrt ? tile * BM : 0;
#pragma unroll
    for (int gi = 0; gi < NG; ++gi) {
      const uint16_t* src = gi ? in2 : in;
#pragma unroll
      for (int i = 0; i < APL; ++i) {
        const int m = min(m0 + arow[i], M - 1);
        glds16(src + (size_t)m * K + aoff[i], sa + (buf * NG + gi) * AEL + (i * NW + wave) * 64 * 8);
      }
    }
#pragma unroll
    for (int i = 0; i < RPL; ++i) {
      const int m = min(m0 + rrow[i], M - 1);
      glds16(res + (size_t)m * ldr + roff[i], sr + buf * REL + (i * NW + wave) * 64 * 8);
    }
  };
  __syncthreads();  // weights in
  int rt = b / ny;
  if (rt < nrt) issue(rt, 0);
  for (int it = 0; rt < nrt; ++it, rt += rstep) {
    const int buf = it & 1;
    // this tile's pieces landed; younger: the previous tile's SL stores
    if (it == 0) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(SL) : "memory");
    issue(rt + rstep, buf ^ 1);  // its readers (the previous tile) passed the barrier
    f32x4 acc[PT][4];
#pragma unroll
    for (int pt = 0; pt < PT; ++pt)
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) acc[pt][ct] = (f32x4)0.f;
#pragma unroll
    for (int gi = 0; gi < NG; ++gi) {
      if (gi == 1) {  // DUAL: conv3 done -> relu(acc + b3) + b_ds, the downsample accumulates on it
#pragma unroll
        for (int pt = 0; pt < PT; ++pt)
#pragma unroll
          for (int ct = 0; ct < 4; ++ct)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int h = ct >> 1, e = ct & 1;
              float x = acc[pt][ct][j] + bv[h][4 * e + j];
              if (relu1) x = relu(x);
              acc[pt][ct][j] = x + bv2[h][4 * e + j];
            }
      }
      const uint16_t* a = sa + (buf * NG + gi) * AEL;
      const uint16_t* wg = sw + gi * WEL;
#pragma unroll
      for (int s = 0; s < KC; ++s) {
        u16x8 wf[4];
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) wf[ct] = *(const u16x8*)(wg + ((wn * KC + s) * 4 + ct) * 512 + lane * 8);
#pragma unroll
        for (int pt = 0; pt < PT; ++pt) {
          const int r = wm * WPOS + pt * 16 + r16;
          const u16x8 pf = *(const u16x8*)(a + (r * PPR + ((s * 4 + g) ^ (r & SWA))) * 8);
#pragma unroll
          for (int ct = 0; ct < 4; ++ct) acc[pt][ct] = T::mfma(wf[ct], pf, acc[pt][ct]);
        }
      }
    }
    // epilogue: v = relu?(acc + b3) + residual, relu? (DUAL: relu?(acc));
    // 16-byte stores of channels n0 + 64 wn + 32 h + 8 g .. +7
#pragma unroll
    for (int pt = 0; pt < PT; ++pt) {
      const int r = wm * WPOS + pt * 16 + r16, m = rt * BM + r;
      uint16_t* o = m < M ? out + (size_t)m * ldo + c_off + n0 + wn * 64 + 8 * g : g_sink + lane * 8;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        u16x8 rv = (u16x8)0;
        if constexpr (RESM) rv = *(const u16x8*)(sr + buf * REL + (r * RPR + ((wn * 8 + 4 * h + g) ^ (r & 15))) * 8);
        u16x4 q[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          f32x4 v;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float x = acc[pt][2 * h + e][j];
            if constexpr (DUAL) {
              if (relu2) x = relu(x);
            } else if constexpr (MODE == 2) {
              x += bv[h][4 * e + j];
              if (relu1) x = relu(x);
            } else {
              x += bv[h][4 * e + j];
              if (relu1) x = relu(x);
              x += T::to_f32(rv[4 * e + j]);
              if (relu2) x = relu(x);
            }
            v[j] = x;
          }
          q[e] = T::pack4(v);
        }
        uint16_t* dst = m < M ? o + 32 * h : o;
        if constexpr (MODE == 2) {  // column segments (8-aligned: a lane's 8 channels never straddle one)
          const int cg = n0 + wn * 64 + 32 * h + 8 * g;
          dst = m >= M || cg >= cout ? g_sink + lane * 8
                : cg >= split2     ? out2 + (size_t)m * ldo2 + (cg - split2)
                : cg >= split1     ? out1 + (size_t)m * ldo1 + (cg - split1)
                                   : dst;
        }
        *(u16x8*)dst = __builtin_shufflevector(q[0], q[1], 0, 1, 2, 3, 4, 5, 6, 7);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing past-the-end pieces landed before LDS is released
}

#ifndef PWD2_BN
#define PWD2_BN 256
#endif
#ifndef PWD2_NB
#define PWD2_NB 2
#endif
// ---- pw_dual2 (round 6): ResNet-50 layer2's first bottleneck end -- conv3
// (1x1 128 -> 512) + bn3 + ReLU, plus the downsample (1x1 256 -> 512,
// stride 2, over the block input at 56^2) + bn, ReLU (ResVitKan.py:146-152).
// One 512-thread workgroup per CU owns a BN-column block (4 waves across,
// 64 columns each; 2 waves down, 16 rows each) and walks BM-row tiles.  Both
// weight blocks live in VGPRs (each wave's 64 columns: K 128 + K 256 = 192
// registers), the biases in LDS, so LDS holds only the input ring: the conv3
// rows and the strided downsample rows (512 B each, every other position of
// the 56^2 map) of the next NB - 1 tiles, issued by global_load_lds.  BN =
// 256 makes each output row's 512 B one workgroup's contiguous stores and
// halves the input re-reads across column blocks against 128-wide blocks
// (measured: 128 columns x 64 rows ran at 3.1 TB/s with HBM traffic equal
// to the algorithmic bytes).  acc -> relu(acc + b3) + b_ds between the two
// GEMMs (the reference's order, as convnd_pt DUAL).
// Layer3's pair (conv3 256 -> 1024 at 14^2, downsample 512 -> 1024 at
// stride 2 over 28^2) runs the same kernel with K3 = 256, KD = 512 and 32
// columns per wave (CW; its two weight blocks are 192 registers again): 8
// waves across the 256 columns, 16-row tiles, one 16-byte store per lane.
template <class T, int K3 = 128, int KD = 256, int CW = 64>
__global__ __launch_bounds__(512, 1) void pw_dual2(const uint16_t* __restrict__ h, const uint16_t* __restrict__ w3,
                                                   const float* __restrict__ b3, const uint16_t* __restrict__ x,
                                                   const uint16_t* __restrict__ wd, const float* __restrict__ bd,
                                                   uint16_t* __restrict__ out, int M, int kp3, int kpd, int ldo,
                                                   int c_off, int ny, int Ho, int Wo, int Hx, int Wx, int sx,
                                                   int relu1, int relu2) {
  constexpr int BN = PWD2_BN, NW = 8, NB = PWD2_NB, CT = CW / 16;          // CT: 16-column tiles per wave
  constexpr int WN = BN / CW, WM = NW / WN, BM = 16 * WM, WPOS = 16;
  constexpr int KC3 = K3 / 32, KCD = KD / 32, PP3 = K3 / 8, PPD = KD / 8;  // k-steps, 16-byte pieces per row
  constexpr int HEL = BM * K3, XEL = BM * KD;
  constexpr int HPL = BM * PP3 / 512, XPL = BM * PPD / 512, PL = HPL + XPL;  // glds pieces per lane per tile
  constexpr int SL = CT / 2;                                                 // 16-byte stores per lane per tile
  static_assert((CW == 32 || CW == 64) && WN * CW == BN && WM * WN == NW && HPL >= 1 && HPL * 512 == BM * PP3 && XPL * 512 == BM * PPD && NB >= 2, "tile shape");
  static_assert(8 * BN + 2 * NB * (HEL + XEL) <= 163840, "LDS");
  __shared__ __attribute__((aligned(16))) uint16_t smem[4 * BN + NB * (HEL + XEL)];
  float* const sbias = (float*)smem;         // [2][BN]: b3, b_ds
  uint16_t* const sh = smem + 4 * BN;        // [NB][BM][K3], piece p at p ^ (row & 15)
  uint16_t* const sx_ = sh + NB * HEL;       // [NB][BM][KD], piece p at p ^ (row & 15)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int wn = wave % WN, wm = wave / WN;
  const int G = gridDim.x;
  int b = blockIdx.x;
  if ((G & 7) == 0) b = (b & 7) * (G >> 3) + (b >> 3);
  const int cb = b % ny, rstep = G / ny, n0 = cb * BN;
  const int nrt = (M + BM - 1) / BM;
  // this wave's CW columns of both weight blocks as lane-ordered fragments
  // (k-step, ct), conv_pw's channel order
  u16x8 w3f[KC3][CT], wdf[KCD][CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int n = n0 + wn * CW + 32 * (ct >> 1) + 8 * (r16 >> 2) + 4 * (ct & 1) + (r16 & 3);
#pragma unroll
    for (int s = 0; s < KC3; ++s) w3f[s][ct] = *(const u16x8*)(w3 + (size_t)n * kp3 + s * 32 + g * 8);
#pragma unroll
    for (int s = 0; s < KCD; ++s) wdf[s][ct] = *(const u16x8*)(wd + (size_t)n * kpd + s * 32 + g * 8);
  }
  for (int i = tid; i < 2 * BN; i += 512) {
    const float* bp = i < BN ? b3 : bd;
    sbias[i] = bp ? bp[n0 + (i & (BN - 1))] : 0.f;
  }
  // the register operands have landed before the first global_load_lds (so
  // no compiler wait on them falls inside the hand-counted loop)
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
#pragma unroll
    for (int s = 0; s < KC3; ++s) asm volatile("" : "+v"(w3f[s][ct]));
#pragma unroll
    for (int s = 0; s < KCD; ++s) asm volatile("" : "+v"(wdf[s][ct]));
  }
  int hrow[HPL], hoff[HPL];
#pragma unroll
  for (int i = 0; i < HPL; ++i) {
    const int q = (i * NW + wave) * 64 + lane, r = q / PP3, j = q - r * PP3;
    hrow[i] = r;
    hoff[i] = (j ^ (r & 15)) * 8;
  }
  // the downsample rows go by a cursor per piece, the output position
  // (nn, oy, ox) of the next tile to issue, advanced by rstep tiles per issue
  // without divisions; rows past M (nn >= N) read image N - 1
  // (piece i is XR rows below piece 0, at the same swizzled column)
  constexpr int XR = NW * 64 / PPD;
  static_assert(PPD % 16 == 0 && PP3 % 16 == 0, "XOR swizzles stay inside a row");
  const int HW = Ho * Wo, N = M / HW, D = rstep * BM, dn = D / HW, doy = (D - dn * HW) / Wo, dox = D % Wo;
  const int rn = XR / HW, roy = (XR - rn * HW) / Wo, rox = XR % Wo;
  int cox, coy, cnn, xoff[XPL];
  {
    const int q = wave * 64 + lane, r = q / PPD, j = q - r * PPD;
#pragma unroll
    for (int i = 0; i < XPL; ++i) xoff[i] = (j ^ ((r + i * XR) & 15)) * 8;
    const int m = (b / ny) * BM + r;
    cox = m % Wo;
    coy = (m / Wo) % Ho;
    cnn = m / HW;
  }
  // rows past M re-read row M - 1 (their stores go to the sink), tiles past
  // the end re-read tile 0: branch-free, every lane issues PL pieces a tile
  auto issue = [&](int tile, int buf) {
    const int m0 = tile < nrt ? tile * BM : 0;
#pragma unroll
    for (int i = 0; i < HPL; ++i) {
      const int m = min(m0 + hrow[i], M - 1);
      glds16(h + (size_t)m * K3 + hoff[i], sh + buf * HEL + (i * NW + wave) * 64 * 8);
    }
    // (ox, oy, nn) + a row step (sox, soy, sn) already reduced mod (Wo, Ho)
    auto step = [&](int& ox, int& oy, int& nn, int sox, int soy, int sn) __attribute__((always_inline)) {
      ox += sox;
      const int c1 = ox >= Wo;
      ox -= c1 ? Wo : 0;
      oy += soy + c1;
      const int c2 = oy >= Ho;
      oy -= c2 ? Ho : 0;
      nn += sn + c2;
    };
    int ox = cox, oy = coy, nn = cnn;
#pragma unroll
    for (int i = 0; i < XPL; ++i) {  // output position (n, oy, ox) reads x at (n, sx oy, sx ox)
      if (i) step(ox, oy, nn, rox, roy, rn);
      const int pos = (min(nn, N - 1) * Hx + oy * sx) * Wx + ox * sx;
      glds16(x + (size_t)pos * KD + xoff[i], sx_ + buf * XEL + (i * NW + wave) * 64 * 8);
    }
    step(cox, coy, cnn, dox, doy, dn);
  };
  __syncthreads();  // biases in
  int rt = b / ny;
  if (rt < nrt) {
#pragma unroll
    for (int i = 0; i < NB - 1; ++i) issue(rt + i * rstep, i);
  }
  for (int it = 0, buf = 0; rt < nrt; ++it, rt += rstep, buf = buf == NB - 1 ? 0 : buf + 1) {
    // this tile's rows landed; younger: the NB - 2 tiles after it and the
    // stores of up to NB - 1 tiles before it (counting at most two of those
    // only waits longer)
    if (it == 0) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"((NB - 2) * PL) : "memory");
    else if (it == 1 || NB == 2) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"((NB - 2) * PL + SL) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"((NB - 2) * PL + 2 * SL) : "memory");
    issue(rt + (NB - 1) * rstep, buf == 0 ? NB - 1 : buf - 1);
    f32x4 acc[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) acc[ct] = (f32x4)0.f;
    const int r = wm * WPOS + r16;
    {
      const uint16_t* a = sh + buf * HEL;
#pragma unroll
      for (int s = 0; s < KC3; ++s) {
        const u16x8 pf = *(const u16x8*)(a + (r * PP3 + ((s * 4 + g) ^ (r & 15))) * 8);
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) acc[ct] = T::mfma(w3f[s][ct], pf, acc[ct]);
      }
    }
    // conv3 done: relu(acc + b3) + b_ds, the downsample accumulates on it
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int nb = wn * CW + 32 * (ct >> 1) + 8 * g + 4 * (ct & 1);
      const f32x4 b3v = *(const f32x4*)(sbias + nb), bdq = *(const f32x4*)(sbias + BN + nb);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v = acc[ct][j] + b3v[j];
        if (relu1) v = relu(v);
        acc[ct][j] = v + bdq[j];
      }
    }
    {
      const uint16_t* a = sx_ + buf * XEL;
#pragma unroll
      for (int s = 0; s < KCD; ++s) {
        const u16x8 pf = *(const u16x8*)(a + (r * PPD + ((s * 4 + g) ^ (r & 15))) * 8);
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) acc[ct] = T::mfma(wdf[s][ct], pf, acc[ct]);
      }
    }
    // epilogue: relu?(acc), 16-byte stores of channels n0 + CW wn + 32 hh + 8 g .. +7
    const int m = rt * BM + r;
    uint16_t* o = m < M ? out + (size_t)m * ldo + c_off + n0 + wn * CW + 8 * g : g_sink + lane * 8;
#pragma unroll
    for (int hh = 0; hh < SL; ++hh) {
      u16x4 q[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        f32x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = relu2 ? relu(acc[2 * hh + e][j]) : acc[2 * hh + e][j];
        q[e] = T::pack4(v);
      }
      *(u16x8*)(m < M ? o + 32 * hh : o) = __builtin_shufflevector(q[0], q[1], 0, 1, 2, 3, 4, 5, 6, 7);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing past-the-end pieces landed before LDS is released
}

// ---- pw_res2 (round 6): ResNet-50 layer4's conv3 + identity, relu(relu(
// conv1x1(h) + b3) + x) with K = 512 -> 2048 at 7^2 (ResVitKan.py:146-152),
// pw_dual2's form with the residual in place of the downsample GEMM: 512
// threads per CU own a 256-column block (8 waves x 32 columns, 16-row tiles),
// each wave's 32 columns x K 512 of weights in VGPRs (128 registers: pw_res's
// LDS-resident block would be 256 KB), biases in LDS, and the next tile's
// input rows (1 KB each) and its 16 x 256 residual block double-buffered in
// LDS by global_load_lds a tile ahead; one 16-byte residual read and one
// 16-byte store per lane per tile.
template <class T, int K = 512, int CW = 32, int BN = 256>
__global__ __launch_bounds__(512, 1) void pw_res2(const uint16_t* __restrict__ h, const uint16_t* __restrict__ w,
                                                  const float* __restrict__ bias, const uint16_t* __restrict__ res,
                                                  uint16_t* __restrict__ out, int M, int kp, int ldo, int c_off,
                                                  int ldr, int r_off, int ny, int relu1, int relu2) {
  constexpr int NW = 8, NB = 2, CT = CW / 16, WN = BN / CW, WM = NW / WN, BM = 16 * WM;
  constexpr int KC = K / 32, PP = K / 8, RPP = BN / 8;  // k-steps, 16-byte pieces per input / residual row
  constexpr int HEL = BM * K, REL = BM * BN;
  constexpr int HPL = BM * PP / 512, RPL = BM * RPP / 512, PL = HPL + RPL;  // glds pieces per lane per tile
  constexpr int SL = CT / 2;                                                // 16-byte stores per lane per tile
  static_assert((CW == 32 || CW == 64) && WN * CW == BN && WM * WN == NW && HPL >= 1 && RPL >= 1 &&
                    HPL * 512 == BM * PP && RPL * 512 == BM * RPP && PP % 16 == 0 && RPP % 16 == 0,
                "tile shape");
  static_assert(4 * BN + 2 * NB * (HEL + REL) <= 163840, "LDS");
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * BN + NB * (HEL + REL)];
  float* const sbias = (float*)smem;     // [BN]
  uint16_t* const sh = smem + 2 * BN;    // [NB][BM][K], piece p at p ^ (row & 15)
  uint16_t* const sr = sh + NB * HEL;    // [NB][BM][BN], piece p at p ^ (row & 15)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int wn = wave % WN, wm = wave / WN;
  const int G = gridDim.x;
  int b = blockIdx.x;
  if ((G & 7) == 0) b = (b & 7) * (G >> 3) + (b >> 3);
  const int cb = b % ny, rstep = G / ny, n0 = cb * BN;
  const int nrt = (M + BM - 1) / BM;
  u16x8 wf[KC][CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int n = n0 + wn * CW + 32 * (ct >> 1) + 8 * (r16 >> 2) + 4 * (ct & 1) + (r16 & 3);
#pragma unroll
    for (int s = 0; s < KC; ++s) wf[s][ct] = *(const u16x8*)(w + (size_t)n * kp + s * 32 + g * 8);
  }
  for (int i = tid; i < BN; i += 512) sbias[i] = bias ? bias[n0 + i] : 0.f;
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int s = 0; s < KC; ++s) asm volatile("" : "+v"(wf[s][ct]));  // landed before the first glds
  // rows past M re-read row M - 1 (their stores go to the sink), tiles past
  // the end re-read tile 0: branch-free, PL pieces per lane per tile
  auto issue = [&](int tile, int buf) {
    const int m0 = tile < nrt ? tile * BM : 0;
#pragma unroll
    for (int i = 0; i < HPL; ++i) {
      const int q = (i * NW + wave) * 64 + lane, r = q / PP, j = q % PP;
      const int m = min(m0 + r, M - 1);
      glds16(h + (size_t)m * K + (j ^ (r & 15)) * 8, sh + buf * HEL + (i * NW + wave) * 64 * 8);
    }
#pragma unroll
    for (int i = 0; i < RPL; ++i) {
      const int q = (i * NW + wave) * 64 + lane, r = q / RPP, j = q % RPP;
      const int m = min(m0 + r, M - 1);
      glds16(res + (size_t)m * ldr + r_off + n0 + (j ^ (r & 15)) * 8, sr + buf * REL + (i * NW + wave) * 64 * 8);
    }
  };
  __syncthreads();  // biases in
  int rt = b / ny;
  if (rt < nrt) issue(rt, 0);
  for (int it = 0; rt < nrt; ++it, rt += rstep) {
    const int buf = it & 1;
    // this tile's rows landed; younger: the previous tile's SL stores
    if (it == 0) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(SL) : "memory");
    issue(rt + rstep, buf ^ 1);
    f32x4 acc[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) acc[ct] = (f32x4)0.f;
    const int r = wm * 16 + r16;
    const uint16_t* a = sh + buf * HEL;
#pragma unroll
    for (int s = 0; s < KC; ++s) {
      const u16x8 pf = *(const u16x8*)(a + (r * PP + ((s * 4 + g) ^ (r & 15))) * 8);
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) acc[ct] = T::mfma(wf[s][ct], pf, acc[ct]);
    }
    // epilogue: relu2?(relu1?(acc + b) + res), 16-byte stores of channels
    // n0 + CW wn + 32 hh + 8 g .. +7
    const int m = rt * BM + r;
    uint16_t* o = m < M ? out + (size_t)m * ldo + c_off + n0 + wn * CW + 8 * g : g_sink + lane * 8;
#pragma unroll
    for (int hh = 0; hh < SL; ++hh) {
      const int pc = (wn * CW + 32 * hh) / 8 + g;  // residual piece of the lane's 8 channels
      const u16x8 rv = *(const u16x8*)(sr + buf * REL + (r * RPP + (pc ^ (r & 15))) * 8);
      const f32x4 b0 = *(const f32x4*)(sbias + wn * CW + 32 * hh + 8 * g);
      const f32x4 b1 = *(const f32x4*)(sbias + wn * CW + 32 * hh + 8 * g + 4);
      u16x4 q[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        f32x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float t = acc[2 * hh + e][j] + (e ? b1[j] : b0[j]);
          if (relu1) t = relu(t);
          t += T::to_f32(rv[4 * e + j]);
          v[j] = relu2 ? relu(t) : t;
        }
        q[e] = T::pack4(v);
      }
      *(u16x8*)(m < M ? o + 32 * hh : o) = __builtin_shufflevector(q[0], q[1], 0, 1, 2, 3, 4, 5, 6, 7);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing past-the-end pieces landed before LDS is released
}

// ---- conv_tk: S3D's temporal (kd,1,1) convs with 8 output frames (model.py:
// 63-82, SepConv3d's conv_t + bn_t + relu_t: base.0's (7,1,1)/(2,1,1) and
// base.3's (3,1,1) at 56^2 / 28^2 positions).  Through the generic implicit
// GEMM every output frame re-gathers its kd input frames (3.5 reads of each
// input element for base.0).  Here a unit is (clip n, 16 consecutive spatial
// positions): its D x 16 x Cin input slab is copied to LDS once (glds,
// double-buffered when it fits: the next unit's slab streams in during this
// one) and wave z computes output frame z for those 16 positions from it,
// the workgroup's 64-channel weight block resident in LDS
// ([k-step][ct][g][r16][8], one 1 KB fragment per read).  MFMAs transposed
// (rows = channels): each lane stores 4 channels of one position straight
// from registers.  Slab pieces are XOR-swizzled by position (piece j of
// position p at slot j ^ (p & 7)) so the 16 positions of a fragment read
// spread over the LDS banks.
template <class T>
__global__ __launch_bounds__(512, 1) void conv_tk(const uint16_t* __restrict__ in, const uint16_t* __restrict__ w,
                                                  const float* __restrict__ bias, uint16_t* __restrict__ out,
                                                  int nunits, int S, int D, int Cin, int kd, int sd, int pd, int kp,
                                                  int ldo, int c_off, int relu_on, int db, int nbk, int nslot) {
  constexpr int LDS_EL = 81920;  // 160 KiB
  __shared__ __attribute__((aligned(16))) uint16_t smem[LDS_EL];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  // workgroup -> (unit slot, 64-channel block): the nbk blocks of one slot
  // have ids 8 apart (same XCD under round-robin placement, dispatched
  // together), so they read each unit's input slab from HBM once and share
  // it through that XCD's L2 instead of streaming the whole input nbk times
  const int b_lo = blockIdx.x & 7, b_hi = blockIdx.x >> 3;
  const int nb = b_hi % nbk, slot = (b_hi / nbk) * 8 + b_lo;
  const int NP = Cin >> 3, CH = Cin >> 5, KS = kd * CH;  // pieces / 32-channel chunks per position, k-steps
  const int SLAB = D * 16 * Cin;                          // elements per slab buffer
  uint16_t* const wts = smem;
  uint16_t* const slab0 = smem + KS * 2048;
  const int units_per_clip = (S + 15) >> 4;  // the last unit of a clip may be partial

  auto issue_slab = [&](uint16_t* dst, int u) {
    const int n = u / units_per_clip, p0 = (u - n * units_per_clip) << 4;
    const int npieces = D * 16 * NP;
    for (int b = wave * 64; b < npieces; b += 512) {
      const int sl = b + lane;
      const int dp = sl / NP, j = sl - dp * NP;     // dp = d * 16 + p
      const int d = dp >> 4, p = dp & 15;
      const uint16_t* src = g_zero16;
      if (d < D && p0 + p < S) src = in + (((size_t)n * D + d) * S + p0 + p) * Cin + ((j ^ (p & 7)) << 3);
      glds16(src, dst + b * 8);
    }
  };

  int u = slot;
  if (u < nunits) issue_slab(slab0, u);
  // this workgroup's 64 output channels, all k-steps
  for (int c = tid; c < 64 * KS * 4; c += 512) {
    const int n = c / (KS * 4), k8 = c - n * (KS * 4);
    *(u16x8*)(wts + ((((k8 >> 2) * 4 + (n >> 4)) * 4 + (k8 & 3)) * 16 + (n & 15)) * 8) =
        *(const u16x8*)(w + (size_t)(nb * 64 + n) * kp + k8 * 8);
  }
  float bv[4][4];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int j = 0; j < 4; ++j) bv[ct][j] = bias ? bias[nb * 64 + ct * 16 + 4 * g + j] : 0.f;
  const int z = wave;  // output frame of this wave (Do == 8)
  for (int it = 0; u < nunits; ++it) {
    const int next = u + nslot;
    uint16_t* const cur = slab0 + (db == 2 ? (it & 1) * SLAB : 0);
    // slab u in; the other buffer's readers done.  lgkmcnt(0) too: the weight
    // block above was written with plain ds_writes, which must have landed
    // before any other wave reads it (first iteration)
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (db == 2 && next < nunits) issue_slab(slab0 + ((it + 1) & 1) * SLAB, next);
    f32x4 acc[4];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) acc[ct] = (f32x4)0.f;
    for (int t = 0; t < kd; ++t) {
      const int d = z * sd + t - pd;
      if ((unsigned)d >= (unsigned)D) continue;     // zero padding (wave-uniform)
      const uint16_t* row = cur + (d * 16 + r16) * Cin;
      const uint16_t* wk = wts + (t * CH * 16 + g) * 128 + r16 * 8;  // [s = t*CH + ch][ct][g][r16][8]
#pragma unroll 2
      for (int ch = 0; ch < CH; ++ch) {
        const u16x8 pf = *(const u16x8*)(row + (((ch * 4 + g) ^ (r16 & 7)) << 3));
        const uint16_t* wb = wk + ch * 16 * 128;
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) acc[ct] = T::mfma(*(const u16x8*)(wb + ct * 4 * 128), pf, acc[ct]);
      }
    }
    {
      const int n = u / units_per_clip, p0 = (u - n * units_per_clip) << 4;
      uint16_t* o = out + (((size_t)n * 8 + z) * S + p0 + r16) * ldo + c_off + nb * 64 + 4 * g;
#pragma unroll
      for (int ct = 0; ct < 4 && p0 + r16 < S; ++ct) {
        f32x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = relu_on ? relu(acc[ct][j] + bv[ct][j]) : acc[ct][j] + bv[ct][j];
        *(u16x4*)(o + ct * 16) = T::pack4(v);
      }
    }
    if (db == 1) {
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // every wave done with the slab
      if (next < nunits) issue_slab(slab0, next);
    }
    u = next;
  }
}

// ---- conv_tk2 (round 3): the same temporal convs as conv_tk, with the unit's
// input streamed as K slices instead of one whole slab.  conv_tk copies a
// unit's D x 16 x Cin slab and then computes on it; for Cin 192 the slab
// (48 KB) and the 64-channel weight block (72 KB) leave no room for a second
// slab, so every unit waited for its slab (base.3's (3,1,1) 192->192 at
// 8x28^2: 0.73 ms for 0.15 ms of HBM and MFMA work).  Here the K loop runs
// 32-channel chunk outer, tap inner: slice c of a unit is D frames x 16
// positions x 32 channels (D KB), all that chunk's taps need, and slices
// stream continuously across units through a 3-slot ring, two ahead of the
// MFMAs, with hand-counted vmcnt waits (DP glds pieces per thread per slice,
// plus the 4 output stores of a unit's last slice).  Positions in a frame
// row are 64 B; piece j of position p sits at 16-byte slot 4p + (j ^ ((p >> 1)
// & 2)), which makes every ds_read_b128 lane group of a fragment read (16
// positions x piece g) hit 16 distinct 4-bank groups.  Wave z computes output
// frame z (Do == 8) for the unit's 16 positions x the workgroup's 64
// channels, MFMAs transposed as in conv_tk; the nbk column blocks of a unit
// slot are 8 workgroup ids apart (see conv_tk).
// vmcnt(BASE + ST*k) + barrier for the wave-uniform k in 0..K (s_waitcnt
// takes an immediate): ST = stores per store batch
template <int BASE, int K, int ST>
__device__ __forceinline__ void wait_vm_stores(int k) {
  if constexpr (K > 0) {
    if (k < K) {
      wait_vm_stores<BASE, K - 1, ST>(k);
      return;
    }
  }
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(BASE + ST * K) : "memory");
}

#ifdef TK2_STAMPS
__device__ unsigned long long tk2_st[4][64][8][4];
#define TK2_STAMP(k)                                                                          \
  do {                                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    unsigned long long t_;                                                                    \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    if (blockIdx.x < 4 && lane == 0 && s < 64) tk2_st[blockIdx.x][s][wave][(k)] = t_;         \
  } while (0)
#else
#define TK2_STAMP(k) \
  do {               \
  } while (0)
#endif

template <class T, int DP, int KD, int SD, int KC, int R, int WR = 0>
__global__ __launch_bounds__(512, 1) void conv_tk2(const uint16_t* __restrict__ in, const uint16_t* __restrict__ w,
                                                   const float* __restrict__ bias, uint16_t* __restrict__ out,
                                                   int nunits, int S, int Cin, int kp, int ldo, int c_off, int relu_on,
                                                   int nbk, int nslot) {
  constexpr int D = DP * 8;             // input frames: one glds piece per thread per chunk per 8 frames
  constexpr int PD = KD / 2;            // 'same' temporal padding (model.py:63-82)
  constexpr int NF = SD + KD;           // input frames two consecutive output frames span
  constexpr int CE = D * 16 * 32;       // elements of one 32-channel chunk of a unit
  constexpr int SL = KC * CE;           // slice (one step) elements
  constexpr int NP = DP * KC;           // glds pieces per thread per slice
  constexpr int LDS_EL = 81920;
  __shared__ __attribute__((aligned(16))) uint16_t smem[LDS_EL];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int b_lo = blockIdx.x & 7, b_hi = blockIdx.x >> 3;
  const int nb = b_hi % nbk, slot = (b_hi / nbk) * 8 + b_lo;
  const int CH = Cin >> 5, KS = KD * CH, SPU = CH / KC;  // chunks, k-steps, steps per unit
  const int upc = (S + 15) >> 4;  // units per clip (the last one may be partial)
  const int wts_el = WR ? 0 : KS * 2048;  // WR: no weight block in LDS, the ring takes its room
  uint16_t* const wts = smem;
  float* const bsm = (float*)(smem + wts_el);
  uint16_t* const ring = smem + wts_el + 128;
  const int my_units = slot < nunits ? (nunits - slot + nslot - 1) / nslot : 0;
  const int nsteps = my_units * SPU;

  // This thread's glds pieces: slice slot sl = k*512 + tid -> (chunk kc,
  // frame d, position p, channel piece j), the same for every slice; per
  // slice only the unit (clip n, first position p0) and the chunk group
  // move, tracked by an incremental cursor (no per-step divisions).
  int toff[NP], tp[NP];
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    const int sl = k * 512 + tid;
    const int kc = sl / (D * 64), r1 = sl - kc * (D * 64);
    const int d = r1 >> 6, rem = r1 & 63, p = rem >> 2, j = (rem & 3) ^ ((p >> 1) & 2);
    toff[k] = (d * S + p) * Cin + kc * 32 + j * 8;
    tp[k] = p;
  }
  int is = 0, ic = 0, iu = slot;
  int in_ = iu / upc, ip0 = (iu - in_ * upc) << 4;
  auto issue = [&]() {  // slice `is` (past the last step: zero pieces, so every step issues the same count)
    uint16_t* dst = ring + (is % R) * SL;
    const bool live = is < nsteps;
    const uint16_t* ub = in + ((size_t)in_ * D * S + ip0) * Cin + ic * KC * 32;
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const uint16_t* src = live && ip0 + tp[k] < S ? ub + toff[k] : g_zero16;
      glds16(src, dst + (k * 512 + wave * 64) * 8);
    }
    ++is;
    if (++ic == SPU) {
      ic = 0;
      iu += nslot;
      in_ = iu / upc;
      ip0 = (iu - in_ * upc) << 4;
    }
  };

  // weight block [k-step t*CH + c][ct][g][r16][8] and biases to LDS (global
  // loads retired here, before the first glds: the loop's counted waits then
  // see only slice pieces and output stores)
  // (row i of the wave's tile cc -- tiles 2h, 2h+1 -- computes channel
  // 32h + 8 (i >> 2) + 4 cc + (i & 3): lane group g ends with channels
  // 32h + 8g .. +7 of its position, one 16-byte store per output frame)
  // WR (round 6; = Cin / 32 when set): the wave's own 32 channels x all KD
  // WR k-steps live in VGPRs instead (2 KD WR fragments), so a k-step's LDS
  // reads are the NF input frames only, not NF + 2 KD
  const int fp = wave & 3, h = wave >> 2;
  u16x8 wreg[WR ? KD * WR : 1][2];
  if constexpr (WR > 0) {
#pragma unroll
    for (int ks = 0; ks < KD * WR; ++ks)
#pragma unroll
      for (int cc = 0; cc < 2; ++cc)
        wreg[ks][cc] = *(const u16x8*)(w + (size_t)(nb * 64 + 32 * h + 8 * (r16 >> 2) + 4 * cc + (r16 & 3)) * kp +
                                       (ks * 4 + g) * 8);
#pragma unroll
    for (int ks = 0; ks < KD * WR; ++ks)
#pragma unroll
      for (int cc = 0; cc < 2; ++cc) asm volatile("" : "+v"(wreg[ks][cc]));  // landed before the first glds
  } else {
    for (int c = tid; c < 64 * KS * 4; c += 512) {
      const int n = c / (KS * 4), k8 = c - n * (KS * 4);
      const int ct = 2 * (n >> 5) + ((n >> 2) & 1), i = 4 * ((n >> 3) & 3) + (n & 3);
      *(u16x8*)(wts + ((((k8 >> 2) * 4 + ct) * 4 + (k8 & 3)) * 16 + i) * 8) =
          *(const u16x8*)(w + (size_t)(nb * 64 + n) * kp + k8 * 8);
    }
  }
  if (tid < 64) bsm[tid] = bias ? bias[nb * 64 + tid] : 0.f;
  __syncthreads();
  // wave (fp, h): output frames 2fp, 2fp+1 x channels 32h .. 32h+31 (tiles 2h, 2h+1)
  f32x4 bv[2];
#pragma unroll
  for (int cc = 0; cc < 2; ++cc) bv[cc] = *(const f32x4*)(bsm + h * 32 + 8 * g + 4 * cc);
#pragma unroll
  for (int i = 0; i < R - 1; ++i) issue();
  const int d0 = 2 * fp * SD - PD;  // input frame of frame 2fp's tap 0
  const int rdoff = r16 * 32 + ((g ^ ((r16 >> 1) & 2)) << 3);  // this lane's piece in a frame row
  const uint16_t* const wl = wts + (h * 2 * 4 + g) * 128 + r16 * 8;  // + kstep*2048 + cc*512
  f32x4 acc[2][2];
#pragma unroll
  for (int j = 0; j < 2; ++j) acc[j][0] = acc[j][1] = (f32x4)0.f;
  // hist bit i: step s-1-i ended a unit (issued its 4 output stores, after
  // that step's slice issue)
  unsigned hist = 0;
  int cs = 0, cu = slot;  // compute cursor: step within the unit, unit
  for (int s = 0; s < nsteps; ++s) {
    // slice s landed: younger than it are slices s+1 .. s+R-2 and the 2
    // output stores of each unit-ending step in s-R+1 .. s-1; every wave is done with slice s-1's slot,
    // which this step's issue refills
    TK2_STAMP(0);
    wait_vm_stores<(R - 2) * NP, R - 1, 2>(__builtin_popcount(hist & ((1u << (R - 1)) - 1)));
    TK2_STAMP(1);
    issue();  // slice s + R - 1
    TK2_STAMP(2);
    const uint16_t* const sbase = ring + (s % R) * SL + rdoff;
    if constexpr (WR > 0) {
      static_assert(WR % KC == 0 && WR / KC <= 2, "WR: one or two steps per unit");
      // the step's k-steps are compile-time per (step within the unit), so
      // the register fragments are indexed statically
      auto kbody = [&](auto csc) __attribute__((always_inline)) {
        constexpr int CS = decltype(csc)::value;
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
          const uint16_t* cur = sbase + kc * CE;
          u16x8 px[NF];
#pragma unroll
          for (int f = 0; f < NF; ++f) {
            const int d = d0 + f;
            px[f] = (unsigned)d < (unsigned)D ? *(const u16x8*)(cur + d * 512) : (u16x8)0;
          }
#pragma unroll
          for (int t = 0; t < KD; ++t)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const int f = j * SD + t;
              if ((unsigned)(d0 + f) < (unsigned)D) {
#pragma unroll
                for (int cc = 0; cc < 2; ++cc)
                  acc[j][cc] = T::mfma(wreg[t * WR + CS * KC + kc][cc], px[f], acc[j][cc]);
              }
            }
        }
      };
      if constexpr (WR / KC == 1) kbody(std::integral_constant<int, 0>{});
      else if (cs == 0) kbody(std::integral_constant<int, 0>{});
      else kbody(std::integral_constant<int, 1>{});
    } else {
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const int c = cs * KC + kc;
      const uint16_t* cur = sbase + kc * CE;
      // every input frame the wave's two output frames read, once (sd = 1:
      // frame 2fp+1's tap t is frame 2fp's tap t+1), then the weights
      u16x8 px[NF], wf[KD][2];
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        const int d = d0 + f;
        px[f] = (unsigned)d < (unsigned)D ? *(const u16x8*)(cur + d * 512) : (u16x8)0;
      }
#pragma unroll
      for (int t = 0; t < KD; ++t)
#pragma unroll
        for (int cc = 0; cc < 2; ++cc) wf[t][cc] = *(const u16x8*)(wl + (t * CH + c) * 2048 + cc * 512);
#pragma unroll
      for (int t = 0; t < KD; ++t)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int f = j * SD + t;
          if ((unsigned)(d0 + f) < (unsigned)D) {  // zero padding: no MFMA (wave-uniform)
#pragma unroll
            for (int cc = 0; cc < 2; ++cc) acc[j][cc] = T::mfma(wf[t][cc], px[f], acc[j][cc]);
          }
        }
    }
    }
    TK2_STAMP(3);
    const bool stored = cs == SPU - 1;
    hist = (hist << 1) | (stored ? 1u : 0u);
    if (stored) {
      const int n = cu / upc, p0 = (cu - n * upc) << 4;
      if (p0 + r16 < S) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          uint16_t* o = out + (((size_t)n * 8 + 2 * fp + j) * S + p0 + r16) * ldo + c_off + nb * 64 + h * 32 + 8 * g;
          u16x4 q2[2];
#pragma unroll
          for (int cc = 0; cc < 2; ++cc) {
            f32x4 v;
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = relu_on ? relu(acc[j][cc][q] + bv[cc][q]) : acc[j][cc][q] + bv[cc][q];
            q2[cc] = T::pack4(v);
          }
          *(u16x8*)o = __builtin_shufflevector(q2[0], q2[1], 0, 1, 2, 3, 4, 5, 6, 7);
        }
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[j][0] = acc[j][1] = (f32x4)0.f;
      cs = 0;
      cu += nslot;
    } else {
      ++cs;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing zero slices landed before LDS is released
}

// ---- convnd_pt: persistent implicit GEMM for the uniform-tap (cin % 64 == 0)
// convs with a dense 16-bit output and no residual (ResNet-50's K >= 256 1x1
// and stride-2 convs, S3D's wide layers): convnd_igemm with three changes.
//   * Persistent: one workgroup per CU walks row tiles of ONE column block
//     (its weights pointer and biases fixed), and the stage ring runs across
//     tile boundaries: the next tile's first stages are already in flight
//     while this tile's last step computes and its outputs are stored.  Per
//     256 x 128 tile convnd_igemm spent ~7-10k cycles in its prologue and ~7k
//     in its LDS-staged epilogue beside 2.4k per K step (s_memtime stamps,
//     tools/ubench/nd_ubench.hip), and with one workgroup per CU nothing
//     overlapped them.
//   * Transposed MFMAs (rows = channels, as conv_pw): a lane ends with 4
//     channels of one position; tile pairs compute channels 32p + 8g + 0..3 /
//     4..7 (weight row i of tile 2p+h is channel 32p + 8(i>>2) + 4h + (i&3)),
//     so each lane stores 16 bytes from registers: no LDS staging, which the
//     ring fills anyway.
//   * BN = 256 (two ring slots of 64 KB): 64 KB through the TA per 4.2M MACs,
//     2/3 of the 256 x 128 tile's bytes per MAC — the CU's glds issue
//     (~37 B/clk) was what bounded that tile's K step.
// LDS images: rows of 64 k (128 B).  A (positions): piece c of row r at
// c ^ ((r >> 1) & 7); B (weights): at c ^ fB(r), fB(r) = ((r >> 1) & 1) |
// (((r >> 3) & 3) << 1), conflict-free for the permuted rows a fragment
// read touches (rows 8(i>>2) + (i&3) + 4h + 32p + 64wn, i = 0..15).
// Stage g's glds go out during step g - D (D = NS - 1), one piece after
// each MFMA group; output stores are counted in the vmcnt waits.
// RES (BN = 128 only): the residual's 16-byte vectors of a tile go out as
// inline-asm loads at the start of its last K step (hipcc would wait
// vmcnt(0) for an ordinary load beside glds in flight) and are waited for
// by count in the epilogue (only that step's glds pieces are younger).
// DUAL (BN = 128, no RES): a second GEMM q over another input into the same
// output positions and channels — ResNet's downsample branch fused into the
// bottleneck's conv3.  A tile runs conv3's K steps, then in registers
// acc = relu(acc + b3) + b_ds (the reference's ReLU after bn3 comes before
// the residual add, ResVitKan.py:146-152), then the downsample's K steps
// (its input gathered with its own geometry and stride), then relu: the
// downsample output never goes through HBM.
template <class T, int BN, bool RES = false, bool DUAL = false>
__global__ __launch_bounds__(512, 1) void convnd_pt(ConvP p, ConvP q) {
  constexpr int BM = 256, BK = 64, NW = 8;
  constexpr int WNW = BN / 64, WMW = NW / WNW;  // waves along N (64 channels each) and M
  constexpr int WTM = BM / WMW, RT = WTM / 16, CT = 4;
  constexpr int NS = BN == 256 ? 2 : 3, D = NS - 1;
  constexpr int SLOT_A = BM * BK, SLOT = (BM + BN) * BK;
  constexpr int NA = BM / 8 / NW, NB = BN / 8 / NW, PER = NA + NB;
  constexpr int KH = BK / 32;
  constexpr int QPK = D == 1 ? PER : (PER + KH - 1) / KH;  // pieces issued per K half (D = 1: all in the first)
  constexpr int NST = RT * CT / 2;                          // output stores per lane per tile
  static_assert(QPK <= RT && NST <= 24 && D * PER + NST <= 63, "piece / store counts");
  static_assert(!RES || BN == 128, "residual: 128-wide tiles (register budget)");
  static_assert(!DUAL || (BN == 128 && !RES), "dual GEMM: 128-wide tiles (register budget), no residual input");
  // the stage ring, then the workgroup's column-block biases (fp32, BN of p's
  // and with DUAL BN of q's): read by the epilogue / the DUAL transition
  // instead of held in 16-32 VGPRs
  constexpr int NBIAS = DUAL ? 2 * BN : BN;
  __shared__ __attribute__((aligned(16))) uint16_t smem[NS * SLOT + 2 * NBIAS];
  float* const sbias = (float*)(smem + NS * SLOT);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int wm = wave / WNW, wn = wave % WNW;
  const int G = gridDim.x;
  int b = blockIdx.x;
  if ((G & 7) == 0) b = (b & 7) * (G >> 3) + (b >> 3);  // consecutive b on one XCD
  // column blocks: the last one partial when BN does not divide Cout (its
  // weight rows and biases past Cout are padding, its stores go to g_sink)
  const int ny = (p.Cout + BN - 1) / BN, nrt = (p.M + BM - 1) / BM;
  const int cb = b % ny, rstep = G / ny;
  const int n0 = cb * BN;
  int rt_first = b / ny;
  const int ntile = rt_first < nrt ? (nrt - 1 - rt_first) / rstep + 1 : 0;
  const int S1 = p.ksteps, S = DUAL ? S1 + q.ksteps : S1, total = ntile * S;

  // glds lane geometry: instruction i of this wave covers image rows
  // 8 (NW i + wave) + (lane >> 3), position lane & 7
  const int pos = lane & 7, rsub = lane >> 3;
  const int jA = pos ^ ((4 * wave + (lane >> 4)) & 7);
  const int jB = pos ^ (((lane >> 4) & 1) | ((wave & 3) << 1));
  // B (weight) glds sources of the GEMM at the issue cursor (DUAL: re-pointed
  // at q's weights for the downsample's steps, which start at step S1)
  const uint16_t* wsrc[NB];
  auto set_wsrc = [&](const uint16_t* w, int kp) {
#pragma unroll
    for (int i = 0; i < NB; ++i) wsrc[i] = w + (size_t)(n0 + 8 * (NW * i + wave) + rsub) * kp + jB * 8;
  };
  set_wsrc(p.w, p.Kp);
  int w_s0 = 0;  // first step of the GEMM wsrc points at
  // biases of the workgroup's column block into LDS, before any glds is in flight
  for (int c = tid; c < NBIAS; c += 512) {
    const float* bsrc = c < BN ? p.bias : q.bias;
    const int cc = c < BN ? c : c - BN;
    sbias[c] = bsrc && n0 + cc < p.Cout ? bsrc[n0 + cc] : 0.f;
  }
  __syncthreads();
  // this lane's 4 channels of channel tile ct (second = q's biases)
  auto bias4 = [&](int ct, bool second) {
    return *(const f32x4*)(sbias + (second ? BN : 0) + wn * 64 + 32 * (ct >> 1) + 8 * g + 4 * (ct & 1));
  };

  // issue cursor: row tile, step, per-A-instruction row offsets and tap bases
  int i_rt = rt_first, i_s = 0, uc = 0, uz = 0, uy = 0, ux = 0, i_stage = 0;
  long long roff[NA];
  int riz[NA], riy[NA], rix[NA];
  // the gather geometry of the GEMM at the cursor (DUAL: p's, then q's)
  const uint16_t* g_in = p.in;
  int gD = p.D, gH = p.H, gW = p.W, gC8 = p.C8, gKH = p.KH, gKW = p.KW;
  int gSD = p.SD, gSH = p.SH, gSW = p.SW, gPD = p.PD, gPH = p.PH, gPW = p.PW;
  auto use_geo = [&](bool second) {
    g_in = second ? q.in : p.in;
    gD = second ? q.D : p.D;
    gH = second ? q.H : p.H;
    gW = second ? q.W : p.W;
    gC8 = second ? q.C8 : p.C8;
    gKH = second ? q.KH : p.KH;
    gKW = second ? q.KW : p.KW;
    gSD = second ? q.SD : p.SD;
    gSH = second ? q.SH : p.SH;
    gSW = second ? q.SW : p.SW;
    gPD = second ? q.PD : p.PD;
    gPH = second ? q.PH : p.PH;
    gPW = second ? q.PW : p.PW;
  };
  long long rowstride = (long long)p.W * p.C8 * 8, planestride = rowstride * p.H;
  auto set_rows = [&](int rt_idx) {
    rowstride = (long long)gW * gC8 * 8;
    planestride = rowstride * gH;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int m = rt_idx * BM + 8 * (NW * i + wave) + rsub;
      const int mm = m < p.M ? m : 0;
      const int ox = mm % p.Wo, t1 = mm / p.Wo;
      const int oy = t1 % p.Ho, t2 = t1 / p.Ho;
      const int oz = t2 % p.Do, n = t2 / p.Do;
      riz[i] = m < p.M ? oz * gSD - gPD : -(1 << 29);
      riy[i] = oy * gSH - gPH;
      rix[i] = ox * gSW - gPW;
      roff[i] = (long long)n * gD * planestride + ((long long)riz[i] * gH + riy[i]) * rowstride +
                (long long)rix[i] * (gC8 * 8) + jA * 8;
    }
  };
  set_rows(i_rt);
  // piece q of the stage at the cursor (A pieces, then B); stages past the
  // workgroup's last copy zeros into slots never read
  auto piece = [&](int qq) {
    uint16_t* slot = smem + (i_stage % NS) * SLOT;
    const bool real = i_stage < total;
    if (qq < NA) {
      const long long toff = uz * planestride + uy * rowstride + (long long)ux * gC8 * 8 + uc;
      const bool ok = real & ((unsigned)(riz[qq] + uz) < (unsigned)gD) & ((unsigned)(riy[qq] + uy) < (unsigned)gH) &
                      ((unsigned)(rix[qq] + ux) < (unsigned)gW);
      glds16(ok ? g_in + (roff[qq] + toff) : g_zero16, slot + (NW * qq + wave) * 64 * 8);
    } else {
      glds16(real ? wsrc[qq - NA] + (size_t)(i_s - w_s0) * BK : g_zero16, slot + SLOT_A + (NW * (qq - NA) + wave) * 64 * 8);
    }
  };
  auto advance = [&] {
    ++i_stage;
    uc += 64;
    if (uc == gC8 * 8) {
      uc = 0;
      if (++ux == gKW) {
        ux = 0;
        if (++uy == gKH) {
          uy = 0;
          ++uz;
        }
      }
    }
    if (++i_s == S) {
      i_s = uc = uz = uy = ux = 0;
      i_rt += rstep;
      if constexpr (DUAL) {
        use_geo(false);
        set_wsrc(p.w, p.Kp);
        w_s0 = 0;
      }
      if (i_stage < total) set_rows(i_rt);
    } else if (DUAL && i_s == S1) {
      uc = uz = uy = ux = 0;
      use_geo(true);
      set_wsrc(q.w, q.Kp);
      w_s0 = S1;
      set_rows(i_rt);
    }
  };

  f32x4 acc[RT][CT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) acc[rt][ct] = (f32x4)0.f;

#pragma unroll
  for (int st = 0; st < D; ++st) {
#pragma unroll
    for (int q = 0; q < PER; ++q) piece(q);
    advance();
  }
  int c_rt = rt_first, c_s = 0;
  // ends[k]: step g-1-k ended a tile (its NST output stores follow stage g-1-k+D's pieces)
  int end1 = 0, end2 = 0;
  for (int gs = 0; gs < total; ++gs) {
#ifdef ND_STAMPS
    const int s = gs;
#endif
    ND_STAMP(0);
    // stage gs landed: younger are stages gs+1 .. gs+D-1 and the stores of
    // the tile ends among steps gs-D .. gs-1
    const int nend = end1 + (D >= 2 ? end2 : 0);
    if (D == 1) {
      if (nend) asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(NST) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    } else {
      if (nend) asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"((D - 1) * PER + NST) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"((D - 1) * PER) : "memory");
    }
    ND_STAMP(1);
    const uint16_t* a = smem + (gs % NS) * SLOT;
    const uint16_t* bw = a + SLOT_A;
    if constexpr (DUAL) {
      if (c_s == S1) {  // conv3 done: relu(acc + b3) + b_ds, then the downsample's K steps accumulate on it
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
          const f32x4 b1 = bias4(ct, false), b2 = bias4(ct, true);
#pragma unroll
          for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              float x = acc[rt][ct][j] + b1[j];
              if (p.flags & FAC_CONV_RELU) x = relu(x);
              acc[rt][ct][j] = x + b2[j];
            }
        }
      }
    }
    // RES: the residual vectors of this tile's lanes, at its last step
    u16x8 rv[RES ? RT : 1][RES ? CT / 2 : 1];
    if constexpr (RES) {
      if (c_s == S - 1) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          const int m = c_rt * BM + wm * WTM + rt * 16 + r16;
#pragma unroll
          for (int pp = 0; pp < CT / 2; ++pp) {
            const uint16_t* src = m < p.M ? p.res + (size_t)m * p.ldr + p.r_off + n0 + wn * 64 + 32 * pp + 8 * g : g_zero16;
            asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(rv[rt][pp]) : "v"(src) : "memory");
          }
        }
      }
    }
#pragma unroll
    for (int ks = 0; ks < KH; ++ks) {
      const int c = ks * 4 + g;
      u16x8 fw[CT], fp[RT];
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const int r = wn * 64 + 32 * (ct >> 1) + 8 * (r16 >> 2) + 4 * (ct & 1) + (r16 & 3);
        const int fB = ((r >> 1) & 1) | (((r >> 3) & 3) << 1);
        fw[ct] = *(const u16x8*)(bw + r * BK + ((c ^ fB) << 3));
      }
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const int r = wm * WTM + rt * 16 + r16;
        fp[rt] = *(const u16x8*)(a + r * BK + ((c ^ ((r >> 1) & 7)) << 3));
      }
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) acc[rt][ct] = T::mfma(fw[ct], fp[rt], acc[rt][ct]);
        __builtin_amdgcn_sched_barrier(0);
        if (rt < QPK && ks * QPK + rt < PER) piece(ks * QPK + rt);
      }
    }
    ND_STAMP(2);
    advance();
    end2 = end1;
    end1 = 0;
    if (++c_s == S) {
      // tile done: bias, ReLU (+ residual, ReLU), 16-byte stores from registers
      if constexpr (RES) {
        // the residual loads landed: younger are this step's PER glds pieces
        static_assert(RT * CT / 2 == 8, "residual wait ties 8 vectors");
        asm volatile("s_waitcnt vmcnt(%8)"
                     : "+v"(rv[0][0]), "+v"(rv[0][1]), "+v"(rv[1][0]), "+v"(rv[1][1]), "+v"(rv[2][0]), "+v"(rv[2][1]),
                       "+v"(rv[3][0]), "+v"(rv[3][1])
                     : "n"(PER)
                     : "memory");
      }
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const int m = c_rt * BM + wm * WTM + rt * 16 + r16;
        if (m < p.M) {
          uint16_t* o = (uint16_t*)p.out + (size_t)m * p.ldo + p.c_off + n0 + wn * 64 + 8 * g;
          const int ch = n0 + wn * 64 + 8 * g;
#pragma unroll
          for (int pp = 0; pp < CT / 2; ++pp) {
            u16x4 q2[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              f32x4 v;
              const f32x4 b1 = DUAL ? (f32x4)0.f : bias4(2 * pp + h, false);
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                float x;
                if constexpr (DUAL) {
                  x = acc[rt][2 * pp + h][j];
                  if (p.flags & FAC_CONV_RELU2) x = relu(x);
                } else {
                  x = acc[rt][2 * pp + h][j] + b1[j];
                  if (p.flags & FAC_CONV_RELU) x = relu(x);
                }
                if constexpr (RES) {
                  x += T::to_f32(rv[rt][pp][4 * h + j]);
                  if (p.flags & FAC_CONV_RELU2) x = relu(x);
                }
                v[j] = x;
              }
              q2[h] = T::pack4(v);
            }
            // channels past Cout (a partial column block): the store still
            // issues, into g_sink, so every tile counts NST stores in the
            // vmcnt waits above.  Column segments (fac_conv_nd_split, 8-aligned):
            // [split1, split2) -> out1 (ldo1), [split2, cout) -> out2 (ldo2)
            const int cg = ch + 32 * pp;
            uint16_t* dst = cg >= p.Cout    ? g_sink + 8 * lane
                            : cg >= p.split2 ? (uint16_t*)p.out2 + (size_t)m * p.ldo2 + (cg - p.split2)
                            : cg >= p.split1 ? (uint16_t*)p.out1 + (size_t)m * p.ldo1 + (cg - p.split1)
                                             : o + 32 * pp;
            *(u16x8*)dst = __builtin_shufflevector(q2[0], q2[1], 0, 1, 2, 3, 4, 5, 6, 7);
          }
        }
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) acc[rt][ct] = (f32x4)0.f;
      }
      c_s = 0;
      c_rt += rstep;
      end1 = 1;
    }
    ND_STAMP(3);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing zero stages landed before LDS is released
}

// grid of gx row tiles x ny column tiles: flat (column tiles of a row tile
// adjacent, see convnd_igemm) unless it would overflow
static dim3 conv_grid(ConvP& p, int gx, int ny) {
  if (ny > 1 && (long long)gx * ny < INT_MAX) {
    p.ny = ny;
    return dim3(gx * ny, 1);
  }
  p.ny = 0;
  return dim3(gx, ny);
}

// process-wide (fac_set_option "nd_pt_wide"): convnd_pt also for cout not a
// multiple of 128 (a partial last column block) from this many 256-row tiles
// on; 0 keeps those on convnd_igemm (A/B)
static int g_nd_pt_wide = 32;
void set_nd_pt_wide(int v) { g_nd_pt_wide = v; }
// process-wide (fac_set_option "nd_occ3"): convnd_igemm's 3-per-CU 2-slot
// 128 x 64 tile also for cout <= 64 up to this many K steps (default 4: S3D's
// narrow SepConv halves, config 4 +0.3 to +0.6 %; 0: K <= 128 only)
static int g_nd_occ3 = 4;
void set_nd_occ3(int v) { g_nd_occ3 = v; }
// process-wide (fac_set_option "pool_roll"): MaxPool3d(3,1,1) on 7-wide
// maps by maxpool3_roll (1: every frame in one thread, k >= 2: k output
// frames per thread), 0: maxpool3_s1 (A/B)
static int g_pool_roll = 1;
void set_pool_roll(int v) { g_pool_roll = v; }
// process-wide (fac_set_option "pool_win"): 1 (default) the strided max pools
// with a compile-time window by pool_max_win, 0 pool_nd (A/B)
static int g_pool_win = 1;
void set_pool_win(int v) { g_pool_win = v; }
// process-wide (fac_set_option "pool3_zg"): output frames per thread of
// maxpool3_s1 (0: all, the default)
static int g_pool3_zg = 0;
void set_pool3_zg(int v) { g_pool3_zg = v; }
// process-wide (fac_set_option "pool_lds14"): 1 (default) MaxPool3d(3,1,1) on
// 14 x 14 maps with 64-multiple channels by maxpool3_lds14, 0 maxpool3_s1
static int g_pool_lds14 = 1;
// process-wide (fac_set_option "pw_res"): 1 (default) the K = 128 / 256
// bottleneck conv3 + identity by pw_res, 0 by convnd_pt (A/B)
static int g_pw_res = 1;
static int g_tk_wreg = 1;  // conv_tk2 with the weights in VGPRs (cin 128 / 192)
// process-wide (fac_set_option "pool3_g"): frames per maxpool3_pw unit on
// 7 x 7 maps, 0 = default (2), else 1 / 2 / 4 (A/B)
static int g_pool3_g = 0;
void set_pool3_g(int v) { g_pool3_g = v; }
void set_pw_res(int v) { g_pw_res = v; }
void set_tk_wreg(int v) { g_tk_wreg = v; }
void set_pool_lds14(int v) { g_pool_lds14 = v; }

template <class T>
static bool launch_convnd_pt(ConvP& p, hipStream_t st) {
  const bool res = p.flags & FAC_CONV_RESID;
  const bool split = p.split1 < p.Cout;
  if (p.ksteps < 2 || !p.vec_out || p.Cout % 8 || (split && res) ||
      (p.flags & FAC_CONV_OUT_F32) || (!res && (p.flags & FAC_CONV_RELU2)) || (res && !p.vec_res))
    return false;
  const int nrt = (p.M + 255) / 256;
  if (p.Cout % 128 || split) {
    // a partial column block or column segments (fac_conv_nd_split): no
    // residual tile, and enough row tiles that every persistent workgroup
    // walks several (small late-block grids keep convnd_igemm's tiles)
    if (!g_nd_pt_wide || res || nrt < g_nd_pt_wide) return false;
  }
  static const int ncu = [] {
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    return n;
  }();
  const int bn = res ? 128 : (p.Cout % 256 == 0 ? 256 : 128);
  const int ny = (p.Cout + bn - 1) / bn;
  int G = ncu / ny * ny;
  if ((long long)nrt * ny < G) G = nrt * ny;
  if (G <= 0) return false;
  p.ny = 0;
  if (res) convnd_pt<T, 128, true><<<G, 512, 0, st>>>(p, p);
  else if (bn == 256) convnd_pt<T, 256><<<G, 512, 0, st>>>(p, p);
  else convnd_pt<T, 128><<<G, 512, 0, st>>>(p, p);
  return true;
}

template <class T, bool UT, bool IL>
static void launch_convnd_t(ConvP p, hipStream_t st) {
  if constexpr (UT) {
    if (launch_convnd_pt<T>(p, st)) return;
  }
  const int gx64 = (p.M + 63) / 64, gx128 = (p.M + 127) / 128, gx256 = (p.M + 255) / 256;
  const int ny64 = (p.Cout + 63) / 64, ny128 = (p.Cout + 127) / 128;
  constexpr int nd256_min = 256;  // 256 x 128 tiles only when they fill the chip at least once
  if (p.ksteps <= 2 || (g_nd_occ3 && p.Cout <= 64 && p.ksteps <= g_nd_occ3)) {
    // K <= 128 (1x1 expansions): memory-bound, so occupancy first — a 2-slot
    // ring (48 KB) lets three 128 x 64 workgroups share a CU
    const dim3 g = conv_grid(p, gx128, ny64);
    convnd_igemm<T, 128, 64, 2, 2, 3, 2, UT, IL><<<g, 256, 0, st>>>(p);
  } else if ((long long)gx128 * ny64 < 512) {
    // small grids (S3D's late 4x7x7 / 2x3x3 stages): 64 x 64 tiles, three per CU
    const dim3 g = conv_grid(p, gx64, ny64);
    convnd_igemm<T, 64, 64, 2, 2, 3, 3, UT, IL><<<g, 256, 0, st>>>(p);
  } else if (p.Cout % 128 == 0 && (long long)gx256 * ny128 >= nd256_min) {
    // 256 x 128 tiles (8 waves, 144 KB ring, one per CU: 48 KB global -> LDS per
    // 4.2 MFLOP, twice the 128 x 64 tile's intensity) when the grid still fills
    // the chip at least once (ResNet's 7x7 layers: 392 tiles, 1.2-1.35x faster
    // than 128 x 64 ones; same-box config 5 +2 %) and no column
    // tile is half empty
    const dim3 g = conv_grid(p, gx256, ny128);
    convnd_igemm<T, 256, 128, 4, 2, 1, 3, UT, IL><<<g, 512, 0, st>>>(p);
  } else {
    const dim3 g = conv_grid(p, gx128, ny64);
    convnd_igemm<T, 128, 64, 2, 2, 2, 3, UT, IL><<<g, 256, 0, st>>>(p);
  }
}

template <class T>
static hipError_t launch_convnd(ConvP p, int cout_pad, hipStream_t st) {
  (void)cout_pad;
  // uniform-tap gather when every 64-deep K step lies in one tap (cin % 64),
  // the per-lane tap gather otherwise; both with the interleaved glds issue
  if (p.C8 % 8 == 0) launch_convnd_t<T, true, true>(p, st);
  else launch_convnd_t<T, false, true>(p, st);
  return hipGetLastError();
}

}  // namespace fac

extern "C" {

int fac_conv_weight_layout(int cout, int cin, int kd, int kh, int kw, int* cout_pad, int* k_pad) {
  if (cout <= 0 || cin <= 0 || kd <= 0 || kh <= 0 || kw <= 0 || !cout_pad || !k_pad) return FAC_ERR_ARG;
  *cout_pad = (cout + 127) / 128 * 128;
  *k_pad = (kd * kh * kw * cin + 63) / 64 * 64;
  return FAC_OK;
}

static int conv_nd_impl(const fac_conv_desc* d, void* out1, int ldo1, int split1, void* out2, int ldo2, int split2,
                        void* stream) {
  using namespace fac;
  if (!d || !d->in || !d->weight || !d->out) return FAC_ERR_ARG;
  if (d->dtype != FAC_DTYPE_BF16 && d->dtype != FAC_DTYPE_F16) return FAC_ERR_ARG;
  if (d->cin <= 0 || d->cin % 8 || d->cout <= 0 || d->n <= 0 || d->d <= 0 || d->h <= 0 || d->w <= 0) return FAC_ERR_SHAPE;
  // MaxPool3d((1,3,3), (1,2,2), (0,1,1)) over the input, then this 1x1x1
  // 64 -> 64 conv (S3D's base.1 + base.2): maxpool2s_pw
  if (d->flags & FAC_CONV_PREPOOL3S2) {
    if ((d->flags & ~(FAC_CONV_RELU | FAC_CONV_PREPOOL3S2)) || out1 || out2 || d->kd != 1 || d->kh != 1 ||
        d->kw != 1 || d->sd != 1 || d->sh != 1 || d->sw != 1 || d->pd || d->ph || d->pw || d->cin != 64 ||
        d->cout != 64 || d->w != 56 || d->k_pad != 64 || d->od != d->d || d->oh != (d->h - 1) / 2 + 1 ||
        d->ow != 28 || d->ldo % 8 || d->c_off % 8 || d->ldo < d->c_off + 64)
      return FAC_ERR_ARG;
    constexpr int RB = 4;
    const int nunits = d->n * d->d * ((d->oh + RB - 1) / RB);
    const int grid = (nunits + 7) / 8 * 8;
    hipStream_t st = (hipStream_t)stream;
    const int relu_on = (d->flags & FAC_CONV_RELU) != 0;
    if (d->dtype == FAC_DTYPE_BF16)
      fac::maxpool2s_pw<fac::BF16, 28, RB><<<grid, 256, 0, st>>>((const uint16_t*)d->in, (const uint16_t*)d->weight,
                                                                 d->bias, (uint16_t*)d->out, nunits, d->h, d->oh,
                                                                 d->ldo, d->c_off, relu_on);
    else
      fac::maxpool2s_pw<fac::F16, 28, RB><<<grid, 256, 0, st>>>((const uint16_t*)d->in, (const uint16_t*)d->weight,
                                                                d->bias, (uint16_t*)d->out, nunits, d->h, d->oh,
                                                                d->ldo, d->c_off, relu_on);
    return hipGetLastError() == hipSuccess ? FAC_OK : FAC_ERR_HIP;
  }
  if (d->kd <= 0 || d->kh <= 0 || d->kw <= 0 || d->sd <= 0 || d->sh <= 0 || d->sw <= 0) return FAC_ERR_SHAPE;
  if (d->pd < 0 || d->ph < 0 || d->pw < 0 || d->od <= 0 || d->oh <= 0 || d->ow <= 0) return FAC_ERR_SHAPE;
  // output dims must be the floor-mode ones (every gathered tap then stays
  // within the padded input)
  if (d->od != (d->d + 2 * d->pd - d->kd) / d->sd + 1 || d->oh != (d->h + 2 * d->ph - d->kh) / d->sh + 1 ||
      d->ow != (d->w + 2 * d->pw - d->kw) / d->sw + 1)
    return FAC_ERR_SHAPE;
  int cout_pad, k_pad;
  fac_conv_weight_layout(d->cout, d->cin, d->kd, d->kh, d->kw, &cout_pad, &k_pad);
  if (d->k_pad != k_pad) return FAC_ERR_SHAPE;
  if (d->ldo < d->c_off + std::min(d->cout, split1) || d->c_off < 0) return FAC_ERR_SHAPE;
  if ((d->flags & FAC_CONV_RESID) && (!d->residual || d->ldr < d->r_off + d->cout || d->r_off < 0)) return FAC_ERR_ARG;
  const long long M = (long long)d->n * d->od * d->oh * d->ow;
  if (M >= (1LL << 31) || (long long)d->n * d->d * d->h * d->w * d->cin >= (1LL << 40)) return FAC_ERR_SHAPE;
  ConvP p;
  p.in = (const uint16_t*)d->in;
  p.w = (const uint16_t*)d->weight;
  p.bias = d->bias;
  p.res = (const uint16_t*)d->residual;
  p.out = d->out;
  p.D = d->d;
  p.H = d->h;
  p.W = d->w;
  p.C8 = d->cin / 8;
  p.Do = d->od;
  p.Ho = d->oh;
  p.Wo = d->ow;
  p.Cout = d->cout;
  p.KD = d->kd;
  p.KH = d->kh;
  p.KW = d->kw;
  p.SD = d->sd;
  p.SH = d->sh;
  p.SW = d->sw;
  p.PD = d->pd;
  p.PH = d->ph;
  p.PW = d->pw;
  p.Kp = k_pad;
  p.ksteps = k_pad / 64;
  p.ktot8 = d->kd * d->kh * d->kw * (d->cin / 8);
  p.ldo = d->ldo;
  p.c_off = d->c_off;
  p.ldr = d->ldr;
  p.r_off = d->r_off;
  p.flags = d->flags;
  p.vec_out = (d->ldo % 8 == 0 && d->c_off % 8 == 0) ? 1 : 0;
  p.vec_res = (d->ldr % 8 == 0 && d->r_off % 8 == 0) ? 1 : 0;
  p.M = (int)M;
  p.out1 = out1;
  p.out2 = out2;
  p.ldo1 = ldo1;
  p.ldo2 = ldo2;
  p.split1 = split1;
  p.split2 = split2;
  const bool split = split1 < d->cout;
  if (split) p.vec_out = p.vec_out && ldo1 % 8 == 0 && ldo2 % 8 == 0;
  hipStream_t st = (hipStream_t)stream;
  const bool s2d4_shape = !split && d->kd == 1 && d->kh == 4 && d->kw == 4 && d->sd == 1 && d->sh == 1 && d->sw == 1 &&
                          d->pd == 0 && d->ph == 0 && d->pw == 0 && d->cin == 16 && d->cout == 64 && k_pad == 256 &&
                          d->oh % 8 == 0 && d->ow % 28 == 0 && d->ldo == 64 && d->c_off == 0;
  auto cu_count = [] {
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
      ncu = 256;
    return ncu;
  };
  // + MaxPool2d(3, 2, 1): only the space-to-depth first conv with ReLU
  // (ResNet-50's conv1 -> bn1 -> relu -> maxpool), conv_s2d4_mp
  if (d->flags & FAC_CONV_MAXPOOL3S2) {
    if (!s2d4_shape || d->flags != (FAC_CONV_RELU | FAC_CONV_MAXPOOL3S2)) return FAC_ERR_ARG;
    const int nimg = d->n * d->od, hp = d->oh / 2, wp = d->ow / 2, nstrip = nimg * (wp / 14);
    const int grid = std::min(nstrip, 2 * cu_count());  // two resident (74 KB of LDS each)
    if (d->dtype == FAC_DTYPE_BF16)
      conv_s2d4_mp<BF16><<<grid, 256, 0, st>>>((const uint16_t*)d->in, (const uint16_t*)d->weight, d->bias,
                                               (uint16_t*)d->out, nstrip, d->h, d->w, hp, wp, k_pad);
    else
      conv_s2d4_mp<F16><<<grid, 256, 0, st>>>((const uint16_t*)d->in, (const uint16_t*)d->weight, d->bias,
                                              (uint16_t*)d->out, nstrip, d->h, d->w, hp, wp, k_pad);
    return hipGetLastError() == hipSuccess ? FAC_OK : FAC_ERR_HIP;
  }
  // MaxPool3d(3, 1, 1) over the input, then this 1x1x1 conv (S3D's
  // Inception branch3): maxpool3_pw
  if (d->flags & FAC_CONV_MAXPOOL3S1) {
    const int S = d->h;
    if (split || (d->flags & ~(FAC_CONV_RELU | FAC_CONV_MAXPOOL3S1)) || d->kd != 1 || d->kh != 1 || d->kw != 1 ||
        d->sd != 1 || d->sh != 1 || d->sw != 1 || d->pd || d->ph || d->pw || d->w != S ||
        !(S == 14 || S == 7 || S == 3) || d->cout % 32 || d->ldo % 8 || d->c_off % 8)
      return FAC_ERR_ARG;
    // frames per unit: 196 positions at 7 x 7 when the clip allows, 18 at 3 x 3
    // frames per unit at 7 x 7: 2 by default (98 positions; fac_set_option
    // "pool3_g" 1 / 2 / 4 forces one where the clip allows), at 3 x 3: 2
    const int g7 = g_pool3_g ? g_pool3_g : 2;
    const int G = S == 14 ? 1 : (S == 7 ? (d->d % g7 == 0 ? g7 : (d->d % 2 == 0 ? 2 : 1)) : (d->d % 2 == 0 ? 2 : 1));
    const int nunits = d->n * (d->d / G);
    // 128 columns per workgroup where cout allows (the pooled image is built
    // once per unit instead of once per 64-column block), else 64 / 32
    const int nct = d->cout % 128 == 0 ? 4 : (d->cout % 64 == 0 ? 2 : 1);
    const dim3 grid((nunits + 7) / 8 * 8, d->cout / (32 * nct));
    const int relu_on = (d->flags & FAC_CONV_RELU) != 0;
    const uint16_t* in = (const uint16_t*)d->in;
    const uint16_t* wt = (const uint16_t*)d->weight;
    uint16_t* o = (uint16_t*)d->out;
#define FAC_MPW(TT, SS, GG, NN)                                                                                     \
  maxpool3_pw<TT, SS, GG, NN><<<grid, 256, 0, st>>>(in, wt, d->bias, o, nunits, d->d, d->cin, k_pad, d->ldo, d->c_off, \
                                                     relu_on)
#define FAC_MPW_S(TT, NN)                      \
  do {                                         \
    if (S == 14) FAC_MPW(TT, 14, 1, NN);       \
    else if (S == 7 && G == 4) FAC_MPW(TT, 7, 4, NN); \
    else if (S == 7 && G == 2) FAC_MPW(TT, 7, 2, NN); \
    else if (S == 7) FAC_MPW(TT, 7, 1, NN);    \
    else if (G == 2) FAC_MPW(TT, 3, 2, NN);    \
    else FAC_MPW(TT, 3, 1, NN);                \
  } while (0)
    if (d->dtype == FAC_DTYPE_BF16) {
      if (nct == 4) FAC_MPW_S(BF16, 4);
      else if (nct == 2) FAC_MPW_S(BF16, 2);
      else FAC_MPW_S(BF16, 1);
    } else {
      if (nct == 4) FAC_MPW_S(F16, 4);
      else if (nct == 2) FAC_MPW_S(F16, 2);
      else FAC_MPW_S(F16, 1);
    }
#undef FAC_MPW_S
#undef FAC_MPW
    return hipGetLastError() == hipSuccess ? FAC_OK : FAC_ERR_HIP;
  }
  // the space-to-depth first conv (4x4/1 over 16-channel cells, cout 64, no
  // residual, dense output): its own kernel (conv_s2d4)
  if (s2d4_shape && (d->flags & ~FAC_CONV_RELU) == 0) {
    const int nimg = d->n * d->od, nbox = nimg * (d->oh / 8) * (d->ow / 28);
    const int grid = std::min(nbox, 2 * cu_count());  // two resident (two halo buffers + weights: 56 KB each)
    const int relu_on = (d->flags & FAC_CONV_RELU) != 0;
    if (d->dtype == FAC_DTYPE_BF16)
      conv_s2d4<BF16><<<grid, 256, 0, st>>>((const uint16_t*)d->in, (const uint16_t*)d->weight, d->bias,
                                            (uint16_t*)d->out, nbox, d->h, d->w, d->oh, d->ow, k_pad, relu_on);
    else
      conv_s2d4<F16><<<grid, 256, 0, st>>>((const uint16_t*)d->in, (const uint16_t*)d->weight, d->bias,
                                           (uint16_t*)d->out, nbox, d->h, d->w, d->oh, d->ow, k_pad, relu_on);
    return hipGetLastError() == hipSuccess ? FAC_OK : FAC_ERR_HIP;
  }
  // S3D's merged Inception heads at K = 192 / 256 (fac_conv_nd_split, 1x1,
  // relu(conv + b) into up to three column segments): pw_res PLAIN, 128-wide
  // column blocks over the zero-padded weight rows
  if (g_pw_res && split && d->kd == 1 && d->kh == 1 && d->kw == 1 && d->sd == 1 && d->sh == 1 && d->sw == 1 &&
      d->pd == 0 && d->ph == 0 && d->pw == 0 && !(d->flags & ~FAC_CONV_RELU) && k_pad == d->cin &&
      (d->cin == 192 || d->cin == 256) && d->ldo % 8 == 0 && d->c_off % 8 == 0 && ldo1 % 8 == 0 && ldo2 % 8 == 0 &&
      split1 % 8 == 0 && (split2 == INT_MAX || split2 % 8 == 0) && cout_pad % 128 == 0) {
    const int ny = cout_pad / 128, ncu = cu_count();
    const int G = std::max(ny, ncu / ny * ny);
    const int r1 = (d->flags & FAC_CONV_RELU) != 0;
    const uint16_t* in = (const uint16_t*)d->in;
    const uint16_t* wt = (const uint16_t*)d->weight;
#define FAC_PWS(TT, KC)                                                                                              \
  pw_res<TT, KC, 128, 64, 2><<<G, 512, 0, st>>>(in, wt, d->bias, nullptr, (uint16_t*)d->out, (int)M, k_pad, d->ldo, \
                                                d->c_off, 0, 0, ny, r1, 0, nullptr, nullptr, nullptr, d->cout,      \
                                                (uint16_t*)out1, ldo1, split1, (uint16_t*)out2, ldo2, split2)
    if (d->dtype == FAC_DTYPE_BF16) {
      if (d->cin == 192) FAC_PWS(BF16, 6);
      else FAC_PWS(BF16, 8);
    } else {
      if (d->cin == 192) FAC_PWS(F16, 6);
      else FAC_PWS(F16, 8);
    }
#undef FAC_PWS
    return hipGetLastError() == hipSuccess ? FAC_OK : FAC_ERR_HIP;
  }
  // the bottleneck conv3 + identity at K = 128 / 256 (ResNet-50 layer2 /
  // layer3, relu(relu(conv + b) + residual)): pw_res
  if (g_pw_res && !split && d->kd == 1 && d->kh == 1 && d->kw == 1 && d->sd == 1 && d->sh == 1 && d->sw == 1 &&
      d->pd == 0 && d->ph == 0 && d->pw == 0 && (d->flags & FAC_CONV_RESID) &&
      !(d->flags & ~(FAC_CONV_RELU | FAC_CONV_RESID | FAC_CONV_RELU2)) && k_pad == d->cin &&
      ((d->cin == 128 && d->cout % 256 == 0) || (d->cin == 256 && d->cout % 128 == 0)) && d->ldo % 8 == 0 &&
      d->c_off % 8 == 0 && d->ldr % 8 == 0 && d->r_off % 8 == 0) {
    const int bn = d->cin == 128 ? 256 : 128, ny = d->cout / bn;
    const int ncu = cu_count();
    const int G = std::max(ny, ncu / ny * ny);
    const int r1 = (d->flags & FAC_CONV_RELU) != 0, r2 = (d->flags & FAC_CONV_RELU2) != 0;
    const uint16_t* in = (const uint16_t*)d->in;
    const uint16_t* wt = (const uint16_t*)d->weight;
    const uint16_t* res = (const uint16_t*)d->residual;
    uint16_t* o = (uint16_t*)d->out;
    const int mi = (int)M;
#define FAC_PWR(TT, KC, BNN) \
  pw_res<TT, KC, BNN, 64><<<G, 512, 0, st>>>(in, wt, d->bias, res, o, mi, k_pad, d->ldo, d->c_off, d->ldr, d->r_off, ny, r1, r2, \
                                             nullptr, nullptr, nullptr, INT_MAX, nullptr, 0, INT_MAX, nullptr, 0, INT_MAX)
    if (d->dtype == FAC_DTYPE_BF16) {
      if (d->cin == 128) FAC_PWR(BF16, 4, 256);
      else FAC_PWR(BF16, 8, 128);
    } else {
      if (d->cin == 128) FAC_PWR(F16, 4, 256);
      else FAC_PWR(F16, 8, 128);
    }
#undef FAC_PWR
    return hipGetLastError() == hipSuccess ? FAC_OK : FAC_ERR_HIP;
  }
  // layer4's conv3 + identity (K 512, cout % 256 == 0): pw_res2, weights in
  // VGPRs ("pw_res" 2 routes it back to convnd_pt for A/B)
  if (g_pw_res == 1 && !split && d->kd == 1 && d->kh == 1 && d->kw == 1 && d->sd == 1 && d->sh == 1 &&
      d->sw == 1 && d->pd == 0 && d->ph == 0 && d->pw == 0 && (d->flags & FAC_CONV_RESID) &&
      !(d->flags & ~(FAC_CONV_RELU | FAC_CONV_RESID | FAC_CONV_RELU2)) && k_pad == d->cin && d->cin == 512 &&
      d->cout % 256 == 0 && d->ldo % 8 == 0 && d->c_off % 8 == 0 && d->ldr % 8 == 0 && d->r_off % 8 == 0) {
    const int ny = d->cout / 256, ncu = cu_count(), G = std::max(ny, ncu / ny * ny);
    const int r1 = (d->flags & FAC_CONV_RELU) != 0, r2 = (d->flags & FAC_CONV_RELU2) != 0;
#define FAC_PWR2(TT)                                                                                            \
  pw_res2<TT><<<G, 512, 0, st>>>((const uint16_t*)d->in, (const uint16_t*)d->weight, d->bias,                 \
                                 (const uint16_t*)d->residual, (uint16_t*)d->out, (int)M, k_pad, d->ldo, d->c_off, \
                                 d->ldr, d->r_off, ny, r1, r2)
    if (d->dtype == FAC_DTYPE_BF16) FAC_PWR2(BF16);
    else FAC_PWR2(F16);
#undef FAC_PWR2
    return hipGetLastError() == hipSuccess ? FAC_OK : FAC_ERR_HIP;
  }
  // stride-1 1x1 convs with K = cin in {64, 128, 256}: conv_pw
  // K 128 / 256 1x1s with cout % 128 == 0 go to convnd_pt instead: config 5
  // +1.2 % same-box (layer3's 256 -> 1024 + residual 160 -> 145 us)
  const bool to_pt = (d->cin == 128 || d->cin == 256) && d->cout % 128 == 0;
  if (!split && !to_pt && d->kd == 1 && d->kh == 1 && d->kw == 1 && d->sd == 1 && d->sh == 1 && d->sw == 1 &&
      d->pd == 0 && d->ph == 0 && d->pw == 0 && (d->cin == 64 || d->cin == 128 || d->cin == 256) &&
      k_pad == d->cin &&
      d->cout % 64 == 0 && d->ldo % 8 == 0 && d->c_off % 8 == 0 && !(d->flags & FAC_CONV_OUT_F32) &&
      (!(d->flags & FAC_CONV_RESID) || (d->ldr % 8 == 0 && d->r_off % 8 == 0))) {
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
      ncu = 256;
    const bool r = d->flags & FAC_CONV_RESID;
    const int ny = d->cout / 64;
    // rows per tile and the LDS-bound residency: weights 64 x cin, two A
    // buffers of bm x cin (+ two residual blocks of bm x 64), 160 KB per CU
    const int bm = d->cin == 64 ? 128 : 64;
    const int lds = 128 * d->cin + 4 * bm * d->cin + (r ? 256 * bm : 0);
    const int occ = std::min(3, 163840 / lds);
    const int ntiles = (int)((M + bm - 1) / bm);
    // one persistent workgroup per resident slot over all column blocks, a
    // multiple of 8 row slots so a row tile's column blocks share an XCD
    int gx = std::max(8, (occ * ncu / ny) / 8 * 8);
    gx = std::min(gx, ntiles);
    const dim3 grid(gx, ny);
    const uint16_t* res = (const uint16_t*)d->residual;
    uint16_t* o = (uint16_t*)d->out;
    const uint16_t* in = (const uint16_t*)d->in;
    const uint16_t* wt = (const uint16_t*)d->weight;
    const int mi = (int)M;
#define FAC_PW(TT, KC, RT, R) \
  conv_pw<TT, KC, RT, R><<<grid, 256, 0, st>>>(in, wt, d->bias, res, o, mi, k_pad, d->ldo, d->c_off, d->ldr, d->r_off, d->flags)
    if (d->dtype == FAC_DTYPE_BF16) {
      if (d->cin == 64) r ? FAC_PW(BF16, 2, 2, true) : FAC_PW(BF16, 2, 2, false);
      else if (d->cin == 128) r ? FAC_PW(BF16, 4, 1, true) : FAC_PW(BF16, 4, 1, false);
      else r ? FAC_PW(BF16, 8, 1, true) : FAC_PW(BF16, 8, 1, false);
    } else {
      if (d->cin == 64) r ? FAC_PW(F16, 2, 2, true) : FAC_PW(F16, 2, 2, false);
      else if (d->cin == 128) r ? FAC_PW(F16, 4, 1, true) : FAC_PW(F16, 4, 1, false);
      else r ? FAC_PW(F16, 8, 1, true) : FAC_PW(F16, 8, 1, false);
    }
#undef FAC_PW
    return hipGetLastError() == hipSuccess ? FAC_OK : FAC_ERR_HIP;
  }
  // S3D's temporal (kd,1,1) convs with 8 output frames: conv_tk (LDS slab per
  // 16 positions, the last one of a clip partial when 16 does not divide h*w)
  if (!split && d->kh == 1 && d->kw == 1 && d->sh == 1 && d->sw == 1 && d->ph == 0 && d->pw == 0 && d->od == 8 &&
      d->cin % 64 == 0 && d->cout % 64 == 0 && d->ldo % 4 == 0 &&
      d->c_off % 4 == 0 &&
      (d->flags & ~FAC_CONV_RELU) == 0 && k_pad == d->kd * d->cin) {
    const int ks = d->kd * d->cin / 32, slab = d->d * 16 * d->cin;
    const int db = ks * 2048 + 2 * slab <= 81920 ? 2 : (ks * 2048 + slab <= 81920 ? 1 : 0);
    const bool k3 = d->kd == 3 && d->sd == 1 && d->pd == 1 && d->d == 8;
    const bool k7 = d->kd == 7 && d->sd == 2 && d->pd == 3 && d->d == 16;
    // slices of KC 32-channel chunks (every chunk of a unit in one or two
    // steps: fewer per-step barriers and slice issues per MFMA), 3 ring slots
    const int tk2_kc = d->cin == 192 ? 3 : (d->cin == 128 ? 4 : 2);
    if ((k3 || k7) && (d->cin == 64 || d->cin == 128 || d->cin == 192) &&
        ks * 2048 + 128 + 3 * tk2_kc * d->d * 512 <= 81920 &&
        d->cin >= 64) {  // >= 2 slices per unit: at most R/2 store batches per wait window
      int dev = 0, ncu = 256;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
        ncu = 256;
      const int nunits = d->n * ((d->h * d->w + 15) / 16);
      const int nbk = d->cout / 64;
      const int nslot = (std::min(nunits, ncu) + 7) / 8 * 8;
      const dim3 grid(nslot * nbk);
      const int relu_on = (d->flags & FAC_CONV_RELU) != 0;
#define FAC_TK2(TT, DP, KD, SD, KC)                                                                          \
  conv_tk2<TT, DP, KD, SD, KC, 3><<<grid, 512, 0, st>>>((const uint16_t*)d->in, (const uint16_t*)d->weight, d->bias,  \
                                                 (uint16_t*)d->out, nunits, d->h * d->w, d->cin, k_pad, d->ldo, \
                                                 d->c_off, relu_on, nbk, nslot)
#define FAC_TK2W(TT, DP, KD, SD, KC, WR)                                                                       \
  conv_tk2<TT, DP, KD, SD, KC, 3, WR><<<grid, 512, 0, st>>>((const uint16_t*)d->in, (const uint16_t*)d->weight,  \
                                                            d->bias, (uint16_t*)d->out, nunits, d->h * d->w,      \
                                                            d->cin, k_pad, d->ldo, d->c_off, relu_on, nbk, nslot)
      if (d->dtype == FAC_DTYPE_BF16) {
        if (k7) FAC_TK2(BF16, 2, 7, 2, 2);
        else if (tk2_kc == 3 && g_tk_wreg) FAC_TK2W(BF16, 1, 3, 1, 6, 6);
        else if (tk2_kc == 3) FAC_TK2(BF16, 1, 3, 1, 3);
        else if (tk2_kc == 4 && g_tk_wreg) FAC_TK2W(BF16, 1, 3, 1, 4, 4);
        else if (tk2_kc == 4) FAC_TK2(BF16, 1, 3, 1, 4);
        else FAC_TK2(BF16, 1, 3, 1, 2);
      } else {
        if (k7) FAC_TK2(F16, 2, 7, 2, 2);
        else if (tk2_kc == 3 && g_tk_wreg) FAC_TK2W(F16, 1, 3, 1, 6, 6);
        else if (tk2_kc == 3) FAC_TK2(F16, 1, 3, 1, 3);
        else if (tk2_kc == 4 && g_tk_wreg) FAC_TK2W(F16, 1, 3, 1, 4, 4);
        else if (tk2_kc == 4) FAC_TK2(F16, 1, 3, 1, 4);
        else FAC_TK2(F16, 1, 3, 1, 2);
      }
#undef FAC_TK2
#undef FAC_TK2W
      return hipGetLastError() == hipSuccess ? FAC_OK : FAC_ERR_HIP;
    }
    if (db) {
      int dev = 0, ncu = 256;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
        ncu = 256;
      const int nunits = d->n * ((d->h * d->w + 15) / 16);
      const int nbk = d->cout / 64;
      // unit slots: a multiple of 8 (slot = 8 * hi + lo, see conv_tk), at most
      // one per CU and per unit
      const int nslot = (std::min(nunits, ncu) + 7) / 8 * 8;
      const dim3 grid(nslot * nbk);
      const int relu_on = (d->flags & FAC_CONV_RELU) != 0;
      if (d->dtype == FAC_DTYPE_BF16)
        conv_tk<BF16><<<grid, 512, 0, st>>>((const uint16_t*)d->in, (const uint16_t*)d->weight, d->bias,
                                            (uint16_t*)d->out, nunits, d->h * d->w, d->d, d->cin, d->kd, d->sd,
                                            d->pd, k_pad, d->ldo, d->c_off, relu_on, db, nbk, nslot);
      else
        conv_tk<F16><<<grid, 512, 0, st>>>((const uint16_t*)d->in, (const uint16_t*)d->weight, d->bias,
                                           (uint16_t*)d->out, nunits, d->h * d->w, d->d, d->cin, d->kd, d->sd,
                                           d->pd, k_pad, d->ldo, d->c_off, relu_on, db, nbk, nslot);
      return hipGetLastError() == hipSuccess ? FAC_OK : FAC_ERR_HIP;
    }
  }
  const hipError_t e = d->dtype == FAC_DTYPE_BF16 ? launch_convnd<BF16>(p, cout_pad, st) : launch_convnd<F16>(p, cout_pad, st);
  return e == hipSuccess ? FAC_OK : FAC_ERR_HIP;
}

int fac_conv_nd(const fac_conv_desc* d, void* stream) {
  return conv_nd_impl(d, nullptr, 0, INT_MAX, nullptr, 0, INT_MAX, stream);
}

static int conv_s2d4_clip_impl(const fac_conv_desc* d, const void* clip, bool u8, int h, int w, int pad_before,
                               void* stream) {
  using namespace fac;
  if (!d || !clip || !d->weight || !d->out || (d->dtype != FAC_DTYPE_BF16 && d->dtype != FAC_DTYPE_F16))
    return FAC_ERR_ARG;
  if ((d->flags & ~FAC_CONV_RELU) != 0 || h <= 0 || w <= 0 || h % 2 || w % 2 || pad_before < 0 || d->n <= 0 ||
      d->d <= 0)
    return FAC_ERR_ARG;
  int cout_pad, k_pad;
  fac_conv_weight_layout(d->cout, d->cin, d->kd, d->kh, d->kw, &cout_pad, &k_pad);
  // the conv fac_conv_nd would run on fac_pack_input_s2d(clip)'s cells: 4x4/1
  // over 16-channel cells, cout 64, no padding, dense output, 8x28 boxes
  const bool shape = d->kd == 1 && d->kh == 4 && d->kw == 4 && d->sd == 1 && d->sh == 1 && d->sw == 1 &&
                     d->pd == 0 && d->ph == 0 && d->pw == 0 && d->cin == 16 && d->cout == 64 && d->k_pad == k_pad &&
                     k_pad == 256 && d->od == d->d && d->oh == d->h - 3 && d->ow == d->w - 3 && d->oh % 8 == 0 &&
                     d->ow % 28 == 0 && d->ldo == 64 && d->c_off == 0 && d->h >= h / 2 + pad_before &&
                     d->w >= w / 2 + pad_before;
  if (!shape) return FAC_ERR_SHAPE;
  if ((long long)d->n * d->d * 3 * h * w >= (1LL << 40)) return FAC_ERR_SHAPE;
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      ncu <= 0)
    ncu = 256;
  const int nimg = d->n * d->od, nbox = nimg * (d->oh / 8) * (d->ow / 28);
  const int grid = std::min(nbox, 2 * ncu);
  const int relu_on = (d->flags & FAC_CONV_RELU) != 0;
  hipStream_t st = (hipStream_t)stream;
#define FAC_S2DC(TT, IN)                                                                                          \
  conv_s2d4<TT, IN><<<grid, 256, 0, st>>>(clip, (const uint16_t*)d->weight, d->bias, (uint16_t*)d->out, nbox, d->h, \
                                          d->w, d->oh, d->ow, k_pad, relu_on, d->d, h, w, pad_before)
  if (d->dtype == FAC_DTYPE_BF16) u8 ? FAC_S2DC(BF16, 2) : FAC_S2DC(BF16, 1);
  else u8 ? FAC_S2DC(F16, 2) : FAC_S2DC(F16, 1);
#undef FAC_S2DC
  return hipGetLastError() == hipSuccess ? FAC_OK : FAC_ERR_HIP;
}

int fac_conv_s2d4_clip(const fac_conv_desc* d, const float* clip, int h, int w, int pad_before, void* stream) {
  return conv_s2d4_clip_impl(d, clip, false, h, w, pad_before, stream);
}

int fac_conv_s2d4_clip_u8(const fac_conv_desc* d, const uint8_t* clip, int h, int w, int pad_before, void* stream) {
  return conv_s2d4_clip_impl(d, clip, true, h, w, pad_before, stream);
}

int fac_s3d_base0_u8(const fac_conv_desc* sdsc, const fac_conv_desc* tdsc, const uint8_t* clip, int h, int w,
                     int pad_before, void* stream) {
  using namespace fac;
  if (!sdsc || !tdsc || !clip || !sdsc->weight || !tdsc->weight || !tdsc->out || sdsc->dtype != tdsc->dtype ||
      (sdsc->dtype != FAC_DTYPE_BF16 && sdsc->dtype != FAC_DTYPE_F16))
    return FAC_ERR_ARG;
  if (((sdsc->flags | tdsc->flags) & ~FAC_CONV_RELU) != 0 || pad_before < 0) return FAC_ERR_ARG;
  int cps, kps, cpt, kpt;
  fac_conv_weight_layout(sdsc->cout, sdsc->cin, sdsc->kd, sdsc->kh, sdsc->kw, &cps, &kps);
  fac_conv_weight_layout(tdsc->cout, tdsc->cin, tdsc->kd, tdsc->kh, tdsc->kw, &cpt, &kpt);
  // the spatial half as fac_conv_s2d4_clip_u8 takes it (4x4/1 over 16-channel
  // cells of 16 frames, a 56 x 56 output), the temporal half as conv_tk2<2,7,2>
  const bool sp = sdsc->kd == 1 && sdsc->kh == 4 && sdsc->kw == 4 && sdsc->sd == 1 && sdsc->sh == 1 && sdsc->sw == 1 &&
                  sdsc->pd == 0 && sdsc->ph == 0 && sdsc->pw == 0 && sdsc->cin == 16 && sdsc->cout == 64 &&
                  sdsc->k_pad == kps && kps == 256 && sdsc->d == 16 && sdsc->od == 16 && sdsc->oh == 56 &&
                  sdsc->ow == 56 && sdsc->h == 59 && sdsc->w == 59 && h % 2 == 0 && w % 2 == 0 &&
                  sdsc->h >= h / 2 + pad_before && sdsc->w >= w / 2 + pad_before;
  const bool tp = tdsc->kd == 7 && tdsc->kh == 1 && tdsc->kw == 1 && tdsc->sd == 2 && tdsc->sh == 1 && tdsc->sw == 1 &&
                  tdsc->pd == 3 && tdsc->ph == 0 && tdsc->pw == 0 && tdsc->cin == 64 && tdsc->cout == 64 &&
                  tdsc->k_pad == kpt && kpt == 7 * 64 && tdsc->n == sdsc->n && tdsc->d == 16 && tdsc->h == 56 &&
                  tdsc->w == 56 && tdsc->od == 8 && tdsc->oh == 56 && tdsc->ow == 56 && tdsc->ldo == 64 &&
                  tdsc->c_off == 0;
  if (!sp || !tp || sdsc->n <= 0) return FAC_ERR_SHAPE;
  if ((long long)sdsc->n * 16 * 3 * h * w >= (1LL << 40)) return FAC_ERR_SHAPE;
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      ncu <= 0)
    ncu = 256;
  const int nunits = sdsc->n * (56 / 2) * (56 / 8);
  const int grid = std::min(nunits, ncu);
  const int rs = (sdsc->flags & FAC_CONV_RELU) != 0, rt = (tdsc->flags & FAC_CONV_RELU) != 0;
  hipStream_t st = (hipStream_t)stream;
  if (sdsc->dtype == FAC_DTYPE_BF16)
    s3d_base0<BF16><<<grid, 512, 0, st>>>(clip, (const uint16_t*)sdsc->weight, sdsc->bias, kps,
                                          (const uint16_t*)tdsc->weight, tdsc->bias, kpt, (uint16_t*)tdsc->out,
                                          nunits, h, w, pad_before, rs, rt);
  else
    s3d_base0<F16><<<grid, 512, 0, st>>>(clip, (const uint16_t*)sdsc->weight, sdsc->bias, kps,
                                         (const uint16_t*)tdsc->weight, tdsc->bias, kpt, (uint16_t*)tdsc->out,
                                         nunits, h, w, pad_before, rs, rt);
  return hipGetLastError() == hipSuccess ? FAC_OK : FAC_ERR_HIP;
}

int fac_sep_tiny(const fac_conv_desc* sdsc, const fac_conv_desc* tdsc, void* stream) {
  using namespace fac;
  if (!sdsc || !tdsc || !sdsc->in || !sdsc->weight || !tdsc->weight || !tdsc->out || sdsc->dtype != tdsc->dtype ||
      (sdsc->dtype != FAC_DTYPE_BF16 && sdsc->dtype != FAC_DTYPE_F16))
    return FAC_ERR_ARG;
  if (((sdsc->flags | tdsc->flags) & ~FAC_CONV_RELU) != 0) return FAC_ERR_ARG;
  int cps, kps, cpt, kpt;
  fac_conv_weight_layout(sdsc->cout, sdsc->cin, sdsc->kd, sdsc->kh, sdsc->kw, &cps, &kps);
  fac_conv_weight_layout(tdsc->cout, tdsc->cin, tdsc->kd, tdsc->kh, tdsc->kw, &cpt, &kpt);
  const bool sp = sdsc->cin == 16 && sdsc->cout == 32 && sdsc->kd == 1 && sdsc->kh == 3 && sdsc->kw == 3 &&
                  sdsc->sd == 1 && sdsc->sh == 1 && sdsc->sw == 1 && sdsc->pd == 0 && sdsc->ph == 1 && sdsc->pw == 1 &&
                  sdsc->d == 8 && sdsc->h == 14 && sdsc->w == 14 && sdsc->od == 8 && sdsc->oh == 14 && sdsc->ow == 14 &&
                  sdsc->k_pad == kps && kps == 192 && sdsc->n > 0;
  const bool tp = tdsc->cin == 32 && tdsc->cout == 32 && tdsc->kd == 3 && tdsc->kh == 1 && tdsc->kw == 1 &&
                  tdsc->sd == 1 && tdsc->sh == 1 && tdsc->sw == 1 && tdsc->pd == 1 && tdsc->ph == 0 && tdsc->pw == 0 &&
                  tdsc->n == sdsc->n && tdsc->d == 8 && tdsc->h == 14 && tdsc->w == 14 && tdsc->od == 8 &&
                  tdsc->oh == 14 && tdsc->ow == 14 && tdsc->k_pad == kpt && kpt == 128 && tdsc->ldo % 8 == 0 &&
                  tdsc->c_off % 8 == 0 && tdsc->ldo >= tdsc->c_off + 32;
  if (!sp || !tp) return FAC_ERR_SHAPE;
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      ncu <= 0)
    ncu = 256;
  const int grid = std::min(sdsc->n, ncu);
  const int rs = (sdsc->flags & FAC_CONV_RELU) != 0, rt = (tdsc->flags & FAC_CONV_RELU) != 0;
  hipStream_t st = (hipStream_t)stream;
  if (sdsc->dtype == FAC_DTYPE_BF16)
    sep_tiny<BF16><<<grid, 512, 0, st>>>((const uint16_t*)sdsc->in, (const uint16_t*)sdsc->weight, sdsc->bias, kps,
                                         (const uint16_t*)tdsc->weight, tdsc->bias, kpt, (uint16_t*)tdsc->out, sdsc->n,
                                         tdsc->ldo, tdsc->c_off, rs, rt);
  else
    sep_tiny<F16><<<grid, 512, 0, st>>>((const uint16_t*)sdsc->in, (const uint16_t*)sdsc->weight, sdsc->bias, kps,
                                        (const uint16_t*)tdsc->weight, tdsc->bias, kpt, (uint16_t*)tdsc->out, sdsc->n,
                                        tdsc->ldo, tdsc->c_off, rs, rt);
  return hipGetLastError() == hipSuccess ? FAC_OK : FAC_ERR_HIP;
}

int fac_sep_mid(const fac_conv_desc* sdsc, const fac_conv_desc* tdsc, void* stream) {
  using namespace fac;
  if (!sdsc || !tdsc || !sdsc->in || !sdsc->weight || !tdsc->weight || !tdsc->out || sdsc->dtype != tdsc->dtype ||
      (sdsc->dtype != FAC_DTYPE_BF16 && sdsc->dtype != FAC_DTYPE_F16))
    return FAC_ERR_ARG;
  if (((sdsc->flags | tdsc->flags) & ~FAC_CONV_RELU) != 0) return FAC_ERR_ARG;
  int cps, kps, cpt, kpt;
  fac_conv_weight_layout(sdsc->cout, sdsc->cin, sdsc->kd, sdsc->kh, sdsc->kw, &cps, &kps);
  fac_conv_weight_layout(tdsc->cout, tdsc->cin, tdsc->kd, tdsc->kh, tdsc->kw, &cpt, &kpt);
  const bool sp = sdsc->cin == 32 && sdsc->cout == 128 && sdsc->kd == 1 && sdsc->kh == 3 && sdsc->kw == 3 &&
                  sdsc->sd == 1 && sdsc->sh == 1 && sdsc->sw == 1 && sdsc->pd == 0 && sdsc->ph == 1 && sdsc->pw == 1 &&
                  sdsc->d == 8 && sdsc->h == 14 && sdsc->w == 14 && sdsc->od == 8 && sdsc->oh == 14 && sdsc->ow == 14 &&
                  sdsc->k_pad == kps && kps == 320 && sdsc->n > 0;
  const bool tp = tdsc->cin == 128 && tdsc->cout == 96 && tdsc->kd == 3 && tdsc->kh == 1 && tdsc->kw == 1 &&
                  tdsc->sd == 1 && tdsc->sh == 1 && tdsc->sw == 1 && tdsc->pd == 1 && tdsc->ph == 0 && tdsc->pw == 0 &&
                  tdsc->n == sdsc->n && tdsc->d == 8 && tdsc->h == 14 && tdsc->w == 14 && tdsc->od == 8 &&
                  tdsc->oh == 14 && tdsc->ow == 14 && tdsc->k_pad == kpt && kpt == 384 && tdsc->ldo % 8 == 0 &&
                  tdsc->c_off % 8 == 0 && tdsc->ldo >= tdsc->c_off + 96;
  if (!sp || !tp) return FAC_ERR_SHAPE;
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      ncu <= 0)
    ncu = 256;
  const int nunits = sdsc->n * 7, grid = std::min(nunits, 2 * ncu);
  const int rs = (sdsc->flags & FAC_CONV_RELU) != 0, rt = (tdsc->flags & FAC_CONV_RELU) != 0;
  hipStream_t st = (hipStream_t)stream;
  if (sdsc->dtype == FAC_DTYPE_BF16)
    sep_mid<BF16><<<grid, 384, 0, st>>>((const uint16_t*)sdsc->in, (const uint16_t*)sdsc->weight, sdsc->bias, kps,
                                        (const uint16_t*)tdsc->weight, tdsc->bias, kpt, (uint16_t*)tdsc->out, nunits,
                                        tdsc->ldo, tdsc->c_off, rs, rt);
  else
    sep_mid<F16><<<grid, 384, 0, st>>>((const uint16_t*)sdsc->in, (const uint16_t*)sdsc->weight, sdsc->bias, kps,
                                       (const uint16_t*)tdsc->weight, tdsc->bias, kpt, (uint16_t*)tdsc->out, nunits,
                                       tdsc->ldo, tdsc->c_off, rs, rt);
  return hipGetLastError() == hipSuccess ? FAC_OK : FAC_ERR_HIP;
}

int fac_conv_nd_split(const fac_conv_desc* d, void* out1, int ldo1, int split1, void* out2, int ldo2, int split2,
                      void* stream) {
  if (!d || !out1 || !out2 || split1 <= 0 || split1 % 8 || split2 <= split1 || split2 % 8 || split2 >= d->cout ||
      ldo1 < split2 - split1 || ldo2 < d->cout - split2 || (d->flags & (FAC_CONV_RESID | FAC_CONV_OUT_F32)) ||
      d->ldo < d->c_off + split1)
    return FAC_ERR_ARG;
  return conv_nd_impl(d, out1, ldo1, split1, out2, ldo2, split2, stream);
}

// the ConvP of a uniform-tap conv for convnd_pt (fac_conv_nd_dual); false if
// the descriptor is malformed or not uniform-tap (cin % 64)
static bool dual_convp(const fac_conv_desc* d, fac::ConvP& p, bool need_out) {
  if (!d || !d->in || !d->weight || (need_out && !d->out)) return false;
  if (d->cin <= 0 || d->cin % 64 || d->cout <= 0 || d->n <= 0 || d->d <= 0 || d->h <= 0 || d->w <= 0) return false;
  if (d->kd <= 0 || d->kh <= 0 || d->kw <= 0 || d->sd <= 0 || d->sh <= 0 || d->sw <= 0) return false;
  if (d->pd < 0 || d->ph < 0 || d->pw < 0) return false;
  if (d->od != (d->d + 2 * d->pd - d->kd) / d->sd + 1 || d->oh != (d->h + 2 * d->ph - d->kh) / d->sh + 1 ||
      d->ow != (d->w + 2 * d->pw - d->kw) / d->sw + 1)
    return false;
  int cout_pad, k_pad;
  fac_conv_weight_layout(d->cout, d->cin, d->kd, d->kh, d->kw, &cout_pad, &k_pad);
  if (d->k_pad != k_pad) return false;
  const long long M = (long long)d->n * d->od * d->oh * d->ow;
  if (M >= (1LL << 31) || (long long)d->n * d->d * d->h * d->w * d->cin >= (1LL << 40)) return false;
  p = fac::ConvP{};
  p.in = (const uint16_t*)d->in;
  p.w = (const uint16_t*)d->weight;
  p.bias = d->bias;
  p.out = d->out;
  p.D = d->d;
  p.H = d->h;
  p.W = d->w;
  p.C8 = d->cin / 8;
  p.Do = d->od;
  p.Ho = d->oh;
  p.Wo = d->ow;
  p.Cout = d->cout;
  p.KD = d->kd;
  p.KH = d->kh;
  p.KW = d->kw;
  p.SD = d->sd;
  p.SH = d->sh;
  p.SW = d->sw;
  p.PD = d->pd;
  p.PH = d->ph;
  p.PW = d->pw;
  p.Kp = k_pad;
  p.ksteps = k_pad / 64;
  p.ktot8 = d->kd * d->kh * d->kw * (d->cin / 8);
  p.ldo = d->ldo;
  p.c_off = d->c_off;
  p.flags = d->flags;
  p.vec_out = (d->ldo % 8 == 0 && d->c_off % 8 == 0) ? 1 : 0;
  p.M = (int)M;
  p.split1 = p.split2 = INT_MAX;
  return true;
}

int fac_conv_nd_dual(const fac_conv_desc* d, const fac_conv_desc* ds, void* stream) {
  using namespace fac;
  if (!d || !ds || d->dtype != ds->dtype || (d->dtype != FAC_DTYPE_BF16 && d->dtype != FAC_DTYPE_F16)) return FAC_ERR_ARG;
  if ((d->flags & ~(FAC_CONV_RELU | FAC_CONV_RELU2)) || ds->flags != 0) return FAC_ERR_ARG;
  ConvP p, q;
  if (!dual_convp(d, p, true) || !dual_convp(ds, q, false)) return FAC_ERR_SHAPE;
  if (d->n != ds->n || d->od != ds->od || d->oh != ds->oh || d->ow != ds->ow || d->cout != ds->cout ||
      d->cout % 128 || !p.vec_out || d->ldo < d->c_off + d->cout)
    return FAC_ERR_SHAPE;
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
    ncu = 256;
  // layer1's first block (64 -> 256 twice, the downsample at stride 1 over
  // the same positions): pw_res DUAL
  if (g_pw_res && d->cin == 64 && ds->cin == 64 && d->cout % 256 == 0 && p.KD * p.KH * p.KW == 1 &&
      q.KD * q.KH * q.KW == 1 && p.SD * p.SH * p.SW == 1 && q.SD * q.SH * q.SW == 1 && !p.PD && !p.PH && !p.PW &&
      !q.PD && !q.PH && !q.PW && p.Kp == 64 && q.Kp == 64) {
    const int ny2 = d->cout / 256, G2 = std::max(ny2, ncu / ny2 * ny2);
    const int r1 = (d->flags & FAC_CONV_RELU) != 0, r2 = (d->flags & FAC_CONV_RELU2) != 0;
    hipStream_t st2 = (hipStream_t)stream;
#define FAC_PWD(TT)                                                                                                     \
  pw_res<TT, 2, 256, 128, 1><<<G2, 512, 0, st2>>>(p.in, p.w, p.bias, nullptr, (uint16_t*)p.out, p.M, 64, p.ldo,           \
                                                   p.c_off, 0, 0, ny2, r1, r2, q.in, q.w, q.bias, INT_MAX, nullptr, 0, INT_MAX, \
                                                   nullptr, 0, INT_MAX)
    if (d->dtype == FAC_DTYPE_BF16) FAC_PWD(BF16);
    else FAC_PWD(F16);
#undef FAC_PWD
    return hipGetLastError() == hipSuccess ? FAC_OK : FAC_ERR_HIP;
  }
  // layer2's first block (conv3 128 -> 512 at 28^2, the downsample 256 -> 512
  // at stride 2 over the 56^2 block input): pw_dual2
  if (g_pw_res == 1 && ((d->cin == 128 && ds->cin == 256) || (d->cin == 256 && ds->cin == 512)) && d->cout % PWD2_BN == 0 && p.KD * p.KH * p.KW == 1 && q.KD * q.KH * q.KW == 1 &&
      p.SD * p.SH * p.SW == 1 && q.SD == 1 && q.SH == q.SW && q.SH >= 1 && !p.PD && !p.PH && !p.PW && !q.PD &&
      !q.PH && !q.PW && p.Kp == d->cin && q.Kp == ds->cin && p.D == 1 && q.D == 1 &&
      (long long)q.H * q.W * d->n < (1LL << 31)) {  // (x positions as int)
    const int ny2 = d->cout / PWD2_BN, G2 = std::max(ny2, ncu / ny2 * ny2);
    const int r1 = (d->flags & FAC_CONV_RELU) != 0, r2 = (d->flags & FAC_CONV_RELU2) != 0;
    hipStream_t st2 = (hipStream_t)stream;
#define FAC_PWD2(TT, K3, KD, CW)                                                                              \
  pw_dual2<TT, K3, KD, CW><<<G2, 512, 0, st2>>>(p.in, p.w, p.bias, q.in, q.w, q.bias, (uint16_t*)p.out, p.M, K3, KD, \
                                                 p.ldo, p.c_off, ny2, p.Ho, p.Wo, q.H, q.W, q.SH, r1, r2)
    if (d->cin == 128) {
      if (d->dtype == FAC_DTYPE_BF16) FAC_PWD2(BF16, 128, 256, 64);
      else FAC_PWD2(F16, 128, 256, 64);
    } else {
      if (d->dtype == FAC_DTYPE_BF16) FAC_PWD2(BF16, 256, 512, 32);
      else FAC_PWD2(F16, 256, 512, 32);
    }
#undef FAC_PWD2
    return hipGetLastError() == hipSuccess ? FAC_OK : FAC_ERR_HIP;
  }
  // 128-wide tiles: the 256-wide DUAL variant needs 256+ VGPRs and spills
  // (scratch traffic would also break the hand-counted vmcnt waits)
  const int nrt = (p.M + 255) / 256, ny = p.Cout / 128;
  int G = ncu / ny * ny;
  if ((long long)nrt * ny < G) G = nrt * ny;
  if (G <= 0) return FAC_ERR_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  if (d->dtype == FAC_DTYPE_BF16) convnd_pt<BF16, 128, false, true><<<G, 512, 0, st>>>(p, q);
  else convnd_pt<F16, 128, false, true><<<G, 512, 0, st>>>(p, q);
  return hipGetLastError() == hipSuccess ? FAC_OK : FAC_ERR_HIP;
}

int fac_bottleneck_pw2(const fac_conv_desc* c3, const fac_conv_desc* c1, void* stream) {
  using namespace fac;
  if (!c3 || !c1 || !c3->in || !c3->weight || !c3->bias || !c3->out || !c3->residual || !c1->weight || !c1->bias ||
      !c1->out)
    return FAC_ERR_ARG;
  if (c3->dtype != c1->dtype || (c3->dtype != FAC_DTYPE_BF16 && c3->dtype != FAC_DTYPE_F16)) return FAC_ERR_ARG;
  if (c3->flags != (FAC_CONV_RELU | FAC_CONV_RESID | FAC_CONV_RELU2) || c1->flags != FAC_CONV_RELU) return FAC_ERR_ARG;
  auto pw = [](const fac_conv_desc* d) {
    return d->kd == 1 && d->kh == 1 && d->kw == 1 && d->sd == 1 && d->sh == 1 && d->sw == 1 && d->pd == 0 &&
           d->ph == 0 && d->pw == 0 && d->od == d->d && d->oh == d->h && d->ow == d->w && d->c_off == 0;
  };
  const bool l1 = c3->cin == 64 && c3->cout == 256 && c3->k_pad == 64 && c1->cin == 256 && c1->k_pad == 256 &&
                  (c1->cout == 64 || c1->cout == 128);
  const bool l2 = c3->cin == 128 && c3->cout == 512 && c3->k_pad == 128 && c1->cin == 512 && c1->k_pad == 512 &&
                  c1->cout == 128;
  if (!pw(c3) || !pw(c1) || !(l1 || l2) || c3->ldo != c3->cout || c1->ldo != c1->cout) return FAC_ERR_SHAPE;
  if (c1->n != c3->n || c1->d != c3->d || c1->h != c3->h || c1->w != c3->w) return FAC_ERR_SHAPE;
  if (c3->ldr % 8 || c3->r_off % 8 || c3->ldr < c3->r_off + c3->cout) return FAC_ERR_SHAPE;
  const long long M = (long long)c3->n * c3->d * c3->h * c3->w;
  if (M <= 0 || M >= (1LL << 31)) return FAC_ERR_SHAPE;
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
    ncu = 256;
  hipStream_t st = (hipStream_t)stream;
  if (l2) {
    const int grid = (int)std::min<long long>((M + 15) / 16, ncu);
    if (c3->dtype == FAC_DTYPE_BF16)
      bneck_pw2_l2<BF16><<<grid, 512, 0, st>>>((const uint16_t*)c3->in, (const uint16_t*)c3->weight, c3->bias,
                                               (const uint16_t*)c3->residual, (const uint16_t*)c1->weight, c1->bias,
                                               (uint16_t*)c3->out, (uint16_t*)c1->out, (int)M, c3->k_pad, c1->k_pad,
                                               c3->ldr, c3->r_off);
    else
      bneck_pw2_l2<F16><<<grid, 512, 0, st>>>((const uint16_t*)c3->in, (const uint16_t*)c3->weight, c3->bias,
                                              (const uint16_t*)c3->residual, (const uint16_t*)c1->weight, c1->bias,
                                              (uint16_t*)c3->out, (uint16_t*)c1->out, (int)M, c3->k_pad, c1->k_pad,
                                              c3->ldr, c3->r_off);
    return hipGetLastError() == hipSuccess ? FAC_OK : FAC_ERR_HIP;
  }
  const int ntiles = (int)((M + 63) / 64), grid = std::min(ntiles, ncu);
#define FAC_PW2(TT, N)                                                                                           \
  bneck_pw2<TT, N><<<grid, 512, 0, st>>>((const uint16_t*)c3->in, (const uint16_t*)c3->weight, c3->bias,         \
                                         (const uint16_t*)c3->residual, (const uint16_t*)c1->weight, c1->bias,   \
                                         (uint16_t*)c3->out, (uint16_t*)c1->out, (int)M, c3->k_pad, c1->k_pad,   \
                                         c3->ldr, c3->r_off)
  if (c3->dtype == FAC_DTYPE_BF16) {
    if (c1->cout == 64) FAC_PW2(BF16, 64);
    else FAC_PW2(BF16, 128);
  } else {
    if (c1->cout == 64) FAC_PW2(F16, 64);
    else FAC_PW2(F16, 128);
  }
#undef FAC_PW2
  return hipGetLastError() == hipSuccess ? FAC_OK : FAC_ERR_HIP;
}

int fac_pool_nd(const fac_pool_desc* d, void* stream) {
  using namespace fac;
  if (!d || !d->in || !d->out) return FAC_ERR_ARG;
  if (d->dtype != FAC_DTYPE_BF16 && d->dtype != FAC_DTYPE_F16) return FAC_ERR_ARG;
  if (d->c <= 0 || d->c % 8 || d->n <= 0 || d->od <= 0 || d->oh <= 0 || d->ow <= 0 || d->mode < 0 || d->mode > 1)
    return FAC_ERR_SHAPE;
  if (d->kd <= 0 || d->kh <= 0 || d->kw <= 0 || d->sd <= 0 || d->sh <= 0 || d->sw <= 0) return FAC_ERR_SHAPE;
  if (d->ldo % 8 || d->c_off % 8 || d->ldo < d->c_off + d->c) return FAC_ERR_SHAPE;
  const long long total = (long long)d->n * d->od * d->oh * d->ow * (d->c / 8);
  if (total >= (1LL << 31)) return FAC_ERR_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  if (d->mode == 0 && d->kd == 3 && d->kh == 3 && d->kw == 3 && d->sd == 1 && d->sh == 1 && d->sw == 1 &&
      d->pd == 1 && d->ph == 1 && d->pw == 1 && d->od == d->d && d->oh == d->h && d->ow == d->w) {
    if (g_pool_lds14 && d->h == 14 && d->w == 14 && d->c % 64 == 0 && d->ldo % 8 == 0) {
      const long long nwg = (long long)d->n * (d->c / 64);
      if (nwg >= (1LL << 31)) return FAC_ERR_SHAPE;
      if (d->dtype == FAC_DTYPE_BF16)
        maxpool3_lds14<BF16><<<(int)nwg, 256, 0, st>>>(*d);
      else
        maxpool3_lds14<F16><<<(int)nwg, 256, 0, st>>>(*d);
      return hipGetLastError() == hipSuccess ? FAC_OK : FAC_ERR_HIP;
    }
    if (g_pool_roll && d->w == 7) {
      const int zg = g_pool_roll == 1 ? d->d : std::min(g_pool_roll, d->d);
      const long long rows = (long long)d->n * ((d->d + zg - 1) / zg) * d->h * (d->c / 8);
      if (rows >= (1LL << 31)) return FAC_ERR_SHAPE;
      const int nb = (int)((rows + 255) / 256);
      if (d->dtype == FAC_DTYPE_BF16)
        maxpool3_roll<BF16, 7><<<nb, 256, 0, st>>>(*d, (int)rows, zg);
      else
        maxpool3_roll<F16, 7><<<nb, 256, 0, st>>>(*d, (int)rows, zg);
      return hipGetLastError() == hipSuccess ? FAC_OK : FAC_ERR_HIP;
    }
    const int zg = g_pool3_zg > 0 ? std::min(g_pool3_zg, d->d) : d->d;  // output frames per thread (default all)
    const long long cols = (long long)d->n * ((d->d + zg - 1) / zg) * d->h * d->w * (d->c / 8);
    if (cols >= (1LL << 31)) return FAC_ERR_SHAPE;
    const int nb = (int)((cols + 255) / 256);
    if (d->dtype == FAC_DTYPE_BF16)
      maxpool3_s1<BF16><<<nb, 256, 0, st>>>(*d, (int)cols, zg);
    else
      maxpool3_s1<F16><<<nb, 256, 0, st>>>(*d, (int)cols, zg);
    return hipGetLastError() == hipSuccess ? FAC_OK : FAC_ERR_HIP;
  }
  const int nb = (int)((total + 255) / 256);
  // compile-time windows (branch-free taps) for the max pools of S3D / ResNet:
  // floor-mode output dims and padding below the window keep a valid tap in
  // every window (pool_nd takes anything else)
  const bool floor_dims = d->od == (d->d + 2 * d->pd - d->kd) / d->sd + 1 &&
                          d->oh == (d->h + 2 * d->ph - d->kh) / d->sh + 1 &&
                          d->ow == (d->w + 2 * d->pw - d->kw) / d->sw + 1 && d->pd >= 0 && d->ph >= 0 &&
                          d->pw >= 0 && d->pd < d->kd && d->ph < d->kh && d->pw < d->kw;
  if (d->mode == 0 && g_pool_win && floor_dims) {
    const bool bf = d->dtype == FAC_DTYPE_BF16;
#define FAC_WIN(KD, KH, KW)                                                                                      \
  if (d->kd == KD && d->kh == KH && d->kw == KW) {                                                            \
    if (bf) pool_max_win<BF16, KD, KH, KW><<<nb, 256, 0, st>>>(*d, (int)total);                               \
    else pool_max_win<F16, KD, KH, KW><<<nb, 256, 0, st>>>(*d, (int)total);                                   \
    return hipGetLastError() == hipSuccess ? FAC_OK : FAC_ERR_HIP;                                            \
  }
    FAC_WIN(1, 3, 3)
    FAC_WIN(3, 3, 3)
    FAC_WIN(2, 2, 2)
#undef FAC_WIN
  }
  if (d->dtype == FAC_DTYPE_BF16)
    pool_nd<BF16><<<nb, 256, 0, st>>>(*d, (int)total);
  else
    pool_nd<F16><<<nb, 256, 0, st>>>(*d, (int)total);
  return hipGetLastError() == hipSuccess ? FAC_OK : FAC_ERR_HIP;
}

int fac_pack_input(int dtype, const void* src, int src_kind, int n, int s, float div, const float* mean3,
                   const float* std3, void* out, int c_pad, void* stream) {
  using namespace fac;
  if (!src || !out || n <= 0 || s <= 0 || c_pad < 8 || c_pad % 8 || (src_kind != 0 && src_kind != 1) || !(div > 0.f))
    return FAC_ERR_ARG;
  if (dtype != FAC_DTYPE_BF16 && dtype != FAC_DTYPE_F16) return FAC_ERR_ARG;
  const float m[3] = {mean3 ? mean3[0] : 0.f, mean3 ? mean3[1] : 0.f, mean3 ? mean3[2] : 0.f};
  const float sd[3] = {std3 ? std3[0] : 1.f, std3 ? std3[1] : 1.f, std3 ? std3[2] : 1.f};
  const long long total = (long long)n * s;
  const int nb = (int)((total + 255) / 256);
  hipStream_t st = (hipStream_t)stream;
  uint16_t* o = (uint16_t*)out;
#define FAC_PACK(TT, U)                                                                                      \
  pack_input<TT, U><<<nb, 256, 0, st>>>(src, n, s, div, m[0], m[1], m[2], sd[0], sd[1], sd[2], o, c_pad)
  if (dtype == FAC_DTYPE_BF16) {
    if (src_kind == 0) FAC_PACK(BF16, true); else FAC_PACK(BF16, false);
  } else {
    if (src_kind == 0) FAC_PACK(F16, true); else FAC_PACK(F16, false);
  }
#undef FAC_PACK
  return hipGetLastError() == hipSuccess ? FAC_OK : FAC_ERR_HIP;
}

int fac_pack_input_s2d(int dtype, const void* src, int src_kind, int n, int frames, int h, int w, int pad_before,
                       int pad_after, float div, const float* mean3, const float* std3, void* out, void* stream) {
  using namespace fac;
  if (!src || !out || n <= 0 || frames <= 0 || h <= 0 || w <= 0 || h % 2 || w % 2 || pad_before < 0 || pad_after < 0 ||
      (src_kind != 0 && src_kind != 1) || !(div > 0.f))
    return FAC_ERR_ARG;
  if (dtype != FAC_DTYPE_BF16 && dtype != FAC_DTYPE_F16) return FAC_ERR_ARG;
  const float m[3] = {mean3 ? mean3[0] : 0.f, mean3 ? mean3[1] : 0.f, mean3 ? mean3[2] : 0.f};
  const float sd[3] = {std3 ? std3[0] : 1.f, std3 ? std3[1] : 1.f, std3 ? std3[2] : 1.f};
  const long long total =
      (long long)n * frames * (h / 2 + pad_before + pad_after) * (w / 2 + pad_before + pad_after);
  if (total >= (1LL << 31) - 256) return FAC_ERR_SHAPE;  // the kernel indexes cells in 32 bits
  const int nb = (int)((total + 255) / 256);
  hipStream_t st = (hipStream_t)stream;
  uint16_t* o = (uint16_t*)out;
#define FAC_PACK(TT, U)                                                                                         \
  pack_input_s2d<TT, U><<<nb, 256, 0, st>>>(src, n * frames, frames, h, w, pad_before, pad_after, div, m[0], \
                                            m[1], m[2], sd[0], sd[1], sd[2], o)
  if (dtype == FAC_DTYPE_BF16) {
    if (src_kind == 0) FAC_PACK(BF16, true); else FAC_PACK(BF16, false);
  } else {
    if (src_kind == 0) FAC_PACK(F16, true); else FAC_PACK(F16, false);
  }
#undef FAC_PACK
  return hipGetLastError() == hipSuccess ? FAC_OK : FAC_ERR_HIP;
}

size_t fac_kan_scratch_bytes(int rows, int in_f, int out_f) {
  if (rows <= 0 || in_f <= 0 || out_f <= 0) return 0;
  const size_t chunks = (in_f + fac::kKanIn - 1) / fac::kKanIn;
  return chunks * rows * out_f * sizeof(float);
}

int fac_kan_linear(const float* x, int rows, int in_f, int out_f, const float* grid, int n_knots, const float* wcat,
                   float* y, void* partial, void* stream) {
  using namespace fac;
  if (!x || !grid || !wcat || !y || !partial || rows <= 0 || in_f <= 0 || out_f <= 0) return FAC_ERR_ARG;
  if (n_knots != kKanNK) return FAC_ERR_SHAPE;  // grid_size 5, spline_order 3 (kan.py:21-22)
  const int chunks = (in_f + kKanIn - 1) / kKanIn;
  hipStream_t st = (hipStream_t)stream;
  kan_partial<<<dim3(chunks, (rows + kKanRows - 1) / kKanRows), 256, 0, st>>>(x, rows, in_f, out_f, grid, wcat,
                                                                              (float*)partial);
  const int n = rows * out_f;
  kan_reduce<<<(n + 255) / 256, 256, 0, st>>>((const float*)partial, chunks, n, y);
  return hipGetLastError() == hipSuccess ? FAC_OK : FAC_ERR_HIP;
}

int fac_sigmoid(const float* x, float* y, int n, void* stream) {
  if (!x || !y || n <= 0) return FAC_ERR_ARG;
  fac::sigmoid_k<<<(n + 255) / 256, 256, 0, (hipStream_t)stream>>>(x, y, n);
  return hipGetLastError() == hipSuccess ? FAC_OK : FAC_ERR_HIP;
}

int fac_ggca(int dtype, const void* x, int n, int h, int w, int c, int groups, const float* w1, const float* b1,
             const float* bn4, const float* w2, const float* b2, void* out, void* stream) {
  if (!x || !out || !w1 || !b1 || !bn4 || !w2 || !b2 || n <= 0 || h <= 0 || w <= 0 || groups <= 0 || c % groups)
    return FAC_ERR_ARG;
  const int cg = c / groups;
  if (h > 16 || w > 16 || cg % 16 || cg > 256 || h * w * cg > 16384 || (2 * h + 2 * w) * cg > 8192 ||
      (2 * h + 2 * w) > 64)
    return FAC_ERR_SHAPE;
  const hipStream_t st = (hipStream_t)stream;
  if (dtype == 0)
    fac::ggca_k<fac::BF16><<<n * groups, 256, 0, st>>>((const uint16_t*)x, h, w, c, groups, w1, b1, bn4, w2, b2,
                                                      (uint16_t*)out);
  else
    fac::ggca_k<fac::F16><<<n * groups, 256, 0, st>>>((const uint16_t*)x, h, w, c, groups, w1, b1, bn4, w2, b2,
                                                     (uint16_t*)out);
  return hipGetLastError() == hipSuccess ? FAC_OK : FAC_ERR_HIP;
}

}  // extern "C"
