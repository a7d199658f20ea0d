// conv3x3_wino: the 14x14 / 28x28 3x3 convs of the CViT stem (cvit.py:110-147,
// conv10..conv17: Conv2d 3x3/1 pad 1 + folded BatchNorm + ReLU, MaxPool 2x2
// after conv13 / conv17) as Winograd F(2,3) along x (Lavin & Gray 2016, the
// one-dimensional minimal filtering algorithm nested in a direct sum over the
// kernel rows).
//
// Per output pair (row y, columns 2p, 2p+1) and input row r = y + ky - 1:
//   d_x = in[r][2p - 1 + x], x = 0..3 (zero padding outside the image)
//   V_0 = d0 - d2, V_1 = d1 + d2, V_2 = d2 - d1, V_3 = d1 - d3   (16-bit)
//   U_0 = g0, U_1 = (g0 + g1 + g2) / 2, U_2 = (g0 - g1 + g2) / 2, U_3 = g2
//   (g = the folded kernel row ky, fp64 on the host, rounded to 16 bits once)
//   M_j = sum over (ky, c) of U_j V_j                               (fp32)
//   out[y][2p] = M_0 + M_1 + M_2,  out[y][2p + 1] = M_1 - M_2 - M_3
// 4 transformed products per 2 outputs and kernel row against 6 direct ones:
// 2/3 of the direct conv's MFMAs.  Error budget (tools/winograd_budget.py):
// the fp16 path stays inside the north star's 1e-3 per-frame bar.
//
// Work split: a workgroup owns a box of output pairs x BN output channels;
// wave j computes position j's accumulator M_j for every pair and channel of
// the box (a GEMM with rows = pairs, cols = channels, k = (ky, channel), so
// the A fragment of a step is V_j of 16 pairs x 32 channels, made from two
// 16-byte LDS reads of the staged input halo and four packed adds), and the
// four positions meet in LDS once per box for the output transform.  Rows of
// pairs are padded to 8 (14x14: 7 real) or 16 (28x28: 14 real) so a 16-row
// MFMA tile covers whole image rows: one lane base address serves every row
// tile and kernel row through immediate offsets.
//
// The halo of each 32-channel chunk is loaded into registers one chunk ahead
// (plain 16-byte loads, written to the other LDS buffer after the chunk's
// first kernel row; one barrier per chunk), the weight fragments straight
// from L2 into registers two steps ahead (conv3x3_db's schedule, conv.hip):
// every vector-memory op in the loop is a plain load, so the compiler's own
// vmcnt waits are exact.
#include "common.hpp"

namespace fac {

// V = a + b (S > 0) or a - b (S < 0) on 8 16-bit values, rounded once.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <int S>
__device__ __forceinline__ u16x8 wino_combine(F16, u16x8 a, u16x8 b) {
  // two-wide pieces, so the backend emits one v_pk_add_f16 (neg modifier for
  // the difference) per pair; on the 8-wide vector it scalarised to
  // v_sub_f16 + v_sub_f16_sdwa + v_pack_b32_f16 per pair
  // (the difference as an explicit v_pk_add_f16 with negated second operand:
  // written in C, the f16x2 subtraction was scalarised too)
  const u32x4 x = __builtin_bit_cast(u32x4, a), y = __builtin_bit_cast(u32x4, b);
  u32x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if constexpr (S > 0)
      asm("v_pk_add_f16 %0, %1, %2" : "=v"(r[i]) : "v"(x[i]), "v"(y[i]));
    else
      asm("v_pk_add_f16 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r[i]) : "v"(x[i]), "v"(y[i]));
  }
  return __builtin_bit_cast(u16x8, r);
}
template <int S>
__device__ __forceinline__ u16x8 wino_combine(BF16, u16x8 a, u16x8 b) {
  u16x8 r;
#pragma unroll
  for (int i = 0; i < 8; i += 2) {
    const f32x2 x = {BF16::to_f32(a[i]), BF16::to_f32(a[i + 1])};
    const f32x2 y = {BF16::to_f32(b[i]), BF16::to_f32(b[i + 1])};
    const bf16x2 v = __builtin_convertvector(S > 0 ? x + y : x - y, bf16x2);  // v_cvt_pk_bf16_f32
    const uint32_t u = __builtin_bit_cast(uint32_t, v);
    r[i] = (uint16_t)u;
    r[i + 1] = (uint16_t)(u >> 16);
  }
  return r;
}

// Box geometry: 14 x 14 output pixels of an IMG x IMG map (IMG = 14, 28, 56,
// ...: (IMG/14)^2 boxes per crop) = 14 rows x 7 pairs, padded to 8 pairs per
// row so each 16-row MFMA tile is exactly two image rows (7 row tiles).
struct WinoGeom {
  static constexpr int TPR = 8, REAL = 7, RPT = 2, RT = 7, TH = 14, TW = 14;
  static constexpr int HH = TH + 2, HWD = TW + 2;   // halo 16 x 16 pixels
  // halo row pitch 17 pixels with the 16-byte piece q of halo column hx at
  // position q ^ ((hx >> 1) & 3): the A-fragment reads (every position,
  // kernel row and row tile) are conflict-free over the ds_read_b128 lane
  // groups (simulated)
  static constexpr int RPX = 17;
  static constexpr int HPIECES = HH * HWD * 4;        // 1024 16-byte pieces per chunk
  static constexpr int HPT = HPIECES / 256;           // 4 per thread
  // one buffer, plus the over-read of the padding pairs (hx up to 17) in the last row
  static constexpr int HBUF = ((HH * RPX + 4) * 4 * 8 + 255) / 256 * 256;  // elements
};

__device__ __forceinline__ int wino_swz(int hx) { return (hx >> 1) & 3; }

template <class T, int IMG, int BN, bool POOL>
__global__ __launch_bounds__(256, 2) void conv3x3_wino(const uint16_t* __restrict__ in,
                                                       const uint16_t* __restrict__ upk,
                                                       const float* __restrict__ bias, uint16_t* __restrict__ out,
                                                       int Cin, int Cout, const uint16_t* __restrict__ zero16) {
  using G = WinoGeom;
  constexpr int CK = 32, CT = BN / 16, RT = G::RT, TPR = G::TPR, RPX = G::RPX;
  constexpr int NT = RT * 16;                   // pair rows of the GEMM (incl. padding pairs)
  constexpr int XP = NT + 4;                    // exchange pitch (floats) per (position, column)
  constexpr int XSZ = 4 * 16 * XP;              // floats: one 16-column slice of all four positions
  constexpr int OH = POOL ? G::TH / 2 : G::TH, OW = POOL ? G::TW / 2 : G::TW;  // box output
  constexpr int OI = POOL ? IMG / 2 : IMG;      // output map size
  constexpr int OPS = BN + 8;                   // output staging pitch (elements)
  constexpr int OSTG = OH * OW * OPS;
  constexpr int EPI = XSZ * 2 + OSTG;           // elements: exchange slice + staging tile
  constexpr int SMEM = 2 * G::HBUF > EPI ? 2 * G::HBUF : EPI;
  constexpr int BX = IMG / G::TW, BPC = BX * BX;  // boxes per crop row / per crop
  static_assert(BN % 16 == 0 && CT >= 1 && IMG % G::TW == 0, "shape");
  __shared__ __attribute__((aligned(16))) uint16_t smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int j = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave = transform position (uniform)
  const int ncb = Cout / BN;
  // XCD-aware order: XCD k takes a contiguous range of (box, column block)
  // pairs, column blocks fastest, so the blocks sharing a box's halo run
  // together on one XCD and read it from its L2
  int id = blockIdx.x;
  if ((gridDim.x & 7) == 0) id = (id & 7) * (gridDim.x >> 3) + (id >> 3);
  const int box = id / ncb, nb = id - box * ncb;
  const int b = box / BPC, bi = box - b * BPC, by = bi / BX;
  const int y0 = by * G::TH, x0 = (bi - by * BX) * G::TW;
  const int nch = Cin / CK, nsteps = nch * 3;
  const uint16_t* in_b = in + (size_t)b * IMG * IMG * Cin;

  // ---- halo map: piece s = i*256 + tid -> (halo row, column, channel piece)
  int hsrc[G::HPT], hdst[G::HPT];
#pragma unroll
  for (int i = 0; i < G::HPT; ++i) {
    const int s = i * 256 + tid;
    const int pix = s >> 2, qq = s & 3;
    const int hr = pix / G::HWD, hx = pix - (pix / G::HWD) * G::HWD;
    const int y = y0 + hr - 1, x = x0 + hx - 1;
    hsrc[i] = (y >= 0 && y < IMG && x >= 0 && x < IMG) ? (y * IMG + x) * Cin + qq * 8 : -1;
    hdst[i] = ((hr * RPX + hx) * 4 + (qq ^ wino_swz(hx))) * 8;
  }
  u16x8 hreg[G::HPT];
  auto load_halo = [&](int c) {
#pragma unroll
    for (int i = 0; i < G::HPT; ++i) hreg[i] = *(const u16x8*)(hsrc[i] >= 0 ? in_b + hsrc[i] + c * CK : zero16);
  };
  auto store_halo = [&](uint16_t* dst) {
#pragma unroll
    for (int i = 0; i < G::HPT; ++i) *(u16x8*)(dst + hdst[i]) = hreg[i];
  };

  // ---- A fragment sources: lane -> pair (row-in-tile, p), channel piece q;
  // position j reads halo columns hx = 2p + {0,1,2,1}[j] and 2p + {2,2,1,3}[j]
  const int tl = lane & 15, q = lane >> 4;
  const int ry = tl / TPR, p = tl - ry * TPR;
  const int ha = 2 * p + (j == 0 ? 0 : (j == 2 ? 2 : 1));
  const int hb = 2 * p + (j == 0 || j == 1 ? 2 : (j == 2 ? 1 : 3));
  const int abase = ((ry * RPX + ha) * 4 + (q ^ wino_swz(ha))) * 8;
  const int bbase = ((ry * RPX + hb) * 4 + (q ^ wino_swz(hb))) * 8;

  // ---- B fragments: U packed [nb][chunk][ky][j][q][BN][8]; this lane reads
  // column ct*16 + (lane & 15), channel piece q, 16 bytes per column tile
  constexpr int USTEP = 4 * 4 * BN * 8;  // elements per (chunk, ky) step: all four positions
  const uint16_t* ub = upk + (size_t)nb * nsteps * USTEP + ((j * 4 + q) * BN + tl) * 8;
  auto load_b = [&](u16x8(&dst)[CT], int s) {
    const uint16_t* sb = ub + (size_t)(s < nsteps ? s : 0) * USTEP;  // past the end: a dummy re-read
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) dst[ct] = *(const u16x8*)(sb + ct * 128);
  };

  f32x4 acc[RT][CT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) acc[rt][ct] = (f32x4)0.f;

  u16x8 bq[3][CT];
  load_halo(0);
  load_b(bq[0], 0);
  load_b(bq[1], 1);
  store_halo(smem);
  __syncthreads();

  // the main loop, instantiated for the sign of the position's combination
  // (V_1 = d1 + d2; the others subtract); j is wave-uniform
  auto main_loop = [&](auto sg) {
    constexpr int SG = decltype(sg)::value;
    for (int c = 0; c < nch; ++c) {
      const uint16_t* hcur = smem + (c & 1) * G::HBUF;
      uint16_t* hnext = smem + ((c + 1) & 1) * G::HBUF;
      const int s0 = c * 3;
      auto step = [&](auto kc) {
        constexpr int ky = decltype(kc)::value;
        load_b(bq[(ky + 2) % 3], s0 + ky + 2);
        if constexpr (ky == 0) load_halo(c + 1 < nch ? c + 1 : c);
        const uint16_t* pa_ = hcur + abase + ky * RPX * 32;
        const uint16_t* pb_ = hcur + bbase + ky * RPX * 32;
        u16x8 pa = *(const u16x8*)pa_, pb = *(const u16x8*)pb_;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          const u16x8 v = wino_combine<SG>(T{}, pa, pb);
          if (rt + 1 < RT) {  // the next row tile's pixels, read behind this tile's MFMAs
            pa = *(const u16x8*)(pa_ + (rt + 1) * G::RPT * RPX * 32);
            pb = *(const u16x8*)(pb_ + (rt + 1) * G::RPT * RPX * 32);
          }
#pragma unroll
          for (int ct = 0; ct < CT; ++ct) acc[rt][ct] = T::mfma(v, bq[ky % 3][ct], acc[rt][ct]);
        }
        if constexpr (ky == 1) store_halo(hnext);
        if constexpr (ky == 2) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      };
      step(std::integral_constant<int, 0>{});
      step(std::integral_constant<int, 1>{});
      step(std::integral_constant<int, 2>{});
    }
  };
  if (j == 1)
    main_loop(std::integral_constant<int, 1>{});
  else
    main_loop(std::integral_constant<int, -1>{});
  __syncthreads();  // the halo buffers are dead: the exchange and staging reuse them

  // ---- output transform, one 16-column slice at a time: each wave stores its
  // M_j slice (fp32, [j][column][pair]), then the workgroup combines the four
  float* const X = (float*)smem;
  uint16_t* const ostg = smem + XSZ * 2;
  const int col = tid & 15;
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) *(f32x4*)(X + (j * 16 + tl) * XP + rt * 16 + q * 4) = acc[rt][ct];
    __syncthreads();
    const int n = ct * 16 + col;
    const float bv = bias[nb * BN + n];
    const float* xc = X + col * XP;
    if constexpr (!POOL) {
#pragma unroll
      for (int k = 0; k < RT; ++k) {
        const int t = (tid >> 4) + 16 * k, ty = t / TPR, tp = t - (t / TPR) * TPR;
        if (tp < G::REAL) {
          const float m0 = xc[t], m1 = xc[16 * XP + t], m2 = xc[32 * XP + t], m3 = xc[48 * XP + t];
          const float o0 = relu(m0 + m1 + m2 + bv), o1 = relu(m1 - m2 - m3 + bv);
          ostg[(ty * G::TW + 2 * tp) * OPS + n] = T::from_f32(o0);
          ostg[(ty * G::TW + 2 * tp + 1) * OPS + n] = T::from_f32(o1);
        }
      }
    } else {
      // pooled pixel (py, tp): the pairs (2py, tp) and (2py + 1, tp)
      for (int k = tid >> 4; k < OH * OW; k += 16) {
        const int py = k / OW, tp = k - (k / OW) * OW;
        const int t0 = 2 * py * TPR + tp, t1 = t0 + TPR;
        const float a0 = xc[t0], a1 = xc[16 * XP + t0], a2 = xc[32 * XP + t0], a3 = xc[48 * XP + t0];
        const float c0 = xc[t1], c1 = xc[16 * XP + t1], c2 = xc[32 * XP + t1], c3 = xc[48 * XP + t1];
        const float mx = fmaxf(fmaxf(a0 + a1 + a2, a1 - a2 - a3), fmaxf(c0 + c1 + c2, c1 - c2 - c3));
        ostg[k * OPS + n] = T::from_f32(relu(mx + bv));
      }
    }
    __syncthreads();  // the next slice overwrites X
  }
  // ---- coalesced 16-byte stores of the staged tile
  const int oy0 = POOL ? y0 / 2 : y0, ox0 = POOL ? x0 / 2 : x0;
  constexpr int QN = BN / 8;
  for (int it = tid; it < OH * OW * QN; it += 256) {
    const int px = it / QN, qq = it - (it / QN) * QN;
    const int oy = px / OW, ox = px - (px / OW) * OW;
    *(u16x8*)(out + (((size_t)b * OI + oy0 + oy) * OI + ox0 + ox) * Cout + nb * BN + qq * 8) =
        *(const u16x8*)(ostg + px * OPS + qq * 8);
  }
}

// Host side: U packed for conv3x3_wino, [nb][chunk][ky][j][q][BN][8] 16-bit,
// from the folded fp32 weights w [co][ci][9] (tap = ky*3 + kx).
void pack_conv3x3_wino(int dtype, int ci, int co, int bn, const float* w, uint16_t* out) {
  const int nch = ci / 32;
  size_t i = 0;
  for (int nb = 0; nb < co / bn; ++nb)
    for (int ch = 0; ch < nch; ++ch)
      for (int ky = 0; ky < 3; ++ky)
        for (int jj = 0; jj < 4; ++jj)
          for (int q = 0; q < 4; ++q)
            for (int nl = 0; nl < bn; ++nl)
              for (int e = 0; e < 8; ++e) {
                const float* g = w + ((size_t)(nb * bn + nl) * ci + ch * 32 + q * 8 + e) * 9 + ky * 3;
                const double g0 = g[0], g1 = g[1], g2 = g[2];
                const double u = jj == 0 ? g0 : (jj == 1 ? (g0 + g1 + g2) * 0.5 : (jj == 2 ? (g0 - g1 + g2) * 0.5 : g2));
                out[i++] = dtype == 0 ? fac_host::f32_to_bf16((float)u) : fac_host::f32_to_f16((float)u);
              }
}

size_t wino_packed_elems(int ci, int co) { return (size_t)co * ci * 12; }

// Winograd conv of [B][H][H][Cin] -> [B][H or H/2][..][Cout]; upk from
// pack_conv3x3_wino with the same bn.  H in {14, 28, 56}.
hipError_t launch_conv3x3_wino(int dtype, const uint16_t* in, const uint16_t* upk, const float* bias, uint16_t* out,
                               int B, int H, int Cin, int Cout, int bn, bool pool, const uint16_t* zero16,
                               hipStream_t st) {
  if (Cin % 32 || bn != 64 || Cout % bn || (H != 14 && H != 28 && H != 56)) return hipErrorInvalidValue;
  const long long nwg = (long long)B * (H / 14) * (H / 14) * (Cout / bn);
  if (nwg <= 0 || nwg >= (1ll << 31)) return hipErrorInvalidValue;
  const dim3 grid((unsigned)nwg);
#define FAC_WINO(TT, HH, P) conv3x3_wino<TT, HH, 64, P><<<grid, 256, 0, st>>>(in, upk, bias, out, Cin, Cout, zero16)
#define FAC_WINO_H(HH)                                                   \
  if (dtype == 0) pool ? FAC_WINO(BF16, HH, true) : FAC_WINO(BF16, HH, false); \
  else pool ? FAC_WINO(F16, HH, true) : FAC_WINO(F16, HH, false);
  switch (H) {
    case 14: FAC_WINO_H(14) break;
    case 28: FAC_WINO_H(28) break;
    default: FAC_WINO_H(56) break;
  }
#undef FAC_WINO_H
#undef FAC_WINO
  return hipGetLastError();
}

}  // namespace fac
