// Conv stem kernels: CViT.features (CViT-main/model/cvit.py:86-148), i.e.
// 17 x [Conv2d 3x3 s1 p1 -> BatchNorm2d(eval) -> ReLU] with MaxPool2d(2,2)
// after convs 3/6/9/13/17, computed as implicit GEMMs on MFMA.
//
// Layout: activations NHWC 16-bit (bf16 or fp16), BN folded into the conv
// weights/bias at load time, fp32 accumulation, fp32 epilogue.
//
// GEMM view per conv: rows = output pixels of a TH x TW spatial box of one
// image, cols = BN output channels, k = (tap, input channel).  A workgroup
// stages the (TH+2) x (TW+2) input halo of a 32-channel chunk in LDS once and
// reads all 9 taps from it (9x less L2 traffic than an im2col gather), while
// per-tap weight slices [BN][32] stream through a second double buffer.
//
// Pixel order inside a box is "window-major" (4 consecutive GEMM rows = one
// 2x2 pooling window), so in the 16x16x32 MFMA C layout (row = 4*(lane>>4) +
// reg) each lane holds a whole window of one channel: the 2x2 max-pool is
// three fmaxf in registers.
#include <cstdlib>
#include <type_traits>

#include "common.hpp"

namespace fac {

constexpr int CONV_CK = 32;  // input channels per K chunk (= 4 x 16-byte "q" pieces)

// LDS images (16-byte units), chosen by simulating the ds_read_b128 lane
// groups of MI355X_MICROARCH.md §LDS over every tap and row tile:
//  * halo: q-major planes [q][hy][hx], row pitch RP = 24 for boxes up to 22
//    wide, 40 for 28-wide boxes (== 8 mod 16, so the 2x8-pixel strip one
//    16-row tile covers hits 16 distinct slots), plane pitch (TH+2)*RP + 8:
//    A-fragment reads conflict-free for 16x16, 1.14-way for 8x28 and 4x28,
//    1.4-way for 14x14 boxes; staging writes 2-way.
//  * weight slice: q-major [q][BN], identical to its global packing
//    [n-block][chunk][tap][q][BN][8], so staging is a linear 16-byte copy and
//    B-fragment reads are conflict-free.
// Async global -> LDS copy of 16 bytes per lane (global_load_lds_dwordx4): the
// wave's 64 pieces land contiguously at the wave-uniform LDS address `ldst`.
__device__ __forceinline__ void glds16(const void* gsrc, void* ldst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gsrc,
                                   (__attribute__((address_space(3))) void*)ldst, 16, 0, 0);
}

template <int TW>
constexpr int halo_rp() { return TW + 2 <= 24 ? 24 : 40; }

// Each box shape serves exactly one image size (launch_conv_t picks the tile
// by resolution): make it a compile-time constant inside the kernels, so the
// box-index divisions and the halo map's address arithmetic fold.
template <int TH, int TW, int BN>
constexpr int tile_res() {
  return TW == 16 ? (BN == 32 ? 224 : 112) : (TH == 8 ? 56 : (TH == 4 ? 28 : (TH == 14 ? 14 : 0)));
}

template <int TW>
__device__ __forceinline__ void box_pixel(int m, int& py, int& px) {
  constexpr int WW = TW / 2;
  const int w = m >> 2, sub = m & 3;
  const int wy = w / WW, wx = w - wy * WW;
  py = 2 * wy + (sub >> 1);
  px = 2 * wx + (sub & 1);
}

// Stage an OPIX x BN tile (row stride OPS, window-major rows) from LDS to
// NHWC global memory with 16-byte stores in raster order.  (Round 5, not
// kept: write-through `sc1` stores, which drop the line from the XCD's L2,
// so the output stream would not evict the halo rows neighbouring boxes
// re-read: conv4-17 within noise, same box.)
template <int TH, int TW, int BN, bool POOL>
__device__ __forceinline__ void store_tile(const uint16_t* ostg, uint16_t* out, int b, int Ho, int Wo,
                                           int oy0, int ox0, int Cout, int n0, int tid) {
  constexpr int OTW = POOL ? TW / 2 : TW;
  constexpr int OTH = POOL ? TH / 2 : TH;
  constexpr int OPS = BN + 8;
  constexpr int QN = BN / 8;
  for (int it = tid; it < OTH * OTW * QN; it += 256) {
    const int r = it / QN, q = it - r * QN;
    const int oy = r / OTW, ox = r - oy * OTW;
    int p;
    if constexpr (POOL) {
      p = oy * OTW + ox;
    } else {
      p = ((oy >> 1) * (TW / 2) + (ox >> 1)) * 4 + (oy & 1) * 2 + (ox & 1);
    }
    const u16x8 v = *(const u16x8*)(ostg + p * OPS + q * 8);
    *(u16x8*)(out + (((size_t)b * Ho + oy0 + oy) * Wo + ox0 + ox) * Cout + n0 + q * 8) = v;
  }
}

// Epilogue part 1: folded-BN bias + ReLU (+ the 2x2 max of a window-major
// row group) of a wave's RTW x CTW accumulator tiles -> 16-bit, into the LDS
// staging tile (rows = window-major pixels, pitch OPS).  RELU is a template
// argument (a runtime flag cost one v_cndmask per value), and the four rows
// of a lane convert as two packed pairs (v_cvt_pk) written as the low and
// high halves (ds_write_b16 / _d16_hi).
template <class T, int RTW, int CTW, int OPS, bool POOL, bool RELU>
__device__ __forceinline__ void stage_tile(const f32x4 (&acc)[RTW][CTW], uint16_t* ostg,
                                           const float* __restrict__ bias_blk, int wm, int wn, int lane) {
#pragma unroll
  for (int ct = 0; ct < CTW; ++ct) {
    const int nl = (wn * CTW + ct) * 16 + (lane & 15);
    const float bv = bias_blk[nl];
#pragma unroll
    for (int rt = 0; rt < RTW; ++rt) {
      const f32x4 v = acc[rt][ct];
      if constexpr (POOL) {
        const float mx = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3])) + bv;
        const int w = (wm * RTW + rt) * 4 + (lane >> 4);
        ostg[w * OPS + nl] = T::from_f32(RELU ? relu(mx) : mx);
      } else {
        f32x4 y;
#pragma unroll
        for (int j = 0; j < 4; ++j) y[j] = RELU ? relu(v[j] + bv) : v[j] + bv;
        // rows (0,1) and (2,3) as two packed dwords: one conversion per pair,
        // the high halves stored by ds_write_b16_d16_hi (as a u16x4 the
        // compiler converted every value on its own, one cvt each)
        const uint32_t p01 = T::pack2(y[0], y[1]), p23 = T::pack2(y[2], y[3]);
        const int m0 = (wm * RTW + rt) * 16 + (lane >> 4) * 4;
        ostg[(m0 + 0) * OPS + nl] = (uint16_t)p01;
        ostg[(m0 + 1) * OPS + nl] = (uint16_t)(p01 >> 16);
        ostg[(m0 + 2) * OPS + nl] = (uint16_t)p23;
        ostg[(m0 + 3) * OPS + nl] = (uint16_t)(p23 >> 16);
      }
    }
  }
}

#ifdef CONV_STAMPS
// Phase timeline of conv3x3_bn_relu (tools/ubench/conv_ubench.hip): s_memtime
// of wave w of workgroup x at stamp k (0 start, 1 prologue landed, 2..10 after
// chunk 0's nine step barriers, 11 last chunk done, 12 staged, 13 stored)
__device__ unsigned long long conv_st[16384][4][14];
#define CONV_STAMP(k)                                                                         \
  do {                                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    unsigned long long t_;                                                                    \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    if (blockIdx.y == 0 && blockIdx.x < 16384 && lane == 0) conv_st[blockIdx.x][wave][(k)] = t_; \
  } while (0)
#else
#define CONV_STAMP(k) \
  do {                \
  } while (0)
#endif

// HB: halo buffers (2: the next chunk's halo streams in during this chunk;
// 1: it is loaded between chunks, exposed, which halves the halo LDS so that
// OCC = 3 workgroups share a CU and hide each other's exposed loads — the
// 112^2 layers, whose 1-2 chunks leave little to pipeline within a box).
// (Round 5, measured and not kept: persistent workgroups walking several
// boxes each, so the per-box setup -- halo map, fragment offsets -- is paid
// once per workgroup.  Bit-identical, but slower on every 112^2 arm, same
// box: the pooled tile at 2 per CU conv6 199 -> 246 us, the unpooled one at
// 3 / 2 per CU conv4 161 -> 185 / 182 us and conv5 240 -> 281 / 297 us: a
// persistent grid loses the overlap of one workgroup's exposed halo load
// with its neighbours' MFMAs that the hardware's dispatch order gives.)
// WR: weight-ring depth in tap slices, 3 or 9.  9 (no PB): slice s+8 is
// issued at step s, so each slice has eight steps to land instead of two --
// for grids of about one workgroup per CU (few crops), where no co-resident
// workgroup covers a step's wait on L2 (past the end: dummy re-reads of
// slice 0 into dead slots, as with 3).  (Round 5: the 9-slice ring for the 112^2 layers, 61 KB of LDS,
// i.e. 2 per CU instead of 4, was slower, conv4 161 -> 188 us: there
// occupancy, not the slice wait, sets the rate.)
template <class T, int TH, int TW, int BN, int WM, int WN, bool POOL, int HB = 2, int OCC = 2, bool PB = true,
          int WR = 3>
__global__ __launch_bounds__(256, OCC) void conv3x3_bn_relu(const uint16_t* __restrict__ in,
                                                       const uint16_t* __restrict__ wpk,
                                                       const float* __restrict__ bias,
                                                       uint16_t* __restrict__ out, int H, int W,
                                                       int Cin, int Cout, const uint16_t* __restrict__ zero16,
                                                       int do_relu) {
  constexpr int CK = CONV_CK;
  constexpr int HH = TH + 2, HWD = TW + 2;
  constexpr int HALO_RP = halo_rp<TW>();
  constexpr int NHP = HH * HALO_RP + 8;     // halo plane pitch (16-byte units)
  constexpr int NPIX = TH * TW;
  constexpr int RT = ((NPIX + 15) / 16 + WM - 1) / WM * WM;
  constexpr int RTW = RT / WM;
  constexpr int CTW = BN / 16 / WN;
  // The halo image is filled by global_load_lds, one 64-slot wave
  // instruction at a time; pad it to whole instructions, a multiple of 4 so
  // every wave issues the same number (HPW).
  // PM (every layer but the 224x224 ones, whose packed weights stem224.hip
  // shares): pixel-major halo image [hy][RPX][4 x 16 B], the 16-byte piece
  // index XOR-swizzled by row parity (position j of pixel (hy,hx) holds
  // channel piece j ^ 2*(hy&1)).  Each glds wave instruction then reads 16
  // consecutive halo pixels' 64 contiguous bytes (a q-major image's
  // instructions touch 64 pixels, i.e. 64 cache lines, for 16 bytes each), and
  // the fragment reads are conflict-free for every tap (simulated over the
  // ds_read_b128 lane groups; 14x14 boxes with RPX = 17: 1.08-way, q-major
  // 1.4).  Lane group g always reads position g ^ 2*(py&1), so on odd kernel
  // rows it holds channel piece g ^ 2: the weight packing swaps pieces
  // q <-> q^2 of those taps to match (pack_conv3x3, stack_ops.hip) -- a
  // permutation of the MFMA's k order.
  constexpr bool PM = !(TH == 16 && TW == 16 && BN == 32);
  constexpr int RPX = TW == 14 ? HWD + 1 : HWD;  // halo row pitch (pixels)
  constexpr int HSLOTS = PM ? (HH * RPX * 4 + 255) / 256 * 256 : (4 * NHP + 255) / 256 * 256;
  constexpr int HPW = HSLOTS / 256;
  constexpr int HALO = HSLOTS * 8;          // elements per halo buffer
  constexpr int WSL = BN * CK;              // elements per tap slice
  constexpr int OPIX = POOL ? NPIX / 4 : NPIX;
  constexpr int OPS = BN + 8;
  constexpr int OPER = HB * HALO + WR * WSL;  // halo buffer(s) + WR-slot weight ring
  static_assert(WR == 3 || WR == 9, "weight ring: 3 or 9 slices");
  constexpr int OSTG = (POOL ? RT * 4 : RT * 16) * OPS;  // padded: epilogue writes unguarded
  constexpr int SMEM = OPER > OSTG ? OPER : OSTG;
  static_assert(WM * WN == 4, "4 waves");
  static_assert(TH % 2 == 0 && TW % 2 == 0, "window-major order needs even boxes");
  static_assert(CTW * 16 * WN == BN, "BN split");
  __shared__ __attribute__((aligned(16))) uint16_t smem[SMEM];

  static_assert(tile_res<TH, TW, BN>() > 0, "tile shape without a resolution");
  H = W = tile_res<TH, TW, BN>();  // == the launch's H (launch_conv_t); folds the index math
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  const int tiles_x = W / TW, tiles_per_img = (H / TH) * tiles_x;
  CONV_STAMP(0);
  // XCD-aware box order: workgroups are dealt round-robin to the 8 XCDs
  // (blockIdx % 8), so give XCD k a contiguous range of boxes; neighbouring
  // boxes then share their halo rows in that XCD's L2 instead of each
  // re-reading them from HBM (measured: the 112^2 layers fetched the full
  // 1.27x halo overhead with the plain order).
  const int nb = blockIdx.y;
  const int nchunks = Cin / CK;
  const uint16_t* wsrc = wpk + (size_t)nb * nchunks * 9 * WSL;
  int bx = blockIdx.x;
  if ((gridDim.x & 7) == 0) bx = (bx & 7) * (gridDim.x >> 3) + (bx >> 3);
  const int b = bx / tiles_per_img;
  const int tile = bx - b * tiles_per_img;
  const int ty = tile / tiles_x, tx = tile - ty * tiles_x;
  const int y0 = ty * TH, x0 = tx * TW;
  const uint16_t* const in_b = in + (size_t)b * H * W * Cin;

  // Halo staging map: each lane of each halo glds instruction owns one
  // 16-byte slot of the LDS image (plane q, row hy, column hx); it copies
  // that piece of the image, or 16 zero bytes for zero padding / pitch
  // padding (a pointer that does not move with c).
  int hsrc[HPW];
#pragma unroll
  for (int i = 0; i < HPW; ++i) {
    const int slot = (i * 4 + wave) * 64 + lane;
    int q, hy, hx;
    if constexpr (PM) {
      const int pix = slot >> 2;
      hy = pix / RPX;
      hx = pix - (pix / RPX) * RPX;
      q = hy < HH ? (slot & 3) ^ ((hy & 1) << 1) : 4;
    } else {
      q = slot / NHP;
      const int j = slot - (slot / NHP) * NHP;
      hy = j / HALO_RP;
      hx = j - (j / HALO_RP) * HALO_RP;
    }
    const int y = y0 + hy - 1, x = x0 + hx - 1;
    hsrc[i] = (q < 4 && hy < HH && hx < HWD && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W)
                  ? (y * W + x) * Cin + q * 8
                  : -1;
  }
  // (the 112x112 pooled variant spills one map entry at its 128-VGPR budget:
  // the store sits in the prologue and the reload at a chunk start, both
  // outside the counted-vmcnt steps; recomputing the map per chunk instead
  // measured slower, conv5 272 -> 286 us)
  auto issue_halo = [&](uint16_t* dst, int c) {
#pragma unroll
    for (int i = 0; i < HPW; ++i) {
      // opaque copy: keeps the per-chunk source addresses from being hoisted
      // into HPW live 64-bit registers across the taps
      int hs;
      asm volatile("v_mov_b32 %0, %1" : "=v"(hs) : "v"(hsrc[i]));
      const uint16_t* src = hs >= 0 ? in_b + hs + c * CK : zero16;
      glds16(src, dst + (i * 4 + wave) * 64 * 8);
    }
  };
  // Weight slices stream global -> LDS by global_load_lds: the packing of a
  // slice in memory IS its LDS image, so wave w copies pieces
  // [256i + 64w, +64) straight into ring slot `slot`.
  constexpr int WPIECES = BN * CK / 8;
  constexpr int WPW = (WPIECES + 255) / 256;  // glds instructions per wave per slice
  uint16_t* const wring = smem + HB * HALO;
  uint16_t* const hbase = smem;  // the halo buffer(s)
  // Every wave issues WPW pieces per slice, so the counted vmcnt waits below
  // hold for every wave: when a slice has fewer than 4 x 64 pieces per
  // instruction row (BN 32: 128 pieces), the waves past its end re-copy a
  // piece another wave copies too -- the same bytes to the same LDS slot,
  // retired by the same wait -- instead of issuing nothing (which left their
  // halo loads uncounted by the per-step waits: ADVICE r05).
  auto issue_w = [&](int slot, const uint16_t* src) {
#pragma unroll
    for (int i = 0; i < WPW; ++i) {
      int pb = i * 256 + wave * 64;
      if (WPIECES % 256 != 0 && pb >= WPIECES) pb %= WPIECES;
      glds16(src + (size_t)(pb + lane) * 8, wring + slot * WSL + pb * 8);
    }
  };

  int abase[RTW];
#pragma unroll
  for (int rt = 0; rt < RTW; ++rt) {
    int m = (wm * RTW + rt) * 16 + (lane & 15);
    if (m >= NPIX) m = 0;  // padding rows: computed on pixel 0, never stored
    int py, px;
    box_pixel<TW>(m, py, px);
    abase[rt] = PM ? ((py * RPX + px) * 4 + ((lane >> 4) ^ ((py & 1) << 1))) * 8
                   : ((lane >> 4) * NHP + py * HALO_RP + px) * 8;
  }
  int bbase[CTW];
#pragma unroll
  for (int ct = 0; ct < CTW; ++ct) bbase[ct] = ((lane >> 4) * BN + (wn * CTW + ct) * 16 + (lane & 15)) * 8;

  f32x4 acc[RTW][CTW];
#pragma unroll
  for (int rt = 0; rt < RTW; ++rt)
#pragma unroll
    for (int ct = 0; ct < CTW; ++ct) acc[rt][ct] = (f32x4)0.f;

  // K loop: chunks of 32 input channels (runtime) x 9 taps (unrolled, so LDS
  // offsets and wait counts are immediates).  Slice s = 9c + t lives in ring
  // slot s % 3 = t % 3; it is issued (glds) at the top of step s-2, so each
  // slice has two steps of MFMA work to land.  The wait before each barrier
  // retires slice s+1 only - the slice issued this step (and the halo loads
  // of t = 0, which are younger than slice s+1 at t = 0 and t = 1) stay in
  // flight across it (cdna_hip_programming.md §5 "Pipelining across
  // barriers": counted vmcnt + raw s_barrier, never __syncthreads here).
  // The next chunk's halo is fetched at t = 0 and written at t = 8.
  const int nsteps = nchunks * 9;
  if constexpr (WR == 9) {
#pragma unroll
    for (int k = 0; k < 8; ++k) issue_w(k, k < nsteps ? wsrc + k * WSL : wsrc);
  } else {
    issue_w(0, wsrc);
    issue_w(1, wsrc + WSL);
    if constexpr (PB) issue_w(2, nsteps > 2 ? wsrc + 2 * WSL : wsrc);
  }
  issue_halo(hbase, 0);
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  CONV_STAMP(1);
  // PB: the B fragments of tap t+1 are read during tap t as well (slice s+1
  // is retired one barrier earlier, slice s+3 is issued at step s into the
  // slot slice s vacated when its fragments went to registers in step s-1).
  u16x8 bcur[CTW];
  if constexpr (PB) {
#pragma unroll
    for (int ct = 0; ct < CTW; ++ct) bcur[ct] = *(const u16x8*)(wring + bbase[ct]);
  }
  // Software pipeline on the halo fragments: tap t multiplies pixel
  // fragments read during tap t-1 and, right behind each row tile's MFMAs,
  // reads that tile's fragment for tap t+1 (at t = 8: tap 0 of the next
  // chunk, whose halo has landed since tap 1).  The reads then overlap the
  // MFMAs instead of bursting after every barrier (tools/ubench: the LDS +
  // MFMA skeleton of this tile goes from 67% to 80% of the MFMA floor).
  u16x8 fa[RTW];
#pragma unroll
  for (int rt = 0; rt < RTW; ++rt) fa[rt] = *(const u16x8*)(hbase + abase[rt]);
  // PB: slot 0 is re-filled at step 0, after every wave has read slice 0
  if constexpr (PB) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");

  for (int c = 0; c < nchunks; ++c) {
    if constexpr (HB == 1) {
      if (c > 0) {  // every wave is past the previous chunk's last barrier
        issue_halo(hbase, c);
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
        for (int rt = 0; rt < RTW; ++rt) fa[rt] = *(const u16x8*)(hbase + abase[rt]);
      }
    }
    const uint16_t* hb = hbase + (HB == 2 ? (c & 1) * HALO : 0);
    const uint16_t* hbn = hbase + (HB == 2 ? ((c + 1) & 1) * HALO : 0);
    const bool next_h = c + 1 < nchunks;
    const uint16_t* wnext = wsrc + (size_t)(c * 9 + WR - 1) * WSL;
    auto step = [&](auto tc) {
      constexpr int t = decltype(tc)::value;
      constexpr int sc = t % WR;  // ring slot of slice s = 9c + t
      // WR = 9: the next chunk's halo goes out first at t = 0, ahead of slice
      // 9c+8, so the step-7 wait (which retires slice 9c+8) retires it too,
      // before step 8 reads it
      if (WR == 9 && HB == 2 && t == 0) issue_halo(hbase + ((c + 1) & 1) * HALO, next_h ? c + 1 : c);
      // slice s+2 (past the end: a dummy re-read of slice 0 into a dead slot)
      // issue order: slice s+2, then (t = 0) the next chunk's halo into the
      // other halo buffer (on the last chunk a dummy re-read of this chunk);
      // glds are LDS writes, so the compiler keeps them in program order
      // (WR = 9: slice s+8 into the slot of slice s-1, read in step s-1, or
      // with PB in step s-2)
      if constexpr (WR == 9)
        issue_w((t + 8) % 9, (c * 9 + t + 8 < nsteps) ? wnext + t * WSL : wsrc);
      else if constexpr (PB)
        issue_w(t % 3, (c * 9 + t + 3 < nsteps) ? wnext + (t + 1) * WSL : wsrc);
      else
        issue_w((t + 2) % 3, (c * 9 + t + 2 < nsteps) ? wnext + t * WSL : wsrc);
      if (WR == 3 && HB == 2 && t == 0) issue_halo(hbase + ((c + 1) & 1) * HALO, next_h ? c + 1 : c);
      u16x8 bfr[CTW], bnx[CTW];
      if constexpr (PB) {
#pragma unroll
        for (int ct = 0; ct < CTW; ++ct) bfr[ct] = bcur[ct];
      } else {
        const uint16_t* wb = wring + sc * WSL;
#pragma unroll
        for (int ct = 0; ct < CTW; ++ct) bfr[ct] = *(const u16x8*)(wb + bbase[ct]);
      }
      constexpr int kyn = t < 8 ? (t + 1) / 3 : 0, kxn = t < 8 ? (t + 1) % 3 : 0;
      constexpr int ntoff = PM ? (kyn * RPX + kxn) * 32 : (kyn * HALO_RP + kxn) * 8;
      const uint16_t* hnx = t < 8 ? hb : hbn;
      const uint16_t* wbn = wring + ((t + 1) % WR) * WSL;
#pragma unroll
      for (int rt = 0; rt < RTW; ++rt) {
#pragma unroll
        for (int ct = 0; ct < CTW; ++ct) acc[rt][ct] = T::mfma(fa[rt], bfr[ct], acc[rt][ct]);
        // (HB = 1: the next chunk's tap-0 fragments are read once its halo is in)
        if (HB == 2 || t < 8) fa[rt] = *(const u16x8*)(hnx + abase[rt] + ntoff);
        if (PB && rt == 0) {
#pragma unroll
          for (int ct = 0; ct < CTW; ++ct) bnx[ct] = *(const u16x8*)(wbn + bbase[ct]);
        }
      }
      if constexpr (PB) {
#pragma unroll
        for (int ct = 0; ct < CTW; ++ct) bcur[ct] = bnx[ct];
      } else {
        __builtin_amdgcn_sched_group_barrier(0x100, CTW, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, CTW, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, PB ? 1 + CTW : 1, 0);
#pragma unroll
      for (int rt = 1; rt < RTW; ++rt) {
        __builtin_amdgcn_sched_group_barrier(0x008, CTW, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      // Retire slice s+1 (and at t = 1 the next halo), leaving younger glds in
      // flight; wait + barrier in ONE asm statement, so no LDS access can be
      // scheduled between this wave's wait and the workgroup barrier.  The LDS
      // wait retires this step's weight-fragment reads (the ring slot the next
      // step refills) and leaves the youngest ones, the A-fragment prefetches
      // for the next tap (halo buffers, not rewritten here), in flight: L of
      // them (with PB, A(0) sits in one group with the bnx reads).
      // (WR = 9: slices s+2 .. s+8 and the next halo while t <= 6; with PB,
      // whose next step reads slice s+2, slices s+3 .. s+8 and the halo
      // while t <= 5)
      constexpr int N = WR == 3 ? WPW + (HB == 2 && t <= 1 ? HPW : 0)
                                : (PB ? 6 * WPW + (HB == 2 && t <= 5 ? HPW : 0) : 7 * WPW + (HB == 2 && t <= 6 ? HPW : 0));
      // The relaxed wait relies on the issue order; fac_fake_amd/isa_check.py
      // verifies it on the built code object (each of the L youngest LDS ops
      // before every such barrier is a ds_read_b128 whose registers next feed
      // an MFMA's A operand, no scalar-memory op in the step) and rebuilds
      // this file with FAC_CONV_STRICT_LGKM (L = 0) if any wait fails.
#ifdef FAC_CONV_STRICT_LGKM
      constexpr int L = 0;
#else
      constexpr int L = (HB == 2 || t < 8) ? (PB ? RTW - 1 : RTW) : 0;
#endif
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(%1)\n\ts_barrier" ::"n"(N), "n"(L) : "memory");
      __builtin_amdgcn_sched_barrier(0);
#ifdef CONV_STAMPS
      if (c == 0) CONV_STAMP(2 + t);
#endif
    };
    step(std::integral_constant<int, 0>{});
    step(std::integral_constant<int, 1>{});
    step(std::integral_constant<int, 2>{});
    step(std::integral_constant<int, 3>{});
    step(std::integral_constant<int, 4>{});
    step(std::integral_constant<int, 5>{});
    step(std::integral_constant<int, 6>{});
    step(std::integral_constant<int, 7>{});
    step(std::integral_constant<int, 8>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // dummy slices land before LDS is reused / the wave ends
  CONV_STAMP(11);
  const int Ho = POOL ? H / 2 : H, Wo = POOL ? W / 2 : W;
  const int oy0 = POOL ? y0 / 2 : y0, ox0 = POOL ? x0 / 2 : x0;
  __syncthreads();

  // Epilogue: folded-BN bias + ReLU (+ 2x2 max) -> 16-bit -> LDS -> global.
  // (Round 4, measured and not kept: the transposed MFMA, D^T = W . A^T, so
  // that each lane holds 4 channels of one pixel and stores them straight to
  // global memory as 8 bytes, the 2x2 max by DPP across a window's 4 lanes.
  // Bit-identical outputs, but 2-23 % slower on every tile, conv4 165 -> 195
  // and conv6 203 -> 249 us: 16 8-byte stores of 32-byte segments per wave
  // against 8 fully coalesced 16-byte ones after the LDS transpose.  Also
  // not kept: the same transposed MFMAs for the unpooled tiles with the LDS
  // staging kept, one ds_write_b64 per tile instead of four ds_write_b16:
  // bit-identical, per-layer sum 2350 -> 2359 us, CViT -1.2 % same box.)
  uint16_t* ostg = smem;
  if (do_relu)
    stage_tile<T, RTW, CTW, OPS, POOL, true>(acc, ostg, bias + nb * BN, wm, wn, lane);
  else
    stage_tile<T, RTW, CTW, OPS, POOL, false>(acc, ostg, bias + nb * BN, wm, wn, lane);
  __syncthreads();
  CONV_STAMP(12);
  store_tile<TH, TW, BN, POOL>(ostg, out, b, Ho, Wo, oy0, ox0, Cout, nb * BN, tid);
#ifdef CONV_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  CONV_STAMP(13);
#endif
}

// ---------------------------------------------------------------------------
// conv3x3_db: the same implicit GEMM with the weight (B) fragments loaded
// straight from global memory (L2) into VGPRs instead of through an LDS ring.
//
// Why: in conv3x3_bn_relu every tap step streams a [BN][32] weight slice into
// LDS with global_load_lds and then needs a workgroup barrier before any wave
// may read it, although with a 1 x WN wave grid each wave reads only its own
// BN/WN columns: the slice is not shared at all.  Round 1 measured the deep
// layers 20-27 % faster without that glds and 4 % without the per-tap barrier
// (DESIGN §3.4).  Here each wave fetches its CTW B fragments (16 columns x 32
// k each = one 16-byte load per lane) two tap steps ahead with
// global_load_dwordx4, so the only LDS traffic left is the shared halo (A)
// and the only barrier is one per 32-channel chunk (halo double buffer).
//
// No LDS-DMA at all: the next chunk's halo is fetched at tap 0 with plain
// 16-byte loads into registers and written to the other halo buffer after
// tap 1.  Every vector-memory op of the loop is then a plain load, and the
// compiler's own `s_waitcnt vmcnt` (before the MFMAs and ds_writes that use
// them) is exact: LLVM counts LDS-DMA and loads as different event types
// and, with both pending, falls back to vmcnt(0).  (An async load must never
// be an inline-asm output either: the compiler takes such a value as written
// at the asm and may reuse its registers -- a dummy load's, once dead --
// before the data lands; a first version faulted that way.)
// BR: depth of the register B ring in tap slices, 3 or 9 (9: each fragment
// is fetched eight steps ahead -- the few-crop grids, where no co-resident
// workgroup covers a step's wait on L2; 9 x CTW x 4 VGPRs).
template <class T, int TH, int TW, int BN, int WM, int WN, bool POOL, int OCC = 2, int BR = 3>
__global__ __launch_bounds__(256, OCC) void conv3x3_db(const uint16_t* __restrict__ in,
                                                       const uint16_t* __restrict__ wpk,
                                                       const float* __restrict__ bias, uint16_t* __restrict__ out,
                                                       int H, int W, int Cin, int Cout,
                                                       const uint16_t* __restrict__ zero16, int do_relu) {
  constexpr int CK = CONV_CK;
  constexpr int HH = TH + 2, HWD = TW + 2;
  constexpr int NPIX = TH * TW;
  constexpr int RT = ((NPIX + 15) / 16 + WM - 1) / WM * WM;
  constexpr int RTW = RT / WM;
  constexpr int CTW = BN / 16 / WN;
  constexpr int RPX = TW == 14 ? HWD + 1 : HWD;  // pixel-major halo row pitch (as conv3x3_bn_relu's PM image)
  constexpr int HSLOTS = (HH * RPX * 4 + 255) / 256 * 256;
  constexpr int HPW = HSLOTS / 256;
  constexpr int HALO = HSLOTS * 8;
  constexpr int WSL = BN * CK;
  constexpr int OPS = BN + 8;
  constexpr int OPER = 2 * HALO;
  constexpr int OSTG = (POOL ? RT * 4 : RT * 16) * OPS;
  constexpr int SMEM = OPER > OSTG ? OPER : OSTG;
  static_assert(WM * WN == 4, "4 waves");
  static_assert(TH % 2 == 0 && TW % 2 == 0, "window-major order needs even boxes");
  static_assert(CTW * 16 * WN == BN, "BN split");
  __shared__ __attribute__((aligned(16))) uint16_t smem[SMEM];

  static_assert(tile_res<TH, TW, BN>() > 0, "tile shape without a resolution");
  H = W = tile_res<TH, TW, BN>();  // == the launch's H (launch_conv_t); folds the index math
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  const int tiles_x = W / TW, tiles_per_img = (H / TH) * tiles_x;
  int bx = blockIdx.x;  // XCD-aware box order (conv3x3_bn_relu)
  if ((gridDim.x & 7) == 0) bx = (bx & 7) * (gridDim.x >> 3) + (bx >> 3);
  const int b = bx / tiles_per_img;
  const int tile = bx - b * tiles_per_img;
  const int ty = tile / tiles_x, tx = tile - ty * tiles_x;
  const int y0 = ty * TH, x0 = tx * TW;
  const int nb = blockIdx.y;
  const int nchunks = Cin / CK;
  const int nsteps = nchunks * 9;
  const uint16_t* in_b = in + (size_t)b * H * W * Cin;
  const uint16_t* wsrc = wpk + (size_t)nb * nchunks * 9 * WSL;

  // Halo map: slot (i*4 + wave)*64 + lane of the pixel-major image holds 16
  // bytes of pixel (hy, hx), channel piece q; out-of-image and pitch-padding
  // slots read the zero page (every lane loads, so the loads stay uniform).
  int hsrc[HPW];
#pragma unroll
  for (int i = 0; i < HPW; ++i) {
    const int slot = (i * 4 + wave) * 64 + lane;
    const int pix = slot >> 2;
    const int hy = pix / RPX, hx = pix - (pix / RPX) * RPX;
    const int q = hy < HH ? (slot & 3) ^ ((hy & 1) << 1) : 4;
    const int y = y0 + hy - 1, x = x0 + hx - 1;
    hsrc[i] = -1;
    if (q < 4 && hx < HWD && y >= 0 && y < H && x >= 0 && x < W) hsrc[i] = (y * W + x) * Cin + q * 8;
  }
  u16x8 hreg[HPW];
  auto load_halo = [&](int c) {
#pragma unroll
    for (int i = 0; i < HPW; ++i) {
      const uint16_t* src = hsrc[i] >= 0 ? in_b + hsrc[i] + c * CK : zero16;
      hreg[i] = *(const u16x8*)src;
    }
  };
  auto store_halo = [&](uint16_t* dst) {
#pragma unroll
    for (int i = 0; i < HPW; ++i) *(u16x8*)(dst + ((i * 4 + wave) * 64 + lane) * 8) = hreg[i];
  };
  // B fragment of column tile ct: lane (n = lane & 15, k piece lane >> 4)
  // reads 16 bytes at ((kq * BN + wn * CTW * 16 + ct * 16 + n) * 8) of the slice
  const int boff = ((lane >> 4) * BN + wn * CTW * 16 + (lane & 15)) * 8;
  auto load_b = [&](u16x8(&dst)[CTW], int s) {
    const uint16_t* sb = wsrc + (size_t)(s < nsteps ? s : 0) * WSL + boff;  // past the end: a dummy re-read
#pragma unroll
    for (int ct = 0; ct < CTW; ++ct) dst[ct] = *(const u16x8*)(sb + ct * 128);
  };

  int abase[RTW];
#pragma unroll
  for (int rt = 0; rt < RTW; ++rt) {
    int m = (wm * RTW + rt) * 16 + (lane & 15);
    if (m >= NPIX) m = 0;
    int py, px;
    box_pixel<TW>(m, py, px);
    abase[rt] = ((py * RPX + px) * 4 + ((lane >> 4) ^ ((py & 1) << 1))) * 8;
  }

  f32x4 acc[RTW][CTW];
#pragma unroll
  for (int rt = 0; rt < RTW; ++rt)
#pragma unroll
    for (int ct = 0; ct < CTW; ++ct) acc[rt][ct] = (f32x4)0.f;

  static_assert(BR == 3 || BR == 9, "B ring: 3 or 9 slices");
  u16x8 bq[BR][CTW];
  load_halo(0);
#pragma unroll
  for (int k = 0; k < BR - 1; ++k) load_b(bq[k], k);
  store_halo(smem);
  __syncthreads();
  u16x8 fa[RTW];
#pragma unroll
  for (int rt = 0; rt < RTW; ++rt) fa[rt] = *(const u16x8*)(smem + abase[rt]);

  // Step s = 9c + t: at its top B(s+2) is fetched into slot (t+2) % 3 and (t
  // = 0) the next chunk's halo into registers; after tap 1 those registers go
  // to the other halo buffer.  Tap t multiplies fragments read during tap t-1
  // and reads tap t+1's behind each row tile's MFMAs.  The end of t = 7 is
  // the chunk's only barrier: after it tap 0 of the next chunk can be read (t
  // = 8), and every wave is past its last read of the buffer the chunk after
  // next overwrites (at its t = 1).
  for (int c = 0; c < nchunks; ++c) {
    const uint16_t* hb = smem + (c & 1) * HALO;
    uint16_t* hbn = smem + ((c + 1) & 1) * HALO;
    const int s0 = c * 9;
    auto step = [&](auto tc) {
      constexpr int t = decltype(tc)::value;
      load_b(bq[(t + BR - 1) % BR], s0 + t + BR - 1);
      if constexpr (t == 0) load_halo(c + 1 < nchunks ? c + 1 : c);
      constexpr int kyn = t < 8 ? (t + 1) / 3 : 0, kxn = t < 8 ? (t + 1) % 3 : 0;
      constexpr int ntoff = (kyn * RPX + kxn) * 32;
      const uint16_t* hnx = t < 8 ? hb : hbn;
#pragma unroll
      for (int rt = 0; rt < RTW; ++rt) {
#pragma unroll
        for (int ct = 0; ct < CTW; ++ct) acc[rt][ct] = T::mfma(fa[rt], bq[t % BR][ct], acc[rt][ct]);
        fa[rt] = *(const u16x8*)(hnx + abase[rt] + ntoff);
      }
      __builtin_amdgcn_sched_group_barrier(0x020, CTW + (t == 0 ? HPW : 0), 0);
#pragma unroll
      for (int rt = 0; rt < RTW; ++rt) {
        __builtin_amdgcn_sched_group_barrier(0x008, CTW, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      if constexpr (t == 1) store_halo(hbn);
      if constexpr (t == 7) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    };
    step(std::integral_constant<int, 0>{});
    step(std::integral_constant<int, 1>{});
    step(std::integral_constant<int, 2>{});
    step(std::integral_constant<int, 3>{});
    step(std::integral_constant<int, 4>{});
    step(std::integral_constant<int, 5>{});
    step(std::integral_constant<int, 6>{});
    step(std::integral_constant<int, 7>{});
    step(std::integral_constant<int, 8>{});
  }
  __syncthreads();

  uint16_t* ostg = smem;
  if (do_relu)
    stage_tile<T, RTW, CTW, OPS, POOL, true>(acc, ostg, bias + nb * BN, wm, wn, lane);
  else
    stage_tile<T, RTW, CTW, OPS, POOL, false>(acc, ostg, bias + nb * BN, wm, wn, lane);
  __syncthreads();
  const int Ho = POOL ? H / 2 : H, Wo = POOL ? W / 2 : W;
  const int oy0 = POOL ? y0 / 2 : y0, ox0 = POOL ? x0 / 2 : x0;
  store_tile<TH, TW, BN, POOL>(ostg, out, b, Ho, Wo, oy0, ox0, Cout, nb * BN, tid);
}

// conv1 (3 -> 32 @224) with the input normalisation of cvit_prediction.py:
// x/255 then (x - mean_c)/std_c (:41-42, :214-215), zero padding applied in
// normalised space exactly like the reference's Conv2d(padding=1).
// k = tap*4 + c (c padded to 4, taps padded to 16 -> K = 64 = two MFMA steps).
// U8 = true: uint8 NHWC crops (the face-crop format, cvit_prediction.py:202);
// U8 = false: already-normalised fp32 NCHW (CViT.forward's input contract).
constexpr float kMean[3] = {0.485f, 0.456f, 0.406f};
constexpr float kStd[3] = {0.229f, 0.224f, 0.225f};

template <class T, bool U8>
__global__ __launch_bounds__(256) void conv1_bn_relu(const void* __restrict__ in_,
                                                     const uint16_t* __restrict__ w1,
                                                     const float* __restrict__ bias,
                                                     uint16_t* __restrict__ out, int H, int W) {
  constexpr int TH = 16, TW = 16, HWD = 18, NH = 18 * 18, BN = 32;
  constexpr int WPS = 64 + 8;
  constexpr int OPS = BN + 8;
  constexpr int HSZ = NH * 4;
  constexpr int SMEM_OPER = HSZ + BN * WPS;
  constexpr int SMEM_OUT = TH * TW * OPS;
  constexpr int SMEM = SMEM_OPER > SMEM_OUT ? SMEM_OPER : SMEM_OUT;
  __shared__ __attribute__((aligned(16))) uint16_t smem[SMEM];
  uint16_t* halo = smem;
  uint16_t* wl = smem + HSZ;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_x = W / TW, tiles_per_img = (H / TH) * tiles_x;
  const int b = blockIdx.x / tiles_per_img;
  const int tile = blockIdx.x - b * tiles_per_img;
  const int ty = tile / tiles_x, tx = tile - ty * tiles_x;
  const int y0 = ty * TH, x0 = tx * TW;

  for (int p = tid; p < NH; p += 256) {
    const int hy = p / HWD, hx = p - (p / HWD) * HWD;
    const int y = y0 + hy - 1, x = x0 + hx - 1;
    float v[3] = {0.f, 0.f, 0.f};
    if (y >= 0 && y < H && x >= 0 && x < W) {
      if constexpr (U8) {
        const uint8_t* src = (const uint8_t*)in_ + (((size_t)b * H + y) * W + x) * 3;
#pragma unroll
        for (int c = 0; c < 3; ++c) v[c] = ((float)src[c] / 255.0f - kMean[c]) / kStd[c];
      } else {
        const float* src = (const float*)in_ + (size_t)b * 3 * H * W + (size_t)y * W + x;
#pragma unroll
        for (int c = 0; c < 3; ++c) v[c] = src[(size_t)c * H * W];
      }
    }
    u16x4 h;
    h[0] = T::from_f32(v[0]);
    h[1] = T::from_f32(v[1]);
    h[2] = T::from_f32(v[2]);
    h[3] = 0;
    *(u16x4*)(halo + p * 4) = h;
  }
  {
    const int n = tid >> 3, q = tid & 7;
    *(u16x8*)(wl + n * WPS + q * 8) = *(const u16x8*)(w1 + n * 64 + q * 8);
  }
  __syncthreads();

  f32x4 acc[4][2];
#pragma unroll
  for (int rt = 0; rt < 4; ++rt) acc[rt][0] = acc[rt][1] = (f32x4)0.f;
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    u16x8 bfr[2];
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
      bfr[ct] = *(const u16x8*)(wl + (ct * 16 + (lane & 15)) * WPS + ks * 32 + (lane >> 4) * 8);
    const int t0 = ks * 8 + (lane >> 4) * 2, t1 = t0 + 1;
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) {
      const int m = (wave * 4 + rt) * 16 + (lane & 15);
      int py, px;
      box_pixel<TW>(m, py, px);
      u16x4 lo = (u16x4)0, hi = (u16x4)0;
      if (t0 < 9) lo = *(const u16x4*)(halo + ((py + t0 / 3) * HWD + px + t0 % 3) * 4);
      if (t1 < 9) hi = *(const u16x4*)(halo + ((py + t1 / 3) * HWD + px + t1 % 3) * 4);
      const u16x8 a = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) acc[rt][ct] = T::mfma(a, bfr[ct], acc[rt][ct]);
    }
  }
  __syncthreads();
  uint16_t* ostg = smem;
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) {
    const int nl = ct * 16 + (lane & 15);
    const float bv = bias[nl];
#pragma unroll
    for (int rt = 0; rt < 4; ++rt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = (wave * 4 + rt) * 16 + (lane >> 4) * 4 + j;
        ostg[m * OPS + nl] = T::from_f32(relu(acc[rt][ct][j] + bv));
      }
  }
  __syncthreads();
  store_tile<TH, TW, BN, false>(ostg, out, b, H, W, y0, x0, BN, 0, tid);
}

}  // namespace fac

// ---------------------------------------------------------------------------
// Host launchers (C++ linkage, used by cvit_abi.hip).
namespace fac {

// Per-resolution kernel configuration (box TH x TW, BN output channels per
// workgroup, WM x WN wave grid); must agree with the weight packing in
// cvit_abi.hip, which asks conv_block_n() for BN.
//   112: 16x16 box, BN  64, 4x1 waves (256 rows, no padding), 1 halo buffer,
//        4 workgroups per CU
//    56:  8x28 box, BN 128, 2x2 waves (224 rows, no padding)
//    28:  4x28 box, BN 256, 1x4 waves (112 rows, no padding)
//    14: 14x14 box, BN 128, 1x4 waves (208 rows for 196 pixels); BN 192 / 64
//        for S3D's 14^2 (1,3,3) convs with cout 192 / 320 (round 3)
// (the 224 layers normally run inside stem224.hip; the 16x16/BN 32 kernel
// serves the unfused debug path)
//
// Other output widths (the ResNet-50 and S3D 3x3 layers routed here by
// fac_fake_amd/ops.py): 56: BN 64 (8x28 box, 2x2 waves); 28: BN 192 / 128
// (4x28 box, 1x4 waves).  0 = shape not supported.
int conv_block_n(int H, int cout) {
  switch (H) {
    case 224: return cout == 32 ? 32 : 0;
    case 112: return cout % 64 == 0 ? 64 : 0;
    case 56: return cout % 128 == 0 ? 128 : (cout % 64 == 0 ? 64 : 0);
    case 28:
      // (BN 128 for cout 256, i.e. 7 rounds of 512 workgroups instead of 3.5,
      // measured 6-8 % slower: the halved A reuse costs more than the tail)
      return cout % 256 == 0 ? 256 : (cout % 192 == 0 ? 192 : (cout % 128 == 0 ? 128 : 0));
    // (round 4: BN 256 as 1 x 4 waves of 208 x 64, half the A reads per MFMA,
    // one workgroup per CU: conv14-17 613 -> 632 us, not kept)
    case 14: return cout % 128 == 0 ? 128 : (cout % 192 == 0 ? 192 : (cout % 64 == 0 ? 64 : 0));
    default: return 0;
  }
}

// POOLED = false: no fused-pool instantiation (the 14x14 / BN 192 tile would
// spill with it; no model pools after such a layer).
template <class T, int TH, int TW, int BN, int WM, int WN, int HB = 2, int OCC = 2, bool PB = true, bool POOLED = true,
          int WR = 3>
static hipError_t launch_box(const uint16_t* in, const uint16_t* wpk, const float* bias, uint16_t* out, int B, int H,
                             int Cin, int Cout, bool pool, const uint16_t* zero16, hipStream_t st, int relu) {
  dim3 grid(B * (H / TH) * (H / TW), Cout / BN);
  if constexpr (POOLED) {
    if (pool) {
      conv3x3_bn_relu<T, TH, TW, BN, WM, WN, true, HB, OCC, PB, WR>
          <<<grid, 256, 0, st>>>(in, wpk, bias, out, H, H, Cin, Cout, zero16, relu);
      return hipSuccess;
    }
  } else if (pool) {
    return hipErrorInvalidValue;
  }
  conv3x3_bn_relu<T, TH, TW, BN, WM, WN, false, HB, OCC, PB, WR>
      <<<grid, 256, 0, st>>>(in, wpk, bias, out, H, H, Cin, Cout, zero16, relu);
  return hipSuccess;
}

// conv3x3_db launch (weights straight to VGPRs, one barrier per chunk)
template <class T, int TH, int TW, int BN, int WM, int WN, int OCC = 2, int BR = 3>
static hipError_t launch_db(const uint16_t* in, const uint16_t* wpk, const float* bias, uint16_t* out, int B, int H,
                            int Cin, int Cout, bool pool, const uint16_t* zero16, hipStream_t st, int relu) {
  dim3 grid(B * (H / TH) * (H / TW), Cout / BN);
  if (pool)
    conv3x3_db<T, TH, TW, BN, WM, WN, true, OCC, BR>
        <<<grid, 256, 0, st>>>(in, wpk, bias, out, H, H, Cin, Cout, zero16, relu);
  else
    conv3x3_db<T, TH, TW, BN, WM, WN, false, OCC, BR>
        <<<grid, 256, 0, st>>>(in, wpk, bias, out, H, H, Cin, Cout, zero16, relu);
  return hipSuccess;
}


// conv3x3_db for the 28^2 tiles.  Same box, bit-identical outputs
// (tools/archive/db_ab.py, round 4): conv10-13 101.7/178.2/177.2/163.2 ->
// 91.1/164.8/165.6/153.4 us against the LDS weight ring (that arm, option
// "conv_db" 0, was removed in round 5).  At 56^2 it was neutral (B shared by
// two waves of the 2x2 grid doubles its L2 reads), at 14^2 slower (the 1x4
// tile needs ~280 VGPRs and spills; the 2x2 tile pads 196 pixels to 224
// rows), at 112^2 15-20 % slower (four waves re-read the same B): those keep
// the LDS weight ring.

// 9-slice weight rings for grids of at most two workgroups per CU (few crops;
// option "conv_ring9", process-wide, A/B): bit 0 = the 14x14 / BN 64 tile
// (the few-crop 14^2 convs, conv_small), bit 1 = it with the B-fragment
// prefetch (PB) too, bit 2 = conv3x3_db's 4x28 / BN 128 tile (the few-crop
// 28^2 convs)
static int g_ring9 = 6;
// (Round 5, not kept: the 14x14 / BN 128 tile at B = 256 with 4- or 5-slice
// rings cycling their slots at run time, 72 / 80 KB of LDS, still two per
// CU: conv15-17 0.186 -> 0.196-0.201 ms.  At two workgroups per CU the slice
// wait is covered; only the one-per-CU grids gain from depth.)
void set_conv_ring9(int v) { g_ring9 = v; }
static int cu_count() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cached[dev]) {
    int n = 0;
    cached[dev] = hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0 ? n : 256;
  }
  return cached[dev];
}

template <class T>
static hipError_t launch_conv_t(const uint16_t* in, const uint16_t* wpk, const float* bias, uint16_t* out,
                                int B, int H, int W, int Cin, int Cout, bool pool, const uint16_t* z, hipStream_t st,
                                int relu, int bn) {
  if (W != H) return hipErrorInvalidValue;
  if (bn == 0) bn = conv_block_n(H, Cout);
  if (bn <= 0 || Cout % bn) return hipErrorInvalidValue;
  const bool few = g_ring9 && (long)B * (Cout / bn) * (H == 14 ? 1 : H == 28 ? 7 : 1 << 30) <= 2L * cu_count();
  const int ring9 = few ? g_ring9 : 0;
  switch (H * 1000 + bn) {
    case 224032: launch_box<T, 16, 16, 32, 4, 1, 2, 2, false>(in, wpk, bias, out, B, H, Cin, Cout, pool, z, st, relu); break;
    // 112: one halo buffer, 4 workgroups per CU (A/B in one process, MI355X:
    // conv4-6 886 -> 769 us vs two halo buffers at 2 per CU)
    case 112064:
      // the pooled tile (conv6) spills at 4 per CU (128 VGPRs): 2 per CU
      // (same box: conv4-6 0.665 -> 0.60 ms)
      if (pool)
        launch_box<T, 16, 16, 64, 4, 1, 1, 2, false>(in, wpk, bias, out, B, H, Cin, Cout, pool, z, st, relu);
      else
        launch_box<T, 16, 16, 64, 4, 1, 1, 4, false>(in, wpk, bias, out, B, H, Cin, Cout, pool, z, st, relu);
      break;
    case 56128: launch_box<T, 8, 28, 128, 2, 2>(in, wpk, bias, out, B, H, Cin, Cout, pool, z, st, relu); break;
    case 56064: launch_box<T, 8, 28, 64, 2, 2>(in, wpk, bias, out, B, H, Cin, Cout, pool, z, st, relu); break;
    case 28256: launch_db<T, 4, 28, 256, 1, 4>(in, wpk, bias, out, B, H, Cin, Cout, pool, z, st, relu); break;
    case 28192: launch_db<T, 4, 28, 192, 1, 4>(in, wpk, bias, out, B, H, Cin, Cout, pool, z, st, relu); break;
    case 28128:
      if (ring9 & 4)
        launch_db<T, 4, 28, 128, 1, 4, 2, 9>(in, wpk, bias, out, B, H, Cin, Cout, pool, z, st, relu);
      else
        launch_db<T, 4, 28, 128, 1, 4>(in, wpk, bias, out, B, H, Cin, Cout, pool, z, st, relu);
      break;
    // (a two-box 14x14 workgroup needs 256+ VGPRs and spills: not built)
    case 14128:
      launch_box<T, 14, 14, 128, 1, 4, 2, 2, false>(in, wpk, bias, out, B, H, Cin, Cout, pool, z, st, relu);
      break;
    case 14192:
      if (launch_box<T, 14, 14, 192, 1, 4, 2, 2, false, false>(in, wpk, bias, out, B, H, Cin, Cout, pool, z, st, relu) != hipSuccess)
        return hipErrorInvalidValue;
      break;
    case 14032:
      if (ring9 & 2)
        launch_box<T, 14, 14, 32, 4, 1, 2, 2, true, true, 9>(in, wpk, bias, out, B, H, Cin, Cout, pool, z, st, relu);
      else
        launch_box<T, 14, 14, 32, 4, 1, 2, 2, true>(in, wpk, bias, out, B, H, Cin, Cout, pool, z, st, relu);
      break;
    case 14064:
      if (ring9 & 2)
        launch_box<T, 14, 14, 64, 1, 4, 2, 2, true, true, 9>(in, wpk, bias, out, B, H, Cin, Cout, pool, z, st, relu);
      else if (ring9 & 1)
        launch_box<T, 14, 14, 64, 1, 4, 2, 2, false, true, 9>(in, wpk, bias, out, B, H, Cin, Cout, pool, z, st, relu);
      else
        launch_box<T, 14, 14, 64, 1, 4, 2, 2, false>(in, wpk, bias, out, B, H, Cin, Cout, pool, z, st, relu);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// bn: the output-channel block (0 = conv_block_n's; the weights must be
// packed for the same block, pack_conv3x3).  Every block gives bit-identical
// outputs (same k order per output channel).
hipError_t launch_conv3x3(int dtype, const uint16_t* in, const uint16_t* wpk, const float* bias, uint16_t* out,
                          int B, int H, int W, int Cin, int Cout, bool pool, const uint16_t* zero16, hipStream_t st,
                          bool relu, int bn) {
  if (dtype == 0) return launch_conv_t<BF16>(in, wpk, bias, out, B, H, W, Cin, Cout, pool, zero16, st, relu, bn);
  return launch_conv_t<F16>(in, wpk, bias, out, B, H, W, Cin, Cout, pool, zero16, st, relu, bn);
}

hipError_t launch_conv1(int dtype, bool u8, const void* in, const uint16_t* w1, const float* bias, uint16_t* out,
                        int B, int H, int W, hipStream_t st) {
  dim3 grid(B * (H / 16) * (W / 16));
  if (dtype == 0) {
    if (u8) conv1_bn_relu<BF16, true><<<grid, 256, 0, st>>>(in, w1, bias, out, H, W);
    else conv1_bn_relu<BF16, false><<<grid, 256, 0, st>>>(in, w1, bias, out, H, W);
  } else {
    if (u8) conv1_bn_relu<F16, true><<<grid, 256, 0, st>>>(in, w1, bias, out, H, W);
    else conv1_bn_relu<F16, false><<<grid, 256, 0, st>>>(in, w1, bias, out, H, W);
  }
  return hipGetLastError();
}

}  // namespace fac
