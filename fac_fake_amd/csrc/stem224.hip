// Fused 224x224 block of the conv stem: conv1 (3->32) -> conv2 (32->32) ->
// conv3 (32->32) -> MaxPool2d(2,2), each conv with folded BN + ReLU
// (CViT-main/model/cvit.py:88-97), plus the input normalisation of
// cvit_prediction.py:41-45,214-215 fused into conv1's staging.
//
// Unfused, this block moves ~13 MB per crop through HBM (three 224x224x32
// activations written and read back); fused, a crop costs its 150 KB of
// uint8 pixels in and 0.8 MB of pooled 112x112x32 out.
//
// One persistent 512-thread workgroup per CU keeps all three weight tensors
// in LDS (40 KB) and walks 16x32 output boxes.  Per box:
//   A: normalised input over the 22x38 region (conv1's receptive field);
//   B: conv1 over the 20x36 region conv2 needs -> LDS image c1;
//   C: conv2 over the 18x34 region conv3 needs -> LDS image c2;
//   D: conv3 over the 16x32 box, 2x2 max in registers -> 8x16x32 tile out.
// Intermediate pixels that fall outside the image are stored as 0, which is
// exactly the zero padding the next conv expects.  Recompute overhead:
// conv1 x1.41, conv2 x1.20 (conv1 is 0.7% of the network's FLOPs).  The
// 16x32 box (vs 16x16) cuts that recompute, gives every wave 4 conv3 row
// tiles per weight fetch (conv3 LDS reads per MFMA 1.0 -> 0.75), balances
// the row tiles over the 8 waves better and halves the barriers per pixel.
//
// conv1 and conv2 run "transposed" (C^T = W . X^T: MFMA rows = channels,
// cols = pixels), so each lane ends with 4 consecutive channels of one pixel
// and writes them to the chunk-major LDS image with one 8-byte store.
// conv3 runs in the normal orientation, where the window-major pixel order
// puts a whole 2x2 pooling window in one lane's 4 accumulators.
#include "common.hpp"

namespace fac {

template <int TW>
__device__ __forceinline__ void win_pixel(int m, int& py, int& px) {
  constexpr int WW = TW / 2;
  const int w = m >> 2, sub = m & 3;
  const int wy = w / WW, wx = w - wy * WW;
  py = 2 * wy + (sub >> 1);
  px = 2 * wx + (sub & 1);
}

// Workgroup barrier that orders LDS only: this wave's LDS accesses retire
// first (lgkmcnt(0)), its global stores and prefetch loads stay in flight
// (__syncthreads' fence would wait for them: vmcnt(0) every phase).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// The nine taps of one 3x3 conv stage over NT row tiles per wave,
// software-pipelined: tap t multiplies fragments read during tap t-1, and
// right behind each row tile's two MFMAs that tile's fragment for tap t+1 is
// read (the weights of tap t+1 ahead of the first tile).  The reads then
// overlap the MFMAs instead of each MFMA pair waiting on the read issued just
// before it (the compiler's own order: one read in flight per wave).
// TR: transposed orientation (C^T = W . X^T, conv2) or normal (conv3).
// img + rd[i]: tile i's fragment for tap 0; tap (ky,kx) is ky*RP + kx pixel
// slots further.  wl: this lane's weight row; tap t, channel tile ct at
// wl + (t*128 + ct*16)*8 (weights [tap][q][32][8]).
// mid(): work issued inside tap 2's MFMA stream (its VALU then issues in the
// MFMAs' shadow instead of ahead of the taps).
template <class T, bool TR, int NT, int RP, class Mid>
__device__ __forceinline__ void tap_pipeline(f32x4 (&acc)[NT][2], const uint16_t* img, const int (&rd)[NT],
                                             const uint16_t* wl, Mid&& mid) {
  u16x8 fa[NT], wf[2];
#pragma unroll
  for (int i = 0; i < NT; ++i) fa[i] = *(const u16x8*)(img + rd[i]);
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) wf[ct] = *(const u16x8*)(wl + ct * 16 * 8);
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int ntoff = (((t + 1) / 3) * RP + (t + 1) % 3) * 8;
    u16x8 wn[2];
    if (t < 8) {
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) wn[ct] = *(const u16x8*)(wl + ((t + 1) * 128 + ct * 16) * 8);
    }
    if (t == 2) mid();
#pragma unroll
    for (int i = 0; i < NT; ++i) {
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
        acc[i][ct] = TR ? T::mfma(wf[ct], fa[i], acc[i][ct]) : T::mfma(fa[i], wf[ct], acc[i][ct]);
      if (t < 8) fa[i] = *(const u16x8*)(img + rd[i] + ntoff);
    }
    if (t < 8) {
      wf[0] = wn[0];
      wf[1] = wn[1];
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

constexpr float kNormMean[3] = {0.485f, 0.456f, 0.406f};  // cvit_prediction.py:41
constexpr float kNormStd[3] = {0.229f, 0.224f, 0.225f};   // cvit_prediction.py:42

// Phase stamps (wave 0, per box, after each barrier) for tools/ubench/stem_ubench.hip only.
#ifdef STEM_STAMPS
__device__ unsigned long long stem_st[4][32][8][8];
#define STEM_STAMP(k)                                                                          \
  do {                                                                                         \
    __builtin_amdgcn_sched_barrier(0);                                                         \
    unsigned long long t_;                                                                     \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                 \
    __builtin_amdgcn_sched_barrier(0);                                                         \
    if (blockIdx.x < 4 && lane == 0 && j < 32) stem_st[blockIdx.x][j][wave][(k)] = t_;         \
  } while (0)
#else
#define STEM_STAMP(k) \
  do {                \
  } while (0)
#endif

template <class T, bool U8>
__global__ __launch_bounds__(512, 1) void stem224_fused(const void* __restrict__ in_,
                                                        const uint16_t* __restrict__ w1g,
                                                        const float* __restrict__ b1,
                                                        const uint16_t* __restrict__ w2g,
                                                        const float* __restrict__ b2,
                                                        const uint16_t* __restrict__ w3g,
                                                        const float* __restrict__ b3,
                                                        uint16_t* __restrict__ out, int ntiles) {
  constexpr int IMG = 224, TPR = 7, TPI = 98;     // 16x32 boxes per box row / per image
  constexpr int BW = 32;                          // box width (height 16)
  constexpr int IW = BW + 6, IN_PIX = 22 * IW;    // input region 22 x 38
  constexpr int C1W = BW + 4, C1_PIX = 20 * C1W;  // conv1 region 20 x 36 (45 row tiles)
  constexpr int C2W = BW + 2, C2_PIX = 18 * C2W;  // conv2 region 18 x 34 (39 row tiles)
  constexpr int RP = 40;                          // LDS image row pitch (16-byte units, == 8 mod 16)
  // plane pitches of c1 / c2, by simulating the ds_read_b128 lane groups:
  // conv2's reads of c1 1.18-way, conv3's reads of c2 conflict-free
  constexpr int P1 = 20 * RP + 8, P2 = 18 * RP;
  constexpr int W1P = 72;                         // conv1 weight row pitch (elements)
  constexpr int WSZ = 9 * 4 * 32 * 8;             // conv2/3 weights: [tap][q][32][8]
  constexpr int OFF_W2 = 32 * W1P, OFF_W3 = OFF_W2 + WSZ, OFF_C1 = OFF_W3 + WSZ;
  constexpr int OFF_C2 = OFF_C1 + 4 * P1 * 8;
  constexpr int OFF_LUT = OFF_C2 + 4 * P2 * 8;    // u8 -> normalised 16-bit value, per channel
  constexpr int SMEM = OFF_LUT + 3 * 256;
  __shared__ __attribute__((aligned(16))) uint16_t smem[SMEM];
  uint16_t* const sw1 = smem;
  uint16_t* const sw2 = smem + OFF_W2;
  uint16_t* const sw3 = smem + OFF_W3;
  uint16_t* const c1 = smem + OFF_C1;
  uint16_t* const c2 = smem + OFF_C2;
  uint16_t* const lut = smem + OFF_LUT;
  uint16_t* const sin = c2;    // 22x38 pixel-pair image (16 B slots): dead before conv2 writes c2
  uint16_t* const ostg = c1;   // 128 x (32+8) pooled tile: c1 is dead after conv2

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;

  for (int i = tid; i < 32 * 8; i += 512)
    *(u16x8*)(sw1 + (i >> 3) * W1P + (i & 7) * 8) = *(const u16x8*)(w1g + i * 8);
  for (int i = tid; i < WSZ / 8; i += 512) {
    *(u16x8*)(sw2 + i * 8) = *(const u16x8*)(w2g + i * 8);
    *(u16x8*)(sw3 + i * 8) = *(const u16x8*)(w3g + i * 8);
  }
  // The normalisation (x/255 - mean_c)/std_c of every possible uint8 value,
  // evaluated once with the reference's IEEE fp32 ops: staging is a lookup.
  if constexpr (U8) {
    for (int i = tid; i < 3 * 256; i += 512) {
      const int c = i >> 8, v = i & 255;
      lut[i] = T::from_f32(((float)v / 255.0f - kNormMean[c]) / kNormStd[c]);
    }
  }
  // Accumulators start at the folded-BN bias of the channels they hold
  // (conv1/conv2 transposed: channel 16ct + 4g + j; conv3: 16ct + r16).
  f32x4 bt1[2], bt2[2], bn3[2];
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bt1[ct][j] = b1[ct * 16 + 4 * g + j];
      bt2[ct][j] = b2[ct * 16 + 4 * g + j];
    }
    bn3[ct] = (f32x4)b3[ct * 16 + r16];
  }
  // Tile-invariant LDS offsets of this lane's rows in each stage.
  constexpr int RT1 = (C1_PIX + 15) / 16, RT2 = (C2_PIX + 15) / 16;  // 45, 39
  constexpr int N1 = (RT1 + 7) / 8, N2 = (RT2 + 7) / 8;              // 6, 5 row tiles per wave (max)
  int in_off[N1][2], c1_wr[N1];
#pragma unroll
  for (int i = 0; i < N1; ++i) {  // conv1: row tiles wave + 8i (< 45), raster over 20x36
    const int rt = wave + 8 * i;
    const int m = (rt < RT1 ? rt : 0) * 16 + r16;
    const int cy = m / C1W, cx = m - (m / C1W) * C1W;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      // lane chunk g of k-step ks = taps (ky, 2*kxp) and (ky, 2*kxp + 1): one
      // pixel-pair slot; chunks past ky = 2 carry zero weights (any slot)
      const int pr = ks * 4 + g, ky = pr < 6 ? pr >> 1 : 2, kxp = pr & 1;
      in_off[i][ks] = ((cy + ky) * IW + cx + 2 * kxp) * 8;
    }
    c1_wr[i] = ((g >> 1) * P1 + cy * RP + cx) * 8 + (g & 1) * 4;  // + ct*2*P1*8 (channels 16ct+4g..)
  }
  int c2_rd[N2], c2_wr[N2];
#pragma unroll
  for (int i = 0; i < N2; ++i) {  // conv2: row tiles wave + 8i (< 39), window-major over 18x34
    int m = (wave + 8 * i) * 16 + r16;
    if (m >= C2_PIX) m = 0;
    int py, px;
    win_pixel<C2W>(m, py, px);
    c2_rd[i] = (g * P1 + py * RP + px) * 8;
    c2_wr[i] = ((g >> 1) * P2 + py * RP + px) * 8 + (g & 1) * 4;
  }
  int c3_rd[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // conv3: row tiles 4*wave + i, window-major over 16x32
    int py, px;
    win_pixel<BW>((wave * 4 + i) * 16 + r16, py, px);
    c3_rd[i] = (g * P2 + py * RP + px) * 8;
  }

  // Raw input pixels of a box's 22x38 receptive field (pixel tid and
  // tid+512 of it), fetched one box ahead (during conv2/conv3 of the previous
  // box) so phase A never waits on HBM.
  // U8: the byte values, kept as integers until phase A (a conversion here
  // would make every wave wait for the loads right after issuing them);
  // F32: normalised floats
  uint32_t raw01[2], raw2[2];  // U8: channels 0|1 (one 2-byte load), channel 2
  float raw[2][3];
  bool raw_in[2];
  // Round 3: the U8 loads are unconditional (out-of-image and past-the-end
  // pixels read a valid pixel that is then discarded), all four issued back to back.  The branchy
  // form made the compiler re-allocate a pending load's registers and put
  // `s_waitcnt vmcnt(0)` between the two pixel pairs (every wave waited for
  // the first pair's HBM round trip, and for its own previous output stores:
  // 600-1400 cycles per box, tools/ubench/stem_ubench.hip stamp 8).
  // this thread's two receptive-field pixels (row, column, byte offset
  // within the box's window), fixed for every box
  int f_iy[2], f_ix[2], f_off[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int p = tid + 512 * k;
    f_iy[k] = p < IN_PIX ? p / IW : 1 << 20;  // past the window: never in the image
    f_ix[k] = p - (p / IW) * IW;
    f_off[k] = (f_iy[k] * IMG + f_ix[k]) * 3;
  }
  auto fetch = [&](int tile) {
    const int b = tile / TPI, rr = tile - (tile / TPI) * TPI;
    const int ty = rr / TPR, tx = rr - (rr / TPR) * TPR;
    if constexpr (U8) {
      // window origin (ty*16 - 3, tx*BW - 3) of crop b: wave-uniform
      const int oy = ty * 16 - 3, ox = tx * BW - 3;
      const long long wbase = ((long long)b * IMG * IMG + oy * IMG + ox) * 3;  // < 0 only for crop 0's top-left box
      const uint8_t* src[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        raw_in[k] = tile < ntiles && (unsigned)(oy + f_iy[k]) < (unsigned)IMG && (unsigned)(ox + f_ix[k]) < (unsigned)IMG;
        // out-of-image / past-the-end pixels load a valid pixel (crop 0's
        // first) whose value phase A discards (raw_in); one address space,
        // so the loads stay global_load (a select with another array made
        // them flat loads, which need vmcnt(0) lgkmcnt(0) waits)
        src[k] = (const uint8_t*)in_ + (raw_in[k] ? wbase + f_off[k] : 0LL);
      }
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        uint16_t v01;
        __builtin_memcpy(&v01, src[k], 2);
        raw01[k] = v01;
        raw2[k] = src[k][2];
      }
      return;
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      raw01[k] = raw2[k] = 0;
      raw[k][0] = raw[k][1] = raw[k][2] = 0.f;
      raw_in[k] = false;
      const int p = tid + 512 * k;
      if (p >= IN_PIX || tile >= ntiles) continue;
      const int iy = p / IW, ix = p - (p / IW) * IW;
      const int y = ty * 16 - 3 + iy, x = tx * BW - 3 + ix;
      if (y < 0 || y >= IMG || x < 0 || x >= IMG) continue;
      raw_in[k] = true;
      if constexpr (U8) {
      } else {
        const float* src = (const float*)in_ + (size_t)b * 3 * IMG * IMG + (size_t)y * IMG + x;
        raw[k][0] = src[0];
        raw[k][1] = src[IMG * IMG];
        raw[k][2] = src[2 * IMG * IMG];
      }
    }
  };
  // Static box schedule: box blockIdx.x + k*gridDim.x.  (Rounds 1-4 also had
  // a dynamic one, boxes claimed from a device counter one box ahead;
  // measured equal, 85.45k vs 85.46k crops/s, and removed in round 5.)
  int tile = blockIdx.x;
  __syncthreads();  // LUT and weights written (the first box reads the LUT before its barrier)
  fetch(tile);

  bool pend = false;  // a pooled tile waiting to be stored
  uint16_t* pend_ptr = out;
  u16x8 pend_v = (u16x8)0;
  for (int j = 0; tile < ntiles; ++j) {
    const int b = tile / TPI, rr = tile - (tile / TPI) * TPI;
    const int ty = rr / TPR, tx = rr - (rr / TPR) * TPR;
    const int y0 = ty * 16, x0 = tx * BW;
    // ---- A: normalised 16-bit input over (y0-3 .. y0+18) x (x0-3 .. x0+34);
    // out-of-image pixels were fetched as 0 (zero padding in normalised space).
    // The LUT lookups go before the box barrier (the LUT is never rewritten),
    // so their latency overlaps the wait for the previous box's last readers.
    u16x4 hv[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      u16x4 h;
      if constexpr (U8) {
        h[0] = raw_in[k] ? lut[raw01[k] & 255] : (uint16_t)0;
        h[1] = raw_in[k] ? lut[256 + (raw01[k] >> 8)] : (uint16_t)0;
        h[2] = raw_in[k] ? lut[512 + raw2[k]] : (uint16_t)0;
      } else {
        h[0] = T::from_f32(raw[k][0]);
        h[1] = T::from_f32(raw[k][1]);
        h[2] = T::from_f32(raw[k][2]);
      }
      h[3] = 0;
      hv[k] = h;
    }
    // the previous box's pooled tile leaves here, after this box's pixel
    // loads were consumed: at the loop head those loads are then the
    // youngest memory operations on every path, so their wait is exact and
    // never waits for a just-issued output store (storing at the end of the
    // box put the store behind the loads, and the compiler's merged wait for
    // the first and later iterations then drained the store too)
    if (pend) *(u16x8*)pend_ptr = pend_v;
    lds_barrier();  // previous tile's readers of sin(=c2) and ostg(=c1) are done
    STEM_STAMP(0);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int p = tid + 512 * k;
      if (p < IN_PIX) {
        const u16x4 h = hv[k];
        // pixel-pair slot p = (pixel p, pixel p+1): left half of slot p, right
        // half of slot p-1 (the last column's right half: zeros, zero weight)
        const int ix = p - (p / IW) * IW;
        *(u16x4*)(sin + p * 8) = h;
        if (ix > 0) *(u16x4*)(sin + p * 8 - 4) = h;
        if (ix == IW - 1) *(u16x4*)(sin + p * 8 + 4) = (u16x4)0;
      }
    }
    lds_barrier();
    STEM_STAMP(1);
    // interior boxes (no receptive field pixel outside the image) skip the zeroing
    const bool interior = ty > 0 && ty < IMG / 16 - 1 && tx > 0 && tx < TPR - 1;

    // ---- B: conv1 over the 20x36 region at (y0-2, x0-2): 45 row tiles, raster order
    u16x8 w1f[2][2];  // this lane's conv1 weight fragments [ks][ct], read once per box
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) w1f[ks][ct] = *(const u16x8*)(sw1 + (ct * 16 + r16) * W1P + ks * 32 + g * 8);
    // All of this wave's row tiles at once (waves 5-7 own five, the sixth is a
    // dummy over in_off's tile-0 slots, computed and not stored): reads, then
    // MFMAs, then the epilogue writes, so neither the LDS read latency nor the
    // MFMA -> store chain of one tile waits on the previous tile's (the c1
    // writes would otherwise pin every later sin read behind them).
    u16x8 pin[N1][2];
#pragma unroll
    for (int i = 0; i < N1; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) pin[i][ks] = *(const u16x8*)(sin + in_off[i][ks]);
    f32x4 acc1[N1][2];
#pragma unroll
    for (int i = 0; i < N1; ++i) {
      acc1[i][0] = bt1[0];
      acc1[i][1] = bt1[1];
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < N1; ++i)
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) acc1[i][ct] = T::mfma(w1f[ks][ct], pin[i][ks], acc1[i][ct]);
    STEM_STAMP(7);
#pragma unroll
    for (int i = 0; i < N1; ++i) {
      const int rt = wave + 8 * i;
      bool inside = rt < RT1;
      if (!interior && inside) {
        const int m = rt * 16 + r16;
        const int cy = m / C1W, cx = m - (m / C1W) * C1W;
        inside = (unsigned)(y0 - 2 + cy) < (unsigned)IMG && (unsigned)(x0 - 2 + cx) < (unsigned)IMG;
      }
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        f32x4 r;
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = relu(acc1[i][ct][j]);
        u16x4 o = T::pack4(r);
        if (!inside) o = (u16x4)0;
        if (rt < RT1) *(u16x4*)(c1 + c1_wr[i] + ct * 2 * P1 * 8) = o;
      }
    }
    lds_barrier();
    STEM_STAMP(2);

    const int next = tile + gridDim.x;

    // ---- C: conv2 over the 18x34 region at (y0-1, x0-1): window-major, 39 row tiles
    // (wave 7's fifth tile is a dummy over pixel 0, computed and not stored:
    // waves 0-6 own five tiles, so it costs no time and keeps the tap steps
    // branch-free for the software pipeline below)
    {
      f32x4 acc[N2][2];
#pragma unroll
      for (int i = 0; i < N2; ++i) {
        acc[i][0] = bt2[0];
        acc[i][1] = bt2[1];
      }
      // the next box's pixels are fetched inside conv2's taps and land while conv2/conv3 run
      tap_pipeline<T, true, N2, RP>(acc, c1, c2_rd, sw2 + (g * 32 + r16) * 8, [&] { fetch(next); });
      STEM_STAMP(5);
#pragma unroll
      for (int i = 0; i < N2; ++i) {
        const int m = (wave + 8 * i) * 16 + r16;
        bool keep = m < C2_PIX;
        if (!interior && keep) {
          int py, px;
          win_pixel<C2W>(m, py, px);
          keep = (unsigned)(y0 - 1 + py) < (unsigned)IMG && (unsigned)(x0 - 1 + px) < (unsigned)IMG;
        }
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
          f32x4 r;
#pragma unroll
          for (int j = 0; j < 4; ++j) r[j] = relu(acc[i][ct][j]);
          u16x4 o = T::pack4(r);
          if (!keep) o = (u16x4)0;
          if (m < C2_PIX) *(u16x4*)(c2 + c2_wr[i] + ct * 2 * P2 * 8) = o;
        }
      }
    }
    lds_barrier();
    STEM_STAMP(3);

    // ---- D: conv3 over the 16x32 box, window-major, 2x2 max-pool in registers
    {
      f32x4 acc[4][2];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        acc[i][0] = bn3[0];
        acc[i][1] = bn3[1];
      }
      tap_pipeline<T, false, 4, RP>(acc, c2, c3_rd, sw3 + (g * 32 + r16) * 8, [] {});
      STEM_STAMP(6);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
          const f32x4 v = acc[i][ct];
          const float mx = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
          ostg[((wave * 4 + i) * 4 + g) * 40 + ct * 16 + r16] = T::from_f32(relu(mx));
        }
    }
    lds_barrier();
    STEM_STAMP(4);
    {  // 128 pooled pixels x 4 16-byte channel quarters = 512 threads: read
       // now (ostg is overwritten in the next box's phase B), stored after
       // the next box's staging
      const int w = tid >> 2, q = tid & 3;
      const int wy = w >> 4, wx = w & 15;
      pend_ptr = out + (((size_t)b * 112 + (y0 >> 1) + wy) * 112 + (x0 >> 1) + wx) * 32 + q * 8;
      pend_v = *(const u16x8*)(ostg + w * 40 + q * 8);
      pend = true;
    }
    tile = next;
  }
  if (pend) *(u16x8*)pend_ptr = pend_v;
}

hipError_t launch_stem224(int dtype, bool u8, const void* in, const uint16_t* w1, const float* b1, const uint16_t* w2,
                          const float* b2, const uint16_t* w3, const float* b3, uint16_t* out, int B, int nwg,
                          hipStream_t st) {
  const int ntiles = B * 98;  // 16x32 boxes
  const int grid = nwg < ntiles ? nwg : ntiles;
#define FAC_STEM(TT, U) stem224_fused<TT, U><<<grid, 512, 0, st>>>(in, w1, b1, w2, b2, w3, b3, out, ntiles)
  if (dtype == 0) u8 ? FAC_STEM(BF16, true) : FAC_STEM(BF16, false);
  else u8 ? FAC_STEM(F16, true) : FAC_STEM(F16, false);
#undef FAC_STEM
  return hipGetLastError();
}

}  // namespace fac
