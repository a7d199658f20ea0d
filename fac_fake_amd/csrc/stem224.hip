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
#include <cstdlib>
#include <utility>

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
template <class T, bool TR, int NT, int RP>
__device__ __forceinline__ void tap_pipeline(f32x4 (&acc)[NT][2], const uint16_t* img, const int (&rd)[NT],
                                             const uint16_t* wl) {
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
                                                        uint16_t* __restrict__ out, int ntiles,
                                                        int* __restrict__ sched) {
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
  auto fetch = [&](int tile) {
    const int b = tile / TPI, rr = tile - (tile / TPI) * TPI;
    const int ty = rr / TPR, tx = rr - (rr / TPR) * TPR;
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
        const uint8_t* src = (const uint8_t*)in_ + (((size_t)b * IMG + y) * IMG + x) * 3;
        uint16_t v01;
        __builtin_memcpy(&v01, src, 2);
        raw01[k] = v01;
        raw2[k] = src[2];
      } else {
        const float* src = (const float*)in_ + (size_t)b * 3 * IMG * IMG + (size_t)y * IMG + x;
        raw[k][0] = src[0];
        raw[k][1] = src[IMG * IMG];
        raw[k][2] = src[2 * IMG * IMG];
      }
    }
  };
  // Box schedule.  sched == nullptr: static, box blockIdx.x + k*gridDim.x.
  // Otherwise dynamic: boxes are claimed from the counter sched[0] one box
  // ahead (the claim for box j+1 is made during box j, so its pixels
  // can be prefetched during box j), and a workgroup that starts late -- its
  // CU still held by another stream's kernel -- simply claims fewer boxes
  // instead of finishing its fixed share last.  s_tile[(j+1)&1] holds the
  // claim for box j+1; every reader of a slot is past two barriers before
  // thread 0 overwrites it.  The last workgroup out resets the counters.
  __shared__ int s_tile[2];
  int tile = blockIdx.x;
  if (sched && tid == 0) s_tile[0] = atomicAdd(sched, 1);
  __syncthreads();  // LUT and weights written (the first box reads the LUT before its barrier), claim published
  if (sched) tile = s_tile[0];
  fetch(tile);

  for (int j = 0; tile < ntiles; ++j) {
    // the claim's round trip overlaps staging and conv1: it is published in
    // LDS only before conv1's closing barrier
    int claim = 0;
    if (sched && tid == 0) claim = atomicAdd(sched, 1);
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
    if (sched && tid == 0) s_tile[(j + 1) & 1] = claim;
    lds_barrier();
    STEM_STAMP(2);

    const int next = sched ? s_tile[(j + 1) & 1] : tile + gridDim.x;
    fetch(next);  // next box's pixels land while conv2/conv3 run

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
      tap_pipeline<T, true, N2, RP>(acc, c1, c2_rd, sw2 + (g * 32 + r16) * 8);
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
      tap_pipeline<T, false, 4, RP>(acc, c2, c3_rd, sw3 + (g * 32 + r16) * 8);
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
    {  // 128 pooled pixels x 4 16-byte channel quarters = 512 threads
      const int w = tid >> 2, q = tid & 3;
      const int wy = w >> 4, wx = w & 15;
      *(u16x8*)(out + (((size_t)b * 112 + (y0 >> 1) + wy) * 112 + (x0 >> 1) + wx) * 32 + q * 8) =
          *(const u16x8*)(ostg + w * 40 + q * 8);
    }
    tile = next;
  }
  // every claim of every workgroup precedes its arrival here: the last one
  // to arrive leaves both counters at zero for the next launch
  if (sched && tid == 0 && atomicAdd(sched + 1, 1) == (int)gridDim.x - 1) {
    atomicExch(sched, 0);
    atomicExch(sched + 1, 0);
  }
}

// ---------------------------------------------------------------------------
// stem224_strip: the same box walk with conv2 and conv3 on strip tiles.
//
// A strip is R vertically stacked 16-pixel row tiles of one 16-column band.
// For a fixed kx the fragment of input row r (16 pixels x 32 channels, one
// ds_read_b128 per lane) is the tap-(ky, kx) operand of output rows r - ky,
// ky = 0..2, so it is read once for up to three row tiles: 3 (R + 2) pixel
// fragment reads per strip instead of 9 R (conv3: 18 instead of 36 per wave,
// conv2: 21-27 instead of 45).  conv2's 18x34 region is two 18-row strips of
// 16 columns (split 5+5+4+4 rows over the waves of a band) plus the two
// right-hand columns, 36 pixels, as three wrapped tiles on waves 4-6 (wave 7
// carries a dummy one, computed and not stored: its SIMD partner wave 3 has
// five strip rows).  The transposed stages (conv1, conv2) compute channel
// 8*(i>>2) + 4*ct + (i&3) in MFMA row i of channel tile ct, so each lane ends
// with channels 8g..8g+7 of its pixel: one conflict-free 16-byte LDS store
// per pixel instead of two 2-way-conflicted 8-byte ones.  conv3 pools a
// strip's row pairs in registers (the two pixels of a window row are
// accumulator elements of one lane, the two rows are consecutive tiles).
// Plane pitches are multiples of 16 slots: the strip reads of every lane
// group then cover 16 distinct 4-bank groups (conflict-free).
// ---------------------------------------------------------------------------

__device__ __forceinline__ int trow(int ct, int i) { return 8 * (i >> 2) + 4 * ct + (i & 3); }

// Taps of one strip (rows 0..R-1 of acc) plus, with LEFT, one wrapped tile
// (acc[R]).  img + sb: this lane's tap-(0,0) fragment of strip row 0; row r,
// kx at + (r*RP + kx)*8.  img + lb: the wrapped tile's.  wl: this lane's
// weight fragment of tap 0, channel tile 0; tap t, tile ct at
// wl + t*1024 + ct*CTOFF.  TR: transposed MFMA (C^T = W . X^T).
template <class F, int... I>
__device__ __forceinline__ void static_for_impl(F& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

template <class T, bool TR, int R, bool LEFT, int RP, int CTOFF>
__device__ __forceinline__ void strip_taps(f32x4 (&acc)[R + (LEFT ? 1 : 0)][2], const uint16_t* img, int sb, int lb,
                                           const uint16_t* wl) {
  // Steps per kx: the strip's R + 2 input rows, then the wrapped tile's 3 rows.
  // All fragments of kx + 1 (and its weights) are read during kx's MFMAs, one
  // per step, so no MFMA waits on a read issued less than a kx earlier.
  constexpr int NS = R + 2 + (LEFT ? 3 : 0);
  u16x8 w[3][2], wn[3][2], fc[NS], fx[NS];
  auto rd = [&](auto sc, int kx) -> u16x8 {
    constexpr int s = decltype(sc)::value;
    if constexpr (s < R + 2) return *(const u16x8*)(img + sb + (s * RP + kx) * 8);
    else return *(const u16x8*)(img + lb + ((s - (R + 2)) * RP + kx) * 8);
  };
#pragma unroll
  for (int ky = 0; ky < 3; ++ky)
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) w[ky][ct] = *(const u16x8*)(wl + ky * 3 * 1024 + ct * CTOFF);
  static_for<NS>([&](auto sc) { fc[decltype(sc)::value] = rd(sc, 0); });
  static_for<3>([&](auto kxc) {
    constexpr int kx = decltype(kxc)::value;
    static_for<NS>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      constexpr bool wload = s == 1 && kx < 2;
      constexpr int nrd = (kx < 2 ? 1 : 0) + (wload ? 6 : 0);
      if constexpr (kx < 2) fx[s] = rd(sc, kx + 1);
      if constexpr (wload) {
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int ct = 0; ct < 2; ++ct) wn[ky][ct] = *(const u16x8*)(wl + (ky * 3 + kx + 1) * 1024 + ct * CTOFF);
      }
      constexpr int nm = s < R + 2 ? 2 * ((s < R ? 1 : 0) + (s >= 1 && s - 1 < R ? 1 : 0) + (s >= 2 && s - 2 < R ? 1 : 0))
                                   : (LEFT ? 2 : 0);
      const u16x8 f = fc[s];
      if constexpr (s < R + 2) {
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const int o = s - ky;
          if (o >= 0 && o < R) {
#pragma unroll
            for (int ct = 0; ct < 2; ++ct)
              acc[o][ct] = TR ? T::mfma(w[ky][ct], f, acc[o][ct]) : T::mfma(f, w[ky][ct], acc[o][ct]);
          }
        }
      } else if constexpr (LEFT) {
        constexpr int ky = s - (R + 2);
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
          acc[R][ct] = TR ? T::mfma(w[ky][ct], f, acc[R][ct]) : T::mfma(f, w[ky][ct], acc[R][ct]);
      }
      if constexpr (nrd > 0) __builtin_amdgcn_sched_group_barrier(0x100, nrd, 0);
      if constexpr (nm > 0) __builtin_amdgcn_sched_group_barrier(0x008, nm, 0);
      __builtin_amdgcn_sched_barrier(0);
    });
    if constexpr (kx < 2) {
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) w[ky][ct] = wn[ky][ct];
#pragma unroll
      for (int i = 0; i < NS; ++i) fc[i] = fx[i];
    }
  });
}

template <class T, int R, bool LEFT, int RP, int P2>
__device__ __forceinline__ void conv2_strip(uint16_t* c1, uint16_t* c2, const uint16_t* sw2, const f32x4 (&bt2)[2],
                                            int wave, int g, int r16, int y0, int x0, bool interior, int lane,
                                            int j) {
  (void)lane;
  (void)j;
  constexpr int P1 = 20 * RP, NL = 36;
  const int xs = 16 * (wave & 1);
  const int rs = (wave >> 1) * 5 - (wave >= 6 ? 1 : 0);
  // wrapped tile (waves 4-7: tiles 0, 1, 2 and a dummy): pixel m = lt*16 + r16
  // of the 2-column remainder, (m >> 1, 32 + (m & 1))
  const int lm = (wave - 4) * 16 + r16;
  const bool lvalid = LEFT && lm < NL;
  const int lmc = lvalid ? lm : 0;
  const int lrow = lmc >> 1, lcol = 32 + (lmc & 1);
  f32x4 acc[R + (LEFT ? 1 : 0)][2];
#pragma unroll
  for (int i = 0; i < R + (LEFT ? 1 : 0); ++i) {
    acc[i][0] = bt2[0];
    acc[i][1] = bt2[1];
  }
  strip_taps<T, true, R, LEFT, RP, 32>(acc, c1, (g * P1 + rs * RP + xs + r16) * 8, (g * P1 + lrow * RP + lcol) * 8,
                                       sw2 + (g * 32 + trow(0, r16)) * 8);
  STEM_STAMP(5);
  auto store = [&](const f32x4& a0, const f32x4& a1, int py, int px) {
    bool keep = true;
    if (!interior) keep = (unsigned)(y0 - 1 + py) < 224u && (unsigned)(x0 - 1 + px) < 224u;
    f32x4 r0, r1;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      r0[j] = relu(a0[j]);
      r1[j] = relu(a1[j]);
    }
    const u16x4 lo = T::pack4(r0), hi = T::pack4(r1);
    u16x8 o = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    if (!keep) o = (u16x8)0;
    *(u16x8*)(c2 + (g * P2 + py * RP + px) * 8) = o;
  };
#pragma unroll
  for (int o = 0; o < R; ++o) store(acc[o][0], acc[o][1], rs + o, xs + r16);
  if constexpr (LEFT) {
    if (lvalid) store(acc[R][0], acc[R][1], lrow, lcol);
  }
}

template <class T, bool U8>
__global__ __launch_bounds__(512, 1) void stem224_strip(const void* __restrict__ in_,
                                                        const uint16_t* __restrict__ w1g,
                                                        const float* __restrict__ b1,
                                                        const uint16_t* __restrict__ w2g,
                                                        const float* __restrict__ b2,
                                                        const uint16_t* __restrict__ w3g,
                                                        const float* __restrict__ b3,
                                                        uint16_t* __restrict__ out, int ntiles,
                                                        int* __restrict__ sched) {
  constexpr int IMG = 224, TPR = 7, TPI = 98;
  constexpr int BW = 32;
  constexpr int IW = BW + 6, IN_PIX = 22 * IW;
  constexpr int C1W = BW + 4, C1_PIX = 20 * C1W;
  constexpr int RP = 40;
  constexpr int P1 = 20 * RP, P2 = 18 * RP;  // multiples of 16 slots (strip reads conflict-free)
  constexpr int W1P = 72;
  constexpr int WSZ = 9 * 4 * 32 * 8;
  constexpr int OFF_W2 = 32 * W1P, OFF_W3 = OFF_W2 + WSZ, OFF_C1 = OFF_W3 + WSZ;
  constexpr int OFF_C2 = OFF_C1 + 4 * P1 * 8;
  constexpr int OFF_LUT = OFF_C2 + 4 * P2 * 8;
  constexpr int SMEM = OFF_LUT + 3 * 256;
  __shared__ __attribute__((aligned(16))) uint16_t smem[SMEM];
  uint16_t* const sw1 = smem;
  uint16_t* const sw2 = smem + OFF_W2;
  uint16_t* const sw3 = smem + OFF_W3;
  uint16_t* const c1 = smem + OFF_C1;
  uint16_t* const c2 = smem + OFF_C2;
  uint16_t* const lut = smem + OFF_LUT;
  uint16_t* const sin = c2;
  uint16_t* const ostg = c1;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;

  for (int i = tid; i < 32 * 8; i += 512)
    *(u16x8*)(sw1 + (i >> 3) * W1P + (i & 7) * 8) = *(const u16x8*)(w1g + i * 8);
  for (int i = tid; i < WSZ / 8; i += 512) {
    *(u16x8*)(sw2 + i * 8) = *(const u16x8*)(w2g + i * 8);
    *(u16x8*)(sw3 + i * 8) = *(const u16x8*)(w3g + i * 8);
  }
  if constexpr (U8) {
    for (int i = tid; i < 3 * 256; i += 512) {
      const int c = i >> 8, v = i & 255;
      lut[i] = T::from_f32(((float)v / 255.0f - kNormMean[c]) / kNormStd[c]);
    }
  }
  // Accumulators start at the folded-BN bias of the channels they hold
  // (conv1/conv2 transposed: channel 8g + 4ct + j; conv3: 16ct + r16).
  f32x4 bt1[2], bt2[2], bn3[2];
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bt1[ct][j] = b1[8 * g + 4 * ct + j];
      bt2[ct][j] = b2[8 * g + 4 * ct + j];
    }
    bn3[ct] = (f32x4)b3[ct * 16 + r16];
  }
  constexpr int RT1 = (C1_PIX + 15) / 16, N1 = (RT1 + 7) / 8;  // 45 row tiles, 6 per wave (max)
  int in_off[N1][2], c1_wr[N1];
#pragma unroll
  for (int i = 0; i < N1; ++i) {
    const int rt = wave + 8 * i;
    const int m = (rt < RT1 ? rt : 0) * 16 + r16;
    const int cy = m / C1W, cx = m - (m / C1W) * C1W;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int pr = ks * 4 + g, ky = pr < 6 ? pr >> 1 : 2, kxp = pr & 1;
      in_off[i][ks] = ((cy + ky) * IW + cx + 2 * kxp) * 8;
    }
    c1_wr[i] = (g * P1 + cy * RP + cx) * 8;
  }

  uint32_t raw01[2], raw2[2];
  float raw[2][3];
  bool raw_in[2];
  auto fetch = [&](int tile) {
    const int b = tile / TPI, rr = tile - (tile / TPI) * TPI;
    const int ty = rr / TPR, tx = rr - (rr / TPR) * TPR;
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
        const uint8_t* src = (const uint8_t*)in_ + (((size_t)b * IMG + y) * IMG + x) * 3;
        uint16_t v01;
        __builtin_memcpy(&v01, src, 2);
        raw01[k] = v01;
        raw2[k] = src[2];
      } else {
        const float* src = (const float*)in_ + (size_t)b * 3 * IMG * IMG + (size_t)y * IMG + x;
        raw[k][0] = src[0];
        raw[k][1] = src[IMG * IMG];
        raw[k][2] = src[2 * IMG * IMG];
      }
    }
  };
  __shared__ int s_tile[2];
  int tile = blockIdx.x;
  if (sched && tid == 0) s_tile[0] = atomicAdd(sched, 1);
  __syncthreads();
  if (sched) tile = s_tile[0];
  fetch(tile);

  for (int j = 0; tile < ntiles; ++j) {
    int claim = 0;
    if (sched && tid == 0) claim = atomicAdd(sched, 1);
    const int b = tile / TPI, rr = tile - (tile / TPI) * TPI;
    const int ty = rr / TPR, tx = rr - (rr / TPR) * TPR;
    const int y0 = ty * 16, x0 = tx * BW;
    // ---- A: normalised input (as stem224_fused)
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
    lds_barrier();
    STEM_STAMP(0);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int p = tid + 512 * k;
      if (p < IN_PIX) {
        const u16x4 h = hv[k];
        const int ix = p - (p / IW) * IW;
        *(u16x4*)(sin + p * 8) = h;
        if (ix > 0) *(u16x4*)(sin + p * 8 - 4) = h;
        if (ix == IW - 1) *(u16x4*)(sin + p * 8 + 4) = (u16x4)0;
      }
    }
    lds_barrier();
    STEM_STAMP(1);
    const bool interior = ty > 0 && ty < IMG / 16 - 1 && tx > 0 && tx < TPR - 1;

    // ---- B: conv1 over the 20x36 region, raster row tiles, transposed, permuted rows
    u16x8 w1f[2][2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) w1f[ks][ct] = *(const u16x8*)(sw1 + trow(ct, r16) * W1P + ks * 32 + g * 8);
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
      f32x4 r0, r1;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        r0[q] = relu(acc1[i][0][q]);
        r1[q] = relu(acc1[i][1][q]);
      }
      const u16x4 lo = T::pack4(r0), hi = T::pack4(r1);
      u16x8 o = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      if (!inside) o = (u16x8)0;
      if (rt < RT1) *(u16x8*)(c1 + c1_wr[i]) = o;
    }
    if (sched && tid == 0) s_tile[(j + 1) & 1] = claim;
    lds_barrier();
    STEM_STAMP(2);

    const int next = sched ? s_tile[(j + 1) & 1] : tile + gridDim.x;
    fetch(next);

    // ---- C: conv2 over the 18x34 region on strips
    if (wave < 4) conv2_strip<T, 5, false, RP, P2>(c1, c2, sw2, bt2, wave, g, r16, y0, x0, interior, lane, j);
    else conv2_strip<T, 4, true, RP, P2>(c1, c2, sw2, bt2, wave, g, r16, y0, x0, interior, lane, j);
    lds_barrier();
    STEM_STAMP(3);

    // ---- D: conv3 over the 16x32 box on strips (band wave&1, rows 4*(wave>>1)..+3),
    // 2x2 max-pool in registers
    {
      f32x4 acc[4][2];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        acc[i][0] = bn3[0];
        acc[i][1] = bn3[1];
      }
      const int xs = 16 * (wave & 1), rs = 4 * (wave >> 1);
      strip_taps<T, false, 4, false, RP, 128>(acc, c2, (g * P2 + rs * RP + xs + r16) * 8, 0,
                                              sw3 + (g * 32 + r16) * 8);
      STEM_STAMP(6);
      // tile o holds pixels (rs + o, xs + 4g + q) of channel 16ct + r16 in acc[o][ct][q]
#pragma unroll
      for (int op = 0; op < 2; ++op)
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const f32x4 a = acc[2 * op][ct], c = acc[2 * op + 1][ct];
            const float mx = fmaxf(fmaxf(a[2 * h], a[2 * h + 1]), fmaxf(c[2 * h], c[2 * h + 1]));
            const int pw = ((wave >> 1) * 2 + op) * 16 + 8 * (wave & 1) + 2 * g + h;
            ostg[pw * 40 + ct * 16 + r16] = T::from_f32(relu(mx));
          }
    }
    lds_barrier();
    STEM_STAMP(4);
    {
      const int w = tid >> 2, q = tid & 3;
      const int wy = w >> 4, wx = w & 15;
      *(u16x8*)(out + (((size_t)b * 112 + (y0 >> 1) + wy) * 112 + (x0 >> 1) + wx) * 32 + q * 8) =
          *(const u16x8*)(ostg + w * 40 + q * 8);
    }
    tile = next;
  }
  if (sched && tid == 0 && atomicAdd(sched + 1, 1) == (int)gridDim.x - 1) {
    atomicExch(sched, 0);
    atomicExch(sched + 1, 0);
  }
}

static int g_stem_version = [] {
  const char* e = std::getenv("FAC_STEM_VERSION");
  return e && e[0] == '1' ? 1 : 0;
}();
void set_stem_version(int v) { g_stem_version = v; }
int stem_version() { return g_stem_version; }

hipError_t launch_stem224(int dtype, bool u8, const void* in, const uint16_t* w1, const float* b1, const uint16_t* w2,
                          const float* b2, const uint16_t* w3, const float* b3, uint16_t* out, int B, int nwg,
                          hipStream_t st, int* sched) {
  const int ntiles = B * 98;  // 16x32 boxes
  const int grid = nwg < ntiles ? nwg : ntiles;
  if (g_stem_version == 1) {
    if (dtype == 0) {
      if (u8) stem224_strip<BF16, true><<<grid, 512, 0, st>>>(in, w1, b1, w2, b2, w3, b3, out, ntiles, sched);
      else stem224_strip<BF16, false><<<grid, 512, 0, st>>>(in, w1, b1, w2, b2, w3, b3, out, ntiles, sched);
    } else {
      if (u8) stem224_strip<F16, true><<<grid, 512, 0, st>>>(in, w1, b1, w2, b2, w3, b3, out, ntiles, sched);
      else stem224_strip<F16, false><<<grid, 512, 0, st>>>(in, w1, b1, w2, b2, w3, b3, out, ntiles, sched);
    }
    return hipGetLastError();
  }
  if (dtype == 0) {
    if (u8) stem224_fused<BF16, true><<<grid, 512, 0, st>>>(in, w1, b1, w2, b2, w3, b3, out, ntiles, sched);
    else stem224_fused<BF16, false><<<grid, 512, 0, st>>>(in, w1, b1, w2, b2, w3, b3, out, ntiles, sched);
  } else {
    if (u8) stem224_fused<F16, true><<<grid, 512, 0, st>>>(in, w1, b1, w2, b2, w3, b3, out, ntiles, sched);
    else stem224_fused<F16, false><<<grid, 512, 0, st>>>(in, w1, b1, w2, b2, w3, b3, out, ntiles, sched);
  }
  return hipGetLastError();
}

}  // namespace fac
