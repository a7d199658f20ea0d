// Face-crop preprocessing of config 3:
// cvit_prediction.py:111-116 takes frame[top:bottom, left:right] of a BGR
// video frame, cv2.resize(.., (224, 224), interpolation=cv2.INTER_AREA),
// then cv2.cvtColor(RGB2BGR), i.e. a channel swap that makes the crop RGB.
//
// INTER_AREA is an area-weighted average: output pixel o of an n-pixel span
// resized to 224 covers the source interval [o*n/224, (o+1)*n/224), and each
// source pixel contributes its overlap with that interval.  In units of
// 1/224 pixel the interval is [o*n, (o+1)*n) and source pixel s covers
// [224 s, 224 s + 224), so every weight is an exact integer overlap ov and
//   out = round( sum_y sum_x ov_y ov_x src / (n_x n_y) )      (round half up)
// in integer arithmetic: the GPU kernel and the numpy restatement
// (oracle/video.py) agree bit for bit.  cv2 itself evaluates the same
// sum with float weights, so it may differ by one count on exact .5 ties
// (cv2 is not in the image: parity with it is unpinned).
// Boxes are clipped to the frame; an empty box gives a zero crop.
//
// cv2 averages areas only when neither axis grows.  A box under 224 px on
// either axis takes cv2's bilinear path with area-mode coefficients on BOTH
// axes (hal::resize, OpenCV 4.x resize.cpp; restated in oracle/video.py
// `linear_area_coeffs` / `_resize_linear_area`): source index
// s = floor(d*scale), fraction (d+1) - (s+1)/scale wrapped to [0,1) in float,
// taps rounded to 1/2048; a horizontal pass in exact integers and the SIMD
// vertical pass for uint8 ((D >> 4) mulhi tap, summed, (+2) >> 2).  The
// coefficient arithmetic is written with explicit _rn intrinsics so nothing is
// contracted into an FMA: every index and tap is bit-identical to the host's.
#include "common.hpp"

namespace fac {

constexpr int kCrop = 224;

// cv2's area-mode bilinear coefficients of output pixel d for an n-pixel
// span: first source index and the two taps in 1/2048 units.
__device__ inline void linear_area_tap(int d, int n, bool clamp_fraction, int& s, int& a0, int& a1) {
  const double inv = __ddiv_rn((double)kCrop, (double)n);
  const double scale = __ddiv_rn(1.0, inv);
  s = (int)floor(__dmul_rn((double)d, scale));
  float f = (float)__dsub_rn((double)(d + 1), __dmul_rn((double)(s + 1), inv));
  f = f <= 0.f ? 0.f : __fsub_rn(f, floorf(f));
  if (clamp_fraction && s >= n - 1) {
    s = n - 1;
    f = 0.f;
  }
  a0 = __float2int_rn(__fmul_rn(__fsub_rn(1.f, f), 2048.f));
  a1 = __float2int_rn(__fmul_rn(f, 2048.f));
}

// One thread per output pixel (all 3 channels); grid (crop, output row).
__global__ __launch_bounds__(256) void crop_resize_area_u8(const uint8_t* __restrict__ frames, int n_frames, int H,
                                                           int W, const int32_t* __restrict__ boxes,
                                                           uint8_t* __restrict__ crops) {
  const int n = blockIdx.x, oy = blockIdx.y, ox = threadIdx.x;
  if (ox >= kCrop) return;
  const int32_t* bx = boxes + 5 * n;  // (frame, left, top, right, bottom)
  const int f = bx[0];
  const int x0 = max(bx[1], 0), y0 = max(bx[2], 0), x1 = min(bx[3], W), y1 = min(bx[4], H);
  uint8_t* dst = crops + (((size_t)n * kCrop + oy) * kCrop + ox) * 3;
  const int nx = x1 - x0, ny = y1 - y0;
  if (f < 0 || f >= n_frames || nx <= 0 || ny <= 0) {
    dst[0] = dst[1] = dst[2] = 0;
    return;
  }
  if (nx < kCrop || ny < kCrop) {
    int sx, a0, a1, sy, b0, b1;
    linear_area_tap(ox, nx, true, sx, a0, a1);
    linear_area_tap(oy, ny, false, sy, b0, b1);
    const int sx1 = min(sx + 1, nx - 1);  // a1 == 0 whenever this clamps
    const int r0 = min(max(sy, 0), ny - 1), r1 = min(max(sy + 1, 0), ny - 1);
    const uint8_t* p0 = frames + (((size_t)f * H + y0 + r0) * W + x0) * 3;
    const uint8_t* p1 = frames + (((size_t)f * H + y0 + r1) * W + x0) * 3;
    int v[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int d0 = p0[sx * 3 + c] * a0 + p0[sx1 * 3 + c] * a1;  // horizontal pass, exact
      const int d1 = p1[sx * 3 + c] * a0 + p1[sx1 * 3 + c] * a1;
      const int h0 = min(d0 >> 4, 32767), h1 = min(d1 >> 4, 32767);
      const int s = ((h0 * b0) >> 16) + ((h1 * b1) >> 16);
      v[c] = min(max((s + 2) >> 2, 0), 255);
    }
    dst[0] = (uint8_t)v[2];  // BGR -> RGB
    dst[1] = (uint8_t)v[1];
    dst[2] = (uint8_t)v[0];
    return;
  }
  // interval of this output pixel in 1/224-pixel units, relative to the box
  const int X0 = ox * nx, X1 = X0 + nx, Y0 = oy * ny, Y1 = Y0 + ny;
  const int sx0 = X0 / kCrop, sx1 = (X1 - 1) / kCrop;  // covered source columns (inclusive)
  const int sy0 = Y0 / kCrop, sy1 = (Y1 - 1) / kCrop;
  const uint8_t* src = frames + (((size_t)f * H + y0) * W + x0) * 3;
  long long acc0 = 0, acc1 = 0, acc2 = 0;
  for (int sy = sy0; sy <= sy1; ++sy) {
    const int ovy = min(Y1, (sy + 1) * kCrop) - max(Y0, sy * kCrop);
    long long r0 = 0, r1 = 0, r2 = 0;
    const uint8_t* row = src + (size_t)sy * W * 3;
    for (int sx = sx0; sx <= sx1; ++sx) {
      const int ovx = min(X1, (sx + 1) * kCrop) - max(X0, sx * kCrop);
      const uint8_t* p = row + sx * 3;
      r0 += ovx * p[0];
      r1 += ovx * p[1];
      r2 += ovx * p[2];
    }
    acc0 += ovy * r0;
    acc1 += ovy * r1;
    acc2 += ovy * r2;
  }
  const long long den = (long long)nx * ny;
  // BGR source -> RGB crop (the cvtColor swap), round half up
  dst[0] = (uint8_t)((2 * acc2 + den) / (2 * den));
  dst[1] = (uint8_t)((2 * acc1 + den) / (2 * den));
  dst[2] = (uint8_t)((2 * acc0 + den) / (2 * den));
}

hipError_t launch_crop_resize(const uint8_t* frames, int n_frames, int H, int W, const int32_t* boxes, int n_boxes,
                              uint8_t* crops, hipStream_t st) {
  if (n_boxes <= 0) return hipSuccess;
  crop_resize_area_u8<<<dim3(n_boxes, kCrop), 256, 0, st>>>(frames, n_frames, H, W, boxes, crops);
  return hipGetLastError();
}

}  // namespace fac
