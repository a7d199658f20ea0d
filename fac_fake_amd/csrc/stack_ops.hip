// The CViT conv-stack kernels (stem224.hip, conv.hip) as layer-level C ABI
// entry points (include/fac_ops.h), plus their host-side weight packing.
//
// fac_cvit.h runs these kernels inside one fused forward for the 17-conv
// CViT; the CViT variants of the reference (RepBn8, whose
// DEConv blocks fold into plain 3x3 convs and whose features1 adds one
// 128->128 conv without BN/ReLU at 56^2) stack the same layers in a different
// order, so they drive them one launch at a time from Python
// (fac_fake_amd/repbn8.py).  The packing functions are also what
// fac_load_weights uses for the CViT itself.
#include <hip/hip_runtime.h>

#include <vector>

#include "../../include/fac_cvit.h"
#include "../../include/fac_ops.h"
#include "common.hpp"

namespace fac {

int conv_block_n(int H, int cout);
hipError_t launch_conv3x3(int dtype, const uint16_t* in, const uint16_t* wpk, const float* bias, uint16_t* out,
                          int B, int H, int W, int Cin, int Cout, bool pool, const uint16_t* zero16, hipStream_t st,
                          bool relu, int bn = 0);
hipError_t launch_stem224(int dtype, bool u8, const void* in, const uint16_t* w1, const float* b1, const uint16_t* w2,
                          const float* b2, const uint16_t* w3, const float* b3, uint16_t* out, int B, int nwg,
                          hipStream_t s);

static inline uint16_t to16(int dtype, float f) {
  return dtype == 0 ? fac_host::f32_to_bf16(f) : fac_host::f32_to_f16(f);
}

// [n-block][32-channel chunk][tap][q][BN][8]: one tap slice of one chunk is
// byte-identical to the LDS image conv3x3_bn_relu streams (conv.hip).
// w: folded fp32 [cout][cin][9].  bn: the output-channel block (0 =
// conv_block_n's), as launch_conv3x3 is given it.
void pack_conv3x3(int dtype, int H, int ci, int co, const float* w, uint16_t* out, int bn) {
  const int BN = bn ? bn : conv_block_n(H, co), CK = 32, nch = ci / CK;
  size_t q = 0;
  for (int nb = 0; nb < co / BN; ++nb)
    for (int ch = 0; ch < nch; ++ch)
      for (int t = 0; t < 9; ++t)
        for (int qq = 0; qq < CK / 8; ++qq) {
          // below 224x224: conv.hip's pixel-major halo hands lane group qq
          // channel piece qq ^ 2 on odd kernel rows (its PM comment)
          const int qs = (H != 224 && (t / 3) % 2 == 1) ? qq ^ 2 : qq;
          for (int nl = 0; nl < BN; ++nl)
            for (int j = 0; j < 8; ++j)
              out[q++] = to16(dtype, w[((size_t)(nb * BN + nl) * ci + ch * CK + qs * 8 + j) * 9 + t]);
        }
}

// stem224's conv1 K order: k = ((ky*2 + kx/2)*2 + kx%2)*4 + cin (kx = 3 and
// k >= 48 zero), so one 16-byte lane chunk = two horizontally adjacent taps.
// w: folded fp32 [32][3][9] -> [32][64].
void pack_stem_conv1(int dtype, const float* w, uint16_t* out) {
  for (int i = 0; i < 32 * 64; ++i) out[i] = 0;
  for (int o = 0; o < 32; ++o)
    for (int t = 0; t < 9; ++t)
      for (int cin = 0; cin < 3; ++cin) {
        const int ky = t / 3, kx = t % 3;
        out[(size_t)o * 64 + ((ky * 2 + kx / 2) * 2 + kx % 2) * 4 + cin] = to16(dtype, w[((size_t)o * 3 + cin) * 9 + t]);
      }
}

static bool conv3x3_shape_ok(int h, int cin, int cout) {
  if (h != 224 && h != 112 && h != 56 && h != 28 && h != 14) return false;
  if (cin < 32 || cin % 32 || cout <= 0) return false;
  return conv_block_n(h, cout) > 0;
}

static int num_cus() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cached[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cached[dev] = n;
  }
  return cached[dev];
}

}  // namespace fac

extern "C" {

size_t fac_conv3x3_packed_elems(int h, int cin, int cout) {
  return fac::conv3x3_shape_ok(h, cin, cout) ? (size_t)cout * cin * 9 : 0;
}

int fac_conv3x3_pack(int dtype, int h, int cin, int cout, const float* w, uint16_t* out) {
  if (!w || !out || (dtype != 0 && dtype != 1)) return FAC_ERR_ARG;
  if (!fac::conv3x3_shape_ok(h, cin, cout)) return FAC_ERR_SHAPE;
  fac::pack_conv3x3(dtype, h, cin, cout, w, out, 0);
  return FAC_OK;
}

int fac_conv3x3(int dtype, const void* in, const void* wpk, const float* bias, void* out, int n, int h, int cin,
                int cout, int pool, int relu, const void* zero256, void* stream) {
  if (!in || !wpk || !bias || !out || !zero256 || n <= 0 || (dtype != 0 && dtype != 1)) return FAC_ERR_ARG;
  if (!fac::conv3x3_shape_ok(h, cin, cout)) return FAC_ERR_SHAPE;
  const hipError_t e = fac::launch_conv3x3(dtype, (const uint16_t*)in, (const uint16_t*)wpk, bias, (uint16_t*)out, n,
                                           h, h, cin, cout, pool != 0, (const uint16_t*)zero256,
                                           (hipStream_t)stream, relu != 0);
  return e == hipSuccess ? FAC_OK : FAC_ERR_HIP;
}

int fac_stem224_pack_conv1(int dtype, const float* w, uint16_t* out) {
  if (!w || !out || (dtype != 0 && dtype != 1)) return FAC_ERR_ARG;
  fac::pack_stem_conv1(dtype, w, out);
  return FAC_OK;
}

int fac_stem224(int dtype, int u8, const void* in, const void* w1p, const float* b1, const void* w2, const float* b2,
                const void* w3, const float* b3, void* out, int n, void* stream) {
  if (!in || !w1p || !b1 || !w2 || !b2 || !w3 || !b3 || !out || n <= 0 || (dtype != 0 && dtype != 1))
    return FAC_ERR_ARG;
  const hipError_t e = fac::launch_stem224(dtype, u8 != 0, in, (const uint16_t*)w1p, b1, (const uint16_t*)w2, b2,
                                           (const uint16_t*)w3, b3, (uint16_t*)out, n, fac::num_cus(),
                                           (hipStream_t)stream);
  return e == hipSuccess ? FAC_OK : FAC_ERR_HIP;
}

}  // extern "C"
