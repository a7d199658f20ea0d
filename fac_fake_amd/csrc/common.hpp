// Shared device/host helpers for the CViT gfx950 kernels.
//
// Every activation and weight operand is a 16-bit value held in memory as
// uint16_t; the two operand types (bf16, fp16) differ only in conversion and
// in which MFMA builtin consumes them.  Both run at the same MFMA rate on
// CDNA4 (v_mfma_f32_16x16x32_{bf16,f16}: 16 cycles/SIMD), accumulate in fp32,
// and every epilogue (bias, BN shift, ReLU, GELU, residual, LN, softmax) is
// fp32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fac {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

// ReLU as one v_max_i32 on the bit pattern (max(x, +0) for every non-NaN x,
// -0 -> +0): fmaxf costs a NaN-canonicalising v_max plus the max.
__device__ __forceinline__ float relu(float x) {
  return __builtin_bit_cast(float, __builtin_elementwise_max(__builtin_bit_cast(int, x), 0));
}

struct BF16 {
  static constexpr int id = 0;
  __device__ __forceinline__ static uint16_t from_f32(float x) {
    __bf16 h = (__bf16)x;  // round-to-nearest-even, v_cvt_pk_bf16_f32
    return __builtin_bit_cast(uint16_t, h);
  }
  __device__ __forceinline__ static float to_f32(uint16_t x) {
    return __builtin_bit_cast(float, (uint32_t)x << 16);
  }
  // 4 floats -> 4 x 16-bit, round-to-nearest-even, two v_cvt_pk_bf16_f32
  __device__ __forceinline__ static u16x4 pack4(f32x4 v) {
    const bf16x2 lo = __builtin_convertvector((f32x2){v[0], v[1]}, bf16x2);
    const bf16x2 hi = __builtin_convertvector((f32x2){v[2], v[3]}, bf16x2);
    return __builtin_bit_cast(u16x4, __builtin_shufflevector(lo, hi, 0, 1, 2, 3));
  }
  // 2 floats -> two 16-bit values in one dword (low = a), one v_cvt_pk_bf16_f32
  __device__ __forceinline__ static uint32_t pack2(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2));
  }
  __device__ __forceinline__ static f32x4 mfma(u16x8 a, u16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  }
};

struct F16 {
  static constexpr int id = 1;
  __device__ __forceinline__ static uint16_t from_f32(float x) {
    _Float16 h = (_Float16)x;  // round-to-nearest-even
    return __builtin_bit_cast(uint16_t, h);
  }
  __device__ __forceinline__ static float to_f32(uint16_t x) {
    return (float)__builtin_bit_cast(_Float16, x);
  }
  // 4 floats -> 4 x 16-bit, round-to-nearest-even, two v_cvt_pk_f16_f32
  __device__ __forceinline__ static u16x4 pack4(f32x4 v) {
    const f16x2 lo = __builtin_convertvector((f32x2){v[0], v[1]}, f16x2);
    const f16x2 hi = __builtin_convertvector((f32x2){v[2], v[3]}, f16x2);
    return __builtin_bit_cast(u16x4, __builtin_shufflevector(lo, hi, 0, 1, 2, 3));
  }
  __device__ __forceinline__ static uint32_t pack2(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, f16x2));
  }
  __device__ __forceinline__ static f32x4 mfma(u16x8 a, u16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  }
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

}  // namespace fac

// Host-side conversions (round-to-nearest-even, matching torch's .to()).
namespace fac_host {
inline uint16_t f32_to_bf16(float f) {
  uint32_t u;
  __builtin_memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
inline uint16_t f32_to_f16(float f) {
  _Float16 h = (_Float16)f;
  uint16_t r;
  __builtin_memcpy(&r, &h, 2);
  return r;
}
}  // namespace fac_host
