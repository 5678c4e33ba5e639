// Shared helpers for the distributedtf_amd CDNA4 (gfx950) kernels.
//
// Conventions:
//  * wave = 64 lanes; blocks are multiples of 64 threads;
//  * bf16 tensors are stored as raw 16-bit words (uint16_t) and converted with
//    the hardware round-to-nearest-even path (`__bf16` casts lower to
//    v_cvt_pk_bf16_f32 on gfx950);
//  * MFMA operand/accumulator vector types follow the gfx950 register maps of
//    v_mfma_f32_16x16x32_bf16 (8 bf16 per lane for A and B, 4 f32 for C/D).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define DTF_API extern "C" __attribute__((visibility("default")))

typedef uint16_t bf16_t;
typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

#define DTF_CHECK_LAUNCH() (int)hipGetLastError()
