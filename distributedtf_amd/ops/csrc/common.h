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
#include <stdio.h>

#define DTF_API extern "C" __attribute__((visibility("default")))

// 16-bit activation / weight-shadow element.  The default build stores bf16; the half build (ops/build.py
// LIB_HALF, -DDTF_HALF=1, selected by --dtype fp16) compiles the SAME kernels for IEEE fp16 storage and the
// v_mfma_f32_16x16x32_f16 matrix op (same rate and operand layout as the bf16 form): every 16-bit <-> fp32
// conversion of the kernels goes through bf2f / f2bf / pack2bf / lo2f / hi2f / pk2 below, and every MFMA through
// dtf_mfma16, so the element type is a build switch rather than a second set of kernels.  (The type keeps its
// bf16_t name: it is "the 16-bit element" of either build.)  Bit tricks the kernels rely on hold for both
// formats: a zero word is +0, bit 15 is the sign (ReLU as a signed-int16 max), 16-byte vectors hold 8 elements.
typedef uint16_t bf16_t;
typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

#ifdef DTF_HALF
typedef _Float16 dtf_h16_t;
typedef _Float16 h16x8_t __attribute__((ext_vector_type(8)));
typedef _Float16 h16x2v_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float bf2f(bf16_t v) { return (float)__builtin_bit_cast(_Float16, v); }
__device__ __forceinline__ bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (_Float16)f); }
__device__ __forceinline__ float lo2f(uint32_t w) { return bf2f((bf16_t)(w & 0xffffu)); }
__device__ __forceinline__ float hi2f(uint32_t w) { return bf2f((bf16_t)(w >> 16)); }
__device__ __forceinline__ uint32_t pk2(f32x2_t v) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, h16x2v_t));
}
__device__ __forceinline__ f32x4_t dtf_mfma16(const bf16x8_t& a, const bf16x8_t& b, const f32x4_t& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h16x8_t, a), __builtin_bit_cast(h16x8_t, b), c,
                                                 0, 0, 0);
}
__device__ __forceinline__ f32x16_t dtf_mfma32(const bf16x8_t& a, const bf16x8_t& b, const f32x16_t& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h16x8_t, a), __builtin_bit_cast(h16x8_t, b), c,
                                                 0, 0, 0);
}
#define DTF_HALF_BUILD 1
#else
typedef __bf16 bf16x2v_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}
// the low / high element of a packed pair as fp32 (one VALU op each for bf16)
__device__ __forceinline__ float lo2f(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi2f(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ uint32_t pk2(f32x2_t v) {  // v_cvt_pk_bf16_f32
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2v_t));
}
__device__ __forceinline__ f32x4_t dtf_mfma16(const bf16x8_t& a, const bf16x8_t& b, const f32x4_t& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16_t dtf_mfma32(const bf16x8_t& a, const bf16x8_t& b, const f32x16_t& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
#define DTF_HALF_BUILD 0
#endif

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

// Debug build (ops/build.py --debug -> libdtf_kernels_debug.so, selected by DTF_DEBUG=1).
// A violated device check never traps (a trapping wave can take the whole GPU down): the workgroup records the
// failing source line in a device error word with a global atomic, prints once, and skips its work, so no
// out-of-range access is issued.  The host reads the word back after each synchronous launch
// (dtf_debug_error(); ops.lib() does this in debug mode) and raises with the launcher's name.
// DTF_WG_CHECK(cond) must be workgroup-uniform and placed before the first barrier.
#ifdef DTF_DEBUG
// One error word per translation unit (no relocatable device code); DTF_DEBUG_EXPORT(tu) defines the host getter
// dtf_debug_error_<tu>() that returns and clears it.
static __device__ int dtf_debug_err;
#define DTF_DEBUG_EXPORT(tu)                                                                        \
  DTF_API int dtf_debug_error_##tu() {                                                              \
    int v = 0, z = 0;                                                                               \
    if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(dtf_debug_err), sizeof(int)) != hipSuccess) return -1;   \
    if (v) (void)hipMemcpyToSymbol(HIP_SYMBOL(dtf_debug_err), &z, sizeof(int));                     \
    return v;                                                                                       \
  }
#define DTF_WG_CHECK(cond)                                                                          \
  do {                                                                                              \
    if (!(cond)) {                                                                                  \
      if (threadIdx.x == 0 && atomicCAS(&dtf_debug_err, 0, __LINE__) == 0)                          \
        printf("DTF_WG_CHECK failed %s:%d: %s (block %d)\n", __FILE__, __LINE__, #cond, (int)blockIdx.x); \
      return;                                                                                       \
    }                                                                                               \
  } while (0)
#define DTF_HOST_CHECK(cond)                                                                        \
  do {                                                                                              \
    if (!(cond)) {                                                                                  \
      fprintf(stderr, "DTF_HOST_CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond);              \
      return 100000 + __LINE__;                                                                     \
    }                                                                                               \
  } while (0)
#else
#define DTF_WG_CHECK(cond) ((void)0)
#define DTF_DEBUG_EXPORT(tu)
#define DTF_HOST_CHECK(cond) ((void)0)
#endif
// BatchNorm statistic accumulators: NREP replicated [2][64] rows per member and BN; a workgroup adds its partial
// sums to replica (blockIdx % NREP) so same-address float atomics serialise NREP-fold less.  Must match
// engine/hip_resnet.py (DTF_NREP).
#ifndef DTF_NREP
#define DTF_NREP 8
#endif
#define DTF_ALIGNED16(p) ((((uintptr_t)(p)) & 15) == 0)

// Order-independent accumulation for the large-channel (ImageNet) kernels of the deterministic build: a float
// partial is rounded to a signed 64-bit multiple of 2^-SHIFT and added with an integer atomic.  Integer addition is
// associative, so the total is the same whatever order the workgroups (and, in LDS, the waves) arrive in.  Buffers
// accumulated this way hold int64 words with the float layout's element indexing; the consumers (bn_final,
// cg_det_finish) convert back.  Scales: BN forward sums 2^24 (sum of y^2 over a member's 1.6M pixels stays below
// 2^39 for |y| < 30); gradients, BN-backward sums and the loss 2^36 (|value| < 1.3e8, resolution 1.5e-11).
#define DTF_FX_STAT 24
#define DTF_FX_GRAD 36
// Non-finite / out-of-range partials.  A fixed-point word cannot hold NaN or Inf, and an integer sum wraps silently,
// so a partial that is not finite or whose scaled magnitude reaches 2^54 (room for 512 such adds below 2^63; at the
// gradient scale |v| >= 2^18, at the statistics scale |v| >= 2^30 -- only a diverging member gets there) adds
// nothing and instead sets its member's flag word.  The flags of every translation unit are read by
// cg_det_finish (convg_aux.hip), which writes NaN into that member's loss and gradient row, so the engine's
// non-finite check culls it exactly as in the float build (a diverged member used to keep a finite loss).
#define DTF_POISON_SLOTS 1024
#define DTF_FX_LIMIT 18014398509481984.0f  // 2^54
__device__ __forceinline__ float dtf_unfx(long long v, int shift) { return (float)ldexp((double)v, -shift); }
#ifdef DTF_DETERMINISTIC
static __device__ unsigned dtf_poison[DTF_POISON_SLOTS];  // one array per translation unit (no relocatable device code)
#define DTF_POISON_EXPORT(tu) \
  DTF_API unsigned* dtf_poison_ptr_##tu() {                                             \
    void* p = nullptr;                                                                  \
    return hipGetSymbolAddress(&p, HIP_SYMBOL(dtf_poison)) == hipSuccess ? (unsigned*)p : nullptr; \
  }
__device__ __forceinline__ long long dtf_fx(float v, int shift, int slot) {
  const float s = ldexpf(v, shift);
  if (!(fabsf(s) < DTF_FX_LIMIT)) {  // also true for NaN
    atomicOr(&dtf_poison[slot & (DTF_POISON_SLOTS - 1)], 1u);
    return 0;
  }
  return __float2ll_rn(s);
}
#else
#define DTF_POISON_EXPORT(tu)
__device__ __forceinline__ long long dtf_fx(float v, int shift, int slot) {
  (void)slot;
  return __float2ll_rn(ldexpf(v, shift));
}
#endif
__device__ __forceinline__ void dtf_fx_add(long long* p, float v, int shift, int slot) {
  atomicAdd(reinterpret_cast<unsigned long long*>(p), (unsigned long long)dtf_fx(v, shift, slot));
}
__device__ __forceinline__ void dtf_fx_addi(long long* p, long long v) {
  atomicAdd(reinterpret_cast<unsigned long long*>(p), (unsigned long long)v);
}
#ifdef DTF_DETERMINISTIC
#define DTF_FIXED_ACC 1
typedef long long dtf_acc_t;  // accumulator word of the ImageNet statistics / gradient sums
#else
#define DTF_FIXED_ACC 0
typedef float dtf_acc_t;
#endif
// acc += v (float partial of member `slot`) / acc += w (an accumulated word, LDS -> global)
__device__ __forceinline__ void dtf_acc_add(dtf_acc_t* p, float v, int shift, int slot) {
#if DTF_FIXED_ACC
  dtf_fx_add(p, v, shift, slot);
#else
  (void)shift;
  (void)slot;
  atomicAdd(p, v);
#endif
}
__device__ __forceinline__ void dtf_acc_addw(dtf_acc_t* p, dtf_acc_t w) {
#if DTF_FIXED_ACC
  dtf_fx_addi(p, w);
#else
  atomicAdd(p, w);
#endif
}
__device__ __forceinline__ float dtf_acc_get(const dtf_acc_t* p, int shift) {
#if DTF_FIXED_ACC
  return dtf_unfx(*p, shift);
#else
  (void)shift;
  return *p;
#endif
}
