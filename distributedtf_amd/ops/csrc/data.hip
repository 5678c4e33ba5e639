// On-device CIFAR input pipeline: gather + pad/crop/flip augmentation + per-image standardization + cast/pack,
// in one launch (reference: cifar10_main.py:71-109 preprocess_image / parse_record, which TF runs on the CPU
// through tf.data; here the uint8 dataset lives in HBM and a batch is produced without leaving the GPU).
//
//   one wave per image: 1024 pixels = 16 per lane, the 48 channel values stay in VGPRs for the two-pass
//   mean / variance (tf.image.per_image_standardization: (x - mean) / max(std, 1/sqrt(N)), N = 3072).
//   Random crop offsets and the flip bit come from a counter-based hash of (seed, counter, batch position);
//   seed/counter are read from device memory so a captured HIP graph draws new crops on every replay.  With
//   per-member keys (key_slot != null: the population step's images) the hash is of (seed, the member's own step
//   counter read from its state row, dataset row) instead: a member's crops then depend only on the member -- not on
//   which other members share its plan, its position in the packed batch, or how many launches its rank ran -- so a
//   PBT run draws the same augmentation at any placement of the population over ranks (tests/test_gpu_placement.py).
//   Outputs: bf16 NHWC with channels zero-padded to 16 (the HIP ResNet stem input) and/or fp32 NHWC (C=3).
#include "common.h"

namespace {

__device__ __forceinline__ uint32_t mix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x7feb352du;
  h ^= h >> 15;
  h *= 0x846ca68bu;
  h ^= h >> 16;
  return h;
}

constexpr int IMG = 32, PAD = 4, CH = 3, NPIX = IMG * IMG, PPL = NPIX / 64;

__global__ __launch_bounds__(256) void augment_cifar_kernel(const uint8_t* __restrict__ images,
                                                            const long* __restrict__ labels_src,
                                                            const long* __restrict__ idx,
                                                            const uint32_t* __restrict__ rng, int n, int augment,
                                                            bf16_t* __restrict__ out16, float* __restrict__ out32,
                                                            int* __restrict__ lab32, long* __restrict__ lab64,
                                                            const int* __restrict__ key_slot,
                                                            const float* __restrict__ key_state, long key_stride,
                                                            long key_col) {
  const int lane = threadIdx.x & 63;
  const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= n) return;
  const long src = idx[p];
  int oy = PAD, ox = PAD, flip = 0;
  if (augment) {
    const uint32_t h =
        key_slot != nullptr
            ? mix32(rng[0] ^ mix32((uint32_t)(int)key_state[(long)key_slot[p] * key_stride + key_col] * 0x9E3779B9u +
                                   (uint32_t)src))
            : mix32(rng[0] ^ mix32(rng[1] * 0x9E3779B9u + (uint32_t)p));
    oy = (int)(h % 9u);
    ox = (int)((h >> 8) % 9u);
    flip = (int)((h >> 16) & 1u);
  }
  const uint8_t* im = images + src * (long)(NPIX * CH);
  float v[PPL][CH];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < PPL; ++j) {
    const int q = lane + 64 * j;
    const int y = q >> 5, x = q & 31;
    const int sy = y + oy - PAD;
    const int sx = (flip ? IMG - 1 - x : x) + ox - PAD;
    const bool in = (unsigned)sy < (unsigned)IMG && (unsigned)sx < (unsigned)IMG;
    const uint8_t* px = im + (sy * IMG + sx) * CH;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      v[j][c] = in ? (float)px[c] : 0.f;
      s += v[j][c];
    }
  }
  const float mean = wave_sum(s) * (1.f / (NPIX * CH));
  float q2 = 0.f;
#pragma unroll
  for (int j = 0; j < PPL; ++j)
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const float d = v[j][c] - mean;
      q2 += d * d;
    }
  const float var = wave_sum(q2) * (1.f / (NPIX * CH));
  const float adj = fmaxf(sqrtf(var), rsqrtf((float)(NPIX * CH)));
  const float inv = 1.f / adj;
#pragma unroll
  for (int j = 0; j < PPL; ++j) {
    const int q = lane + 64 * j;
    const float a = (v[j][0] - mean) * inv, b = (v[j][1] - mean) * inv, c = (v[j][2] - mean) * inv;
    if (out16) {
      uint4* dst = reinterpret_cast<uint4*>(out16 + ((long)p * NPIX + q) * 16);
      dst[0] = make_uint4(pack2bf(a, b), pack2bf(c, 0.f), 0u, 0u);
      dst[1] = make_uint4(0u, 0u, 0u, 0u);
    }
    if (out32) {
      float* d = out32 + ((long)p * NPIX + q) * CH;
      d[0] = a;
      d[1] = b;
      d[2] = c;
    }
  }
  if (lane == 0) {
    const long l = labels_src[src];
    if (lab32) lab32[p] = (int)l;
    if (lab64) lab64[p] = l;
  }
}

}  // namespace

DTF_API int dtf_augment_cifar(const uint8_t* images, const long* labels_src, const long* idx, const uint32_t* rng,
                              int n, int augment, bf16_t* out16, float* out32, int* lab32, long* lab64,
                              const int* key_slot, const float* key_state, long key_stride, long key_col,
                              hipStream_t stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(augment_cifar_kernel, dim3((n + 3) / 4), dim3(256), 0, stream, images, labels_src, idx, rng, n,
                     augment, out16, out32, lab32, lab64, key_slot, key_state, key_stride, key_col);
  return DTF_CHECK_LAUNCH();
}
