// Population-batched MNIST CNN training step (gfx950), reference mnist_model.py:62-126:
//   conv5x5 1->32 SAME +b +ReLU -> maxpool 2/2 -> conv5x5 32->64 SAME +b +ReLU -> maxpool 2/2
//   -> dense 3136->1024 +b +ReLU -> dropout 0.4 -> dense 1024->10 -> softmax CE
//
// Images of ALL members are packed along N (img_slot[n] = member row); weights are per member.
//   conv1_fwd   VALU direct conv (K = 25) in fp32 from an LDS image tile; bias+ReLU+2x2 max-pool fused,
//               2-bit pool argmax kept per output (uint8) for the backward.
//   conv2_fwd   implicit GEMM on v_mfma_f32_16x16x32_bf16: one K-step = one 5x5 tap x 32 input channels,
//               A = weights (16 couts, held in VGPRs for all 25 taps), B = 16 pixels of the LDS tile.
//               The 16 pixels of an MFMA column tile are 4 pooling quads, so bias+ReLU+max-pool+argmax
//               are two cross-lane max steps in the epilogue (no pre-pool tensor is ever written).
//   dense1      grouped bf16 GEMM (gemm.hip) on the bf16 shadow of the fp32 master weights.
//   head        bias+ReLU+dropout (counter hash, recomputed -- no mask tensor) + dense2 + softmax CE +
//               all dense2 gradients + dL/d(dense1 pre-activation), one workgroup per image chunk.
//   conv2_dgrad implicit GEMM on the unpooled/masked gradient tile (flipped, transposed weights).
//   conv2_wgrad k = pixel MFMA fragments via ds_read_b64_tr_b16 from NHWC LDS tiles.
//   conv1_wgrad VALU, K = 25.
#include "common.h"

namespace {

typedef short s16x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4_t mfma16(const bf16x8_t& a, const bf16x8_t& b, const f32x4_t& c) {
  return dtf_mfma16(a, b, c);
}

__device__ __forceinline__ s16x4_t ds_read_tr(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(p));
}

__device__ __forceinline__ uint32_t mix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x7FEB352Du;
  h ^= h >> 15;
  h *= 0x846CA68Bu;
  h ^= h >> 16;
  return h;
}

struct MnistArgs {
  const float* x;        // [N, 28, 28] fp32 images
  const int* labels;     // [N]
  const int* img_slot;   // [N]
  const int4* work;      // (img0, nimg, 0, slot): image chunks of one member
  const float* params;   // fp32 state rows
  long p_mstride;
  float* grads;          // fp32 gradient rows
  long g_mstride;
  const bf16_t* shadow;  // bf16 shadow rows of the params (conv2 fwd weights, dense1 weights)
  long s_mstride;
  bf16_t* wd;            // per-member conv2 dgrad weights [32 ci][25 tap'][64 co]
  long wd_mstride;
  bf16_t* p1;            // [N, 196, 32] pooled conv1
  uint8_t* am1;          // [N, 196, 32] pool argmax (dy*2+dx)
  bf16_t* p2;            // [N, 49, 64] pooled conv2 (= dense1 input, TF flatten order h, w, c)
  uint8_t* am2;          // [N, 49, 64]
  const float* z;        // [N, 1024] dense1 output (pre-bias)
  bf16_t* dz;            // [N, 1024] dL/d(dense1 pre-activation)
  const bf16_t* dp2;     // [N, 3136]
  bf16_t* dp1;           // [N, 196, 32]
  float* loss;           // [cap]
  float* correct;        // [cap]
  const float* cnt;      // [cap] images per member this step
  const int* rng;        // [2] (seed, counter), read on the device
  float* logits_out;     // optional [N, 10]
  int off_c1w, off_c1b, off_c2w, off_c2b, off_d1w, off_d1b, off_d2w, off_d2b;
  float drop_rate;
  int train;
  float* dz32;           // fp32 step (engine/hip_mnist_f32.py): dz stored fp32 here instead of bf16 in ``dz``
};

// ------------------------------------------------------------------------------------------ conv1
// One workgroup per image.  Work item = (pooled pixel, 8-channel group): 4 pre-pool sums x 25 taps x 8 ch.
__global__ __launch_bounds__(256) void mnist_conv1_kernel(MnistArgs a) {
  __shared__ float xs[32 * 33];
  __shared__ float ws[25 * 32];  // [tap][c]
  __shared__ float bs[32];
  const int img = blockIdx.x, tid = threadIdx.x;
  const int slot = a.img_slot[img];
  const float* prow = a.params + (long)slot * a.p_mstride;
  const float* xi = a.x + (long)img * 784;
  for (int i = tid; i < 32 * 32; i += 256) {
    const int r = i >> 5, c = i & 31, y = r - 2, x = c - 2;
    xs[r * 33 + c] = (y >= 0 && y < 28 && x >= 0 && x < 28) ? xi[y * 28 + x] : 0.f;
  }
  for (int i = tid; i < 800; i += 256) ws[(i % 25) * 32 + i / 25] = prow[a.off_c1w + i];
  if (tid < 32) bs[tid] = prow[a.off_c1b + tid];
  __syncthreads();
  for (int it = tid; it < 196 * 4; it += 256) {
    const int q = it >> 2, cg = it & 3;
    const int py = q / 14, px = q - 14 * (q / 14);
    float patch[6][6];
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
      for (int c = 0; c < 6; ++c) patch[r][c] = xs[(2 * py + r) * 33 + 2 * px + c];
    uint32_t outw[4];
    uint32_t amw[2] = {0u, 0u};
#pragma unroll
    for (int ch = 0; ch < 8; ch += 2) {
      float v2[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int c = cg * 8 + ch + u;
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
        for (int ky = 0; ky < 5; ++ky)
#pragma unroll
          for (int kx = 0; kx < 5; ++kx) {
            const float w = ws[(ky * 5 + kx) * 32 + c];
            s0 += w * patch[ky][kx];
            s1 += w * patch[ky][kx + 1];
            s2 += w * patch[ky + 1][kx];
            s3 += w * patch[ky + 1][kx + 1];
          }
        float m = s0;
        uint32_t am = 0;
        if (s1 > m) { m = s1; am = 1; }
        if (s2 > m) { m = s2; am = 2; }
        if (s3 > m) { m = s3; am = 3; }
        v2[u] = fmaxf(m + bs[c], 0.f);
        const int byte = ch + u;
        amw[byte >> 2] |= am << (8 * (byte & 3));
      }
      outw[ch >> 1] = pack2bf(v2[0], v2[1]);
    }
    const long o = ((long)img * 196 + q) * 32 + cg * 8;
    *reinterpret_cast<uint4*>(a.p1 + o) = make_uint4(outw[0], outw[1], outw[2], outw[3]);
    *reinterpret_cast<uint2*>(a.am1 + o) = make_uint2(amw[0], amw[1]);
  }
}

// ------------------------------------------------------------------------------------------ conv2 fwd
// LDS tile [18][18][40] bf16 (2-pixel zero halo, 8 bf16 pad per pixel).  Wave w owns couts 16w..16w+15;
// MFMA column tile t (16 pixels) = pooling quads 4t..4t+3 (lane col j: quad 4t + j/4, sub-pixel j%4).
constexpr int C2_TP = 40;  // tile pixel pitch (bf16)

__global__ __launch_bounds__(256) void mnist_conv2_fwd_kernel(MnistArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t tile[18 * 18 * C2_TP];
  const int4 wk = a.work[blockIdx.x];
  DTF_WG_CHECK(wk.x >= 0 && wk.y >= 1 && wk.w >= 0);
  const int img0 = wk.x, nimg = wk.y, slot = wk.w;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, kg = lane >> 4, j = lane & 15;
  for (int i = tid; i < 18 * 18 * C2_TP / 8; i += 256) reinterpret_cast<uint4*>(tile)[i] = make_uint4(0, 0, 0, 0);
  const bf16_t* wrow = a.shadow + (long)slot * a.s_mstride + a.off_c2w;  // OHWI [64][25][32]
  const int co_a = wave * 16 + j;
  bf16x8_t wa[25];
#pragma unroll
  for (int t = 0; t < 25; ++t) wa[t] = *reinterpret_cast<const bf16x8_t*>(wrow + (co_a * 25 + t) * 32 + 8 * kg);
  const float* prow = a.params + (long)slot * a.p_mstride;
  float bias[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) bias[r] = prow[a.off_c2b + wave * 16 + 4 * kg + r];
  int boff[13];
#pragma unroll
  for (int t = 0; t < 13; ++t) {
    const int q = 4 * t + (j >> 2);
    int y = 0, x = 0;
    if (q < 49) {
      y = 2 * (q / 7) + ((j >> 1) & 1);
      x = 2 * (q % 7) + (j & 1);
    }
    boff[t] = (y * 18 + x) * C2_TP + 8 * kg;
  }
  for (int im = 0; im < nimg; ++im) {
    const int img = img0 + im;
    __syncthreads();
    const bf16_t* src = a.p1 + (long)img * 196 * 32;
    for (int i = tid; i < 196 * 4; i += 256) {
      const int p = i >> 2, ch = i & 3, y = p / 14, x = p - 14 * (p / 14);
      *reinterpret_cast<uint4*>(tile + ((y + 2) * 18 + x + 2) * C2_TP + 8 * ch) =
          *reinterpret_cast<const uint4*>(src + p * 32 + 8 * ch);
    }
    __syncthreads();
    f32x4_t acc[13];
#pragma unroll
    for (int t = 0; t < 13; ++t) acc[t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < 25; ++tap) {
      const int toff = ((tap / 5) * 18 + tap % 5) * C2_TP;
#pragma unroll
      for (int t = 0; t < 13; ++t)
        acc[t] = mfma16(wa[tap], *reinterpret_cast<const bf16x8_t*>(tile + boff[t] + toff), acc[t]);
    }
#pragma unroll
    for (int t = 0; t < 13; ++t) {
      const int q = 4 * t + (j >> 2);
      float m[4];
      int am[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        m[r] = acc[t][r] + bias[r];
        am[r] = j & 3;
#pragma unroll
        for (int sh = 1; sh <= 2; sh <<= 1) {
          const float om = __shfl_xor(m[r], sh, 64);
          const int oa = __shfl_xor(am[r], sh, 64);
          if (om > m[r] || (om == m[r] && oa < am[r])) {
            m[r] = om;
            am[r] = oa;
          }
        }
      }
      if ((j & 3) == 0 && q < 49) {
        const long o = ((long)img * 49 + q) * 64 + wave * 16 + 4 * kg;
        *reinterpret_cast<uint2*>(a.p2 + o) =
            make_uint2(pack2bf(fmaxf(m[0], 0.f), fmaxf(m[1], 0.f)), pack2bf(fmaxf(m[2], 0.f), fmaxf(m[3], 0.f)));
        *reinterpret_cast<uint32_t*>(a.am2 + o) =
            (uint32_t)am[0] | ((uint32_t)am[1] << 8) | ((uint32_t)am[2] << 16) | ((uint32_t)am[3] << 24);
      }
    }
  }
}

// Un-pool + ReLU mask of the pooled gradient of conv2: writes the 4 pre-pool pixels of pooled output q,
// channels 8ch..8ch+7, through `put(y, x, uint4)`.
template <typename Put>
__device__ __forceinline__ void unpool_item(const MnistArgs& a, int img, int q, int ch, Put put) {
  const long o = ((long)img * 49 + q) * 64 + 8 * ch;
  const uint4 dv = *reinterpret_cast<const uint4*>(a.dp2 + o);
  const uint4 pv = *reinterpret_cast<const uint4*>(a.p2 + o);
  const uint2 av = *reinterpret_cast<const uint2*>(a.am2 + o);
  const uint32_t d32[4] = {dv.x, dv.y, dv.z, dv.w}, p32[4] = {pv.x, pv.y, pv.z, pv.w};
  const int py = q / 7, px = q - 7 * (q / 7);
#pragma unroll
  for (int sub = 0; sub < 4; ++sub) {
    uint32_t r32[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint32_t w = 0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = 2 * k + h;
        const uint32_t amc = ((c < 4 ? av.x : av.y) >> (8 * (c & 3))) & 0xffu;
        const bool live = (amc == (uint32_t)sub) && (((p32[k] >> (16 * h)) & 0x7fffu) != 0u) &&
                          !((p32[k] >> (16 * h)) & 0x8000u);
        if (live) w |= ((d32[k] >> (16 * h)) & 0xffffu) << (16 * h);
      }
      r32[k] = w;
    }
    put(2 * py + (sub >> 1), 2 * px + (sub & 1), make_uint4(r32[0], r32[1], r32[2], r32[3]));
  }
}

// ------------------------------------------------------------------------------------------ conv2 dgrad
// dP1[y][x][ci] = sum_{tap', co} dYpad[y+ky'][x+kx'][co] * Wd[ci][tap'][co]   (Wd = flipped, transposed W)
// LDS tile [18][18][72] holds the un-pooled, ReLU-masked gradient with a 2-pixel zero halo.
constexpr int D2_TP = 72;

__global__ __launch_bounds__(256) void mnist_conv2_dgrad_kernel(MnistArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t tile[18 * 18 * D2_TP];
  const int4 wk = a.work[blockIdx.x];
  DTF_WG_CHECK(wk.x >= 0 && wk.y >= 1 && wk.w >= 0);
  const int img0 = wk.x, nimg = wk.y, slot = wk.w;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, kg = lane >> 4, j = lane & 15;
  for (int i = tid; i < 18 * 18 * D2_TP / 8; i += 256) reinterpret_cast<uint4*>(tile)[i] = make_uint4(0, 0, 0, 0);
  const int ct = wave & 1, mp = wave >> 1;
  const bf16_t* wrow = a.wd + (long)slot * a.wd_mstride + (long)(16 * ct + j) * 25 * 64 + 8 * kg;
  int boff[7];
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    const int p = 16 * (mp + 2 * i) + j;
    const int y = p < 196 ? p / 14 : 0, x = p < 196 ? p % 14 : 0;
    boff[i] = (y * 18 + x) * D2_TP + 8 * kg;
  }
  const int ntile = mp == 0 ? 7 : 6;
  for (int im = 0; im < nimg; ++im) {
    const int img = img0 + im;
    __syncthreads();
    for (int it = tid; it < 49 * 8; it += 256) {
      unpool_item(a, img, it >> 3, it & 7, [&](int y, int x, uint4 v) {
        *reinterpret_cast<uint4*>(tile + ((y + 2) * 18 + x + 2) * D2_TP + 8 * (it & 7)) = v;
      });
    }
    __syncthreads();
    f32x4_t acc[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) acc[i] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll 5
    for (int tap = 0; tap < 25; ++tap) {
      const int toff = ((tap / 5) * 18 + tap % 5) * D2_TP;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const bf16x8_t wa = *reinterpret_cast<const bf16x8_t*>(wrow + tap * 64 + 32 * h);
#pragma unroll
        for (int i = 0; i < 7; ++i)
          if (i < ntile)
            acc[i] = mfma16(wa, *reinterpret_cast<const bf16x8_t*>(tile + boff[i] + toff + 32 * h), acc[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      const int p = 16 * (mp + 2 * i) + j;
      if (i < ntile && p < 196) {
        const long o = ((long)img * 196 + p) * 32 + 16 * ct + 4 * kg;
        *reinterpret_cast<uint2*>(a.dp1 + o) =
            make_uint2(pack2bf(acc[i][0], acc[i][1]), pack2bf(acc[i][2], acc[i][3]));
      }
    }
  }
}

// ------------------------------------------------------------------------------------------ conv2 wgrad
// dW2[co][tap][ci] += sum_p dY[p][co] * X1pad[p + tap][ci],  db2[co] += sum_p dY[p][co]
// grid.y = 5 tap groups (5 taps x 32 ci = 10 n-tiles); wave = (co pair mh, n-tile half nh): 2 x 5 accumulators.
constexpr int W2_DP = 72;  // dY tile pixel pitch
constexpr int W2_XP = 40;  // X tile pixel pitch

__global__ __launch_bounds__(256) void mnist_conv2_wgrad_kernel(MnistArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t dyt[224 * W2_DP];
  __shared__ __attribute__((aligned(16))) bf16_t xt[18 * 18 * W2_XP];
  __shared__ float dbred[4][64];
  const int4 wk = a.work[blockIdx.x];
  DTF_WG_CHECK(wk.x >= 0 && wk.y >= 1 && wk.w >= 0);
  const int img0 = wk.x, nimg = wk.y, slot = wk.w;
  const int ng = blockIdx.y;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p4 = i16 & 3;
  const int mh = wave & 1, nh = wave >> 1;
  for (int i = tid; i < 224 * W2_DP / 8; i += 256) reinterpret_cast<uint4*>(dyt)[i] = make_uint4(0, 0, 0, 0);
  for (int i = tid; i < 18 * 18 * W2_XP / 8; i += 256) reinterpret_cast<uint4*>(xt)[i] = make_uint4(0, 0, 0, 0);
  f32x4_t acc[2][5];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 5; ++n) acc[m][n] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  int xoff[5];
#pragma unroll
  for (int n = 0; n < 5; ++n) {
    const int nl = nh * 5 + n, tap = 5 * ng + (nl >> 1);
    xoff[n] = ((tap / 5) * 18 + tap % 5) * W2_XP + 16 * (nl & 1) + 4 * p4;
  }
  float dbacc = 0.f;
  for (int im = 0; im < nimg; ++im) {
    const int img = img0 + im;
    __syncthreads();
    for (int it = tid; it < 49 * 8; it += 256) {
      unpool_item(a, img, it >> 3, it & 7, [&](int y, int x, uint4 v) {
        *reinterpret_cast<uint4*>(dyt + (y * 14 + x) * W2_DP + 8 * (it & 7)) = v;
      });
    }
    const bf16_t* src = a.p1 + (long)img * 196 * 32;
    for (int i = tid; i < 196 * 4; i += 256) {
      const int p = i >> 2, ch = i & 3, y = p / 14, x = p - 14 * (p / 14);
      *reinterpret_cast<uint4*>(xt + ((y + 2) * 18 + x + 2) * W2_XP + 8 * ch) =
          *reinterpret_cast<const uint4*>(src + p * 32 + 8 * ch);
    }
    __syncthreads();
    if (ng == 0) {
      // db2 partial: 4 waves x 49 pixels each, lane = channel
      float s = 0.f;
      for (int p = wave; p < 196; p += 4) s += bf2f(dyt[p * W2_DP + lane]);
      dbacc += s;
    }
#pragma unroll
    for (int ks = 0; ks < 7; ++ks) {
      const int pa = 32 * ks + 8 * g + q, pb = pa + 4;
      bf16x8_t af[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int co0 = 16 * (2 * mh + m);
        const s16x4_t lo = ds_read_tr(dyt + pa * W2_DP + co0 + 4 * p4);
        const s16x4_t hi = ds_read_tr(dyt + pb * W2_DP + co0 + 4 * p4);
        af[m] = (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
      const int ya = pa < 196 ? pa / 14 : 0, xa = pa < 196 ? pa % 14 : 0;
      const int yb = pb < 196 ? pb / 14 : 0, xb = pb < 196 ? pb % 14 : 0;
      const bf16_t* xa_ = xt + (ya * 18 + xa) * W2_XP;
      const bf16_t* xb_ = xt + (yb * 18 + xb) * W2_XP;
#pragma unroll
      for (int n = 0; n < 5; ++n) {
        const s16x4_t lo = ds_read_tr(xa_ + xoff[n]);
        const s16x4_t hi = ds_read_tr(xb_ + xoff[n]);
        const bf16x8_t bfr = (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int m = 0; m < 2; ++m) acc[m][n] = mfma16(af[m], bfr, acc[m][n]);
      }
    }
  }
  float* gr = a.grads + (long)slot * a.g_mstride;
#pragma unroll
  for (int n = 0; n < 5; ++n) {
    const int nl = nh * 5 + n, tap = 5 * ng + (nl >> 1), ci = 16 * (nl & 1) + i16;
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = 16 * (2 * mh + m) + 4 * g + r;
        atomicAdd(gr + a.off_c2w + (co * 25 + tap) * 32 + ci, acc[m][n][r]);
      }
  }
  if (ng == 0) {
    dbred[wave][lane] = dbacc;
    __syncthreads();
    if (tid < 64) atomicAdd(gr + a.off_c2b + tid, dbred[0][tid] + dbred[1][tid] + dbred[2][tid] + dbred[3][tid]);
  }
}

// ------------------------------------------------------------------------------------------ conv1 wgrad
__global__ __launch_bounds__(256) void mnist_conv1_wgrad_kernel(MnistArgs a) {
  __shared__ float xs[32 * 33];
  __shared__ float red[8][32][27];
  const int4 wk = a.work[blockIdx.x];
  DTF_WG_CHECK(wk.x >= 0 && wk.y >= 1 && wk.w >= 0);
  const int img0 = wk.x, nimg = wk.y, slot = wk.w;
  const int tid = threadIdx.x, c = tid & 31, qg = tid >> 5;
  float acc[26];
#pragma unroll
  for (int k = 0; k < 26; ++k) acc[k] = 0.f;
  for (int im = 0; im < nimg; ++im) {
    const int img = img0 + im;
    const float* xi = a.x + (long)img * 784;
    __syncthreads();
    for (int i = tid; i < 32 * 32; i += 256) {
      const int r = i >> 5, cc = i & 31, y = r - 2, x = cc - 2;
      xs[r * 33 + cc] = (y >= 0 && y < 28 && x >= 0 && x < 28) ? xi[y * 28 + x] : 0.f;
    }
    __syncthreads();
    for (int q = qg; q < 196; q += 8) {
      const long o = ((long)img * 196 + q) * 32 + c;
      const float pv = bf2f(a.p1[o]);
      const float gv = bf2f(a.dp1[o]);
      if (pv > 0.f && gv != 0.f) {
        const int s = a.am1[o];
        const int iy = 2 * (q / 14) + (s >> 1), ix = 2 * (q % 14) + (s & 1);
#pragma unroll
        for (int ky = 0; ky < 5; ++ky)
#pragma unroll
          for (int kx = 0; kx < 5; ++kx) acc[ky * 5 + kx] += gv * xs[(iy + ky) * 33 + ix + kx];
        acc[25] += gv;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 26; ++k) red[qg][c][k] = acc[k];
  __syncthreads();
  float* gr = a.grads + (long)slot * a.g_mstride;
  for (int i = tid; i < 32 * 26; i += 256) {
    const int cc = i / 26, k = i % 26;
    float s = 0.f;
#pragma unroll
    for (int gq = 0; gq < 8; ++gq) s += red[gq][cc][k];
    atomicAdd(gr + (k < 25 ? a.off_c1w + cc * 25 + k : a.off_c1b + cc), s);
  }
}

// ------------------------------------------------------------------------------------------ head
// Thread t owns dense1 features 4t..4t+3 (256 threads = 1024 features); one image per iteration.
__global__ __launch_bounds__(256) void mnist_head_kernel(MnistArgs a) {
  __shared__ float red[2][4][10];
  const int4 wk = a.work[blockIdx.x];
  DTF_WG_CHECK(wk.x >= 0 && wk.y >= 1 && wk.w >= 0);
  const int img0 = wk.x, nimg = wk.y, slot = wk.w;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, f0 = 4 * tid;
  const float* prow = a.params + (long)slot * a.p_mstride;
  float w[10][4], b2[10], b1[4];
#pragma unroll
  for (int jj = 0; jj < 10; ++jj) {
    const float4 v = *reinterpret_cast<const float4*>(prow + a.off_d2w + jj * 1024 + f0);
    w[jj][0] = v.x;
    w[jj][1] = v.y;
    w[jj][2] = v.z;
    w[jj][3] = v.w;
    b2[jj] = prow[a.off_d2b + jj];
  }
  {
    const float4 v = *reinterpret_cast<const float4*>(prow + a.off_d1b + f0);
    b1[0] = v.x;
    b1[1] = v.y;
    b1[2] = v.z;
    b1[3] = v.w;
  }
  float dw[10][4], db1[4] = {0.f, 0.f, 0.f, 0.f}, db2 = 0.f, loss = 0.f, corr = 0.f;
#pragma unroll
  for (int jj = 0; jj < 10; ++jj)
#pragma unroll
    for (int k = 0; k < 4; ++k) dw[jj][k] = 0.f;
  const float bsz = a.cnt[slot];
  const bool drop = a.train && a.drop_rate > 0.f;
  const uint32_t thresh = drop ? (uint32_t)(a.drop_rate * 4294967296.0) : 0u;
  const float scale = drop ? 1.f / (1.f - a.drop_rate) : 1.f;
  const uint32_t seed = drop ? (uint32_t)a.rng[0] : 0u, ctr = drop ? (uint32_t)a.rng[1] : 0u;
  const uint32_t cmix = ctr * 0x9E3779B9u;
  for (int im = 0; im < nimg; ++im) {
    const int img = img0 + im;
    const float4 zv = *reinterpret_cast<const float4*>(a.z + (long)img * 1024 + f0);
    const float zz[4] = {zv.x, zv.y, zv.z, zv.w};
    float pre[4], hd[4], keep[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      pre[k] = zz[k] + b1[k];
      keep[k] = 1.f;
      if (drop) {
        const uint32_t hsh = mix32(seed ^ mix32(cmix + (uint32_t)img * 1024u + (uint32_t)(f0 + k)));
        keep[k] = hsh >= thresh ? scale : 0.f;
      }
      hd[k] = fmaxf(pre[k], 0.f) * keep[k];
    }
    float lg[10];
#pragma unroll
    for (int jj = 0; jj < 10; ++jj) {
      float s = w[jj][0] * hd[0] + w[jj][1] * hd[1] + w[jj][2] * hd[2] + w[jj][3] * hd[3];
      s = wave_sum(s);
      if (lane == 0) red[im & 1][wave][jj] = s;
    }
    __syncthreads();
    float mx = -3.0e38f;
    int arg = 0;
#pragma unroll
    for (int jj = 0; jj < 10; ++jj) {
      lg[jj] = red[im & 1][0][jj] + red[im & 1][1][jj] + red[im & 1][2][jj] + red[im & 1][3][jj] + b2[jj];
      if (lg[jj] > mx) {
        mx = lg[jj];
        arg = jj;
      }
    }
    float se = 0.f;
#pragma unroll
    for (int jj = 0; jj < 10; ++jj) se += __expf(lg[jj] - mx);
    const float lse = mx + __logf(se);
    const int lab = a.labels[img];
    float lgl = 0.f;
#pragma unroll
    for (int jj = 0; jj < 10; ++jj) lgl = jj == lab ? lg[jj] : lgl;
    if (tid == 0) {
      loss += lse - lgl;
      corr += arg == lab ? 1.f : 0.f;
    }
    if (a.logits_out && tid < 10) {
#pragma unroll
      for (int jj = 0; jj < 10; ++jj)
        if (jj == tid) a.logits_out[(long)img * 10 + jj] = lg[jj];
    }
    if (a.train) {
      float dl[10];
#pragma unroll
      for (int jj = 0; jj < 10; ++jj) {
        dl[jj] = (__expf(lg[jj] - lse) - (jj == lab ? 1.f : 0.f)) / bsz;
        if (jj == tid) db2 += dl[jj];
      }
      float dzv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float dh = 0.f;
#pragma unroll
        for (int jj = 0; jj < 10; ++jj) {
          dw[jj][k] += dl[jj] * hd[k];
          dh += w[jj][k] * dl[jj];
        }
        dzv[k] = pre[k] > 0.f ? dh * keep[k] : 0.f;
        db1[k] += dzv[k];
      }
      if (a.dz32)
        *reinterpret_cast<float4*>(a.dz32 + (long)img * 1024 + f0) = make_float4(dzv[0], dzv[1], dzv[2], dzv[3]);
      else
        *reinterpret_cast<uint2*>(a.dz + (long)img * 1024 + f0) =
            make_uint2(pack2bf(dzv[0], dzv[1]), pack2bf(dzv[2], dzv[3]));
    }
  }
  if (tid == 0) {
    atomicAdd(&a.loss[slot], loss / bsz);
    atomicAdd(&a.correct[slot], corr);
  }
  if (a.train) {
    float* gr = a.grads + (long)slot * a.g_mstride;
#pragma unroll
    for (int jj = 0; jj < 10; ++jj)
#pragma unroll
      for (int k = 0; k < 4; ++k) atomicAdd(gr + a.off_d2w + jj * 1024 + f0 + k, dw[jj][k]);
#pragma unroll
    for (int k = 0; k < 4; ++k) atomicAdd(gr + a.off_d1b + f0 + k, db1[k]);
    if (tid < 10) atomicAdd(gr + a.off_d2b + tid, db2);
  }
}

// ------------------------------------------------------------------------------------------ weight prep
// Wd[ci][tap'][co] = W[co][24 - tap'][ci] from the fp32 master rows (51200 per member).
__global__ __launch_bounds__(256) void mnist_wd_prep_kernel(MnistArgs a, const int* slots) {
  const int slot = slots[blockIdx.y];
  const float* w = a.params + (long)slot * a.p_mstride + a.off_c2w;
  bf16_t* d = a.wd + (long)slot * a.wd_mstride;
  for (int e = blockIdx.x * 256 + threadIdx.x; e < 51200; e += gridDim.x * 256) {
    const int co = e & 63, rest = e >> 6, tp = rest % 25, ci = rest / 25;
    d[e] = f2bf(w[(co * 25 + 24 - tp) * 32 + ci]);
  }
}

// ------------------------------------------------------------------------------------------ fp32 step helpers
// The fp32 step (engine/hip_mnist_f32.py) runs conv1 / conv2 / dense1 and their gradients on the generic fp32
// MFMA conv kernels (f32conv.hip, v_mfma_f32_16x16x4_f32); these are the pieces around them: the 1 -> 4 channel
// input packing, bias + ReLU + 2x2 max-pool (argmax kept) and its backward (un-pool, ReLU mask, bias gradient).
struct PoolArgs {
  const float* h;       // [N, H, H, C] conv output before the bias
  float* p;             // [N, H/2, H/2, C] max-pool of relu(h + b)
  uint8_t* am;          // [N, H/2, H/2, C] argmax (dy * 2 + dx)
  const float* dp;      // backward: dL/dp
  float* dh;            // backward: dL/dh
  const int* img_slot;  // [N]
  const int4* work;     // backward: (img0, nimg, 0, slot) image chunks of one member
  const float* params;
  long p_mstride;
  dtf_acc_t* grads;     // bias gradient rows (the int64 accumulator rows in the deterministic build)
  long g_mstride;
  int b_off, H, C, pad_;
  long nimg;
};

__global__ __launch_bounds__(256) void mnist_f32_prep_kernel(const float* __restrict__ x, float* __restrict__ x4,
                                                             long npix) {
  for (long p = (long)blockIdx.x * 256 + threadIdx.x; p < npix; p += (long)gridDim.x * 256)
    *reinterpret_cast<float4*>(x4 + 4 * p) = make_float4(x[p], 0.f, 0.f, 0.f);
}

// one thread per pooled pixel and 4 channels; ties keep the first window position (the ReLU zeros carry no gradient)
__global__ __launch_bounds__(256) void mnist_f32_pool_kernel(PoolArgs a) {
  const int Ho = a.H >> 1, C4 = a.C >> 2;
  const long total = a.nimg * Ho * Ho * C4;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int c = (int)(e % C4) * 4;
    const long q = e / C4;
    const long img = q / (Ho * Ho);
    const int pix = (int)(q - img * Ho * Ho), oy = pix / Ho, ox = pix - oy * Ho;
    const float* br = a.params + (long)a.img_slot[img] * a.p_mstride + a.b_off + c;
    const float b[4] = {br[0], br[1], br[2], br[3]};
    float best[4] = {-3.0e38f, -3.0e38f, -3.0e38f, -3.0e38f};
    uint32_t arg[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const float4 v = *reinterpret_cast<const float4*>(
          a.h + ((img * a.H + 2 * oy + (d >> 1)) * a.H + 2 * ox + (d & 1)) * a.C + c);
      const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float t = fmaxf(vv[i] + b[i], 0.f);
        if (t > best[i]) {
          best[i] = t;
          arg[i] = (uint32_t)d;
        }
      }
    }
    *reinterpret_cast<float4*>(a.p + q * a.C + c) = make_float4(best[0], best[1], best[2], best[3]);
    *reinterpret_cast<uint32_t*>(a.am + q * a.C + c) = arg[0] | (arg[1] << 8) | (arg[2] << 16) | (arg[3] << 24);
  }
}

// dh = un-pool(dp masked by p > 0); bias gradient = sum of the masked dp over the chunk's pixels (fixed in-workgroup
// order, one accumulator add per workgroup and channel).  C in {32, 64}: thread = (pixel group, channel).
__global__ __launch_bounds__(256) void mnist_f32_unpool_kernel(PoolArgs a) {
  __shared__ float red[256];
  const int4 wk = a.work[blockIdx.x];
  DTF_WG_CHECK(wk.x >= 0 && wk.y >= 1 && wk.w >= 0);
  const int img0 = wk.x, nimg = wk.y, slot = wk.w;
  const int Ho = a.H >> 1, C = a.C, tid = threadIdx.x;
  const int c = tid % C, G = 256 / C;
  const long base = (long)img0 * Ho * Ho, n = (long)nimg * Ho * Ho;
  float db = 0.f;
  for (long q = tid / C; q < n; q += G) {
    const long e = (base + q) * C + c;
    const float v = a.p[e] > 0.f ? a.dp[e] : 0.f;
    const int am = a.am[e];
    db += v;
    const long pq = base + q, img = pq / (Ho * Ho);
    const int pix = (int)(pq - img * Ho * Ho), oy = pix / Ho, ox = pix - oy * Ho;
#pragma unroll
    for (int d = 0; d < 4; ++d)
      a.dh[((img * a.H + 2 * oy + (d >> 1)) * a.H + 2 * ox + (d & 1)) * C + c] = d == am ? v : 0.f;
  }
  red[tid] = db;
  __syncthreads();
  if (tid < C) {
    float s = 0.f;
    for (int g = 0; g < G; ++g) s += red[g * C + tid];
    dtf_acc_add(a.grads + (long)slot * a.g_mstride + a.b_off + tid, s, DTF_FX_GRAD, slot);
  }
}

}  // namespace

DTF_API int dtf_mnist_args_size() { return (int)sizeof(MnistArgs); }

DTF_API int dtf_mnist_wd_prep(const MnistArgs* a, const int* slots, int nslots, hipStream_t stream) {
  if (nslots <= 0) return 0;
  hipLaunchKernelGGL(mnist_wd_prep_kernel, dim3(50, nslots), dim3(256), 0, stream, *a, slots);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_mnist_conv1(const MnistArgs* a, int nimg, hipStream_t stream) {
  if (nimg <= 0) return 0;
  hipLaunchKernelGGL(mnist_conv1_kernel, dim3(nimg), dim3(256), 0, stream, *a);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_mnist_conv2_fwd(const MnistArgs* a, int nwork, hipStream_t stream) {
  if (nwork <= 0) return 0;
  hipLaunchKernelGGL(mnist_conv2_fwd_kernel, dim3(nwork), dim3(256), 0, stream, *a);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_mnist_head(const MnistArgs* a, int nwork, hipStream_t stream) {
  if (nwork <= 0) return 0;
  hipLaunchKernelGGL(mnist_head_kernel, dim3(nwork), dim3(256), 0, stream, *a);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_mnist_conv2_dgrad(const MnistArgs* a, int nwork, hipStream_t stream) {
  if (nwork <= 0) return 0;
  hipLaunchKernelGGL(mnist_conv2_dgrad_kernel, dim3(nwork), dim3(256), 0, stream, *a);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_mnist_conv2_wgrad(const MnistArgs* a, int nwork, hipStream_t stream) {
  if (nwork <= 0) return 0;
  hipLaunchKernelGGL(mnist_conv2_wgrad_kernel, dim3(nwork, 5), dim3(256), 0, stream, *a);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_mnist_conv1_wgrad(const MnistArgs* a, int nwork, hipStream_t stream) {
  if (nwork <= 0) return 0;
  hipLaunchKernelGGL(mnist_conv1_wgrad_kernel, dim3(nwork), dim3(256), 0, stream, *a);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_mnist_pool_args_size() { return (int)sizeof(PoolArgs); }

DTF_API int dtf_mnist_f32_prep(const float* x, float* x4, long npix, hipStream_t stream) {
  long blocks = (npix + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks <= 0) return 0;
  DTF_HOST_CHECK(DTF_ALIGNED16(x4));
  hipLaunchKernelGGL(mnist_f32_prep_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, x, x4, npix);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_mnist_f32_pool(const PoolArgs* a, hipStream_t stream) {
  if (a->nimg <= 0) return 0;
  if ((a->C & 3) != 0 || (a->H & 1) != 0) return -2;
  DTF_HOST_CHECK(DTF_ALIGNED16(a->h) && DTF_ALIGNED16(a->p));
  long blocks = (a->nimg * (a->H / 2) * (a->H / 2) * (a->C / 4) + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(mnist_f32_pool_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, *a);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_mnist_f32_unpool(const PoolArgs* a, int nwork, hipStream_t stream) {
  if (nwork <= 0) return 0;
  if (a->C != 32 && a->C != 64) return -2;
  hipLaunchKernelGGL(mnist_f32_unpool_kernel, dim3(nwork), dim3(256), 0, stream, *a);
  return DTF_CHECK_LAUNCH();
}

DTF_DEBUG_EXPORT(mnist)
