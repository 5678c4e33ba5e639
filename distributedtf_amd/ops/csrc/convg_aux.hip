// Auxiliary population-batched kernels of the ImageNet-shape ResNet step (gfx950).
//   cg_weight_prep  : fp32 master rows -> bf16 conv weights (forward [o][tap][i], input channels padded) and
//                     flipped/transposed dgrad weights [i][K*K-1-tap][o]; dense weights padded to 1024 rows
//   cg_bn_fwd_final : per (member, channel) BN forward coefficients from the conv-epilogue sums
//                     (scale, shift, mean, inv) + TF moving averages (momentum 0.997, unbiased variance)
//   cg_bn_bwd_final : BN backward coefficients A, B, C of dh = A dz + B h + C from (sum dz, sum dz*xhat),
//                     and dgamma / dbeta into the gradient row
//   cg_bn_bwd_apply : g = A dz + B h + C (+ add)   (the residual-stream gradient through the first BN of a block)
//   cg_prep_input   : fp32 NHWC images -> bf16 with channels zero-padded to 8
//   cg_maxpool_fwd / cg_maxpool_bwd : 3x3/2 'SAME' (TF pads the end) max-pool with a per-output argmax byte;
//                     the backward gathers (no atomics): every input pixel sums the <= 4 windows choosing it
//   cg_gap          : final BN+ReLU + global average pool -> bf16 features (dense GEMM operand)
//   cg_softmax_ce   : + bias, softmax cross-entropy, loss / correct count, dlogits (bf16, padded), dbias
//   cg_gap_bwd_reduce / cg_gap_bwd_apply : backward of GAP + final BN + ReLU
#include "common.h"

#include <cstdlib>

#define BN_EPS 1e-5f
#define BN_MOM 0.997f

namespace {

// conv table row: {w_off, cout, cin, k, cin_pad, fwd_off, dgr_off, 0}
__global__ __launch_bounds__(256) void cg_weight_prep_kernel(const float* __restrict__ state, long s_mstride,
                                                              const int* __restrict__ table,
                                                              const int* __restrict__ slots, bf16_t* __restrict__ wf,
                                                              bf16_t* __restrict__ wd, long w_mstride) {
  const int* t = table + blockIdx.x * 8;
  const int slot = slots[blockIdx.z];
  const int w_off = t[0], cout = t[1], cin = t[2], k = t[3], cin_pad = t[4], fwd_off = t[5], dgr_off = t[6];
  const int kk = k * k;
  const float* p = state + (long)slot * s_mstride + w_off;
  bf16_t* f = wf + (long)slot * w_mstride + fwd_off;
  const int t0 = blockIdx.y * blockDim.x + threadIdx.x, ts = gridDim.y * blockDim.x;
  if (t[7] == 1) {
    // space-to-depth stem: the 7x7/2 kernel W[co][ky][kx][c] (c < cin = 3) as a 4x4/1 kernel over 2x2 pixel blocks,
    // W'[co][a][b][(2 dy + dx) * cin + c] = W[co][2a + dy - 1][2b + dx - 1][c] (zero outside 0..6 and for the pad
    // channels): input row 2 oy + ky - 3 = 2 (oy + a - 2) + dy
    const int nf = cout * 16 * cin_pad;
    for (int i = t0; i < nf; i += ts) {
      const int ci = i % cin_pad, rest = i / cin_pad, tap = rest % 16, co = rest / 16;
      const int q = ci / cin, c = ci - q * cin;
      const int ky = 2 * (tap >> 2) + (q >> 1) - 1, kx = 2 * (tap & 3) + (q & 1) - 1;
      const bool ok = q < 4 && ky >= 0 && ky < k && kx >= 0 && kx < k;
      f[i] = ok ? f2bf(p[((co * k + ky) * k + kx) * cin + c]) : (bf16_t)0;
    }
    return;
  }
  const int nf = cout * kk * cin_pad;
  if (cin_pad == cin && (nf & 3) == 0) {
    for (int i = 4 * t0; i < nf; i += 4 * ts) {
      const float4 v = *reinterpret_cast<const float4*>(p + i);
      *reinterpret_cast<uint2*>(f + i) = make_uint2(pack2bf(v.x, v.y), pack2bf(v.z, v.w));
    }
  } else {
    for (int i = t0; i < nf; i += ts) {
      const int ci = i % cin_pad, rest = i / cin_pad;
      f[i] = ci < cin ? f2bf(p[rest * cin + ci]) : (bf16_t)0;
    }
  }
  if (dgr_off >= 0) {
    bf16_t* d = wd + (long)slot * w_mstride + dgr_off;
    const int nd = cin * kk * cout;
    for (int i = t0; i < nd; i += ts) {
      const int co = i % cout, rest = i / cout;  // rest = ci*kk + tap'
      const int tp = rest % kk, ci = rest / kk;
      d[i] = f2bf(p[(co * kk + (kk - 1 - tp)) * cin + ci]);
    }
  }
}

// dense [ncls][C] fp32 -> bf16 [npad][C] (rows >= ncls zero)
__global__ __launch_bounds__(256) void cg_dense_prep_kernel(const float* __restrict__ state, long s_mstride, int w_off,
                                                             int ncls, int npad, int C, const int* __restrict__ slots,
                                                             bf16_t* __restrict__ out, long o_mstride) {
  const int slot = slots[blockIdx.y];
  const float* p = state + (long)slot * s_mstride + w_off;
  bf16_t* o = out + (long)slot * o_mstride;
  const int n = npad * C;
  for (int i = (blockIdx.x * blockDim.x + threadIdx.x) * 2; i < n; i += gridDim.x * blockDim.x * 2) {
    const int r = i / C;
    const float v0 = r < ncls ? p[i] : 0.f, v1 = r < ncls ? p[i + 1] : 0.f;
    *reinterpret_cast<uint32_t*>(o + i) = pack2bf(v0, v1);
  }
}

struct BnFinArgs {
  float* state;        // fp32 state rows (gamma/beta in params, running stats at run_base)
  long s_mstride;
  const dtf_acc_t* sums;  // [cap][2][cmax]
  float* coef;         // [cap][4][cmax] out
  const float* fcoef;  // bwd: forward coefficients of the same BN
  float* grads;        // bwd: dgamma / dbeta
  long g_mstride;
  const int* slots;
  const float* cnt;    // images per member
  int gamma_off, beta_off, run_off;  // run_off: absolute float index of running mean in the state row
  int C, hw, cmax;
};

__global__ __launch_bounds__(256) void cg_bn_fwd_final_kernel(BnFinArgs a) {
  const int slot = a.slots[blockIdx.y];
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= a.C) return;
  const dtf_acc_t* su = a.sums + (long)slot * 2 * a.cmax;
  const float n = a.cnt[slot] * (float)a.hw;
  const float mean = dtf_acc_get(su + c, DTF_FX_STAT) / n;
  const float var = fmaxf(dtf_acc_get(su + a.cmax + c, DTF_FX_STAT) / n - mean * mean, 0.f);
  const float inv = rsqrtf(var + BN_EPS);
  float* row = a.state + (long)slot * a.s_mstride;
  const float scale = row[a.gamma_off + c] * inv;
  float* co = a.coef + (long)slot * 4 * a.cmax;
  co[c] = scale;
  co[a.cmax + c] = row[a.beta_off + c] - mean * scale;
  co[2 * a.cmax + c] = mean;
  co[3 * a.cmax + c] = inv;
  float* run = row + a.run_off;
  const float unb = n > 1.f ? var * n / (n - 1.f) : var;
  run[c] = BN_MOM * run[c] + (1.f - BN_MOM) * mean;
  run[a.C + c] = BN_MOM * run[a.C + c] + (1.f - BN_MOM) * unb;
}

// Eval mode: coefficients from the moving statistics (no update): scale, shift, mean, inv
__global__ __launch_bounds__(256) void cg_bn_eval_final_kernel(BnFinArgs a) {
  const int slot = a.slots[blockIdx.y];
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= a.C) return;
  const float* row = a.state + (long)slot * a.s_mstride;
  const float mean = row[a.run_off + c], var = row[a.run_off + a.C + c];
  const float inv = rsqrtf(var + BN_EPS);
  const float scale = row[a.gamma_off + c] * inv;
  float* co = a.coef + (long)slot * 4 * a.cmax;
  co[c] = scale;
  co[a.cmax + c] = row[a.beta_off + c] - mean * scale;
  co[2 * a.cmax + c] = mean;
  co[3 * a.cmax + c] = inv;
}

__global__ __launch_bounds__(256) void cg_bn_bwd_final_kernel(BnFinArgs a) {
  const int slot = a.slots[blockIdx.y];
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= a.C) return;
  const dtf_acc_t* su = a.sums + (long)slot * 2 * a.cmax;
  const float* fc = a.fcoef + (long)slot * 4 * a.cmax;
  const float n = a.cnt[slot] * (float)a.hw;
  const float sdz = dtf_acc_get(su + c, DTF_FX_GRAD), sdzx = dtf_acc_get(su + a.cmax + c, DTF_FX_GRAD);
  const float mean = fc[2 * a.cmax + c], inv = fc[3 * a.cmax + c];
  const float* row = a.state + (long)slot * a.s_mstride;
  const float scale = row[a.gamma_off + c] * inv;
  const float m1 = sdz / n, m2 = sdzx / n;
  float* co = a.coef + (long)slot * 4 * a.cmax;
  co[c] = scale;
  co[a.cmax + c] = -scale * inv * m2;
  co[2 * a.cmax + c] = -scale * m1 + scale * inv * mean * m2;
  float* g = a.grads + (long)slot * a.g_mstride;
  g[a.gamma_off + c] += sdzx;
  g[a.beta_off + c] += sdz;
}

struct EwArgs {
  const bf16_t* dz;
  const bf16_t* h;
  const bf16_t* add;
  bf16_t* out;
  const float* coef;   // [cap][4][cmax]
  const int* img_slot;
  long hw;
  int C, cmax;
  long nimg;
};

// 8 consecutive per-channel coefficients (c0 % 8 == 0: two 16-byte loads)
__device__ __forceinline__ void coef8(const float* p, float (&v)[8]) {
  const float4 u = *reinterpret_cast<const float4*>(p), w = *reinterpret_cast<const float4*>(p + 4);
  v[0] = u.x; v[1] = u.y; v[2] = u.z; v[3] = u.w; v[4] = w.x; v[5] = w.y; v[6] = w.z; v[7] = w.w;
}

// Channel of element 8*i of an image (32-bit: one image holds < 2^31 elements; a mask for power-of-two C).
__device__ __forceinline__ int chan8(long i, int C) {
  const int e = (int)i * 8;
  return (C & (C - 1)) == 0 ? (e & (C - 1)) : e % C;
}

// 16-byte output store; NT: non-temporal (measured 86.7 vs 86.9 ms per ResNet-50 step, so the launchers use plain
// stores: the next conv reads the output right away, partly from the caches; profiles/r2_s3_imagenet_ew_nt_ab.log)
template <bool NT>
__device__ __forceinline__ void ew_store(bf16_t* p, uint4 v) {
  if constexpr (NT) {
    uint32_t* q = reinterpret_cast<uint32_t*>(p);
    __builtin_nontemporal_store(v.x, q);
    __builtin_nontemporal_store(v.y, q + 1);
    __builtin_nontemporal_store(v.z, q + 2);
    __builtin_nontemporal_store(v.w, q + 3);
  } else {
    *reinterpret_cast<uint4*>(p) = v;
  }
}

// Both apply kernels stream U 16-byte chunks per thread and outer iteration, all loads issued before the first
// store (the output may alias an input for the compiler), so each thread keeps U (x 2-3 operands) loads in flight.
constexpr int EW_U = 4;

template <bool NT>
__global__ __launch_bounds__(256) void cg_bn_bwd_apply_kernel(EwArgs a) {
  const int img = blockIdx.x;
  const int slot = a.img_slot[img];
  const float* co = a.coef + (long)slot * 4 * a.cmax;
  const long base = (long)img * a.hw * a.C;
  const long n8 = a.hw * a.C / 8;
  const long stride = (long)gridDim.y * blockDim.x;
  const bf16_t* __restrict__ dz = a.dz + base;
  const bf16_t* __restrict__ h = a.h + base;
  const bf16_t* __restrict__ add = a.add ? a.add + base : nullptr;
  bf16_t* __restrict__ out = a.out + base;
  for (long i0 = (long)blockIdx.y * blockDim.x + threadIdx.x; i0 < n8; i0 += EW_U * stride) {
    uint4 dv[EW_U], hv[EW_U], av[EW_U];
#pragma unroll
    for (int u = 0; u < EW_U; ++u) {
      const long i = i0 + u * stride;
      dv[u] = hv[u] = av[u] = make_uint4(0, 0, 0, 0);
      if (i < n8) {
        dv[u] = *reinterpret_cast<const uint4*>(dz + i * 8);
        hv[u] = *reinterpret_cast<const uint4*>(h + i * 8);
        if (add) av[u] = *reinterpret_cast<const uint4*>(add + i * 8);
      }
    }
#pragma unroll
    for (int u = 0; u < EW_U; ++u) {
      const long i = i0 + u * stride;
      if (i >= n8) break;
      const int c0 = chan8(i, a.C);
      float ca[8], cbv[8], cc[8];
      coef8(co + c0, ca);
      coef8(co + a.cmax + c0, cbv);
      coef8(co + 2 * a.cmax + c0, cc);
      const uint32_t d32[4] = {dv[u].x, dv[u].y, dv[u].z, dv[u].w}, h32[4] = {hv[u].x, hv[u].y, hv[u].z, hv[u].w},
                     a32[4] = {av[u].x, av[u].y, av[u].z, av[u].w};
      uint32_t r[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float v0 = ca[2 * q] * lo2f(d32[q]) + cbv[2 * q] * lo2f(h32[q]) +
                         cc[2 * q] + lo2f(a32[q]);
        const float v1 = ca[2 * q + 1] * hi2f(d32[q]) +
                         cbv[2 * q + 1] * hi2f(h32[q]) + cc[2 * q + 1] +
                         hi2f(a32[q]);
        r[q] = pack2bf(v0, v1);
      }
      ew_store<NT>(out + i * 8, make_uint4(r[0], r[1], r[2], r[3]));
    }
  }
}

// a = relu(BN(h)) with the member's forward coefficients (the activation every consumer conv stages as-is)
template <bool NT>
__global__ __launch_bounds__(256) void cg_bn_relu_apply_kernel(EwArgs a) {
  const int img = blockIdx.x;
  const int slot = a.img_slot[img];
  const float* co = a.coef + (long)slot * 4 * a.cmax;
  const long base = (long)img * a.hw * a.C;
  const long n8 = a.hw * a.C / 8;
  const long stride = (long)gridDim.y * blockDim.x;
  const bf16_t* __restrict__ h = a.h + base;
  bf16_t* __restrict__ out = a.out + base;
  for (long i0 = (long)blockIdx.y * blockDim.x + threadIdx.x; i0 < n8; i0 += EW_U * stride) {
    uint4 hv[EW_U];
#pragma unroll
    for (int u = 0; u < EW_U; ++u) {
      const long i = i0 + u * stride;
      hv[u] = i < n8 ? *reinterpret_cast<const uint4*>(h + i * 8) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < EW_U; ++u) {
      const long i = i0 + u * stride;
      if (i >= n8) break;
      const int c0 = chan8(i, a.C);
      float sc[8], sh[8];
      coef8(co + c0, sc);
      coef8(co + a.cmax + c0, sh);
      const uint32_t h32[4] = {hv[u].x, hv[u].y, hv[u].z, hv[u].w};
      uint32_t r[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float v0 = fmaxf(lo2f(h32[q]) * sc[2 * q] + sh[2 * q], 0.f);
        const float v1 = fmaxf(hi2f(h32[q]) * sc[2 * q + 1] + sh[2 * q + 1], 0.f);
        r[q] = pack2bf(v0, v1);
      }
      ew_store<NT>(out + i * 8, make_uint4(r[0], r[1], r[2], r[3]));
    }
  }
}

// Channel-fixed forms of the two apply kernels (C / 8 a power of two <= 256): thread t always owns the 16-byte
// channel chunk t % (C / 8) and walks pixels, so its 8 channels' coefficients are loaded ONCE into registers instead
// of with every data chunk (the chunk-walking kernels above issue 2-3 coefficient loads of 32 bytes per 16-byte data
// load; at C >= 1024 they streamed at 3.9-4.1 TB/s: profiles/r5_imagenet_roofline_epi.txt).  A wave still covers
// 64 consecutive chunks (1 KB contiguous: the pixel rows are contiguous).  grid (images, pixel splits).
#ifndef CG_EW_CF
#define CG_EW_CF 1
#endif
template <bool RELU_APPLY>
__global__ __launch_bounds__(256) void cg_ew_apply_cf_kernel(EwArgs a) {
  const int img = blockIdx.x;
  const int slot = a.img_slot[img];
  const float* co = a.coef + (long)slot * 4 * a.cmax;
  const int cpp = a.C >> 3, ppi = 256 / cpp;  // chunks per pixel, pixels per workgroup pass
  const int cc = threadIdx.x & (cpp - 1);
  const long P = a.hw, pstep = (long)gridDim.y * ppi;
  const long base = (long)img * P * a.C + 8 * cc;
  float c0[8], c1[8], c2[8];
  coef8(co + 8 * cc, c0);
  coef8(co + a.cmax + 8 * cc, c1);
  if constexpr (!RELU_APPLY) coef8(co + 2 * a.cmax + 8 * cc, c2);
  const bf16_t* __restrict__ h = a.h + base;
  const bf16_t* __restrict__ dz = RELU_APPLY ? nullptr : a.dz + base;
  const bf16_t* __restrict__ add = (!RELU_APPLY && a.add) ? a.add + base : nullptr;
  bf16_t* __restrict__ out = a.out + base;
  for (long p = (long)blockIdx.y * ppi + threadIdx.x / cpp; p < P; p += EW_U * pstep) {
    uint4 hv[EW_U], dv[EW_U], av[EW_U];
#pragma unroll
    for (int u = 0; u < EW_U; ++u) {
      const long pp = p + u * pstep;
      hv[u] = dv[u] = av[u] = make_uint4(0, 0, 0, 0);
      if (pp < P) {
        hv[u] = *reinterpret_cast<const uint4*>(h + pp * a.C);
        if constexpr (!RELU_APPLY) {
          dv[u] = *reinterpret_cast<const uint4*>(dz + pp * a.C);
          if (add) av[u] = *reinterpret_cast<const uint4*>(add + pp * a.C);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < EW_U; ++u) {
      const long pp = p + u * pstep;
      if (pp >= P) break;
      const uint32_t h32[4] = {hv[u].x, hv[u].y, hv[u].z, hv[u].w}, d32[4] = {dv[u].x, dv[u].y, dv[u].z, dv[u].w},
                     a32[4] = {av[u].x, av[u].y, av[u].z, av[u].w};
      uint32_t r[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float v0, v1;
        if constexpr (RELU_APPLY) {
          v0 = fmaxf(lo2f(h32[q]) * c0[2 * q] + c1[2 * q], 0.f);
          v1 = fmaxf(hi2f(h32[q]) * c0[2 * q + 1] + c1[2 * q + 1], 0.f);
        } else {
          v0 = c0[2 * q] * lo2f(d32[q]) + c1[2 * q] * lo2f(h32[q]) + c2[2 * q] + lo2f(a32[q]);
          v1 = c0[2 * q + 1] * hi2f(d32[q]) + c1[2 * q + 1] * hi2f(h32[q]) + c2[2 * q + 1] + hi2f(a32[q]);
        }
        r[q] = pack2bf(v0, v1);
      }
      *reinterpret_cast<uint4*>(out + pp * a.C) = make_uint4(r[0], r[1], r[2], r[3]);
    }
  }
}

__device__ __host__ inline bool ew_cf_ok(int C) {
  const int cpp = C >> 3;
  return CG_EW_CF && (C & 7) == 0 && cpp >= 1 && cpp <= 256 && (cpp & (cpp - 1)) == 0;
}

__global__ __launch_bounds__(256) void cg_prep_input_kernel(const float* __restrict__ x, bf16_t* __restrict__ y,
                                                             long npix, int c_in) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long p = (long)blockIdx.x * blockDim.x + threadIdx.x; p < npix; p += stride) {
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < c_in; ++c) v[c] = x[p * c_in + c];
    *reinterpret_cast<uint4*>(y + p * 8) =
        make_uint4(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]), pack2bf(v[6], v[7]));
  }
}

// space-to-depth stem input: x [N][H][W][c_in] fp32 -> y [N][H/2][W/2][16] with channel (2 dy + dx) * c_in + c =
// x[2 by + dy][2 bx + dx][c] (channels 4 c_in .. 15 zero); thread = one 2x2 block
__global__ __launch_bounds__(256) void cg_prep_input_s2d_kernel(const float* __restrict__ x, bf16_t* __restrict__ y,
                                                                long nblk, int H, int W, int c_in) {
  const long stride = (long)gridDim.x * blockDim.x;
  const int Wb = W / 2, Hb = H / 2;
  for (long b = (long)blockIdx.x * blockDim.x + threadIdx.x; b < nblk; b += stride) {
    const long img = b / ((long)Hb * Wb);
    const int r = (int)(b - img * Hb * Wb), by = r / Wb, bx = r - by * Wb;
    float v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = 0.f;
    if (c_in == 3) {  // the image case: per input row the block's 2 pixels are 6 contiguous floats (3 x 8-byte loads)
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const float2* src = reinterpret_cast<const float2*>(x + ((img * H + 2 * by + r) * W + 2 * bx) * 3);
        const float2 a = src[0], b = src[1], c = src[2];
        v[6 * r] = a.x; v[6 * r + 1] = a.y; v[6 * r + 2] = b.x; v[6 * r + 3] = b.y; v[6 * r + 4] = c.x; v[6 * r + 5] = c.y;
      }
    } else {
      for (int q = 0; q < 4; ++q) {
        const float* src = x + ((img * H + 2 * by + (q >> 1)) * W + 2 * bx + (q & 1)) * c_in;
        for (int c = 0; c < c_in; ++c) v[q * c_in + c] = src[c];
      }
    }
    uint4* dst = reinterpret_cast<uint4*>(y + b * 16);
    dst[0] = make_uint4(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]), pack2bf(v[6], v[7]));
    dst[1] = make_uint4(pack2bf(v[8], v[9]), pack2bf(v[10], v[11]), pack2bf(v[12], v[13]), pack2bf(v[14], v[15]));
  }
}

// 3x3 stride-2 max-pool, output o covers input rows / cols 2o .. 2o+2 (TF 'SAME': the pad is at the end)
__global__ __launch_bounds__(256) void cg_maxpool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                              uint8_t* __restrict__ am, int H, int W, int Ho, int Wo,
                                                              int C, long total8) {
  // 32-bit index math (the host checks total8 < 2^31; 64-bit division per element cost more than the loads)
  const unsigned stride = gridDim.x * blockDim.x, C8 = (unsigned)C / 8;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < (unsigned)total8; i += stride) {
    const unsigned pix = i / C8;
    const int c0 = (int)(i - pix * C8) * 8;
    const unsigned pr = pix / (unsigned)Wo;
    const int ox = (int)(pix - pr * Wo), oy = (int)(pr % (unsigned)Ho);
    const long img = pr / (unsigned)Ho;
    float best[8];
    uint32_t arg[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      best[k] = -3.0e38f;
      arg[k] = 0;
    }
    for (int t = 0; t < 9; ++t) {
      const int iy = 2 * oy + t / 3, ix = 2 * ox + t % 3;
      if (iy >= H || ix >= W) continue;
      const uint4 v = *reinterpret_cast<const uint4*>(x + ((img * H + iy) * W + ix) * C + c0);
      const uint32_t w32[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float f = bf2f((bf16_t)((w32[k >> 1] >> (16 * (k & 1))) & 0xffff));
        if (f > best[k]) {
          best[k] = f;
          arg[k] = (uint32_t)t;
        }
      }
    }
    const long o = (long)pix * C + c0;
    *reinterpret_cast<uint4*>(y + o) = make_uint4(pack2bf(best[0], best[1]), pack2bf(best[2], best[3]),
                                                  pack2bf(best[4], best[5]), pack2bf(best[6], best[7]));
    *reinterpret_cast<uint2*>(am + o) = make_uint2(arg[0] | (arg[1] << 8) | (arg[2] << 16) | (arg[3] << 24),
                                                   arg[4] | (arg[5] << 8) | (arg[6] << 16) | (arg[7] << 24));
  }
}

__device__ uint4 g_mp_zero16 = {0u, 0u, 0u, 0u};  // what a masked-off candidate window reads (never written)
__device__ uint2 g_mp_ff8 = {0xffffffffu, 0xffffffffu};  // ... and its argmax (matches no tap)

__global__ __launch_bounds__(256) void cg_maxpool_bwd_kernel(const bf16_t* __restrict__ g, const uint8_t* __restrict__ am,
                                                              bf16_t* __restrict__ dx, int H, int W, int Ho, int Wo,
                                                              int C, long total8) {
  const unsigned stride = gridDim.x * blockDim.x, C8 = (unsigned)C / 8;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < (unsigned)total8; i += stride) {
    const unsigned pix = i / C8;
    const int c0 = (int)(i - pix * C8) * 8;
    const unsigned pr = pix / (unsigned)W;
    const int ix = (int)(pix - pr * W), iy = (int)(pr % (unsigned)H);
    const long img = pr / (unsigned)H;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // the (at most 2 x 2) windows containing (iy, ix): oy = iy / 2 (tap row iy % 2) and, for even iy >= 2,
    // oy = iy / 2 - 1 (tap row 2); likewise in x.  All four candidates' loads are issued before any is used
    // (branch-free: a missing window reads a zero vector / an argmax that matches no tap) -- the former loop
    // issued one window's loads at a time (2.9 TB/s, profiles/r3_s2_imagenet_roofline.txt)
    const int oyA = iy >> 1, oxA = ix >> 1;
    const bool yA = oyA < Ho, xA = oxA < Wo, yB = !(iy & 1) && iy >= 2, xB = !(ix & 1) && ix >= 2;
    const int oy_[2] = {oyA, oyA - 1}, ox_[2] = {oxA, oxA - 1};
    const uint32_t ty_[2] = {(uint32_t)(iy & 1), 2u}, tx_[2] = {(uint32_t)(ix & 1), 2u};
    const bool oky[2] = {yA, yB}, okx[2] = {xA, xB};
    uint2 av[4];
    uint4 gv[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const int a_ = w >> 1, b_ = w & 1;
      const bool ok = oky[a_] && okx[b_];
      const long o = ok ? ((img * Ho + oy_[a_]) * Wo + ox_[b_]) * C + c0 : 0;
      av[w] = *(ok ? reinterpret_cast<const uint2*>(am + o) : &g_mp_ff8);
      gv[w] = *(ok ? reinterpret_cast<const uint4*>(g + o) : &g_mp_zero16);
    }
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const uint32_t t = ty_[w >> 1] * 3 + tx_[w & 1];
      const uint32_t g32[4] = {gv[w].x, gv[w].y, gv[w].z, gv[w].w};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t ak = ((k < 4 ? av[w].x : av[w].y) >> (8 * (k & 3))) & 0xffu;
        if (ak == t) acc[k] += bf2f((bf16_t)((g32[k >> 1] >> (16 * (k & 1))) & 0xffff));
      }
    }
    *reinterpret_cast<uint4*>(dx + (long)pix * C + c0) = make_uint4(pack2bf(acc[0], acc[1]), pack2bf(acc[2], acc[3]),
                                                              pack2bf(acc[4], acc[5]), pack2bf(acc[6], acc[7]));
  }
}

// The same backward for even H, W with Ho = H / 2 (every ImageNet shape): thread = one 2 x 2 input block (by, bx)
// and 8 channels.  The block's 4 pixels draw only on the windows {by - 1, by} x {bx - 1, bx}, so each window's
// gradient / argmax is loaded once for 4 pixels (the per-pixel form above loads ~2.25 windows per pixel) and the
// 4 output rows are written as 16-byte stores.  Pixel (dy, dx) of the block receives window (by - a, bx - b)'s
// gradient when its argmax is tap (dy + 2a) * 3 + (dx + 2b) (a, b in {0, 1}; a = 1 only for dy = 0).
__global__ __launch_bounds__(256) void cg_maxpool_bwd2_kernel(const bf16_t* __restrict__ g, const uint8_t* __restrict__ am,
                                                               bf16_t* __restrict__ dx, int Ho, int Wo, int C,
                                                               long total8) {
  const unsigned stride = gridDim.x * blockDim.x, C8 = (unsigned)C / 8;
  const int W = 2 * Wo;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < (unsigned)total8; i += stride) {
    const unsigned blk = i / C8;
    const int c0 = (int)(i - blk * C8) * 8;
    const unsigned pr = blk / (unsigned)Wo;
    const int bx = (int)(blk - pr * Wo), by = (int)(pr % (unsigned)Ho);
    const long img = pr / (unsigned)Ho;
    uint2 av[2][2];
    uint4 gv[2][2];
#pragma unroll
    for (int a_ = 0; a_ < 2; ++a_)
#pragma unroll
      for (int b_ = 0; b_ < 2; ++b_) {
        const bool ok = by - a_ >= 0 && bx - b_ >= 0;
        const long o = ok ? ((img * Ho + by - a_) * Wo + bx - b_) * C + c0 : 0;
        av[a_][b_] = *(ok ? reinterpret_cast<const uint2*>(am + o) : &g_mp_ff8);
        gv[a_][b_] = *(ok ? reinterpret_cast<const uint4*>(g + o) : &g_mp_zero16);
      }
#pragma unroll
    for (int py = 0; py < 2; ++py)
#pragma unroll
      for (int px = 0; px < 2; ++px) {
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int a_ = 0; a_ < 2; ++a_)
#pragma unroll
          for (int b_ = 0; b_ < 2; ++b_) {
            if ((a_ && py) || (b_ && px)) continue;  // window by - 1 / bx - 1 covers only the block's first row / col
            const uint32_t t = (uint32_t)((py + 2 * a_) * 3 + px + 2 * b_);
            const uint32_t g32[4] = {gv[a_][b_].x, gv[a_][b_].y, gv[a_][b_].z, gv[a_][b_].w};
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const uint32_t ak = ((k < 4 ? av[a_][b_].x : av[a_][b_].y) >> (8 * (k & 3))) & 0xffu;
              if (ak == t) acc[k] += bf2f((bf16_t)((g32[k >> 1] >> (16 * (k & 1))) & 0xffff));
            }
          }
        const long o = ((img * 2 * Ho + 2 * by + py) * W + 2 * bx + px) * C + c0;
        *reinterpret_cast<uint4*>(dx + o) = make_uint4(pack2bf(acc[0], acc[1]), pack2bf(acc[2], acc[3]),
                                                       pack2bf(acc[4], acc[5]), pack2bf(acc[6], acc[7]));
      }
  }
}

struct GapArgs {
  const bf16_t* x;      // [N][hw][C] last block output (pre final BN)
  const float* coef;    // final BN forward coefficients [cap][4][cmax] (nullptr: identity, v1)
  const int* img_slot;
  bf16_t* feat;         // [N][C] bf16
  const float* dfeat;   // bwd: [N][C] fp32 (dL/dfeat)
  dtf_acc_t* sums;      // bwd: final-BN backward sums [cap][2][cmax]
  const float* bcoef;   // bwd apply: A, B, C
  bf16_t* out;          // bwd apply: gradient at x
  int hw, C, cmax;
};

// one workgroup per image, thread = channel group of 8 (C <= 2048)
__global__ __launch_bounds__(256) void cg_gap_kernel(GapArgs a) {
  const int img = blockIdx.x, slot = a.img_slot[img];
  const float* co = a.coef ? a.coef + (long)slot * 4 * a.cmax : nullptr;
  for (int c0 = threadIdx.x * 8; c0 < a.C; c0 += blockDim.x * 8) {
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 7  // several independent loads per round trip (hw = 49 for the 224x224 net)
    for (int p = 0; p < a.hw; ++p) {
      const uint4 v = *reinterpret_cast<const uint4*>(a.x + ((long)img * a.hw + p) * a.C + c0);
      const uint32_t w32[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float f = bf2f((bf16_t)((w32[k >> 1] >> (16 * (k & 1))) & 0xffff));
        if (co) f = fmaxf(f * co[c0 + k] + co[a.cmax + c0 + k], 0.f);
        s[k] += f;
      }
    }
    const float inv = 1.f / (float)a.hw;
    *reinterpret_cast<uint4*>(a.feat + (long)img * a.C + c0) =
        make_uint4(pack2bf(s[0] * inv, s[1] * inv), pack2bf(s[2] * inv, s[3] * inv), pack2bf(s[4] * inv, s[5] * inv),
                   pack2bf(s[6] * inv, s[7] * inv));
  }
}

// final-BN backward sums: dz = dfeat/hw * [BN(x) > 0]; sum dz, sum dz*xhat
__global__ __launch_bounds__(256) void cg_gap_bwd_reduce_kernel(GapArgs a) {
  const int img = blockIdx.x, slot = a.img_slot[img];
  const float* co = a.coef + (long)slot * 4 * a.cmax;
  dtf_acc_t* su = a.sums + (long)slot * 2 * a.cmax;
  const float inv_hw = 1.f / (float)a.hw;
  for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
    const float g = a.dfeat[(long)img * a.C + c] * inv_hw;
    const float sc = co[c], sh = co[a.cmax + c], mu = co[2 * a.cmax + c], iv = co[3 * a.cmax + c];
    float s = 0.f, q = 0.f;
#pragma unroll 7
    for (int p = 0; p < a.hw; ++p) {
      const float xv = bf2f(a.x[((long)img * a.hw + p) * a.C + c]);
      if (xv * sc + sh > 0.f) {
        s += g;
        q += g * (xv - mu) * iv;
      }
    }
    dtf_acc_add(su + c, s, DTF_FX_GRAD, slot);
    dtf_acc_add(su + a.cmax + c, q, DTF_FX_GRAD, slot);
  }
}

__global__ __launch_bounds__(256) void cg_gap_bwd_apply_kernel(GapArgs a) {
  const int img = blockIdx.x, slot = a.img_slot[img];
  const float* co = a.coef ? a.coef + (long)slot * 4 * a.cmax : nullptr;
  const float* bc = a.bcoef ? a.bcoef + (long)slot * 4 * a.cmax : nullptr;
  const float inv_hw = 1.f / (float)a.hw;
  const long n = (long)a.hw * a.C;
  for (long i = threadIdx.x; i < n; i += blockDim.x) {
    const int c = (int)(i % a.C);
    const long o = (long)img * n + i;
    const float xv = bf2f(a.x[o]);
    const float g = a.dfeat[(long)img * a.C + c] * inv_hw;
    float r;
    if (co) {
      const float dz = (xv * co[c] + co[a.cmax + c] > 0.f) ? g : 0.f;
      r = bc[c] * dz + bc[a.cmax + c] * xv + bc[2 * a.cmax + c];
    } else {
      r = xv > 0.f ? g : 0.f;  // v1: the last block's ReLU
    }
    a.out[o] = f2bf(r);
  }
}

// one wave per image: logits [N][ld] fp32 (+ bias) -> loss / correct / dlogits bf16 [N][ld] / dbias
__global__ __launch_bounds__(256) void cg_softmax_ce_kernel(const float* __restrict__ logits, int ld, int ncls,
                                                             const int* __restrict__ labels,
                                                             const int* __restrict__ img_slot,
                                                             const float* __restrict__ state, long s_mstride, int b_off,
                                                             dtf_acc_t* __restrict__ grads, long g_mstride,
                                                             const float* __restrict__ cnt, dtf_acc_t* __restrict__ loss,
                                                             float* __restrict__ correct, bf16_t* __restrict__ dl,
                                                             long nimg, float loss_scale) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long img = (long)blockIdx.x * 4 + wave;
  if (img >= nimg) return;
  const int slot = img_slot[img];
  const float* bias = state + (long)slot * s_mstride + b_off;
  const float* lr = logits + img * ld;
  float mx = -3.0e38f;
  int arg = 0;
  for (int j = lane; j < ncls; j += 64) {
    const float v = lr[j] + bias[j];
    if (v > mx) {
      mx = v;
      arg = j;
    }
  }
  for (int o = 32; o >= 1; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64);
    const int oa = __shfl_xor(arg, o, 64);
    if (om > mx || (om == mx && oa < arg)) {
      mx = om;
      arg = oa;
    }
  }
  float se = 0.f;
  for (int j = lane; j < ncls; j += 64) se += __expf(lr[j] + bias[j] - mx);
  se = wave_sum(se);
  const float lse = mx + __logf(se);
  const int lab = labels[img];
  const float bsz = cnt[slot];
  const float gsc = loss_scale / bsz;  // gradients of loss_scale * loss (fp16 static loss scaling; else 1)
  dtf_acc_t* gb = grads != nullptr ? grads + (long)slot * g_mstride + b_off : nullptr;
  for (int j = lane; j < ld; j += 64) {
    float d = 0.f;
    if (j < ncls) {
      d = (__expf(lr[j] + bias[j] - lse) - (j == lab ? 1.f : 0.f)) * gsc;
      if (grads != nullptr) dtf_acc_add(gb + j, d, DTF_FX_GRAD, slot);
    }
    if (dl != nullptr) dl[img * ld + j] = f2bf(d);  // eval (no grads / dlogits): loss and correct count only
  }
  if (lane == 0) {
    dtf_acc_add(loss + slot, (lse - (lr[lab] + bias[lab])) / bsz, DTF_FX_GRAD, slot);
    atomicAdd(correct + slot, arg == lab ? 1.f : 0.f);  // integer-valued: exact in any order
  }
}

// per-channel sum / second moment of a [N][hw][C] tensor into [cap][2][cmax] (BN statistics of a tensor no conv
// epilogue produced, e.g. the max-pool output); thread = 8 fixed channels, LDS reduction, one atomic per WG
__global__ __launch_bounds__(256) void cg_chan_stats_kernel(const bf16_t* __restrict__ x, const int* __restrict__ img_slot,
                                                             dtf_acc_t* __restrict__ sums, int hw, int C, int cmax) {
  __shared__ dtf_acc_t acc[2][2048];
  const int img = blockIdx.x, slot = img_slot[img];
  for (int i = threadIdx.x; i < 2 * C; i += blockDim.x) (&acc[0][0])[(i / C) * 2048 + i % C] = 0;
  __syncthreads();
  const long n8 = (long)hw * C / 8;
  const long i0 = (long)blockIdx.y * blockDim.x + threadIdx.x, st = (long)gridDim.y * blockDim.x;
  if (i0 < n8 && (st * 8) % C == 0) {
    const int c0 = (int)((i0 * 8) % C);
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, q[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (long i = i0; i < n8; i += st) {
      const uint4 v = *reinterpret_cast<const uint4*>(x + (long)img * hw * C + i * 8);
      const uint32_t w32[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float f = bf2f((bf16_t)((w32[k >> 1] >> (16 * (k & 1))) & 0xffff));
        s[k] += f;
        q[k] += f * f;
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      dtf_acc_add(&acc[0][c0 + k], s[k], DTF_FX_STAT, slot);
      dtf_acc_add(&acc[1][c0 + k], q[k], DTF_FX_STAT, slot);
    }
  }
  __syncthreads();
  dtf_acc_t* su = sums + (long)slot * 2 * cmax;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    dtf_acc_addw(su + c, acc[0][c]);
    dtf_acc_addw(su + cmax + c, acc[1][c]);
  }
}

// ---- ResNet v1 (post-activation) bottleneck blocks (reference resnet_model.py:215-264)
// Block output y = relu(BN3(h3) + shortcut), shortcut = BN_p(s) (projection conv output s) or the block input.
struct BnAddArgs {
  const bf16_t* h;       // conv3 output (BN3 input)
  const bf16_t* s;       // projection conv output (coef_s) or the block input (coef_s == null: identity)
  bf16_t* out;
  const float* coef_h;   // [cap][4][cmax] forward coefficients of BN3
  const float* coef_s;   // ... of the projection BN, or null
  const int* img_slot;
  long hw;
  int C, cmax;
  long nimg;
};

__global__ __launch_bounds__(256) void cg_bn_add_relu_kernel(BnAddArgs a) {
  const int img = blockIdx.x;
  const int slot = a.img_slot[img];
  const float* ch = a.coef_h + (long)slot * 4 * a.cmax;
  const float* cs = a.coef_s ? a.coef_s + (long)slot * 4 * a.cmax : nullptr;
  const long base = (long)img * a.hw * a.C;
  const long n8 = a.hw * a.C / 8;
  const long stride = (long)gridDim.y * blockDim.x;
  const bf16_t* __restrict__ h = a.h + base;
  const bf16_t* __restrict__ s = a.s + base;
  bf16_t* __restrict__ out = a.out + base;
  for (long i0 = (long)blockIdx.y * blockDim.x + threadIdx.x; i0 < n8; i0 += EW_U * stride) {
    uint4 hv[EW_U], sv[EW_U];
#pragma unroll
    for (int u = 0; u < EW_U; ++u) {
      const long i = i0 + u * stride;
      hv[u] = sv[u] = make_uint4(0, 0, 0, 0);
      if (i < n8) {
        hv[u] = *reinterpret_cast<const uint4*>(h + i * 8);
        sv[u] = *reinterpret_cast<const uint4*>(s + i * 8);
      }
    }
#pragma unroll
    for (int u = 0; u < EW_U; ++u) {
      const long i = i0 + u * stride;
      if (i >= n8) break;
      const int c0 = chan8(i, a.C);
      float sc[8], sh[8], ps[8], pt[8];
      coef8(ch + c0, sc);
      coef8(ch + a.cmax + c0, sh);
      if (cs) {
        coef8(cs + c0, ps);
        coef8(cs + a.cmax + c0, pt);
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) ps[k] = 1.f, pt[k] = 0.f;
      }
      const uint32_t h32[4] = {hv[u].x, hv[u].y, hv[u].z, hv[u].w}, s32[4] = {sv[u].x, sv[u].y, sv[u].z, sv[u].w};
      uint32_t r[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float v0 = lo2f(h32[q]) * sc[2 * q] + sh[2 * q] +
                         lo2f(s32[q]) * ps[2 * q] + pt[2 * q];
        const float v1 = hi2f(h32[q]) * sc[2 * q + 1] + sh[2 * q + 1] +
                         hi2f(s32[q]) * ps[2 * q + 1] + pt[2 * q + 1];
        r[q] = pack2bf(fmaxf(v0, 0.f), fmaxf(v1, 0.f));
      }
      *reinterpret_cast<uint4*>(out + i * 8) = make_uint4(r[0], r[1], r[2], r[3]);
    }
  }
}

// Channel-fixed form (the layout of cg_ew_apply_cf_kernel): the 4 coefficient vectors of the thread's 8 channels are
// loaded once instead of 4 x 32 bytes per 16-byte data chunk
__global__ __launch_bounds__(256) void cg_bn_add_relu_cf_kernel(BnAddArgs a) {
  const int img = blockIdx.x;
  const int slot = a.img_slot[img];
  const int cpp = a.C >> 3, ppi = 256 / cpp;
  const int cc = threadIdx.x & (cpp - 1);
  const long P = a.hw, pstep = (long)gridDim.y * ppi;
  const float* ch = a.coef_h + (long)slot * 4 * a.cmax + 8 * cc;
  float sc[8], sh[8], ps[8], pt[8];
  coef8(ch, sc);
  coef8(ch + a.cmax, sh);
  if (a.coef_s) {
    const float* cs = a.coef_s + (long)slot * 4 * a.cmax + 8 * cc;
    coef8(cs, ps);
    coef8(cs + a.cmax, pt);
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) ps[k] = 1.f, pt[k] = 0.f;
  }
  const long base = (long)img * P * a.C + 8 * cc;
  const bf16_t* __restrict__ h = a.h + base;
  const bf16_t* __restrict__ s = a.s + base;
  bf16_t* __restrict__ out = a.out + base;
  for (long p = (long)blockIdx.y * ppi + threadIdx.x / cpp; p < P; p += EW_U * pstep) {
    uint4 hv[EW_U], sv[EW_U];
#pragma unroll
    for (int u = 0; u < EW_U; ++u) {
      const long pp = p + u * pstep;
      hv[u] = sv[u] = make_uint4(0, 0, 0, 0);
      if (pp < P) {
        hv[u] = *reinterpret_cast<const uint4*>(h + pp * a.C);
        sv[u] = *reinterpret_cast<const uint4*>(s + pp * a.C);
      }
    }
#pragma unroll
    for (int u = 0; u < EW_U; ++u) {
      const long pp = p + u * pstep;
      if (pp >= P) break;
      const uint32_t h32[4] = {hv[u].x, hv[u].y, hv[u].z, hv[u].w}, s32[4] = {sv[u].x, sv[u].y, sv[u].z, sv[u].w};
      uint32_t r[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float v0 = lo2f(h32[q]) * sc[2 * q] + sh[2 * q] + lo2f(s32[q]) * ps[2 * q] + pt[2 * q];
        const float v1 = hi2f(h32[q]) * sc[2 * q + 1] + sh[2 * q + 1] + hi2f(s32[q]) * ps[2 * q + 1] + pt[2 * q + 1];
        r[q] = pack2bf(fmaxf(v0, 0.f), fmaxf(v1, 0.f));
      }
      *reinterpret_cast<uint4*>(out + pp * a.C) = make_uint4(r[0], r[1], r[2], r[3]);
    }
  }
}

// BN-backward sums of post-activation BNs whose output gradient dz is already ReLU-masked (v1: the block output's
// mask is applied by the consumer's data-gradient epilogue): sum dz and sum dz * xhat into [cap][2][cmax], for
// the BN of h and optionally a second BN of h2 that received the same dz (v1 projection BN of the shortcut).
// Layout as cg_chan_stats: thread = 8 fixed channels, LDS accumulators, one global atomic per workgroup+channel.
struct BnSumArgs {
  const bf16_t* dz;
  const bf16_t* h;
  const bf16_t* h2;     // null: one BN
  const float* fc;      // forward coefficients of h's BN (mean at 2*cmax, inv at 3*cmax)
  const float* fc2;
  dtf_acc_t* sums;
  dtf_acc_t* sums2;
  const int* img_slot;
  int hw, C, cmax, pad;
};

__global__ __launch_bounds__(256) void cg_bn_bwd_sums_kernel(BnSumArgs a) {
  __shared__ dtf_acc_t acc[3][2048];
  const int img = blockIdx.x, slot = a.img_slot[img];
  const bool two = a.h2 != nullptr;
  for (int i = threadIdx.x; i < 3 * a.C; i += blockDim.x) (&acc[0][0])[(i / a.C) * 2048 + i % a.C] = 0;
  __syncthreads();
  const long n8 = (long)a.hw * a.C / 8;
  const long i0 = (long)blockIdx.y * blockDim.x + threadIdx.x, st = (long)gridDim.y * blockDim.x;
  if (i0 < n8 && (st * 8) % a.C == 0) {
    const int c0 = (int)((i0 * 8) % a.C);
    const float* f1 = a.fc + (long)slot * 4 * a.cmax;
    float mu[8], iv[8], mu2[8], iv2[8];
    coef8(f1 + 2 * a.cmax + c0, mu);
    coef8(f1 + 3 * a.cmax + c0, iv);
    if (two) {
      const float* f2 = a.fc2 + (long)slot * 4 * a.cmax;
      coef8(f2 + 2 * a.cmax + c0, mu2);
      coef8(f2 + 3 * a.cmax + c0, iv2);
    }
    float s[8], q[8], q2[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) s[k] = q[k] = q2[k] = 0.f;
    const long base = (long)img * a.hw * a.C;
    for (long i = i0; i < n8; i += st) {
      const uint4 dv = *reinterpret_cast<const uint4*>(a.dz + base + i * 8);
      const uint4 hv = *reinterpret_cast<const uint4*>(a.h + base + i * 8);
      const uint4 gv = two ? *reinterpret_cast<const uint4*>(a.h2 + base + i * 8) : make_uint4(0, 0, 0, 0);
      const uint32_t d32[4] = {dv.x, dv.y, dv.z, dv.w}, h32[4] = {hv.x, hv.y, hv.z, hv.w},
                     g32[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int sh = 16 * (k & 1);
        const float d = bf2f((bf16_t)((d32[k >> 1] >> sh) & 0xffff));
        const float hx = bf2f((bf16_t)((h32[k >> 1] >> sh) & 0xffff));
        s[k] += d;
        q[k] += d * (hx - mu[k]) * iv[k];
        if (two) {
          const float gx = bf2f((bf16_t)((g32[k >> 1] >> sh) & 0xffff));
          q2[k] += d * (gx - mu2[k]) * iv2[k];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      dtf_acc_add(&acc[0][c0 + k], s[k], DTF_FX_GRAD, slot);
      dtf_acc_add(&acc[1][c0 + k], q[k], DTF_FX_GRAD, slot);
      if (two) dtf_acc_add(&acc[2][c0 + k], q2[k], DTF_FX_GRAD, slot);
    }
  }
  __syncthreads();
  dtf_acc_t* su = a.sums + (long)slot * 2 * a.cmax;
  dtf_acc_t* su2 = two ? a.sums2 + (long)slot * 2 * a.cmax : nullptr;
  for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
    dtf_acc_addw(su + c, acc[0][c]);
    dtf_acc_addw(su + a.cmax + c, acc[1][c]);
    if (two) {
      dtf_acc_addw(su2 + c, acc[0][c]);
      dtf_acc_addw(su2 + a.cmax + c, acc[2][c]);
    }
  }
}

// Deterministic build: fold the fixed-point gradient accumulators of the step into the fp32 gradient rows (which
// already hold the order-free contributions: the dense-layer GEMM and the BN gamma / beta sums) and the loss, and
// clear the accumulators for the next step.  A member whose step produced a non-finite or out-of-range partial
// (flag words of convg.hip / this file, common.h dtf_fx) gets a NaN loss and NaN gradients instead.  grid (chunks,
// members); the flags are cleared by cg_poison_clear_kernel after every block has read them.
__global__ __launch_bounds__(256) void cg_det_finish_kernel(long long* __restrict__ gacc, float* __restrict__ grads,
                                                             long stride, long n, const int* __restrict__ slots,
                                                             long long* __restrict__ loss64, float* __restrict__ loss,
                                                             const unsigned* __restrict__ pz0,
                                                             const unsigned* __restrict__ pz1,
                                                             const unsigned* __restrict__ pz2) {
  const int slot = slots[blockIdx.y];
  const int ps = slot & (DTF_POISON_SLOTS - 1);
  const bool bad = (pz0 != nullptr && pz0[ps] != 0u) || (pz1 != nullptr && pz1[ps] != 0u) ||
                   (pz2 != nullptr && pz2[ps] != 0u);
  long long* ga = gacc + (long)slot * stride;
  float* g = grads + (long)slot * stride;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long long v = ga[i];
    if (bad) {
      g[i] = __builtin_nanf("");
      ga[i] = 0;
    } else if (v != 0) {
      g[i] += dtf_unfx(v, DTF_FX_GRAD);
      ga[i] = 0;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    loss[slot] = bad ? __builtin_nanf("") : dtf_unfx(loss64[slot], DTF_FX_GRAD);
    loss64[slot] = 0;
  }
}

__global__ void cg_poison_clear_kernel(unsigned* __restrict__ pz0, unsigned* __restrict__ pz1,
                                       unsigned* __restrict__ pz2, const int* __restrict__ slots, int nslots) {
  for (int i = threadIdx.x; i < nslots; i += blockDim.x) {
    const int ps = slots[i] & (DTF_POISON_SLOTS - 1);
    if (pz0 != nullptr) pz0[ps] = 0u;
    if (pz1 != nullptr) pz1[ps] = 0u;
    if (pz2 != nullptr) pz2[ps] = 0u;
  }
}

}  // namespace

#ifdef DTF_DETERMINISTIC
DTF_API unsigned* dtf_poison_ptr_convg();  // convg.hip
DTF_API unsigned* dtf_poison_ptr_convg_aux();
DTF_API unsigned* dtf_poison_ptr_f32conv();  // f32conv.hip (the fp32 CIFAR step)
#else
static unsigned* dtf_poison_ptr_convg() { return nullptr; }
static unsigned* dtf_poison_ptr_convg_aux() { return nullptr; }
static unsigned* dtf_poison_ptr_f32conv() { return nullptr; }
#endif

DTF_API int dtf_cg_det_finish(long long* gacc, float* grads, long stride, long n, const int* slots, int nslots,
                              long long* loss64, float* loss, hipStream_t stream) {
  if (nslots <= 0) return 0;
  long blocks = (n + 255) / 256;
  if (blocks > 512) blocks = 512;
  static unsigned* const pz0 = dtf_poison_ptr_convg();  // looked up once (not inside a graph capture's hot path)
  static unsigned* const pz1 = dtf_poison_ptr_convg_aux();
  static unsigned* const pz2 = dtf_poison_ptr_f32conv();
  hipLaunchKernelGGL(cg_det_finish_kernel, dim3((unsigned)blocks, nslots), dim3(256), 0, stream, gacc, grads, stride, n,
                     slots, loss64, loss, pz0, pz1, pz2);
  if (pz0 != nullptr || pz1 != nullptr || pz2 != nullptr)
    hipLaunchKernelGGL(cg_poison_clear_kernel, dim3(1), dim3(256), 0, stream, pz0, pz1, pz2, slots, nslots);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_fixed_acc() { return DTF_FIXED_ACC; }

DTF_POISON_EXPORT(convg_aux)

DTF_API int dtf_bnadd_args_size() { return (int)sizeof(BnAddArgs); }
DTF_API int dtf_bnsum_args_size() { return (int)sizeof(BnSumArgs); }

DTF_API int dtf_cg_bn_add_relu(const BnAddArgs* a, hipStream_t stream) {
  if (a->nimg <= 0) return 0;
  if (a->C % 8) return -2;
  const long n8 = a->hw * a->C / 8;
  long split = (4096 + a->nimg - 1) / a->nimg;
  const long ms = (n8 + 255) / 256;
  if (split > ms) split = ms;
  if (split < 1) split = 1;
  if (ew_cf_ok(a->C)) {
    const long ppi = 256 / (a->C >> 3), mp = (a->hw + ppi - 1) / ppi;
    const long sp = split < mp ? split : mp;
    hipLaunchKernelGGL(cg_bn_add_relu_cf_kernel, dim3((unsigned)a->nimg, (unsigned)sp), dim3(256), 0, stream, *a);
    return DTF_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(cg_bn_add_relu_kernel, dim3((unsigned)a->nimg, (unsigned)split), dim3(256), 0, stream, *a);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_cg_bn_bwd_sums(const BnSumArgs* a, int nimg, hipStream_t stream) {
  if (nimg <= 0) return 0;
  if (a->C > 2048 || a->C % 8 || 2048 % a->C) return -2;
  // workgroups per image: every workgroup ends with 2-3 x C global atomic adds, so wide layers get fewer (C = 2048:
  // 1 instead of 8 -- 6.3M instead of 50M atomics per launch); split * 2048 stays a multiple of C (the kernel's
  // fixed-channel condition)
  int split = 2048 / a->C;
  split = split < 1 ? 1 : (split > 8 ? 8 : split);
  hipLaunchKernelGGL(cg_bn_bwd_sums_kernel, dim3(nimg, split), dim3(256), 0, stream, *a);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_cg_chan_stats(const bf16_t* x, const int* img_slot, dtf_acc_t* sums, int nimg, int hw, int C, int cmax,
                              hipStream_t stream) {
  if (nimg <= 0) return 0;
  if (C > 2048 || C % 8 || 2048 % C) return -2;
  int split = 2048 / C;  // as dtf_cg_bn_bwd_sums: fewer workgroups (each ends with 2 x C global atomics) for wide C
  split = split < 1 ? 1 : (split > 8 ? 8 : split);
  hipLaunchKernelGGL(cg_chan_stats_kernel, dim3(nimg, split), dim3(256), 0, stream, x, img_slot, sums, hw, C, cmax);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_bnfin_args_size() { return (int)sizeof(BnFinArgs); }
DTF_API int dtf_ew_args_size() { return (int)sizeof(EwArgs); }
DTF_API int dtf_gap_args_size() { return (int)sizeof(GapArgs); }

DTF_API int dtf_cg_weight_prep(const float* state, long s_mstride, const int* table, int nconv, const int* slots,
                               int nslots, bf16_t* wf, bf16_t* wd, long w_mstride, hipStream_t stream) {
  if (nconv <= 0 || nslots <= 0) return 0;
  hipLaunchKernelGGL(cg_weight_prep_kernel, dim3(nconv, 32, nslots), dim3(256), 0, stream, state, s_mstride, table,
                     slots, wf, wd, w_mstride);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_cg_dense_prep(const float* state, long s_mstride, int w_off, int ncls, int npad, int C,
                              const int* slots, int nslots, bf16_t* out, long o_mstride, hipStream_t stream) {
  if (nslots <= 0) return 0;
  hipLaunchKernelGGL(cg_dense_prep_kernel, dim3(256, nslots), dim3(256), 0, stream, state, s_mstride, w_off, ncls,
                     npad, C, slots, out, o_mstride);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_cg_bn_final(const BnFinArgs* a, int backward, int nslots, hipStream_t stream) {
  if (nslots <= 0) return 0;
  dim3 grid((a->C + 255) / 256, nslots);
  if (backward == 2)  // eval: moving statistics
    hipLaunchKernelGGL(cg_bn_eval_final_kernel, grid, dim3(256), 0, stream, *a);
  else if (backward)
    hipLaunchKernelGGL(cg_bn_bwd_final_kernel, grid, dim3(256), 0, stream, *a);
  else
    hipLaunchKernelGGL(cg_bn_fwd_final_kernel, grid, dim3(256), 0, stream, *a);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_cg_bn_bwd_apply(const EwArgs* a, hipStream_t stream) {
  if (a->nimg <= 0) return 0;
  const long n8 = a->hw * a->C / 8;
  long split = (4096 + a->nimg - 1) / a->nimg;
  const long ms = (n8 + 255) / 256;
  if (split > ms) split = ms;
  if (split < 1) split = 1;
  if (ew_cf_ok(a->C)) {
    const long ppi = 256 / (a->C >> 3), mp = (a->hw + ppi - 1) / ppi;  // at most one pass of pixels per thread row
    const long sp = split < mp ? split : mp;
    hipLaunchKernelGGL(cg_ew_apply_cf_kernel<false>, dim3((unsigned)a->nimg, (unsigned)sp), dim3(256), 0, stream, *a);
    return DTF_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(cg_bn_bwd_apply_kernel<false>, dim3((unsigned)a->nimg, (unsigned)split), dim3(256), 0, stream, *a);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_cg_bn_relu_apply(const EwArgs* a, hipStream_t stream) {
  if (a->nimg <= 0) return 0;
  const long n8 = a->hw * a->C / 8;
  long split = (4096 + a->nimg - 1) / a->nimg;
  const long ms = (n8 + 255) / 256;
  if (split > ms) split = ms;
  if (split < 1) split = 1;
  if (ew_cf_ok(a->C)) {
    const long ppi = 256 / (a->C >> 3), mp = (a->hw + ppi - 1) / ppi;  // at most one pass of pixels per thread row
    const long sp = split < mp ? split : mp;
    hipLaunchKernelGGL(cg_ew_apply_cf_kernel<true>, dim3((unsigned)a->nimg, (unsigned)sp), dim3(256), 0, stream, *a);
    return DTF_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(cg_bn_relu_apply_kernel<false>, dim3((unsigned)a->nimg, (unsigned)split), dim3(256), 0, stream, *a);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_cg_prep_input(const float* x, bf16_t* y, long npix, int c_in, hipStream_t stream) {
  long blocks = (npix + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(cg_prep_input_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, x, y, npix, c_in);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_cg_prep_input_s2d(const float* x, bf16_t* y, int N, int H, int W, int c_in, hipStream_t stream) {
  if (N <= 0) return 0;
  if ((H & 1) || (W & 1) || c_in * 4 > 16) return -2;
  const long nblk = (long)N * (H / 2) * (W / 2);
  long blocks = (nblk + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(cg_prep_input_s2d_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, x, y, nblk, H, W, c_in);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_cg_maxpool(const bf16_t* x, bf16_t* y, uint8_t* am, const bf16_t* g, bf16_t* dx, int N, int H, int W,
                           int Ho, int Wo, int C, int backward, hipStream_t stream) {
  if (C % 8) return -2;
  const long total8 = (long)N * (backward ? H * W : Ho * Wo) * C / 8;
  if (total8 >= (1L << 31)) return -2;  // 32-bit element indices in the kernels
  long blocks = (total8 + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  if (backward && H == 2 * Ho && W == 2 * Wo) {  // 2 x 2 input blocks per thread
    const long tb8 = total8 / 4;
    long b2 = (tb8 + 255) / 256;
    if (b2 > 16384) b2 = 16384;
    hipLaunchKernelGGL(cg_maxpool_bwd2_kernel, dim3((unsigned)b2), dim3(256), 0, stream, g, am, dx, Ho, Wo, C, tb8);
  } else if (backward)
    hipLaunchKernelGGL(cg_maxpool_bwd_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, g, am, dx, H, W, Ho, Wo, C,
                       total8);
  else
    hipLaunchKernelGGL(cg_maxpool_fwd_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, x, y, am, H, W, Ho, Wo, C,
                       total8);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_cg_gap(const GapArgs* a, int which, int nimg, hipStream_t stream) {
  if (nimg <= 0) return 0;
  if (which == 0)
    hipLaunchKernelGGL(cg_gap_kernel, dim3(nimg), dim3(256), 0, stream, *a);
  else if (which == 1)
    hipLaunchKernelGGL(cg_gap_bwd_reduce_kernel, dim3(nimg), dim3(256), 0, stream, *a);
  else
    hipLaunchKernelGGL(cg_gap_bwd_apply_kernel, dim3(nimg), dim3(256), 0, stream, *a);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_cg_softmax_ce(const float* logits, int ld, int ncls, const int* labels, const int* img_slot,
                              const float* state, long s_mstride, int b_off, dtf_acc_t* grads, long g_mstride,
                              const float* cnt, dtf_acc_t* loss, float* correct, bf16_t* dl, long nimg,
                              float loss_scale, hipStream_t stream) {
  if (nimg <= 0) return 0;
  hipLaunchKernelGGL(cg_softmax_ce_kernel, dim3((unsigned)((nimg + 3) / 4)), dim3(256), 0, stream, logits, ld, ncls,
                     labels, img_slot, state, s_mstride, b_off, grads, g_mstride, cnt, loss, correct, dl, nimg,
                     loss_scale);
  return DTF_CHECK_LAUNCH();
}
