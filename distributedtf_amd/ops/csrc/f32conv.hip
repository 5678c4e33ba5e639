// fp32 population-batched CIFAR ResNet kernels (gfx950): the --dtype fp32 path (the reference's default dtype,
// resnet/official/utils/flags/_performance.py:30-33), accurate to fp32 rounding instead of bf16.
//
// Tensors are NHWC fp32 with the images of every member packed along N; weights are read straight from the fp32
// master state rows (OHWI at the conv's offset) -- no weight-prep pass, no bf16 shadow.  Matrix products run on
// v_mfma_f32_16x16x4_f32 (fp32 inputs, fp32 accumulation): A = 16 rows x 4 k (one float per lane: row lane % 16,
// k lane / 16), B = 4 k x 16 columns (k lane / 16, column lane % 16), D = 16 x 16 (lane holds rows
// 4 (lane / 16) + i, column lane % 16).
//
//  f32conv  : out[p][o] = sum_k A[k][o] * T(gathered)[p][k], forward (k = (tap, ci), any stride) or data gradient
//             (k = (tap, o) over dy; dx pixel (y, x) reads dy at ((y + P - ky) / S, (x + P - kx) / S) when
//             divisible -- the transposed convolution without a flipped weight copy).  T: identity | relu(x s + t)
//             | A dz + B h + C (BN backward).  Epilogue: [+ residual] [mask by BN(xm) + ReLU > 0] [per-channel
//             statistics: y, y^2 (forward) or dz, dz * xhat (with the mask)] -> fp32 sums [cap][2][cmax] that the
//             shared bn_final kernel (convg_aux.hip) turns into coefficients.
//  f32wgrad : dW[o][k] += sum_p T_dy(dy)[p][o] * T_x(gather(x))[p][k], split over pixel chunks, fp32 atomics into
//             the member's gradient row.
//  elementwise / head: BN-backward apply, ReLU(BN) apply, v1 block output and BN-backward sums, global average
//             pool (+ final BN + ReLU), dense + softmax CE, dense gradient (fixed-order per member), GAP backward.
#include "common.h"

namespace {

__device__ __forceinline__ f32x4_t mfma4(float a, float b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

struct F32Args {
  const float* x;     // gathered operand (fwd: input; dgrad: dy; wgrad: x)
  const float* x2;    // MODE 2: the BN input h of the gathered operand's BN-backward transform
  const float* dy;    // wgrad: output-side operand
  const float* dy2;   // wgrad: BN input of dy's BN-backward transform
  const float* w;     // fp32 master rows; OHWI weights at w_off
  long w_mstride, w_off;
  float* y;
  const float* res;   // residual added in the epilogue
  const float* xm;    // epilogue mask source
  float* grads;
  long g_mstride, g_off;
  const float* c_in;  // [cap][4][cmax] transform coefficients of the gathered operand
  const float* c_dy;  // wgrad: of dy
  const float* c_ep;  // epilogue mask BN (scale, shift, mean, inv)
  dtf_acc_t* st_out;  // [cap][2][cmax] statistics (atomics; int64 fixed point in the deterministic build)
  const int4* work;   // (slot, p0, p1, o0 [| n0 / 16 << 16 for wgrad])
  int Hi, Wi, Ci;     // gathered tensor (fwd: x, dgrad: dy)
  int Ho, Wo, Co;     // output tensor (wgrad: dy)
  int kh, kw, stride, pad;  // FORWARD conv geometry
  int cmax, log2ci;
  int wci;            // input channels of the weight row (the stem's 3; Ci is its 4-channel padded gather)
  int wrows;          // rows of the weight matrix present (0: all).  A dense layer run as a 1x1 conv with its
                      // class count padded (1001 -> 1024): forward output channels / data-gradient dy channels /
                      // weight-gradient rows past it read zero weights and write nothing
};

constexpr int F_BK = 16;  // k per LDS stage
// LDS row pitch (floats): the 4 row groups (lane / 16) of a fragment read land 16 banks apart
constexpr int f_pitch(int n) { return n == 16 ? 16 : (n == 32 ? 48 : n + 16); }
// conv tile: TC output channels x TP = 16 * 4 * NT pixels, NT = 64 / TC pixel tiles per wave -- every wave runs
// MT x NT = 4 MFMA tiles per k-step whatever the channel width (a C = 16 layer would otherwise get one)
constexpr int f_tp(int tc) { return 64 * (64 / tc); }

// ---- shared epilogue of the conv kernels: one lane's 4 output channels co .. co + 3 of pixel p (MFMA D layout):
// [+ residual] [mask by BN(xm) + ReLU > 0], fp32 store, per-channel statistics (y, y^2; with the mask dz, dz * xhat)
template <int EPI>
__device__ __forceinline__ void f32_epi4(const F32Args& a, int slot, long p, int co, bool ok, const f32x4_t& acc,
                                         float (&ss)[4], float (&sq)[4]) {
  const long o = p * a.Co + co;
  float v[4] = {acc[0], acc[1], acc[2], acc[3]};
  float xv[4] = {0.f, 0.f, 0.f, 0.f};
  if constexpr (EPI & 1) {
    if (ok) {
      const float4 r = *reinterpret_cast<const float4*>(a.res + o);
      v[0] += r.x, v[1] += r.y, v[2] += r.z, v[3] += r.w;
    }
  }
  const float* ep = (EPI & 2) ? a.c_ep + (long)slot * 4 * a.cmax + (ok ? co : 0) : nullptr;
  if constexpr (EPI & 2) {
    if (ok) {
      const float4 xr = *reinterpret_cast<const float4*>(a.xm + o);
      xv[0] = xr.x, xv[1] = xr.y, xv[2] = xr.z, xv[3] = xr.w;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = (xv[i] * ep[i] + ep[a.cmax + i] > 0.f) ? v[i] : 0.f;
  }
  if (ok) *reinterpret_cast<float4*>(a.y + o) = make_float4(v[0], v[1], v[2], v[3]);
  if constexpr (EPI & 4) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float vv = ok ? v[i] : 0.f;
      ss[i] += vv;
      if constexpr (EPI & 2)
        sq[i] += ok ? vv * (xv[i] - ep[2 * a.cmax + i]) * ep[3 * a.cmax + i] : 0.f;
      else
        sq[i] += vv * vv;
    }
  }
}

// Workgroup statistics: the 16 lanes of one lane / 16 group hold the same 4 channels -- butterfly, one LDS atomic
// per group and channel, one global atomic per workgroup and channel.  acc_lds [2][TC] zeroed before the k loop.
template <int TC, int FX, int MT>
__device__ __forceinline__ void f32_stats_flush(const F32Args& a, int slot, int o0, float (&ss)[MT][4],
                                                float (&sq)[MT][4], dtf_acc_t (&acc_lds)[2][TC]) {
  const int tid = threadIdx.x, lane = tid & 63;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float s_ = ss[m][i], q_ = sq[m][i];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        s_ += __shfl_xor(s_, o, 64);
        q_ += __shfl_xor(q_, o, 64);
      }
      if ((lane & 15) == 0) {
        dtf_acc_add(&acc_lds[0][16 * m + 4 * (lane >> 4) + i], s_, FX, slot);
        dtf_acc_add(&acc_lds[1][16 * m + 4 * (lane >> 4) + i], q_, FX, slot);
      }
    }
  __syncthreads();
  if (tid < TC && o0 + tid < a.Co) {
    dtf_acc_t* st = a.st_out + (long)slot * 2 * a.cmax;
    dtf_acc_addw(st + o0 + tid, acc_lds[0][tid]);
    dtf_acc_addw(st + a.cmax + o0 + tid, acc_lds[1][tid]);
  }
}

// ------------------------------------------------------------------------------------------------ fwd / dgrad
template <int TC, int MODE, int EPI, bool DGRAD>
__global__ __launch_bounds__(256) void f32conv_kernel(F32Args a) {
  constexpr int MT = TC / 16, NT = 64 / TC, TP = f_tp(TC);
  constexpr int PA = f_pitch(TC), PB = f_pitch(TP);
  constexpr int AE = TC * F_BK / 256;  // A elements per thread per stage
  __shared__ __attribute__((aligned(16))) float sA[2][F_BK * PA];
  __shared__ __attribute__((aligned(16))) float sB[2][F_BK * PB];
  __shared__ dtf_acc_t acc_lds[2][TC];
  extern __shared__ float dyn[];  // transform coefficients: MODE 1: 2 * Ci, MODE 2: 3 * Ci
  const int4 wk = a.work[blockIdx.x];
  DTF_WG_CHECK(wk.x >= 0 && wk.y >= 0 && wk.z >= wk.y && wk.z - wk.y <= TP);
  const int slot = wk.x, p0 = wk.y, p1 = wk.z, o0 = wk.w;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int Ci = a.Ci, kk = a.kh * a.kw;
  const int K = kk * Ci;
  if constexpr (MODE != 0) {
    const float* cb = a.c_in + (long)slot * 4 * a.cmax;
    for (int i = tid; i < Ci; i += 256) {
      dyn[i] = cb[i];
      dyn[Ci + i] = cb[a.cmax + i];
      if constexpr (MODE == 2) dyn[2 * Ci + i] = cb[2 * a.cmax + i];
    }
  }
  for (int i = tid; i < 2 * TC; i += 256) (&acc_lds[0][0])[i] = 0;
  // this thread's B rows (pixels rB + 64 j) and k chunk (4 consecutive k of one tap: Ci % 4 == 0)
  const int rB = tid >> 2, cB = tid & 3;
  const int HWo = a.Ho * a.Wo;
  int by[NT], bx[NT];
  long ibase[NT];
  bool okp[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int pB = p0 + rB + 64 * j;
    okp[j] = pB < p1;
    const int pp = okp[j] ? pB : p0;
    const int img = pp / HWo, rem = pp - img * HWo, oy = rem / a.Wo, ox = rem - oy * a.Wo;
    by[j] = DGRAD ? oy + a.pad : oy * a.stride - a.pad;
    bx[j] = DGRAD ? ox + a.pad : ox * a.stride - a.pad;
    ibase[j] = (long)img * a.Hi * a.Wi * Ci;
  }
  const float* wrow = a.w + (long)slot * a.w_mstride + a.w_off;
  float4 rb[NT], rb2[NT];
  unsigned okb;
  int cb_;
  auto load_b = [&](int k0) {
    const int k = k0 + 4 * cB;
    const int tap = k >> a.log2ci, ci = k & (Ci - 1);
    const int ky = a.kw == 1 ? tap : tap / a.kw, kx = tap - ky * a.kw;
    okb = 0;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      int iy, ix;
      bool ok;
      if constexpr (DGRAD) {
        const int ny = by[j] - ky, nx = bx[j] - kx;
        iy = ny / a.stride;
        ix = nx / a.stride;
        ok = ny >= 0 && nx >= 0 && iy * a.stride == ny && ix * a.stride == nx && iy < a.Hi && ix < a.Wi;
      } else {
        iy = by[j] + ky;
        ix = bx[j] + kx;
        ok = iy >= 0 && ix >= 0 && iy < a.Hi && ix < a.Wi;
      }
      ok = ok && okp[j] && k < K;
      const long off = ibase[j] + ((long)iy * a.Wi + ix) * Ci + ci;
      rb[j] = ok ? *reinterpret_cast<const float4*>(a.x + off) : make_float4(0.f, 0.f, 0.f, 0.f);
      if constexpr (MODE == 2)
        rb2[j] = ok ? *reinterpret_cast<const float4*>(a.x2 + off) : make_float4(0.f, 0.f, 0.f, 0.f);
      okb |= (unsigned)ok << j;
    }
    cb_ = ci;
  };
  auto store_b = [&](float* dst) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      float v[4] = {rb[j].x, rb[j].y, rb[j].z, rb[j].w};
      if constexpr (MODE != 0) {
        const float h[4] = {rb2[j].x, rb2[j].y, rb2[j].z, rb2[j].w};
        const bool ok = (okb >> j) & 1u;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int c = cb_ + q;
          float t;
          if constexpr (MODE == 1)
            t = fmaxf(v[q] * dyn[c] + dyn[Ci + c], 0.f);
          else
            t = dyn[c] * v[q] + dyn[Ci + c] * h[q] + dyn[2 * Ci + c];
          v[q] = ok ? t : 0.f;  // zero padding stays zero after the transform
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) dst[(4 * cB + q) * PB + rB + 64 * j] = v[q];
    }
  };
  float ra[AE];
  auto load_a = [&](int k0) {
#pragma unroll
    for (int j = 0; j < AE; ++j) {
      const int idx = tid + 256 * j;
      int m, kl;
      if constexpr (DGRAD) {  // A[k = (tap, o)][m = dx channel i] = W[o][tap][o0 + m]: contiguous in m
        m = idx % TC;
        kl = idx / TC;
      } else {                // A[k][m = o] = W[o0 + m][k]: contiguous in k
        m = idx / F_BK;
        kl = idx % F_BK;
      }
      const int k = k0 + kl;
      bool ok = k < K && o0 + m < a.Co;
      long off;
      const int tap = k >> a.log2ci, ci = k & (Ci - 1);
      if constexpr (DGRAD) {  // ci = dy channel o
        ok = ok && (a.wrows == 0 || ci < a.wrows);
        off = ((long)ci * kk + tap) * a.Co + o0 + m;
      } else {
        ok = ok && ci < a.wci && (a.wrows == 0 || o0 + m < a.wrows);
        off = ((long)(o0 + m) * kk + tap) * a.wci + ci;
      }
      ra[j] = ok ? wrow[off] : 0.f;
    }
  };
  auto store_a = [&](float* dst) {
#pragma unroll
    for (int j = 0; j < AE; ++j) {
      const int idx = tid + 256 * j;
      const int m = DGRAD ? idx % TC : idx / F_BK, kl = DGRAD ? idx / TC : idx % F_BK;
      dst[kl * PA + m] = ra[j];
    }
  };
  f32x4_t acc[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[m][n] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  __syncthreads();  // coefficients
  const int nk = (K + F_BK - 1) / F_BK;
  load_a(0);
  load_b(0);
  store_a(sA[0]);
  store_b(sB[0]);
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    const int cur = ks & 1;
    const bool more = ks + 1 < nk;
    if (more) {
      load_a(F_BK * (ks + 1));
      load_b(F_BK * (ks + 1));
    }
    const float* A = sA[cur];
    const float* B = sB[cur];
#pragma unroll
    for (int q = 0; q < F_BK / 4; ++q) {
      const int kr = 4 * q + (lane >> 4);
      float av[MT], bv[NT];
#pragma unroll
      for (int m = 0; m < MT; ++m) av[m] = A[kr * PA + 16 * m + (lane & 15)];
#pragma unroll
      for (int n = 0; n < NT; ++n) bv[n] = B[kr * PB + 16 * (wave * NT + n) + (lane & 15)];
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[m][n] = mfma4(av[m], bv[n], acc[m][n]);
    }
    if (more) {
      store_a(sA[cur ^ 1]);
      store_b(sB[cur ^ 1]);
    }
    __syncthreads();
  }
  // ---- epilogue: lane holds channels o0 + 16 m + 4 (lane / 16) + i of pixel p0 + 16 (wave NT + n) + lane % 16
  float ss[MT][4], sq[MT][4];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int i = 0; i < 4; ++i) ss[m][i] = sq[m][i] = 0.f;
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int p = p0 + 16 * (wave * NT + n) + (lane & 15);
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int co = o0 + 16 * m + 4 * (lane >> 4);
      f32_epi4<EPI>(a, slot, p, co, p < p1 && co < a.Co, acc[m][n], ss[m], sq[m]);
    }
  }
  // forward statistics (y, y^2) or, with the mask, BN-backward sums (dz, dz * xhat): fixed-point scales of the
  // deterministic build (common.h)
  if constexpr (EPI & 4) f32_stats_flush<TC, (EPI & 2) ? DTF_FX_GRAD : DTF_FX_STAT>(a, slot, o0, ss, sq, acc_lds);
}

// ------------------------------------------------------------------------------------------ band fwd / dgrad
// Forward or data gradient of a stride-1 3x3 conv with Ci = Co = C on W x W images from LDS-resident row bands: the
// workgroup stages its TCB output rows of the weights once ([tap][row][k], k contiguous; the data gradient's
// transposed operand W[o][t][i] -> [t][i][o] is transposed while staging), then per band of R output rows the
// gathered operand (x, or dy) with its zero halo, transform applied once; all 9 taps read B fragments from that tile
// at a (ky, kx) offset (data gradient: the flipped (2 - ky, 2 - kx) offset).  The gather kernel above re-reads the
// operand from memory per tap and per output-channel tile.
// Both operands are read as float4 along k: lane l takes k = base + 4 (l / 16) .. + 3, and MFMA q of the four uses
// element q -- the 4 MFMAs cover k = base .. base + 15 in a permuted order that A and B share.  Pitches C + 8
// (k rows of one pixel / one weight row) make those ds_read_b128 conflict-free (the W = 8 tile: 2-way).
// work: (slot, first band, end band, o0); band b = image b / (W / R), rows (b % (W / R)) R ..
template <int C, int W, int TCB, int MODE, int EPI, bool DGRAD>
__global__ __launch_bounds__(256) void f32conv_band_kernel(F32Args a) {
  constexpr int R = (128 / W < W) ? 128 / W : W;
  constexpr int BPI = W / R;
  constexpr int NPX = R * W;
  constexpr int XW = W + 2, XR = R + 2, XP = C + 8, WP = C + 8;
  constexpr int MT = TCB / 16, NT = NPX / 64;     // row tiles; 16-pixel tiles per wave
  constexpr int XCH = XR * XW * C / 4;
  constexpr int XQ = (XCH + 255) / 256;
  constexpr int SW = 9 * TCB * WP, SX = XR * XW * XP;
  static_assert(NPX % 64 == 0 && W % 4 == 0 && C % 16 == 0 && TCB % 16 == 0, "band geometry");
  __shared__ __attribute__((aligned(16))) float wL[SW];
  __shared__ __attribute__((aligned(16))) float xL[SX];
  __shared__ dtf_acc_t acc_lds[2][TCB];
  __shared__ float cf[3 * C];
  const int4 wk = a.work[blockIdx.x];
  DTF_WG_CHECK(wk.x >= 0 && wk.y >= 0 && wk.z >= wk.y && wk.w >= 0 && wk.w + TCB <= C);
  const int slot = wk.x, b0 = wk.y, b1 = wk.z, o0 = wk.w;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int j4 = lane >> 4, i16 = lane & 15;
  if constexpr (MODE != 0) {
    const float* cb = a.c_in + (long)slot * 4 * a.cmax;
    for (int i = tid; i < C; i += 256) {
      cf[i] = cb[i];
      cf[C + i] = cb[a.cmax + i];
      if constexpr (MODE == 2) cf[2 * C + i] = cb[2 * a.cmax + i];
    }
  }
  for (int i = tid; i < 2 * TCB; i += 256) (&acc_lds[0][0])[i] = 0;
  // ---- weights: wL[t][r][k] (r = output row o0 + r, k = reduction channel)
  const float* wrow = a.w + (long)slot * a.w_mstride + a.w_off;
  if constexpr (!DGRAD) {
    for (int q = tid; q < 9 * TCB * C / 4; q += 256) {  // (r, t, k4): global W[o0 + r][t][4 k4 ..] contiguous
      const int k4 = q % (C / 4), rt = q / (C / 4), t = rt % 9, r = rt / 9;
      const float4 v = *reinterpret_cast<const float4*>(wrow + ((long)(o0 + r) * 9 + t) * C + 4 * k4);
      *reinterpret_cast<float4*>(wL + (t * TCB + r) * WP + 4 * k4) = v;
    }
  } else {
    for (int q = tid; q < 9 * TCB * C; q += 256) {  // (o, t, r): global W[o][t][o0 + r], r fastest
      const int r = q % TCB, ot = q / TCB, t = ot % 9, o = ot / 9;
      wL[(t * TCB + r) * WP + o] = wrow[((long)o * 9 + t) * C + o0 + r];
    }
  }
  // ---- per-lane pixel of each of the wave's 16-pixel tiles (band-relative) and its halo-tile index
  int pxl[NT], xb[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    pxl[n] = 16 * (wave * NT + n) + i16;
    const int r = pxl[n] / W, c = pxl[n] - r * W;
    xb[n] = (r * XW + c) * XP + 4 * j4;
  }
  float4 rx[XQ], rx2[XQ];
  unsigned okx = 0;
  auto load = [&](int b) {
    const int img = b / BPI, y0 = (b - img * BPI) * R;
    okx = 0;
#pragma unroll
    for (int j = 0; j < XQ; ++j) {
      const int q = tid + 256 * j;
      const int pix = q / (C / 4), c4 = q - pix * (C / 4);
      const int r = pix / XW, c = pix - r * XW;
      const int iy = y0 - 1 + r, ix = c - 1;
      const bool ok = q < XCH && iy >= 0 && iy < W && ix >= 0 && ix < W;
      const long off = (((long)img * W + iy) * W + ix) * C + 4 * c4;
      rx[j] = ok ? *reinterpret_cast<const float4*>(a.x + off) : make_float4(0.f, 0.f, 0.f, 0.f);
      if constexpr (MODE == 2)
        rx2[j] = ok ? *reinterpret_cast<const float4*>(a.x2 + off) : make_float4(0.f, 0.f, 0.f, 0.f);
      okx |= (unsigned)ok << j;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int j = 0; j < XQ; ++j) {
      const int q = tid + 256 * j;
      if (q >= XCH) break;
      const int pix = q / (C / 4), c4 = q - pix * (C / 4);
      float v[4] = {rx[j].x, rx[j].y, rx[j].z, rx[j].w};
      if constexpr (MODE != 0) {
        const float h[4] = {rx2[j].x, rx2[j].y, rx2[j].z, rx2[j].w};
        const bool ok = (okx >> j) & 1u;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int ch = 4 * c4 + i;
          float t;
          if constexpr (MODE == 1)
            t = fmaxf(v[i] * cf[ch] + cf[C + ch], 0.f);
          else
            t = cf[ch] * v[i] + cf[C + ch] * h[i] + cf[2 * C + ch];
          v[i] = ok ? t : 0.f;  // the zero padding stays zero after the transform
        }
      }
      *reinterpret_cast<float4*>(xL + pix * XP + 4 * c4) = make_float4(v[0], v[1], v[2], v[3]);
    }
  };
  float ss[MT][4], sq[MT][4];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int i = 0; i < 4; ++i) ss[m][i] = sq[m][i] = 0.f;
  if (b0 < b1) load(b0);
  for (int b = b0; b < b1; ++b) {
    __syncthreads();  // (first band: weights / coefficients staged) the previous band's tile is consumed
    store();
    __syncthreads();
    if (b + 1 < b1) load(b + 1);  // the next band's loads stay in flight under this band's MFMAs
    f32x4_t acc[MT][NT];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int n = 0; n < NT; ++n) acc[m][n] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll 3
    for (int t = 0; t < 9; ++t) {
      const int ky = t / 3, kx = t - 3 * (t / 3);
      const int boff = DGRAD ? ((2 - ky) * XW + 2 - kx) * XP : (ky * XW + kx) * XP;
      const float* wt = wL + (t * TCB + i16) * WP + 4 * j4;
#pragma unroll
      for (int kc = 0; kc < C / 16; ++kc) {
        float4 av[MT], bv[NT];
#pragma unroll
        for (int m = 0; m < MT; ++m) av[m] = *reinterpret_cast<const float4*>(wt + 16 * m * WP + 16 * kc);
#pragma unroll
        for (int n = 0; n < NT; ++n) bv[n] = *reinterpret_cast<const float4*>(xL + xb[n] + boff + 16 * kc);
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
          for (int n = 0; n < NT; ++n) {
            acc[m][n] = mfma4(av[m].x, bv[n].x, acc[m][n]);
            acc[m][n] = mfma4(av[m].y, bv[n].y, acc[m][n]);
            acc[m][n] = mfma4(av[m].z, bv[n].z, acc[m][n]);
            acc[m][n] = mfma4(av[m].w, bv[n].w, acc[m][n]);
          }
      }
    }
    const int img = b / BPI, y0 = (b - img * BPI) * R;
    const long pbase = ((long)img * W + y0) * W;
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int m = 0; m < MT; ++m)
        f32_epi4<EPI>(a, slot, pbase + pxl[n], o0 + 16 * m + 4 * j4, true, acc[m][n], ss[m], sq[m]);
  }
  if constexpr (EPI & 4) f32_stats_flush<TCB, (EPI & 2) ? DTF_FX_GRAD : DTF_FX_STAT>(a, slot, o0, ss, sq, acc_lds);
}

// ------------------------------------------------------------------------------------------------------ wgrad
// work: (slot, p0, p1, o0 | (n0 / 16) << 16); rows o0 .. o0 + TC of dW, columns n0 .. n0 + 64 of K; pixels p0..p1 of
// the OUTPUT grid (dy), BP per stage.  Each wave owns 16 columns and every row tile: BP / 4 x MT MFMAs per stage.
constexpr int W_BP = 32;
template <int TC, int MODE_X, int MODE_DY>
__global__ __launch_bounds__(256) void f32wgrad_kernel(F32Args a) {
  constexpr int MT = TC / 16, TN = 64, BP = W_BP;
  constexpr int PA = f_pitch(TC), PB = f_pitch(TN);
  constexpr int DCH = BP * TC / 4;               // dy float4 chunks per stage
  constexpr int DQ = (DCH + 255) / 256;          // ... per thread
  constexpr int XQ = BP * TN / 1024;   // x float4 chunks per thread per stage
  __shared__ __attribute__((aligned(16))) float sA[2][BP * PA];  // [pixel][o]
  __shared__ __attribute__((aligned(16))) float sB[2][BP * PB];  // [pixel][k]
  extern __shared__ float dyn[];  // x coefficients (2 Ci) | dy coefficients (3 Co)
  const int4 wk = a.work[blockIdx.x];
  DTF_WG_CHECK(wk.x >= 0 && wk.y >= 0 && wk.z >= wk.y);
  const int slot = wk.x, p0 = wk.y, p1 = wk.z, o0 = wk.w & 0xffff, n0 = (wk.w >> 16) * 16;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int Ci = a.Ci, K = a.kh * a.kw * Ci;
  float* cx = dyn;
  float* cd = dyn + 2 * Ci;
  if constexpr (MODE_X != 0) {
    const float* cb = a.c_in + (long)slot * 4 * a.cmax;
    for (int i = tid; i < Ci; i += 256) {
      cx[i] = cb[i];
      cx[Ci + i] = cb[a.cmax + i];
    }
  }
  if constexpr (MODE_DY != 0) {
    const float* cb = a.c_dy + (long)slot * 4 * a.cmax;
    for (int i = tid; i < a.Co; i += 256) {
      cd[i] = cb[i];
      cd[a.Co + i] = cb[a.cmax + i];
      cd[2 * a.Co + i] = cb[2 * a.cmax + i];
    }
  }
  const int HWo = a.Ho * a.Wo;
  // dy chunk q = tid + 256 j: pixel q / (TC / 4), channels o0 + 4 (q % (TC / 4)) ..
  // x chunk q = tid + 256 j: pixel q / 16, columns n0 + 4 (tid % 16) .. (the same columns for every j)
  const int kX = n0 + 4 * (tid & 15);
  const int tapX = kX >> a.log2ci, ciX = kX & (Ci - 1);
  const int kyX = a.kw == 1 ? tapX : tapX / a.kw, kxX = tapX - kyX * a.kw;
  const bool kok = kX < K;
  float4 rd[DQ], rd2[DQ], rx[XQ];
  unsigned okd, okx;
  auto load = [&](int s0) {
    okd = 0;
#pragma unroll
    for (int j = 0; j < DQ; ++j) {
      const int q = tid + 256 * j;
      const int p = s0 + q / (TC / 4), oc = o0 + 4 * (q % (TC / 4));
      const bool ok = q < DCH && p < p1 && oc < a.Co;
      const long o = (long)p * a.Co + oc;
      rd[j] = ok ? *reinterpret_cast<const float4*>(a.dy + o) : make_float4(0.f, 0.f, 0.f, 0.f);
      if constexpr (MODE_DY == 2)
        rd2[j] = ok ? *reinterpret_cast<const float4*>(a.dy2 + o) : make_float4(0.f, 0.f, 0.f, 0.f);
      okd |= (unsigned)ok << j;
    }
    okx = 0;
#pragma unroll
    for (int j = 0; j < XQ; ++j) {
      const int px = s0 + (tid >> 4) + 16 * j;
      const int pp = px < p1 ? px : p0;
      const int img = pp / HWo, rem = pp - img * HWo, oy = rem / a.Wo, ox = rem - oy * a.Wo;
      const int iy = oy * a.stride - a.pad + kyX, ix = ox * a.stride - a.pad + kxX;
      const bool ok = px < p1 && kok && iy >= 0 && ix >= 0 && iy < a.Hi && ix < a.Wi;
      const long xo = (((long)img * a.Hi + iy) * a.Wi + ix) * Ci + ciX;
      rx[j] = ok ? *reinterpret_cast<const float4*>(a.x + xo) : make_float4(0.f, 0.f, 0.f, 0.f);
      okx |= (unsigned)ok << j;
    }
  };
  auto store = [&](float* A, float* B) {
#pragma unroll
    for (int j = 0; j < DQ; ++j) {
      const int q = tid + 256 * j;
      if (q >= DCH) break;
      const int pr = q / (TC / 4), oc = 4 * (q % (TC / 4));
      float v[4] = {rd[j].x, rd[j].y, rd[j].z, rd[j].w};
      if constexpr (MODE_DY == 2) {
        const float h[4] = {rd2[j].x, rd2[j].y, rd2[j].z, rd2[j].w};
        const bool ok = (okd >> j) & 1u;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = o0 + oc + i;
          v[i] = ok ? cd[c] * v[i] + cd[a.Co + c] * h[i] + cd[2 * a.Co + c] : 0.f;
        }
      }
      *reinterpret_cast<float4*>(A + pr * PA + oc) = make_float4(v[0], v[1], v[2], v[3]);
    }
#pragma unroll
    for (int j = 0; j < XQ; ++j) {
      float v[4] = {rx[j].x, rx[j].y, rx[j].z, rx[j].w};
      if constexpr (MODE_X == 1) {
        const bool ok = (okx >> j) & 1u;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = ok ? fmaxf(v[i] * cx[ciX + i] + cx[Ci + ciX + i], 0.f) : 0.f;
      }
      *reinterpret_cast<float4*>(B + ((tid >> 4) + 16 * j) * PB + 4 * (tid & 15)) = make_float4(v[0], v[1], v[2],
                                                                                               v[3]);
    }
  };
  f32x4_t acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  __syncthreads();  // coefficients
  const int ns = (p1 - p0 + BP - 1) / BP;
  load(p0);
  store(sA[0], sB[0]);
  __syncthreads();
  for (int s = 0; s < ns; ++s) {
    const int cur = s & 1;
    const bool more = s + 1 < ns;
    if (more) load(p0 + BP * (s + 1));
    const float* A = sA[cur];
    const float* B = sB[cur];
#pragma unroll
    for (int q = 0; q < BP / 4; ++q) {
      const int pr = 4 * q + (lane >> 4);
      const float bv = B[pr * PB + 16 * wave + (lane & 15)];
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[m] = mfma4(A[pr * PA + 16 * m + (lane & 15)], bv, acc[m]);
    }
    if (more) store(sA[cur ^ 1], sB[cur ^ 1]);
    __syncthreads();
  }
  const int kcol = n0 + 16 * wave + (lane & 15);
  const int tapc = kcol >> a.log2ci, cic = kcol & (Ci - 1);
  if (kcol < K && cic < a.wci) {  // the stem's padded 4th channel has no weight
    dtf_acc_t* g = reinterpret_cast<dtf_acc_t*>(a.grads) + (long)slot * a.g_mstride + a.g_off;
    const long Kw = (long)a.kh * a.kw * a.wci;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int o = o0 + 16 * m + 4 * (lane >> 4) + i;
        if (o < a.Co && (a.wrows == 0 || o < a.wrows))
          dtf_acc_add(g + (long)o * Kw + (long)tapc * a.wci + cic, acc[m][i], DTF_FX_GRAD, slot);
      }
  }
}

// --------------------------------------------------------------------------------------------- band wgrad
// Weight gradient of the stride-1 3x3 convs with Ci = Co = C (every CIFAR ResNet conv but the stem and the stride-2
// / projection convs) from LDS-resident row bands: a band of R output rows of one image stages dy (all C channels,
// BN-backward transform applied once) and x (one 16-channel tile `ct`, R + 2 rows x W + 2 columns with the zero
// halo, ReLU(BN) applied once), and all 9 taps read their B fragments from the same x tile at a (ky, kx) offset.
// The gather kernel above re-reads x from memory once per tap and per 64-column tile (9-27x the bytes) and
// re-applies the transforms per read.
// MFMA: A = dy^T (16 o x 4 pixels), B = x (4 pixels x 16 ci of tap t), acc[m][t] = dW[16 m .. +16][t][16 ct .. +16].
// The 4 waves split each band's 4-pixel groups and are summed through LDS at the end; then one fp32 atomic per
// weight and workgroup.  work: (slot, first band, end band, ct); band b = image b / (W / R), rows (b % (W / R)) R ..
template <int C, int W, int MODE_X, int MODE_DY>
__global__ __launch_bounds__(256) void f32wgrad_band_kernel(F32Args a) {
  constexpr int R = (128 / W < W) ? 128 / W : W;  // output rows per band: W 32 -> 4, 16 -> 8, 8 -> 8
  constexpr int BPI = W / R;                      // bands per image
  constexpr int NPX = R * W;                      // output pixels per band
  constexpr int XW = W + 2, XR = R + 2;
  constexpr int XCH = XR * XW * 4;                // x float4 chunks per band (16 channels)
  constexpr int XQ = (XCH + 255) / 256;
  constexpr int DP = f_pitch(C);                  // dy pixel pitch (floats): A-fragment reads conflict-free
  constexpr int DCH = NPX * C / 4;
  constexpr int DQ = (DCH + 255) / 256;
  constexpr int MT = C / 16;
  constexpr int GPW = NPX / 16;                   // 4-pixel groups per wave and band
  constexpr int SX = XR * XW * 16, SD = NPX * DP, SRED = MT * 9 * 256;
  constexpr int SM = (SX + SD > SRED) ? SX + SD : SRED;
  static_assert(NPX % 16 == 0 && W % 4 == 0, "band geometry");
  __shared__ __attribute__((aligned(16))) float smem[SM];
  __shared__ float cx[32];
  __shared__ float cd[3 * C];
  float* xL = smem;
  float* dL = smem + SX;
  const int4 wk = a.work[blockIdx.x];
  DTF_WG_CHECK(wk.x >= 0 && wk.y >= 0 && wk.z >= wk.y && wk.w >= 0 && wk.w < MT);
  const int slot = wk.x, b0 = wk.y, b1 = wk.z, ct = wk.w;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  if constexpr (MODE_X != 0) {
    const float* cb = a.c_in + (long)slot * 4 * a.cmax + 16 * ct;
    if (tid < 16) {
      cx[tid] = cb[tid];
      cx[16 + tid] = cb[a.cmax + tid];
    }
  }
  if constexpr (MODE_DY != 0) {
    const float* cb = a.c_dy + (long)slot * 4 * a.cmax;
    for (int i = tid; i < C; i += 256) {
      cd[i] = cb[i];
      cd[C + i] = cb[a.cmax + i];
      cd[2 * C + i] = cb[2 * a.cmax + i];
    }
  }
  float4 rx[XQ], rd[DQ], rd2[DQ];
  unsigned okx = 0;
  auto load = [&](int b) {
    const int img = b / BPI, y0 = (b - img * BPI) * R;
    okx = 0;
#pragma unroll
    for (int j = 0; j < XQ; ++j) {
      const int q = tid + 256 * j;
      const int pix = q >> 2, c4 = q & 3;
      const int r = pix / XW, c = pix - r * XW;
      const int iy = y0 - 1 + r, ix = c - 1;
      const bool ok = q < XCH && iy >= 0 && iy < W && ix >= 0 && ix < W;
      const long off = (((long)img * W + iy) * W + ix) * C + 16 * ct + 4 * c4;
      rx[j] = ok ? *reinterpret_cast<const float4*>(a.x + off) : make_float4(0.f, 0.f, 0.f, 0.f);
      okx |= (unsigned)ok << j;
    }
    const long dbase = ((long)img * W + y0) * W * C;  // the band's rows are contiguous in NHWC
#pragma unroll
    for (int j = 0; j < DQ; ++j) {
      const int q = tid + 256 * j;
      const bool ok = q < DCH;
      const long off = dbase + 4L * (ok ? q : 0);
      rd[j] = ok ? *reinterpret_cast<const float4*>(a.dy + off) : make_float4(0.f, 0.f, 0.f, 0.f);
      if constexpr (MODE_DY == 2)
        rd2[j] = ok ? *reinterpret_cast<const float4*>(a.dy2 + off) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int j = 0; j < XQ; ++j) {
      const int q = tid + 256 * j;
      if (q >= XCH) break;
      const int pix = q >> 2, c4 = q & 3;
      float v[4] = {rx[j].x, rx[j].y, rx[j].z, rx[j].w};
      if constexpr (MODE_X == 1) {
        const bool ok = (okx >> j) & 1u;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = ok ? fmaxf(v[i] * cx[4 * c4 + i] + cx[16 + 4 * c4 + i], 0.f) : 0.f;
      }
      *reinterpret_cast<float4*>(xL + pix * 16 + 4 * c4) = make_float4(v[0], v[1], v[2], v[3]);
    }
#pragma unroll
    for (int j = 0; j < DQ; ++j) {
      const int q = tid + 256 * j;
      if (q >= DCH) break;
      const int pix = q / (C / 4), oc = 4 * (q % (C / 4));
      float v[4] = {rd[j].x, rd[j].y, rd[j].z, rd[j].w};
      if constexpr (MODE_DY == 2) {
        const float h[4] = {rd2[j].x, rd2[j].y, rd2[j].z, rd2[j].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = cd[oc + i] * v[i] + cd[C + oc + i] * h[i] + cd[2 * C + oc + i];
      }
      *reinterpret_cast<float4*>(dL + pix * DP + oc) = make_float4(v[0], v[1], v[2], v[3]);
    }
  };
  f32x4_t acc[MT][9];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[m][t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  const int j4 = lane >> 4, i16 = lane & 15;
  __syncthreads();  // coefficients
  if (b0 < b1) load(b0);
  for (int b = b0; b < b1; ++b) {
    store();
    __syncthreads();
    if (b + 1 < b1) load(b + 1);  // next band's loads in flight under this band's MFMAs
#pragma unroll 2
    for (int gi = 0; gi < GPW; ++gi) {
      const int pb = 4 * (wave * GPW + gi);  // first pixel of the group (one output row: W % 4 == 0)
      const int row = pb / W, col = pb - row * W;
      float av[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) av[m] = dL[(pb + j4) * DP + 16 * m + i16];
      const float* xb = xL + (row * XW + col + j4) * 16 + i16;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const float bv = xb[((t / 3) * XW + t % 3) * 16];
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[m][t] = mfma4(av[m], bv, acc[m][t]);
      }
    }
    __syncthreads();
  }
  // ---- sum the 4 waves' partials through LDS (the band buffers are free), then one atomic per weight
  float* red = smem;
  for (int w = 1; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) red[((m * 9 + t) * 4 + r) * 64 + lane] = acc[m][t][r];
    }
    __syncthreads();
    if (wave == 0) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[m][t][r] += red[((m * 9 + t) * 4 + r) * 64 + lane];
    }
    __syncthreads();
  }
  if (wave == 0) {
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[((m * 9 + t) * 4 + r) * 64 + lane] = acc[m][t][r];
  }
  __syncthreads();
  dtf_acc_t* g = reinterpret_cast<dtf_acc_t*>(a.grads) + (long)slot * a.g_mstride + a.g_off;
  for (int idx = tid; idx < SRED; idx += 256) {
    const int l = idx & 63, r = (idx >> 6) & 3, mt = idx >> 8;
    const int m = mt / 9, t = mt - m * 9;
    const int o = 16 * m + 4 * (l >> 4) + r, ci = 16 * ct + (l & 15);
    dtf_acc_add(g + (long)o * 9 * C + t * C + ci, red[idx], DTF_FX_GRAD, slot);
  }
}

// ------------------------------------------------------------------------------------------------ elementwise
struct F32Ew {
  const float* dz;
  const float* h;
  const float* add;    // bwd apply: added; add_relu: the shortcut
  float* out;
  const float* coef;   // [cap][4][cmax]
  const float* coef2;  // add_relu: shortcut BN (null: identity shortcut)
  const int* img_slot;
  long hw;
  int C, cmax;
  long nimg;
};

// which: 0 out = A dz + B h + C (+ add); 1 out = relu(h s + t); 2 out = relu(BN(h) + BN2(add) | add)
template <int WHICH>
__global__ __launch_bounds__(256) void f32_ew_kernel(F32Ew a) {
  const long n4 = a.nimg * a.hw * a.C / 4;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    const long e = 4 * i;
    const long img = e / (a.hw * a.C);
    const int c0 = (int)(e % a.C);
    const int slot = a.img_slot[img];
    const float* co = a.coef + (long)slot * 4 * a.cmax + c0;
    const float4 hv = *reinterpret_cast<const float4*>(a.h + e);
    const float h[4] = {hv.x, hv.y, hv.z, hv.w};
    float r[4];
    if constexpr (WHICH == 0) {
      const float4 dv = *reinterpret_cast<const float4*>(a.dz + e);
      const float d[4] = {dv.x, dv.y, dv.z, dv.w};
      float4 av = make_float4(0.f, 0.f, 0.f, 0.f);
      if (a.add) av = *reinterpret_cast<const float4*>(a.add + e);
      const float ad[4] = {av.x, av.y, av.z, av.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) r[j] = co[j] * d[j] + co[a.cmax + j] * h[j] + co[2 * a.cmax + j] + ad[j];
    } else if constexpr (WHICH == 1) {
#pragma unroll
      for (int j = 0; j < 4; ++j) r[j] = fmaxf(h[j] * co[j] + co[a.cmax + j], 0.f);
    } else {
      const float4 sv = *reinterpret_cast<const float4*>(a.add + e);
      const float s[4] = {sv.x, sv.y, sv.z, sv.w};
      const float* c2 = a.coef2 ? a.coef2 + (long)slot * 4 * a.cmax + c0 : nullptr;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        r[j] = fmaxf(h[j] * co[j] + co[a.cmax + j] + (c2 ? s[j] * c2[j] + c2[a.cmax + j] : s[j]), 0.f);
    }
    *reinterpret_cast<float4*>(a.out + e) = make_float4(r[0], r[1], r[2], r[3]);
  }
}

// v1 BN-backward sums of a post-activation BN (dz already ReLU-masked): sum dz, sum dz * xhat of h [and of h2 for
// a second BN fed the same dz].  One workgroup per image, thread = channel (C <= 256), LDS-free.
struct F32Sum {
  const float* dz;
  const float* h;
  const float* h2;
  const float* fc;
  const float* fc2;
  dtf_acc_t* sums;
  dtf_acc_t* sums2;
  const int* img_slot;
  int hw, C, cmax, pad;
};

__device__ __forceinline__ void kahan_add(float& s, float& c, float v) {
  const float y = v - c;
  const float t = s + y;
  c = (t - s) - y;
  s = t;
}

// One workgroup per image: thread (channel c, part) sums the pixels part, part + P, .. (P = 256 / C parts) with
// compensated (Kahan) accumulation, then the parts combine in LDS: a long serial fp32 sum over the image's pixels
// loses ~1e-3 of these cancellation-heavy BN-backward sums.
// C > 256 (the bottleneck nets): blockIdx.y = group of 256 channels, one part.  pad = 1: forward statistics (sum x,
// sum x^2 with dz = h and identity coefficients) at the statistics fixed-point scale (a tensor no conv produced).
__global__ __launch_bounds__(256) void f32_bwd_sums_kernel(F32Sum a) {
  __shared__ float red[3][256];
  const int img = blockIdx.x, slot = a.img_slot[img];
  const int Cg = a.C < 256 ? a.C : 256;
  const int P = 256 / Cg;
  const int c = blockIdx.y * Cg + threadIdx.x % Cg, part = threadIdx.x / Cg;
  const int cl = threadIdx.x % Cg;  // this thread's channel within the group (LDS column)
  const float* f1 = a.fc + (long)slot * 4 * a.cmax;
  const float mu = f1[2 * a.cmax + c], iv = f1[3 * a.cmax + c];
  float mu2 = 0.f, iv2 = 0.f;
  if (a.h2) {
    const float* f2 = a.fc2 + (long)slot * 4 * a.cmax;
    mu2 = f2[2 * a.cmax + c];
    iv2 = f2[3 * a.cmax + c];
  }
  float s = 0.f, q = 0.f, q2 = 0.f, cs = 0.f, cq = 0.f, cq2 = 0.f;
  const long base = (long)img * a.hw * a.C + c;
  if (part < P) {
    for (int p = part; p < a.hw; p += P) {
      const float d = a.dz[base + (long)p * a.C];
      kahan_add(s, cs, d);
      kahan_add(q, cq, d * (a.h[base + (long)p * a.C] - mu) * iv);
      if (a.h2) kahan_add(q2, cq2, d * (a.h2[base + (long)p * a.C] - mu2) * iv2);
    }
  }
  red[0][threadIdx.x] = s;
  red[1][threadIdx.x] = q;
  red[2][threadIdx.x] = q2;
  __syncthreads();
  for (int w = P / 2; w >= 1; w >>= 1) {  // pairwise over the parts (P is a power of two)
    if (part < w) {
      red[0][threadIdx.x] += red[0][threadIdx.x + w * Cg];
      red[1][threadIdx.x] += red[1][threadIdx.x + w * Cg];
      red[2][threadIdx.x] += red[2][threadIdx.x + w * Cg];
    }
    __syncthreads();
  }
  if (part != 0) return;
  dtf_acc_t* su = a.sums + (long)slot * 2 * a.cmax;
  if (a.pad == 1) {
    dtf_acc_add(su + c, red[0][cl], DTF_FX_STAT, slot);
    dtf_acc_add(su + a.cmax + c, red[1][cl], DTF_FX_STAT, slot);
    return;
  }
  dtf_acc_add(su + c, red[0][cl], DTF_FX_GRAD, slot);
  dtf_acc_add(su + a.cmax + c, red[1][cl], DTF_FX_GRAD, slot);
  if (a.h2) {
    dtf_acc_t* s2 = a.sums2 + (long)slot * 2 * a.cmax;
    dtf_acc_add(s2 + c, red[0][cl], DTF_FX_GRAD, slot);
    dtf_acc_add(s2 + a.cmax + c, red[2][cl], DTF_FX_GRAD, slot);
  }
}

// ------------------------------------------------------------------------------------------------------- head
struct F32Head {
  const float* x;       // [N][hw][C] last block output
  const float* coef;    // final BN forward coefficients (v2) or null (v1: x is already a ReLU output)
  const int* img_slot;
  const int* labels;
  const float* state;   // master rows: dense W [ncls][C] at w_off, bias at b_off
  long s_mstride;
  int w_off, b_off;
  float* feat;          // [N][C]
  float* dlog;          // [N][ncls]
  float* dfeat;         // [N][C]
  const float* cnt;     // images per member
  dtf_acc_t* loss;      // summed mean CE (int64 fixed point in the deterministic build: cg_det_finish converts)
  float* correct;
  dtf_acc_t* sums;      // final-BN backward sums [cap][2][cmax]
  const float* bcoef;   // final-BN backward coefficients
  float* gout;          // gradient at x
  int hw, C, ncls, cmax;
  int train, pad;
};

// one workgroup per image: feat = mean_p T(x); logits = W feat + b; softmax CE -> loss / correct (/ member batch),
// dlogits, dfeat = W^T dlogits (train)
__global__ __launch_bounds__(256) void f32_head_kernel(F32Head a) {
  __shared__ float f[256];
  __shared__ float lg[64];
  const int img = blockIdx.x, slot = a.img_slot[img];
  const int t = threadIdx.x;
  if (t < a.C) {
    const float* co = a.coef ? a.coef + (long)slot * 4 * a.cmax : nullptr;
    float s = 0.f;
    for (int p = 0; p < a.hw; ++p) {
      float v = a.x[((long)img * a.hw + p) * a.C + t];
      if (co) v = fmaxf(v * co[t] + co[a.cmax + t], 0.f);
      s += v;
    }
    f[t] = s / (float)a.hw;
    a.feat[(long)img * a.C + t] = f[t];
  }
  __syncthreads();
  const float* row = a.state + (long)slot * a.s_mstride;
  if (t < a.ncls) {
    float z = row[a.b_off + t];
    for (int c = 0; c < a.C; ++c) z += row[a.w_off + t * a.C + c] * f[c];
    lg[t] = z;
  }
  __syncthreads();
  if (t == 0) {
    float mx = lg[0];
    int arg = 0;
    for (int j = 1; j < a.ncls; ++j)
      if (lg[j] > mx) mx = lg[j], arg = j;
    float se = 0.f;
    for (int j = 0; j < a.ncls; ++j) se += expf(lg[j] - mx);
    const float lse = mx + logf(se);
    const int lab = a.labels[img];
    const float bsz = a.cnt[slot];
    dtf_acc_add(a.loss + slot, (lse - lg[lab]) / bsz, DTF_FX_GRAD, slot);
    atomicAdd(a.correct + slot, arg == lab ? 1.f : 0.f);
    for (int j = 0; j < a.ncls; ++j) lg[j] = (expf(lg[j] - lse) - (j == lab ? 1.f : 0.f)) / bsz;
  }
  __syncthreads();
  if (!a.train) return;
  if (t < a.ncls) a.dlog[(long)img * a.ncls + t] = lg[t];
  if (t < a.C) {
    float d = 0.f;
    for (int j = 0; j < a.ncls; ++j) d += row[a.w_off + j * a.C + t] * lg[j];
    a.dfeat[(long)img * a.C + t] = d;
  }
}

// dense gradient, fixed summation order: workgroup = (member, 256 elements of [ncls][C] + ncls bias)
__global__ __launch_bounds__(256) void f32_dense_grad_kernel(F32Head a, const int* slots, const int* first,
                                                             float* grads, long g_mstride) {
  const int m = blockIdx.y, slot = slots[m], i0 = first[m];
  const int n = (int)a.cnt[slot];
  const int e = blockIdx.x * 256 + threadIdx.x;
  const int nw = a.ncls * a.C;
  if (e >= nw + a.ncls) return;
  float s = 0.f;
  if (e < nw) {
    const int j = e / a.C, c = e - j * a.C;
    for (int i = i0; i < i0 + n; ++i) s += a.dlog[(long)i * a.ncls + j] * a.feat[(long)i * a.C + c];
    grads[(long)slot * g_mstride + a.w_off + e] += s;
  } else {
    const int j = e - nw;
    for (int i = i0; i < i0 + n; ++i) s += a.dlog[(long)i * a.ncls + j];
    grads[(long)slot * g_mstride + a.b_off + j] += s;
  }
}

// GAP backward: which 0 -> final-BN backward sums (dz = dfeat / hw masked by BN(x) + ReLU > 0); which 1 -> gradient
// at x: A dz + B x + C (v2) or dfeat / hw masked by x > 0 (v1: coef null)
template <int WHICH>
__global__ __launch_bounds__(256) void f32_gap_bwd_kernel(F32Head a) {
  const int img = blockIdx.x, slot = a.img_slot[img];
  const float* co = a.coef ? a.coef + (long)slot * 4 * a.cmax : nullptr;
  const float inv_hw = 1.f / (float)a.hw;
  if constexpr (WHICH == 0) {
    const int c = threadIdx.x;
    if (c >= a.C) return;
    const float g = a.dfeat[(long)img * a.C + c] * inv_hw;
    const float sc = co[c], sh = co[a.cmax + c], mu = co[2 * a.cmax + c], iv = co[3 * a.cmax + c];
    float s = 0.f, q = 0.f;
    for (int p = 0; p < a.hw; ++p) {
      const float xv = a.x[((long)img * a.hw + p) * a.C + c];
      if (xv * sc + sh > 0.f) {
        s += g;
        q += g * (xv - mu) * iv;
      }
    }
    dtf_acc_t* su = a.sums + (long)slot * 2 * a.cmax;
    dtf_acc_add(su + c, s, DTF_FX_GRAD, slot);
    dtf_acc_add(su + a.cmax + c, q, DTF_FX_GRAD, slot);
  } else {
    const float* bc = a.bcoef ? a.bcoef + (long)slot * 4 * a.cmax : nullptr;
    const long n = (long)a.hw * a.C;
    for (long i = threadIdx.x; i < n; i += blockDim.x) {
      const int c = (int)(i % a.C);
      const long o = (long)img * n + i;
      const float xv = a.x[o];
      const float g = a.dfeat[(long)img * a.C + c] * inv_hw;
      float r;
      if (co) {
        const float dz = (xv * co[c] + co[a.cmax + c] > 0.f) ? g : 0.f;
        r = bc[c] * dz + bc[a.cmax + c] * xv + bc[2 * a.cmax + c];
      } else {
        r = xv > 0.f ? g : 0.f;
      }
      a.gout[o] = r;
    }
  }
}

// [N][hw][3] fp32 -> [N][hw][4] (channel 3 zero: the stem gathers 4-channel chunks)
__global__ __launch_bounds__(256) void f32_prep_input_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                             long npix) {
  for (long p = (long)blockIdx.x * 256 + threadIdx.x; p < npix; p += (long)gridDim.x * 256)
    *reinterpret_cast<float4*>(y + 4 * p) = make_float4(x[3 * p], x[3 * p + 1], x[3 * p + 2], 0.f);
}

}  // namespace

DTF_API int dtf_f32_args_size() { return (int)sizeof(F32Args); }
DTF_API int dtf_f32_ew_size() { return (int)sizeof(F32Ew); }
DTF_API int dtf_f32_sum_size() { return (int)sizeof(F32Sum); }
DTF_API int dtf_f32_head_size() { return (int)sizeof(F32Head); }

// conv / data gradient: tc (16 | 32 | 64), mode (0 | 1 | 2), epi (bits: 1 residual, 2 mask, 4 statistics)
DTF_API int dtf_f32_conv(const F32Args* a, int tc, int mode, int epi, int dgrad, int nwork, hipStream_t stream) {
  if (nwork <= 0) return 0;
  if ((a->Ci & (a->Ci - 1)) != 0 || a->Ci < 4 || (a->Co & 3) != 0 || (1 << a->log2ci) != a->Ci) return -2;
  DTF_HOST_CHECK(DTF_ALIGNED16(a->x) && DTF_ALIGNED16(a->y));
  const size_t dyn = (size_t)(mode == 0 ? 0 : (mode == 1 ? 2 : 3)) * a->Ci * sizeof(float);
#define F_CASE(TC_, M_, E_, D_)                                                                          \
  if (tc == TC_ && mode == M_ && epi == E_ && dgrad == D_) {                                             \
    hipLaunchKernelGGL((f32conv_kernel<TC_, M_, E_, D_>), dim3(nwork), dim3(256), dyn, stream, *a);      \
    return DTF_CHECK_LAUNCH();                                                                           \
  }
#define F_TCS(M_, E_, D_) F_CASE(16, M_, E_, D_) F_CASE(32, M_, E_, D_) F_CASE(64, M_, E_, D_)
  // forward: stem / v1 (identity), v2 BN+ReLU prologue; statistics; + residual
  F_TCS(0, 4, false) F_TCS(0, 0, false) F_TCS(1, 4, false) F_TCS(1, 0, false) F_TCS(1, 5, false)
  F_TCS(0, 5, false)  // bottleneck v2 conv3 (materialised BN+ReLU input) + shortcut (engine/hip_imagenet_f32.py)
  // data gradient: mask + statistics [+ residual], plain, residual + mask (v1)
  F_TCS(0, 6, true) F_TCS(0, 7, true) F_TCS(0, 0, true) F_TCS(2, 3, true) F_TCS(2, 6, true) F_TCS(2, 7, true)
  F_TCS(2, 0, true) F_TCS(0, 3, true)
#undef F_TCS
#undef F_CASE
  return -1;
}

DTF_API int dtf_f32_wgrad(const F32Args* a, int tc, int mode_x, int mode_dy, int nwork, hipStream_t stream) {
  if (nwork <= 0) return 0;
  if ((a->Ci & (a->Ci - 1)) != 0 || a->Ci < 4 || (a->Co % tc) != 0 || (1 << a->log2ci) != a->Ci) return -2;
  // coefficient LDS only for the transforms that run (dy's start at 2 Ci either way)
  const size_t dyn = (size_t)(mode_dy ? 2 * a->Ci + 3 * a->Co : (mode_x ? 2 * a->Ci : 0)) * sizeof(float);
#define W_CASE(TC_, MX, MD)                                                                              \
  if (tc == TC_ && mode_x == MX && mode_dy == MD) {                                                      \
    hipLaunchKernelGGL((f32wgrad_kernel<TC_, MX, MD>), dim3(nwork), dim3(256), dyn, stream, *a);         \
    return DTF_CHECK_LAUNCH();                                                                           \
  }
#define W_TCS(MX, MD) W_CASE(16, MX, MD) W_CASE(32, MX, MD) W_CASE(64, MX, MD)
  W_TCS(0, 0) W_TCS(1, 0) W_TCS(0, 2) W_TCS(1, 2)
#undef W_TCS
#undef W_CASE
  return -1;
}

// band fwd / dgrad of a stride-1 3x3 conv with Ci = Co = C on W x W images (the dtf_f32_conv modes / epilogues);
// rows per workgroup: C (C <= 32) or 16 (C = 64: the 9 x 64 x 72 weight tile of all 64 rows would not fit twice)
DTF_API int dtf_f32_conv_band_rows(int C) { return C <= 32 ? C : 16; }

DTF_API int dtf_f32_conv_band(const F32Args* a, int mode, int epi, int dgrad, int nwork, hipStream_t stream) {
  if (nwork <= 0) return 0;
  if (a->Ci != a->Co || a->kh != 3 || a->kw != 3 || a->stride != 1 || a->pad != 1 || a->Hi != a->Wi ||
      a->Ho != a->Hi || a->Wo != a->Wi || a->wci != a->Ci)
    return -2;
  DTF_HOST_CHECK(DTF_ALIGNED16(a->x) && DTF_ALIGNED16(a->y));
#define CB_CASE(C_, W_, M_, E_, D_)                                                                                \
  if (a->Ci == C_ && a->Wi == W_ && mode == M_ && epi == E_ && dgrad == D_) {                                      \
    hipLaunchKernelGGL((f32conv_band_kernel<C_, W_, (C_ <= 32 ? C_ : 16), M_, E_, D_>), dim3(nwork), dim3(256), 0, \
                       stream, *a);                                                                               \
    return DTF_CHECK_LAUNCH();                                                                                     \
  }
#define CB_CWS(M_, E_, D_) CB_CASE(16, 32, M_, E_, D_) CB_CASE(32, 16, M_, E_, D_) CB_CASE(64, 8, M_, E_, D_)
  CB_CWS(0, 4, false) CB_CWS(0, 0, false) CB_CWS(1, 4, false) CB_CWS(1, 0, false) CB_CWS(1, 5, false)
  CB_CWS(0, 6, true) CB_CWS(0, 7, true) CB_CWS(0, 0, true) CB_CWS(2, 3, true) CB_CWS(2, 6, true) CB_CWS(2, 7, true)
  CB_CWS(2, 0, true)
#undef CB_CWS
#undef CB_CASE
  return -1;
}

// band wgrad of a stride-1 3x3 conv with Ci = Co = C on W x W images: (C, W) in (16, 32) (32, 16) (64, 8)
DTF_API int dtf_f32_wgrad_band(const F32Args* a, int mode_x, int mode_dy, int nwork, hipStream_t stream) {
  if (nwork <= 0) return 0;
  if (a->Ci != a->Co || a->kh != 3 || a->kw != 3 || a->stride != 1 || a->pad != 1 || a->Hi != a->Wi ||
      a->Ho != a->Hi || a->Wo != a->Wi || a->wci != a->Ci)
    return -2;
  DTF_HOST_CHECK(DTF_ALIGNED16(a->x) && DTF_ALIGNED16(a->dy));
#define B_CASE(C_, W_, MX, MD)                                                                           \
  if (a->Ci == C_ && a->Wi == W_ && mode_x == MX && mode_dy == MD) {                                     \
    hipLaunchKernelGGL((f32wgrad_band_kernel<C_, W_, MX, MD>), dim3(nwork), dim3(256), 0, stream, *a);   \
    return DTF_CHECK_LAUNCH();                                                                           \
  }
#define B_CWS(MX, MD) B_CASE(16, 32, MX, MD) B_CASE(32, 16, MX, MD) B_CASE(64, 8, MX, MD)
  B_CWS(0, 0) B_CWS(1, 0) B_CWS(0, 2) B_CWS(1, 2)
#undef B_CWS
#undef B_CASE
  return -1;
}

DTF_API int dtf_f32_wgrad_band_ok(int C, int W) {
  return (C == 16 && W == 32) || (C == 32 && W == 16) || (C == 64 && W == 8);
}

DTF_API int dtf_f32_ew(const F32Ew* a, int which, hipStream_t stream) {
  if (a->nimg <= 0) return 0;
  if (a->C % 4) return -2;
  const long n4 = a->nimg * a->hw * a->C / 4;
  long blocks = (n4 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (which == 0)
    hipLaunchKernelGGL(f32_ew_kernel<0>, dim3((unsigned)blocks), dim3(256), 0, stream, *a);
  else if (which == 1)
    hipLaunchKernelGGL(f32_ew_kernel<1>, dim3((unsigned)blocks), dim3(256), 0, stream, *a);
  else
    hipLaunchKernelGGL(f32_ew_kernel<2>, dim3((unsigned)blocks), dim3(256), 0, stream, *a);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_f32_bwd_sums(const F32Sum* a, int nimg, hipStream_t stream) {
  if (nimg <= 0) return 0;
  if (a->C > 256 ? (a->C % 256) != 0 : (256 % a->C) != 0) return -2;
  hipLaunchKernelGGL(f32_bwd_sums_kernel, dim3(nimg, a->C > 256 ? a->C / 256 : 1), dim3(256), 0, stream, *a);
  return DTF_CHECK_LAUNCH();
}

// which 0: GAP + dense + CE (+ dlogits / dfeat when train); 1: dense gradient; 2: GAP-backward sums; 3: gradient at x
DTF_API int dtf_f32_head(const F32Head* a, int which, int nimg, const int* slots, const int* first, int nslots,
                         float* grads, long g_mstride, hipStream_t stream) {
  if (nimg <= 0) return 0;
  if (a->C > 256 || a->ncls > 64) return -2;
  if (which == 0)
    hipLaunchKernelGGL(f32_head_kernel, dim3(nimg), dim3(256), 0, stream, *a);
  else if (which == 1)
    hipLaunchKernelGGL(f32_dense_grad_kernel, dim3((a->ncls * a->C + a->ncls + 255) / 256, nslots), dim3(256), 0,
                       stream, *a, slots, first, grads, g_mstride);
  else if (which == 2)
    hipLaunchKernelGGL(f32_gap_bwd_kernel<0>, dim3(nimg), dim3(256), 0, stream, *a);
  else
    hipLaunchKernelGGL(f32_gap_bwd_kernel<1>, dim3(nimg), dim3(256), 0, stream, *a);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_f32_prep_input(const float* x, float* y, long npix, hipStream_t stream) {
  long blocks = (npix + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(f32_prep_input_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, x, y, npix);
  return DTF_CHECK_LAUNCH();
}

DTF_DEBUG_EXPORT(f32conv)
DTF_POISON_EXPORT(f32conv)
