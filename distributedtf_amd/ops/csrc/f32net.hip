// fp32 helpers of the ImageNet-shape bottleneck nets' fp32 step (engine/hip_imagenet_f32.py, --dtype fp32
// --model imagenet): the pieces of the network that are not convolutions, at fp32.  The convolutions (7x7/2 stem,
// 1x1 / 3x3 / strided, the dense layer as a 1x1 conv) run on f32conv.hip's v_mfma_f32_16x16x4_f32 kernels, BN
// finalize on convg_aux.hip cg_bn_final, elementwise BN applies and BN-backward sums on f32conv.hip.
//
//   f32_maxpool_fwd / _bwd : 3x3/2 'SAME' max-pool (TF pads the end: output o covers input 2o .. 2o+2) with a
//                            per-output argmax byte; the backward gathers the (at most 2 x 2) windows of an input
//                            pixel (no atomics)
//   f32_gap / _gap_bwd_reduce / _gap_bwd_apply : [final BN + ReLU +] global average pool and its backward
//   f32_softmax_ce         : + bias, softmax cross-entropy, loss / correct count, dlogits (fp32, zero padding
//                            columns), dbias
// Semantics follow the bf16 kernels of convg_aux.hip one for one (reference resnet_model.py:504-525,
// resnet_run_loop.py:228-236).
#include "common.h"

namespace {

struct F32GapArgs {  // layout of convg_aux.hip GapArgs (engine/hip_imagenet.py GapArgs) with fp32 tensors
  const float* x;       // [N][hw][C] last block output (pre final BN)
  const float* coef;    // final BN forward coefficients [cap][4][cmax] (nullptr: identity, v1)
  const int* img_slot;
  float* feat;          // [N][C]
  const float* dfeat;   // bwd: [N][C] dL/dfeat
  dtf_acc_t* sums;      // bwd: final-BN backward sums [cap][2][cmax]
  const float* bcoef;   // bwd apply: A, B, C
  float* out;           // bwd apply: gradient at x
  int hw, C, cmax;
};

// thread = (output pixel, 4 channels)
__global__ __launch_bounds__(256) void f32_maxpool_fwd_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                              uint8_t* __restrict__ am, int H, int W, int Ho, int Wo,
                                                              int C, long total4) {
  const long stride = (long)gridDim.x * blockDim.x;
  const int C4 = C / 4;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total4; i += stride) {
    const long pix = i / C4;
    const int c0 = (int)(i - pix * C4) * 4;
    const long pr = pix / Wo;
    const int ox = (int)(pix - pr * Wo), oy = (int)(pr % Ho);
    const long img = pr / Ho;
    float best[4] = {-3.0e38f, -3.0e38f, -3.0e38f, -3.0e38f};
    uint32_t arg[4] = {0u, 0u, 0u, 0u};
    for (int t = 0; t < 9; ++t) {
      const int iy = 2 * oy + t / 3, ix = 2 * ox + t % 3;
      if (iy >= H || ix >= W) continue;
      const float4 v = *reinterpret_cast<const float4*>(x + ((img * H + iy) * W + ix) * C + c0);
      const float f[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (f[k] > best[k]) {
          best[k] = f[k];
          arg[k] = (uint32_t)t;
        }
    }
    const long o = pix * C + c0;
    *reinterpret_cast<float4*>(y + o) = make_float4(best[0], best[1], best[2], best[3]);
    *reinterpret_cast<uint32_t*>(am + o) = arg[0] | (arg[1] << 8) | (arg[2] << 16) | (arg[3] << 24);
  }
}

// thread = (input pixel, 4 channels): the windows containing (iy, ix) are oy = iy / 2 (tap row iy % 2) and, for
// even iy >= 2, oy = iy / 2 - 1 (tap row 2); likewise in x
__global__ __launch_bounds__(256) void f32_maxpool_bwd_kernel(const float* __restrict__ g, const uint8_t* __restrict__ am,
                                                              float* __restrict__ dx, int H, int W, int Ho, int Wo,
                                                              int C, long total4) {
  const long stride = (long)gridDim.x * blockDim.x;
  const int C4 = C / 4;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total4; i += stride) {
    const long pix = i / C4;
    const int c0 = (int)(i - pix * C4) * 4;
    const long pr = pix / W;
    const int ix = (int)(pix - pr * W), iy = (int)(pr % H);
    const long img = pr / H;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    const int oy_[2] = {iy >> 1, (iy >> 1) - 1}, ox_[2] = {ix >> 1, (ix >> 1) - 1};
    const bool oky[2] = {(iy >> 1) < Ho, !(iy & 1) && iy >= 2}, okx[2] = {(ix >> 1) < Wo, !(ix & 1) && ix >= 2};
    const uint32_t ty_[2] = {(uint32_t)(iy & 1), 2u}, tx_[2] = {(uint32_t)(ix & 1), 2u};
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const int a_ = w >> 1, b_ = w & 1;
      if (!(oky[a_] && okx[b_])) continue;
      const long o = ((img * Ho + oy_[a_]) * Wo + ox_[b_]) * C + c0;
      const uint32_t av = *reinterpret_cast<const uint32_t*>(am + o);
      const float4 gv = *reinterpret_cast<const float4*>(g + o);
      const float gg[4] = {gv.x, gv.y, gv.z, gv.w};
      const uint32_t t = ty_[a_] * 3 + tx_[b_];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (((av >> (8 * k)) & 0xffu) == t) acc[k] += gg[k];
    }
    *reinterpret_cast<float4*>(dx + pix * C + c0) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  }
}

// one workgroup per image, thread = 4-channel group
__global__ __launch_bounds__(256) void f32_gap_kernel(F32GapArgs a) {
  const int img = blockIdx.x, slot = a.img_slot[img];
  const float* co = a.coef ? a.coef + (long)slot * 4 * a.cmax : nullptr;
  const float inv = 1.f / (float)a.hw;
  for (int c0 = threadIdx.x * 4; c0 < a.C; c0 += blockDim.x * 4) {
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    for (int p = 0; p < a.hw; ++p) {
      const float4 v = *reinterpret_cast<const float4*>(a.x + ((long)img * a.hw + p) * a.C + c0);
      const float f[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) s[k] += co ? fmaxf(f[k] * co[c0 + k] + co[a.cmax + c0 + k], 0.f) : f[k];
    }
    *reinterpret_cast<float4*>(a.feat + (long)img * a.C + c0) = make_float4(s[0] * inv, s[1] * inv, s[2] * inv,
                                                                            s[3] * inv);
  }
}

// final-BN backward sums: dz = dfeat / hw * [BN(x) > 0]; sum dz, sum dz * xhat
__global__ __launch_bounds__(256) void f32_gap_bwd_reduce_kernel(F32GapArgs a) {
  const int img = blockIdx.x, slot = a.img_slot[img];
  const float* co = a.coef + (long)slot * 4 * a.cmax;
  dtf_acc_t* su = a.sums + (long)slot * 2 * a.cmax;
  const float inv_hw = 1.f / (float)a.hw;
  for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
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
    dtf_acc_add(su + c, s, DTF_FX_GRAD, slot);
    dtf_acc_add(su + a.cmax + c, q, DTF_FX_GRAD, slot);
  }
}

__global__ __launch_bounds__(256) void f32_gap_bwd_apply_kernel(F32GapArgs a) {
  const int img = blockIdx.x, slot = a.img_slot[img];
  const float* co = a.coef ? a.coef + (long)slot * 4 * a.cmax : nullptr;
  const float* bc = a.bcoef ? a.bcoef + (long)slot * 4 * a.cmax : nullptr;
  const float inv_hw = 1.f / (float)a.hw;
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
      r = xv > 0.f ? g : 0.f;  // v1: the last block's ReLU
    }
    a.out[o] = r;
  }
}

// one wave per image: logits [N][ld] (+ bias) -> loss / correct / dlogits [N][ld] (0 past ncls) / dbias
__global__ __launch_bounds__(256) void f32_softmax_ce_kernel(const float* __restrict__ logits, int ld, int ncls,
                                                             const int* __restrict__ labels,
                                                             const int* __restrict__ img_slot,
                                                             const float* __restrict__ state, long s_mstride, int b_off,
                                                             dtf_acc_t* __restrict__ grads, long g_mstride,
                                                             const float* __restrict__ cnt, dtf_acc_t* __restrict__ loss,
                                                             float* __restrict__ correct, float* __restrict__ dl,
                                                             long nimg) {
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
  for (int j = lane; j < ncls; j += 64) se += expf(lr[j] + bias[j] - mx);
  se = wave_sum(se);
  const float lse = mx + logf(se);
  const int lab = labels[img];
  const float bsz = cnt[slot];
  dtf_acc_t* gb = grads != nullptr ? grads + (long)slot * g_mstride + b_off : nullptr;
  for (int j = lane; j < ld; j += 64) {
    float d = 0.f;
    if (j < ncls) {
      d = (expf(lr[j] + bias[j] - lse) - (j == lab ? 1.f : 0.f)) / bsz;
      if (grads != nullptr) dtf_acc_add(gb + j, d, DTF_FX_GRAD, slot);
    }
    if (dl != nullptr) dl[img * ld + j] = d;
  }
  if (lane == 0) {
    dtf_acc_add(loss + slot, (lse - (lr[lab] + bias[lab])) / bsz, DTF_FX_GRAD, slot);
    atomicAdd(correct + slot, arg == lab ? 1.f : 0.f);  // integer-valued: exact in any order
  }
}

}  // namespace

DTF_API int dtf_f32_gap_args_size() { return (int)sizeof(F32GapArgs); }

// dx == nullptr: forward (x -> y, am); else backward (g, am -> dx)
DTF_API int dtf_f32_maxpool(const float* x, float* y, uint8_t* am, const float* g, float* dx, int N, int H, int W,
                            int Ho, int Wo, int C, int bwd, hipStream_t stream) {
  if (N <= 0) return 0;
  if (C % 4) return -2;
  const long total4 = bwd ? (long)N * H * W * C / 4 : (long)N * Ho * Wo * C / 4;
  long blocks = (total4 + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  if (bwd)
    hipLaunchKernelGGL(f32_maxpool_bwd_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, g, am, dx, H, W, Ho, Wo,
                       C, total4);
  else
    hipLaunchKernelGGL(f32_maxpool_fwd_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, x, y, am, H, W, Ho, Wo,
                       C, total4);
  return DTF_CHECK_LAUNCH();
}

// which 0: GAP forward, 1: final-BN backward sums, 2: gradient at x
DTF_API int dtf_f32_gap(const F32GapArgs* a, int which, int nimg, hipStream_t stream) {
  if (nimg <= 0) return 0;
  if (a->C % 4) return -2;
  if (which == 0)
    hipLaunchKernelGGL(f32_gap_kernel, dim3(nimg), dim3(256), 0, stream, *a);
  else if (which == 1)
    hipLaunchKernelGGL(f32_gap_bwd_reduce_kernel, dim3(nimg), dim3(256), 0, stream, *a);
  else
    hipLaunchKernelGGL(f32_gap_bwd_apply_kernel, dim3(nimg), dim3(256), 0, stream, *a);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_f32_softmax_ce(const float* logits, int ld, int ncls, const int* labels, const int* img_slot,
                               const float* state, long s_mstride, int b_off, dtf_acc_t* grads, long g_mstride,
                               const float* cnt, dtf_acc_t* loss, float* correct, float* dl, long nimg,
                               hipStream_t stream) {
  if (nimg <= 0) return 0;
  if (ncls > ld) return -2;
  hipLaunchKernelGGL(f32_softmax_ce_kernel, dim3((unsigned)((nimg + 3) / 4)), dim3(256), 0, stream, logits, ld, ncls,
                     labels, img_slot, state, s_mstride, b_off, grads, g_mstride, cnt, loss, correct, dl, nimg);
  return DTF_CHECK_LAUNCH();
}

DTF_DEBUG_EXPORT(f32net)
