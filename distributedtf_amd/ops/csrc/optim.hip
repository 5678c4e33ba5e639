// Fused population optimizer (gfx950).
//
// One launch updates EVERY member of a GPU: state rows are
//   state[g] = [ w (Pp) | slot1 (Pp) | slot2 (Pp) | running stats ... ]
// and grads[g] = [ g (Pp) ].  Per-member hyper row (8 floats):
//   [opt_code, lr, momentum, grad_decay, weight_decay, reg_code, step t (1-based), active]
// Optimizer codes: 0 gd, 1 Momentum, 2 Adam, 3 Adagrad, 4 Adadelta, 5 RMSProp
// (TF1 semantics, see engine/optim.py).  Regularizer codes: 0 none, 1 l1, 2 l2, 3 l1_l2,
// applied to the conv-kernel prefix [0, n_reg).
// In the same pass the kernel writes the bf16 shadow copy of the new weights
// (read by the conv kernels) and zeroes the gradient buffer for the next step,
// so weights are touched once per step: ~30 B/param of HBM traffic in total.
// Memory-bound: float4 (16 B/lane) accesses, grid-stride over the row,
// blockIdx.y = member (optimizer branch is block-uniform: no divergence).
#include "common.h"

namespace {

struct Hyper {
  int opt, reg;
  float lr, mom, dec, wd, t;
};

__device__ __forceinline__ float reg_grad(float g, float w, float wd, int reg) {
  if (reg == 2 || reg == 3) g += wd * w;
  if (reg == 1 || reg == 3) g += wd * ((w > 0.f) ? 1.f : ((w < 0.f) ? -1.f : 0.f));
  return g;
}

template <int OPT>
__device__ __forceinline__ void update1(float& w, float& a, float& b, float g, const Hyper& h, float lr_t) {
  if constexpr (OPT == 0) {
    w -= h.lr * g;
  } else if constexpr (OPT == 1) {
    a = h.mom * a + g;
    w -= h.lr * a;
  } else if constexpr (OPT == 2) {
    a = 0.9f * a + 0.1f * g;
    b = 0.999f * b + 0.001f * g * g;
    w -= lr_t * a / (sqrtf(b) + 1e-8f);
  } else if constexpr (OPT == 3) {
    a += g * g;
    w -= h.lr * g * rsqrtf(a);
  } else if constexpr (OPT == 4) {
    a = 0.95f * a + 0.05f * g * g;
    float u = sqrtf(b + 1e-8f) * rsqrtf(a + 1e-8f) * g;
    b = 0.95f * b + 0.05f * u * u;
    w -= h.lr * u;
  } else {
    a = h.dec * a + (1.f - h.dec) * g * g;
    b = h.mom * b + h.lr * g * rsqrtf(a + 1e-10f);
    w -= b;
  }
}

template <int OPT>
__device__ void run_row(float* __restrict__ w, float* __restrict__ a, float* __restrict__ b, float* __restrict__ gr,
                        bf16_t* __restrict__ sh, long P, long n_reg, const Hyper& h, int zero_grads, float gscale) {
  float lr_t = h.lr;
  if constexpr (OPT == 2) lr_t = h.lr * sqrtf(1.f - powf(0.999f, h.t)) / (1.f - powf(0.9f, h.t));
  const long stride = (long)gridDim.x * blockDim.x * 4;
  for (long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < P; i += stride) {
    float4 wv = *reinterpret_cast<float4*>(w + i);
    float4 gv = *reinterpret_cast<float4*>(gr + i);
    float4 av = make_float4(0.f, 0.f, 0.f, 0.f), bv = av;
    if constexpr (OPT != 0) av = *reinterpret_cast<float4*>(a + i);
    if constexpr (OPT == 2 || OPT == 4 || OPT == 5) bv = *reinterpret_cast<float4*>(b + i);
    float ww[4] = {wv.x, wv.y, wv.z, wv.w};
    float gg[4] = {gv.x, gv.y, gv.z, gv.w};
    float aa[4] = {av.x, av.y, av.z, av.w};
    float bb[4] = {bv.x, bv.y, bv.z, bv.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float g = gg[j] * gscale;  // static loss scaling (fp16): the gradients of S * loss, unscaled here
      if (h.reg != 0 && i + j < n_reg) g = reg_grad(g, ww[j], h.wd, h.reg);
      update1<OPT>(ww[j], aa[j], bb[j], g, h, lr_t);
    }
    *reinterpret_cast<float4*>(w + i) = make_float4(ww[0], ww[1], ww[2], ww[3]);
    if constexpr (OPT != 0) *reinterpret_cast<float4*>(a + i) = make_float4(aa[0], aa[1], aa[2], aa[3]);
    if constexpr (OPT == 2 || OPT == 4 || OPT == 5) *reinterpret_cast<float4*>(b + i) = make_float4(bb[0], bb[1], bb[2], bb[3]);
    if (sh) {
      uint2 p;
      p.x = pack2bf(ww[0], ww[1]);
      p.y = pack2bf(ww[2], ww[3]);
      *reinterpret_cast<uint2*>(sh + i) = p;
    }
    if (zero_grads) *reinterpret_cast<float4*>(gr + i) = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

__global__ __launch_bounds__(256) void fused_optimizer_kernel(float* __restrict__ state, float* __restrict__ grads,
                                                               const float* __restrict__ hyper, bf16_t* __restrict__ shadow,
                                                               long S, long Pp, long P, long n_reg, int zero_grads,
                                                               float gscale) {
  const int g = blockIdx.y;
  const float* hp = hyper + g * 8;
  if (hp[7] == 0.f) return;
  Hyper h;
  h.opt = (int)hp[0];
  h.lr = hp[1];
  h.mom = hp[2];
  h.dec = hp[3];
  h.wd = hp[4];
  h.reg = (int)hp[5];
  h.t = hp[6];
  float* w = state + (long)g * S;
  float* a = w + Pp;
  float* b = w + 2 * Pp;
  float* gr = grads + (long)g * Pp;
  bf16_t* sh = shadow ? shadow + (long)g * Pp : nullptr;
  switch (h.opt) {
    case 0: run_row<0>(w, a, b, gr, sh, P, n_reg, h, zero_grads, gscale); break;
    case 1: run_row<1>(w, a, b, gr, sh, P, n_reg, h, zero_grads, gscale); break;
    case 2: run_row<2>(w, a, b, gr, sh, P, n_reg, h, zero_grads, gscale); break;
    case 3: run_row<3>(w, a, b, gr, sh, P, n_reg, h, zero_grads, gscale); break;
    case 4: run_row<4>(w, a, b, gr, sh, P, n_reg, h, zero_grads, gscale); break;
    default: run_row<5>(w, a, b, gr, sh, P, n_reg, h, zero_grads, gscale); break;
  }
}

// bf16 shadow refresh for rows whose weights changed outside the optimizer
// (initialisation, exploit import).
__global__ __launch_bounds__(256) void shadow_refresh_kernel(const float* __restrict__ state, bf16_t* __restrict__ shadow,
                                                              const int* __restrict__ rows, long S, long Pp, long P) {
  const int g = rows[blockIdx.y];
  const float* w = state + (long)g * S;
  bf16_t* sh = shadow + (long)g * Pp;
  const long stride = (long)gridDim.x * blockDim.x * 4;
  for (long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < P; i += stride) {
    float4 v = *reinterpret_cast<const float4*>(w + i);
    uint2 p;
    p.x = pack2bf(v.x, v.y);
    p.y = pack2bf(v.z, v.w);
    *reinterpret_cast<uint2*>(sh + i) = p;
  }
}

// Per-member step counters after a captured step: state[slot][col] += 1 and hyper[slot][h_step] += 1 for every
// ACTIVE listed member (hyper column 7; an elastic plan replayed for a subset of its members leaves the others
// untouched); optionally the step's per-member losses gathered in slot-list order (loss_sel[i] = loss[slots[i]]).
// ring (optional, single-block launches): the losses go to row (*ring_idx % ring_rows) of a [ring_rows][n] ring and
// the index advances -- every replay of a captured step leaves its losses in a row of their own, so the host keeps
// per-step loss views without a per-step copy launch
__global__ void step_advance_kernel(float* __restrict__ state, long S, long col, float* __restrict__ hyper,
                                    int h_step, const int* __restrict__ slots, int n, const float* __restrict__ loss,
                                    float* __restrict__ loss_sel, float* __restrict__ ring, int* __restrict__ ring_idx,
                                    int ring_rows) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int r = ring != nullptr ? *ring_idx : 0;
  if (i < n) {
    const int s = slots[i];
    const float inc = hyper[s * 8 + 7] != 0.f ? 1.f : 0.f;
    state[(long)s * S + col] += inc;
    hyper[s * 8 + h_step] += inc;
    if (loss_sel != nullptr) loss_sel[i] = loss[s];
    if (ring != nullptr) ring[(long)(r % ring_rows) * n + i] = loss[s];
  }
  if (ring != nullptr) {
    __syncthreads();  // every thread has read the index
    if (threadIdx.x == 0) *ring_idx = r + 1;
  }
}

}  // namespace

DTF_API int dtf_step_advance(float* state, long S, long col, float* hyper, int h_step, const int* slots, int n,
                             hipStream_t stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(step_advance_kernel, dim3((n + 63) / 64), dim3(64), 0, stream, state, S, col, hyper, h_step,
                     slots, n, (const float*)nullptr, (float*)nullptr, (float*)nullptr, (int*)nullptr, 1);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_step_end(float* state, long S, long col, float* hyper, int h_step, const int* slots, int n,
                         const float* loss, float* loss_sel, float* ring, int* ring_idx, int ring_rows,
                         hipStream_t stream) {
  if (n <= 0) return 0;
  if (ring != nullptr && (n > 1024 || ring_idx == nullptr || ring_rows <= 0)) return -2;  // one block
  const int threads = ring != nullptr ? ((n + 63) / 64) * 64 : 64;
  hipLaunchKernelGGL(step_advance_kernel, dim3(ring != nullptr ? 1 : (n + 63) / 64), dim3(threads), 0, stream, state,
                     S, col, hyper, h_step, slots, n, loss, loss_sel, ring, ring_idx, ring_rows);
  return DTF_CHECK_LAUNCH();
}

// gscale: factor on every gradient before the update (1 / the static loss scale of the fp16 mode, else 1)
DTF_API int dtf_fused_optimizer(float* state, float* grads, const float* hyper, bf16_t* shadow, int G, long S, long Pp,
                                long P, long n_reg, int zero_grads, float gscale, hipStream_t stream) {
  if (G <= 0) return 0;
  long per_block = 256 * 4;
  long blocks = (P + per_block - 1) / per_block;
  if (blocks > 512) blocks = 512;  // grid-stride; G*512 blocks >> 256 CUs
  dim3 grid((unsigned)blocks, (unsigned)G);
  hipLaunchKernelGGL(fused_optimizer_kernel, grid, dim3(256), 0, stream, state, grads, hyper, shadow, S, Pp, P, n_reg,
                     zero_grads, gscale);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_shadow_refresh(const float* state, bf16_t* shadow, const int* rows, int nrows, long S, long Pp, long P,
                               hipStream_t stream) {
  if (nrows <= 0) return 0;
  long blocks = (P + 1023) / 1024;
  if (blocks > 512) blocks = 512;
  hipLaunchKernelGGL(shadow_refresh_kernel, dim3((unsigned)blocks, (unsigned)nrows), dim3(256), 0, stream, state, shadow,
                     rows, S, Pp, P);
  return DTF_CHECK_LAUNCH();
}
