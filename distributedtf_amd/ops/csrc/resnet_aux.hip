// Auxiliary population-batched kernels of the CIFAR ResNet step (gfx950):
//   * prep_input       : fp32 NHWC images -> bf16 NHWC with channels zero-padded to 16
//   * weight_prep      : fp32 master weights -> bf16 forward (OHWI) + dgrad (IHWO) layouts, all convs x members
//   * bn_running_update: TF-style moving averages (momentum 0.997, unbiased var) for every BN x member
//   * bn_bwd_apply     : g = A*dz + B*x + C (+ add): finishes a BatchNorm backward once its reductions are done
//   * head_fwd_bwd     : final BN+ReLU -> global avg pool -> dense -> softmax CE -> all gradients of the head,
//                        BN-final backward reductions, per-member loss / correct count
//   * head_bwd_apply   : residual-stream gradient entering the last block
#include "common.h"

#define BN_EPS 1e-5f
#define BN_MOM 0.997f
#define NREP DTF_NREP

namespace {

__device__ __forceinline__ void stats_sum(const float* row, int c, float& s, float& q) {
  s = 0.f;
  q = 0.f;
#pragma unroll
  for (int r = 0; r < NREP; ++r) {
    s += row[r * 128 + c];
    q += row[r * 128 + 64 + c];
  }
}

__global__ __launch_bounds__(256) void prep_input_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, long npix,
                                                          int c_in) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long p = (long)blockIdx.x * blockDim.x + threadIdx.x; p < npix; p += stride) {
    uint32_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    float v[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) v[c] = 0.f;
    for (int c = 0; c < c_in; ++c) v[c] = x[p * c_in + c];
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = pack2bf(v[2 * j], v[2 * j + 1]);
    uint4* dst = reinterpret_cast<uint4*>(y + p * 16);
    dst[0] = make_uint4(w[0], w[1], w[2], w[3]);
    dst[1] = make_uint4(w[4], w[5], w[6], w[7]);
  }
}

// conv table row: {w_off, cout, cin, k, cin_pad, fwd_off, dgr_off, 0} (int32)
__global__ __launch_bounds__(256) void weight_prep_kernel(const float* __restrict__ state, long s_mstride,
                                                           const int* __restrict__ table, const int* __restrict__ slots,
                                                           bf16_t* __restrict__ wf, bf16_t* __restrict__ wd,
                                                           long w_mstride, float* __restrict__ zbuf, long zn) {
  {  // the step's accumulators (BN statistics, loss, correct) start at zero: folded into this first launch
    const long nb = (long)gridDim.x * gridDim.y * gridDim.z;
    const long b = blockIdx.x + (long)gridDim.x * (blockIdx.y + (long)gridDim.y * blockIdx.z);
    const long z4 = zn >> 2;
    for (long i = b * blockDim.x + threadIdx.x; i < z4; i += nb * blockDim.x)
      reinterpret_cast<float4*>(zbuf)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (b == 0 && (long)threadIdx.x < zn - 4 * z4) zbuf[4 * z4 + threadIdx.x] = 0.f;
  }
  // grid (conv, chunk, member): every conv is split over gridDim.y workgroups so the launch fills the GPU
  // even for a single member (it sits at the head of the step's critical path).
  const int* t = table + blockIdx.x * 8;
  const int slot = slots[blockIdx.z];
  const int w_off = t[0], cout = t[1], cin = t[2], k = t[3], cin_pad = t[4], fwd_off = t[5], dgr_off = t[6];
  const int kk = k * k;
  const float* p = state + (long)slot * s_mstride + w_off;
  bf16_t* f = wf + (long)slot * w_mstride + fwd_off;
  bf16_t* d = wd + (long)slot * w_mstride + dgr_off;
  const int nf = cout * kk * cin_pad;
  const int t0 = blockIdx.y * blockDim.x + threadIdx.x, tstride = gridDim.y * blockDim.x;
  if (cin_pad == cin && (nf & 3) == 0 && (w_off & 3) == 0) {
    // same OHWI order: 4 elements per thread (float4 in, 4 x bf16 out)
    for (int i = 4 * t0; i < nf; i += 4 * tstride) {
      const float4 v = *reinterpret_cast<const float4*>(p + i);
      *reinterpret_cast<uint2*>(f + i) = make_uint2(pack2bf(v.x, v.y), pack2bf(v.z, v.w));
    }
  } else {
    for (int i = t0; i < nf; i += tstride) {
      const int ci = i % cin_pad, rest = i / cin_pad;  // rest = co*kk + tap
      f[i] = ci < cin ? f2bf(p[rest * cin + ci]) : (bf16_t)0;
    }
  }
  if (dgr_off >= 0) {
    if (cout <= 64 && cin <= 64) {
      // IHWO = per-tap [co][ci] -> [ci][co] transposes through LDS: coalesced reads along ci, coalesced writes
      // along co (the direct gather read one cache line per element)
      __shared__ float tt[64][65];
      for (int tap = blockIdx.y; tap < kk; tap += gridDim.y) {
        for (int e = threadIdx.x; e < cout * cin; e += blockDim.x) {
          const int co = e / cin, ci = e - co * cin;
          tt[co][ci] = p[(co * kk + tap) * cin + ci];
        }
        __syncthreads();
        for (int e = threadIdx.x; e < cout * cin; e += blockDim.x) {
          const int ci = e / cout, co = e - ci * cout;
          d[(ci * kk + tap) * cout + co] = f2bf(tt[co][ci]);
        }
        __syncthreads();
      }
    } else {
      const int nd = cin * kk * cout;
      for (int i = t0; i < nd; i += tstride) {
        const int co = i % cout, rest = i / cout;  // rest = ci*kk + tap
        const int tap = rest % kk, ci = rest / kk;
        d[i] = f2bf(p[(co * kk + tap) * cin + ci]);
      }
    }
  }
}

// bn table row: {run_off (float index into state row), C, hw, stats index, gamma_off, beta_off, 0, 0}
// grads == nullptr: moving-average update from forward statistics;
// grads != nullptr: accumulate dgamma / dbeta from backward statistics.
__global__ __launch_bounds__(64) void bn_running_update_kernel(float* __restrict__ state, long s_mstride, long run_base,
                                                                const int* __restrict__ table,
                                                                const float* __restrict__ stats, long stats_bn_stride,
                                                                const int* __restrict__ slots,
                                                                const float* __restrict__ cnt,
                                                                float* __restrict__ grads, long g_mstride,
                                                                const float* __restrict__ stats_fwd) {
  const int* t = table + blockIdx.x * 8;
  const int slot = slots[blockIdx.y];
  const int c = threadIdx.x;
  const int C = t[1];
  if (c >= C || cnt[slot] <= 0.f) return;  // (a member without images this step: an elastic plan's idle slot)
  if (blockIdx.z == 1) {  // combined launch: z = 1 is the moving-statistics update from the forward statistics
    stats = stats_fwd;
    grads = nullptr;
  }
  const float* row = stats + (long)t[3] * stats_bn_stride + (long)slot * NREP * 128;
  float s, q;
  stats_sum(row, c, s, q);
  if (grads != nullptr) {
    // parameter gradients of the BN: dgamma = sum(dz * xhat), dbeta = sum(dz) (backward reductions)
    float* g = grads + (long)slot * g_mstride;
    g[t[4] + c] += q;
    g[t[5] + c] += s;
    return;
  }
  const float n = cnt[slot] * (float)t[2];
  const float mean = s / n;
  const float var = fmaxf(q / n - mean * mean, 0.f);
  const float unbiased = n > 1.f ? var * n / (n - 1.f) : var;
  float* run = state + (long)slot * s_mstride + run_base + t[0];
  run[c] = BN_MOM * run[c] + (1.f - BN_MOM) * mean;
  run[C + c] = BN_MOM * run[C + c] + (1.f - BN_MOM) * unbiased;
}

// Elastic (capacity-keyed) step plans: every work table of the captured step is regenerated on the device from
// the per-member batch sizes (cnt) at the start of each replay, so a batch-size change needs no new plan or graph.
// The table holds R = per * M rows (x2 entries per row for a split table) for M members.
//  prop = 0 (the deterministic build, whose replay needs <= `per` rows per member): member m owns rows
//    [m*per, m*per + per); row j covers iterations [j*chunk_m, j*chunk_m + chunk_m) of the member's n * bands
//    (image, band) iterations, chunk_m = max(min_chunk, ceil(n * bands / per)).
//  prop = 1 (default): rows are dealt out in proportion to the members' sizes with ONE chunk for the whole table,
//    chunk = max(min_chunk, ceil(sum_m n_m * bands / (R - M))), member m gets max(1, ceil(total_m / chunk)) rows
//    (sum <= R) in member order and the last member also owns the unused tail.  With fixed rows per member a ragged
//    population (PBT samples batch sizes 65..255, constants.py:91-93) ran every launch at the pace of its largest
//    member: that member's rows carried up to 4x the iterations of the smallest member's.
// Rows past a member's iterations get nit = 0 (the kernels skip their loop and write zero partials) and point at
// the member's first iteration.  `red` (optional): the per-member (first entry, entries, 0, slot) table of the dW
// slab reductions over this work table, rewritten to match.
struct WorkGenDesc {
  int4* dst;
  int4* red;
  int per, bands, min_chunk, split;
  int prop, pad;
};

__global__ __launch_bounds__(256) void work_gen_kernel(const WorkGenDesc* __restrict__ descs,
                                                       const int* __restrict__ slots, const int* __restrict__ first,
                                                       const float* __restrict__ cnt, int nslots) {
  const WorkGenDesc d = descs[blockIdx.x];
  const int m = blockIdx.y;
  const int slot = slots[m];
  const int total = (int)cnt[slot] * d.bands;
  const int f = first[m] * d.bands;
  const int rows = d.split ? 2 : 1;
  const int R = d.per * nslots;
  int chunk, row0, nrows;
  if (d.prop && R > nslots) {
    int sum = 0, before = 0;  // rows of the members ahead of m (every member computes the same chunk)
    for (int k = 0; k < nslots; ++k) sum += (int)cnt[slots[k]] * d.bands;
    chunk = (sum + (R - nslots) - 1) / (R - nslots);
    if (chunk < d.min_chunk) chunk = d.min_chunk;
    if (chunk < 1) chunk = 1;
    for (int k = 0; k < m; ++k) {
      const int tk = (int)cnt[slots[k]] * d.bands;
      before += max(1, (tk + chunk - 1) / chunk);
    }
    row0 = before;
    nrows = m + 1 < nslots ? max(1, (total + chunk - 1) / chunk) : R - before;  // the last member takes the tail
  } else {
    chunk = (total + d.per - 1) / d.per;
    if (chunk < d.min_chunk) chunk = d.min_chunk;
    if (chunk < 1) chunk = 1;
    row0 = m * d.per;
    nrows = d.per;
  }
  for (int j = threadIdx.x; j < nrows; j += blockDim.x) {
    const int start = j * chunk;
    const int nit = start < total ? min(chunk, total - start) : 0;
    const int it0 = nit > 0 ? f + start : f;
    for (int z = 0; z < rows; ++z) d.dst[((long)row0 + j) * rows + z] = make_int4(it0, nit, z, slot);
  }
  if (d.red != nullptr && threadIdx.x == 0) d.red[m] = make_int4(row0 * rows, nrows * rows, 0, slot);
}

// Eval mode: BatchNorm with the moving statistics.  Every consumer derives its coefficients from replicated
// (sum, sum of squares) accumulators and the per-member count n = cnt * hw, so the moving mean / variance are
// written in that form (replica 0: n*mean, n*(var + mean^2); replicas 1.. zero) and the training kernels
// normalise with them unchanged.  Relative error of the recovered variance ~ 1e-7 * mean^2 / var (fp32).
__global__ __launch_bounds__(64) void bn_eval_stats_kernel(const float* __restrict__ state, long s_mstride,
                                                            long run_base, const int* __restrict__ table,
                                                            float* __restrict__ stats, long stats_bn_stride,
                                                            const int* __restrict__ slots,
                                                            const float* __restrict__ cnt) {
  const int* t = table + blockIdx.x * 8;
  const int slot = slots[blockIdx.y];
  const int c = threadIdx.x;
  const int C = t[1];
  float* row = stats + (long)t[3] * stats_bn_stride + (long)slot * NREP * 128;
  if (c >= C) return;
  const float* run = state + (long)slot * s_mstride + run_base + t[0];
  const float n = cnt[slot] * (float)t[2];
  const float mean = run[c], var = run[C + c];
  row[c] = n * mean;
  row[64 + c] = n * (var + mean * mean);
#pragma unroll
  for (int r = 1; r < NREP; ++r) {
    row[r * 128 + c] = 0.f;
    row[r * 128 + 64 + c] = 0.f;
  }
}

struct BnBwdArgs {
  const bf16_t* dz;
  const bf16_t* x;
  const bf16_t* add;
  bf16_t* out;
  const int* img_slot;
  const float* params;
  long p_mstride;
  int gamma_off;
  const float* st_f;
  const float* st_b;
  const float* cnt;
  int hw;
  int C;
  long nimg;
};

__device__ __forceinline__ void bwd_coef(const float* stf, const float* stb, float n, float gamma, int c, float& A,
                                         float& B, float& Cc) {
  float s, q;
  stats_sum(stf, c, s, q);
  const float mean = s / n;
  const float var = fmaxf(q / n - mean * mean, 0.f);
  const float inv = rsqrtf(var + BN_EPS);
  const float scale = gamma * inv;
  float sdz, sdzx;
  stats_sum(stb, c, sdz, sdzx);
  const float mdz = sdz / n, mdzx = sdzx / n;
  A = scale;
  B = -scale * inv * mdzx;
  Cc = -scale * mdz + scale * inv * mean * mdzx;
}

// One workgroup per image: coefficients of the image's member in LDS, then 8 bf16 per thread.
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(BnBwdArgs a) {
  __shared__ float co[3 * 64];
  const int img = blockIdx.x;
  const int slot = a.img_slot[img];
  const int C = a.C;
  if (threadIdx.x < C) {
    const float* prow = a.params + (long)slot * a.p_mstride;
    float A, B, Cc;
    bwd_coef(a.st_f + (long)slot * NREP * 128, a.st_b + (long)slot * NREP * 128, a.cnt[slot] * (float)a.hw,
             prow[a.gamma_off + threadIdx.x], threadIdx.x, A, B, Cc);
    co[threadIdx.x] = A;
    co[64 + threadIdx.x] = B;
    co[128 + threadIdx.x] = Cc;
  }
  __syncthreads();
  const long base = (long)img * a.hw * C;
  const int n8 = a.hw * C / 8;
  for (int i = blockIdx.y * blockDim.x + threadIdx.x; i < n8; i += gridDim.y * blockDim.x) {
    const long o = base + (long)i * 8;
    const int c0 = (i * 8) % C;
    uint4 dz = *reinterpret_cast<const uint4*>(a.dz + o);
    uint4 xv = *reinterpret_cast<const uint4*>(a.x + o);
    uint4 ad = make_uint4(0, 0, 0, 0);
    if (a.add) ad = *reinterpret_cast<const uint4*>(a.add + o);
    uint32_t d32[4] = {dz.x, dz.y, dz.z, dz.w}, x32[4] = {xv.x, xv.y, xv.z, xv.w}, a32[4] = {ad.x, ad.y, ad.z, ad.w};
    uint32_t r32[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = c0 + 2 * j;
      float v0 = co[c] * bf2f((bf16_t)(d32[j] & 0xffff)) + co[64 + c] * bf2f((bf16_t)(x32[j] & 0xffff)) + co[128 + c];
      float v1 = co[c + 1] * bf2f((bf16_t)(d32[j] >> 16)) + co[64 + c + 1] * bf2f((bf16_t)(x32[j] >> 16)) +
                 co[128 + c + 1];
      v0 += bf2f((bf16_t)(a32[j] & 0xffff));
      v1 += bf2f((bf16_t)(a32[j] >> 16));
      r32[j] = pack2bf(v0, v1);
    }
    *reinterpret_cast<uint4*>(a.out + o) = make_uint4(r32[0], r32[1], r32[2], r32[3]);
  }
}

struct HeadArgs {
  const bf16_t* x;        // [N, hw, C] last residual-stream tensor (pre final-BN)
  const int* labels;      // [N]
  const int4* work;       // (img0, nimg, 0, slot)
  const float* params;
  long p_mstride;
  int gamma_off, beta_off, dw_off, db_off;
  float* grads;
  long g_mstride;
  const float* st_f;      // final-BN forward stats
  float* st_b;            // final-BN backward reductions (out)
  const float* cnt;       // per-slot batch size (float)
  float* dfeat;           // [N, C] fp32 (out): dL/dfeat / hw
  float* loss;            // [cap] (out, summed mean CE)
  float* correct;         // [cap] (out)
  float* logits_out;      // [N, ncls] optional
  int hw, C, ncls;
  int train;
  float* slab;            // optional [nblocks][ncls * C] per-workgroup dense-weight gradients (else atomics)
  float* slab_b;          // optional [nblocks][ncls] per-workgroup bias gradients
  float loss_scale;       // the loss gradient is taken of loss_scale * loss (fp16 static loss scaling; else 1)
};

// Head of the CIFAR ResNet (C == 64 final channels, hw % 32 == 0, hw <= 128, ncls <= 16).  One image at a time
// per workgroup, all 4 waves on it: thread t stages pixels t/8 + 32k, channels 8*(t%8)..+7 as 16-byte loads (the
// whole 8 KB image in two load instructions per thread), keeps them in registers for the backward reductions, and
// the pooled feature is summed lane-group -> wave (xor shuffles) -> workgroup (LDS, one barrier per image; the
// LDS buffer alternates by image parity).  Every wave then computes the logits / softmax / dL/dfeat redundantly
// (no second barrier); wave 0 accumulates the dense gradients, written as a per-workgroup slab (reduced after the
// backward in fixed order) instead of thousands of same-address fp32 atomics.
constexpr int HEAD_MAXK = 4;  // 32-pixel rounds per image (hw <= 128)

__device__ __forceinline__ float xor_sum_8_16_32(float v) {
  v += __shfl_xor(v, 8, 64);
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}

__global__ __launch_bounds__(256) void head_kernel(HeadArgs a) {
  __shared__ float sc[64], sh[64], mu[64], iv[64];
  __shared__ float fpart[2][4][64];
  __shared__ float red[4][2][64];
  const int4 wk = a.work[blockIdx.x];
  DTF_WG_CHECK(wk.x >= 0 && wk.y >= 0 && wk.w >= 0 && a.C == 64 && a.hw % 32 == 0 && a.hw <= 32 * HEAD_MAXK &&
               a.ncls <= 16);
  const int img0 = wk.x, nimg = wk.y, slot = wk.w;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane;
  const int cg = threadIdx.x & 7, c8 = cg * 8, pix0 = threadIdx.x >> 3;  // this thread's 8 channels / first pixel
  const float* prow = a.params + (long)slot * a.p_mstride;
  const float bsz = a.cnt[slot];
  const float gsc = a.loss_scale / bsz;
  const int nk = a.hw / 32;
  // first image's loads before the coefficient math
  uint4 xv[HEAD_MAXK];
  auto load_img = [&](int img) {
    const bf16_t* xp = a.x + (long)img * a.hw * 64 + c8;
#pragma unroll
    for (int k = 0; k < HEAD_MAXK; ++k)
      if (k < nk) xv[k] = *reinterpret_cast<const uint4*>(xp + (long)(pix0 + 32 * k) * 64);
  };
  load_img(img0);
  if (threadIdx.x < 64) {
    if (a.gamma_off < 0) {  // ResNet v1: no final BN (input is the last block's ReLU output)
      sc[c] = 1.f;
      sh[c] = 0.f;
      mu[c] = 0.f;
      iv[c] = 1.f;
    } else {
      float s, q;
      stats_sum(a.st_f + (long)slot * NREP * 128, c, s, q);
      const float n = bsz * (float)a.hw;
      const float mean = s / n;
      const float var = fmaxf(q / n - mean * mean, 0.f);
      const float inv = rsqrtf(var + BN_EPS);
      sc[c] = prow[a.gamma_off + c] * inv;
      sh[c] = prow[a.beta_off + c] - mean * sc[c];
      mu[c] = mean;
      iv[c] = inv;
    }
  }
  const int ncls = a.ncls;
  float wcol[16];  // W[j][c] for lane c
#pragma unroll
  for (int j = 0; j < 16; ++j) wcol[j] = j < ncls ? prow[a.dw_off + j * 64 + c] : 0.f;
  const float bias = lane < ncls ? prow[a.db_off + lane] : 0.f;
  __syncthreads();
  float s8[8], t8[8], m8[8], i8[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    s8[i] = sc[c8 + i];
    t8[i] = sh[c8 + i];
    m8[i] = mu[c8 + i];
    i8[i] = iv[c8 + i];
  }
  float dw[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) dw[j] = 0.f;
  float db = 0.f;  // lane j < ncls of wave 0: db[j]
  float sdz[8], sdzx[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) sdz[i] = sdzx[i] = 0.f;
  float loss_acc = 0.f, corr = 0.f;
  const float inv_hw = 1.f / (float)a.hw;
  for (int im = 0; im < nimg; ++im) {
    const int img = img0 + im;
    // ---- pooled relu(BN(x)) of this thread's pixels, 8 channels
    float f8[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) f8[i] = 0.f;
#pragma unroll
    for (int k = 0; k < HEAD_MAXK; ++k) {
      if (k < nk) {
        const uint32_t w4[4] = {xv[k].x, xv[k].y, xv[k].z, xv[k].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          f8[2 * j] += fmaxf(bf2f((bf16_t)(w4[j] & 0xffff)) * s8[2 * j] + t8[2 * j], 0.f);
          f8[2 * j + 1] += fmaxf(bf2f((bf16_t)(w4[j] >> 16)) * s8[2 * j + 1] + t8[2 * j + 1], 0.f);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) f8[i] = xor_sum_8_16_32(f8[i]);
    float* fp = fpart[im & 1][wave];
    if (lane < 8) {
      *reinterpret_cast<float4*>(fp + c8) = make_float4(f8[0], f8[1], f8[2], f8[3]);
      *reinterpret_cast<float4*>(fp + c8 + 4) = make_float4(f8[4], f8[5], f8[6], f8[7]);
    }
    __syncthreads();
    const float f = (fpart[im & 1][0][c] + fpart[im & 1][1][c] + fpart[im & 1][2][c] + fpart[im & 1][3][c]) * inv_hw;
    uint4 xcur[HEAD_MAXK];
#pragma unroll
    for (int k = 0; k < HEAD_MAXK; ++k) xcur[k] = xv[k];
    if (im + 1 < nimg) load_img(img + 1);  // next image in flight during the softmax / backward math
    // ---- logits / softmax / CE (every wave, redundantly)
    float logit[16];
    float mx = -3.0e38f;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if (j < ncls) {
        logit[j] = wave_sum(wcol[j] * f) + __shfl(bias, j, 64);
        mx = fmaxf(mx, logit[j]);
      }
    }
    float se = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (j < ncls) se += __expf(logit[j] - mx);
    const float lse = mx + __logf(se);
    const int lab = a.labels[img];
    if (wave == 0) {
      float best = -3.0e38f;
      int arg = 0;
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (j < ncls && logit[j] > best) {
          best = logit[j];
          arg = j;
        }
      if (lane == 0) {
        float ll = 0.f;
#pragma unroll
        for (int j = 0; j < 16; ++j)
          if (j == lab) ll = logit[j];
        loss_acc += lse - ll;
        corr += (arg == lab) ? 1.f : 0.f;
      }
      if (a.logits_out && lane < ncls) {
#pragma unroll
        for (int j = 0; j < 16; ++j)
          if (j == lane) a.logits_out[(long)img * ncls + j] = logit[j];
      }
    }
    if (a.train) {
      float dfeat = 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        if (j < ncls) {
          const float dl = (__expf(logit[j] - lse) - (j == lab ? 1.f : 0.f)) * gsc;
          dfeat += wcol[j] * dl;
          if (wave == 0) {
            dw[j] += dl * f;
            if (lane == j) db += dl;
          }
        }
      }
      const float g = dfeat * inv_hw;  // dL/d(post-relu activation), identical for every pixel
      if (wave == 0) a.dfeat[(long)img * 64 + c] = g;
      float g8[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) g8[i] = __shfl(g, c8 + i, 64);
#pragma unroll
      for (int k = 0; k < HEAD_MAXK; ++k) {
        if (k < nk) {
          const uint32_t w4[4] = {xcur[k].x, xcur[k].y, xcur[k].z, xcur[k].w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int i = 2 * j + h;
              const float x = bf2f((bf16_t)(h ? (w4[j] >> 16) : (w4[j] & 0xffff)));
              if (x * s8[i] + t8[i] > 0.f) {
                sdz[i] += g8[i];
                sdzx[i] += g8[i] * (x - m8[i]) * i8[i];
              }
            }
          }
        }
      }
    }
  }
  // ---- workgroup reductions: BN-final backward sums (per channel), dense gradients, loss / correct
  if (a.train) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      sdz[i] = xor_sum_8_16_32(sdz[i]);
      sdzx[i] = xor_sum_8_16_32(sdzx[i]);
    }
    if (lane < 8) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        red[wave][0][c8 + i] = sdz[i];
        red[wave][1][c8 + i] = sdzx[i];
      }
    }
  }
  __syncthreads();
  if (wave == 0) {
    if (lane == 0) {
#ifdef DTF_DETERMINISTIC
      // partials rounded to multiples of 2^-16: their float sum is exact (so order-free) while the member's loss
      // stays below 2^8
      atomicAdd(&a.loss[slot], rintf(ldexpf(loss_acc / bsz, 16)) * (1.f / 65536.f));
#else
      atomicAdd(&a.loss[slot], loss_acc / bsz);
#endif
      atomicAdd(&a.correct[slot], corr);
    }
    if (a.train) {
      if (a.gamma_off >= 0) {
        const float v0 = red[0][0][c] + red[1][0][c] + red[2][0][c] + red[3][0][c];
        const float v1 = red[0][1][c] + red[1][1][c] + red[2][1][c] + red[3][1][c];
        float* row = a.st_b + (long)slot * NREP * 128 + (blockIdx.x & (NREP - 1)) * 128;
        atomicAdd(&row[c], v0);
        atomicAdd(&row[64 + c], v1);
      }
      if (a.slab != nullptr) {
        float* sl = a.slab + (long)blockIdx.x * ncls * 64;
#pragma unroll
        for (int j = 0; j < 16; ++j)
          if (j < ncls) sl[j * 64 + c] = dw[j];
        if (lane < ncls) a.slab_b[(long)blockIdx.x * ncls + lane] = db;
      } else {
        float* g = a.grads + (long)slot * a.g_mstride;
#pragma unroll
        for (int j = 0; j < 16; ++j)
          if (j < ncls) atomicAdd(&g[a.dw_off + j * 64 + c], dw[j]);
        if (lane < ncls) atomicAdd(&g[a.db_off + lane], db);
      }
    }
  }
}

// g[n,p,c] = A_c * dz + B_c * x + C_c  with  dz = dfeat[n,c] * [x*s+t > 0]  (final BN backward)
__global__ __launch_bounds__(256) void head_bwd_apply_kernel(const bf16_t* __restrict__ x, const float* __restrict__ dfeat,
                                                              bf16_t* __restrict__ out, const int* __restrict__ img_slot,
                                                              const float* __restrict__ params, long p_mstride,
                                                              int gamma_off, int beta_off, const float* __restrict__ st_f,
                                                              const float* __restrict__ st_b,
                                                              const float* __restrict__ cnt, int hw, int C) {
  __shared__ float co[5 * 64];
  const int img = blockIdx.x;
  const int slot = img_slot[img];
  const int c = threadIdx.x;
  if (c < C && gamma_off < 0) {  // v1: identity -> g = dfeat * [x > 0] (the last block's ReLU backward)
    co[c] = 1.f;
    co[64 + c] = 0.f;
    co[128 + c] = 0.f;
    co[192 + c] = 1.f;
    co[256 + c] = 0.f;
  } else if (c < C) {
    const float* prow = params + (long)slot * p_mstride;
    const float n = cnt[slot] * (float)hw;
    float s, q;
    stats_sum(st_f + (long)slot * NREP * 128, c, s, q);
    const float mean = s / n;
    const float var = fmaxf(q / n - mean * mean, 0.f);
    const float inv = rsqrtf(var + BN_EPS);
    const float scale = prow[gamma_off + c] * inv;
    float sdz, sdzx;
    stats_sum(st_b + (long)slot * NREP * 128, c, sdz, sdzx);
    const float mdz = sdz / n, mdzx = sdzx / n;
    co[c] = scale;
    co[64 + c] = -scale * inv * mdzx;
    co[128 + c] = -scale * mdz + scale * inv * mean * mdzx;
    co[192 + c] = scale;                                 // forward scale
    co[256 + c] = prow[beta_off + c] - mean * scale;     // forward shift
  }
  __syncthreads();
  const long base = (long)img * hw * C;
  const float* df = dfeat + (long)img * C;
  for (int i = threadIdx.x; i < hw * C; i += blockDim.x) {
    const int cc = i % C;
    const float xv = bf2f(x[base + i]);
    const float dz = (xv * co[192 + cc] + co[256 + cc] > 0.f) ? df[cc] : 0.f;
    out[base + i] = f2bf(co[cc] * dz + co[64 + cc] * xv + co[128 + cc]);
  }
}

// ---------------------------------------------------------------------------------------------- ResNet v1
// BN-apply + residual + ReLU of a v1 block output (also the stem: no addend):
//   out = relu(BN1(h1) + [BN2(h2) | add | 0])
struct BnEwArgs {
  const bf16_t* h1;
  const bf16_t* h2;
  const bf16_t* add;
  bf16_t* out;
  const bf16_t* d;    // bn_bwd_reduce: gradient w.r.t. the BN outputs (post-ReLU-mask)
  const int* img_slot;
  const float* params;
  long p_mstride;
  int g1, b1, g2, b2;
  const float* st1;   // forward stats of BN1 / BN2
  const float* st2;
  float* sb1;         // backward reductions of BN1 / BN2 (out)
  float* sb2;
  const float* cnt;
  int hw, C;
  long nimg;
  int cap;            // elastic plan: images per member region (an image is real iff img % cap < cnt[slot]); 0: exact
  int pad_;
  float* slab;        // deterministic build, bn_bwd_reduce: per-image partial sums [nimg][3][64]
};

// Elastic plans lay member k's images at [k * cap, (k + 1) * cap) and only the first cnt[slot] of them are real:
// the per-image BN kernels skip the rest (a capacity-padded image must not enter the BatchNorm reductions)
__device__ __forceinline__ bool idle_image(const BnEwArgs& a, int img, int slot) {
  return a.cap > 0 && (float)(img % a.cap) >= a.cnt[slot];
}

__device__ __forceinline__ void fwd_coef2(const float* st, float n, float gamma, float beta, int c, float& scale,
                                          float& shift, float& mean, float& inv) {
  float s, q;
  stats_sum(st, c, s, q);
  mean = s / n;
  const float var = fmaxf(q / n - mean * mean, 0.f);
  inv = rsqrtf(var + BN_EPS);
  scale = gamma * inv;
  shift = beta - mean * scale;
}

__global__ __launch_bounds__(256) void bn_add_relu_kernel(BnEwArgs a) {
  __shared__ float co[4 * 64];
  const int img = blockIdx.x;
  const int slot = a.img_slot[img];
  if (idle_image(a, img, slot)) return;  // workgroup-uniform
  const int C = a.C;
  if (threadIdx.x < C) {
    const int c = threadIdx.x;
    const float* prow = a.params + (long)slot * a.p_mstride;
    const float n = a.cnt[slot] * (float)a.hw;
    float sc, sh, mean, inv;
    fwd_coef2(a.st1 + (long)slot * NREP * 128, n, prow[a.g1 + c], prow[a.b1 + c], c, sc, sh, mean, inv);
    co[c] = sc;
    co[64 + c] = sh;
    if (a.h2) {
      fwd_coef2(a.st2 + (long)slot * NREP * 128, n, prow[a.g2 + c], prow[a.b2 + c], c, sc, sh, mean, inv);
      co[128 + c] = sc;
      co[192 + c] = sh;
    }
  }
  __syncthreads();
  const long base = (long)img * a.hw * C;
  const int n8 = a.hw * C / 8;
  for (int i = blockIdx.y * blockDim.x + threadIdx.x; i < n8; i += gridDim.y * blockDim.x) {
    const long o = base + (long)i * 8;
    const int c0 = (i * 8) % C;
    const uint4 hv = *reinterpret_cast<const uint4*>(a.h1 + o);
    uint4 av = make_uint4(0, 0, 0, 0);
    if (a.h2) av = *reinterpret_cast<const uint4*>(a.h2 + o);
    else if (a.add) av = *reinterpret_cast<const uint4*>(a.add + o);
    const uint32_t h32[4] = {hv.x, hv.y, hv.z, hv.w}, a32[4] = {av.x, av.y, av.z, av.w};
    uint32_t r32[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = c0 + 2 * j;
      float v0 = bf2f((bf16_t)(h32[j] & 0xffff)) * co[c] + co[64 + c];
      float v1 = bf2f((bf16_t)(h32[j] >> 16)) * co[c + 1] + co[64 + c + 1];
      const float x0 = bf2f((bf16_t)(a32[j] & 0xffff)), x1 = bf2f((bf16_t)(a32[j] >> 16));
      if (a.h2) {
        v0 += x0 * co[128 + c] + co[192 + c];
        v1 += x1 * co[128 + c + 1] + co[192 + c + 1];
      } else {
        v0 += x0;
        v1 += x1;
      }
      r32[j] = pack2bf(fmaxf(v0, 0.f), fmaxf(v1, 0.f));
    }
    *reinterpret_cast<uint4*>(a.out + o) = make_uint4(r32[0], r32[1], r32[2], r32[3]);
  }
}

// Backward reductions of the BN(s) feeding a v1 block output: sum(d), sum(d * xhat1) [, sum(d * xhat2)], with
// d = dL/d(pre-ReLU sum) (already masked).  Each thread keeps 8 fixed channels (2048 % C == 0), LDS reduction,
// one replicated atomic per channel and workgroup.
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(BnEwArgs a) {
  __shared__ float co[4 * 64];
  __shared__ float acc[3 * 64];
  const int img = blockIdx.x;
  const int slot = a.img_slot[img];
  if (idle_image(a, img, slot)) return;  // workgroup-uniform
  const int C = a.C;
  if (threadIdx.x < C) {
    const int c = threadIdx.x;
    const float* prow = a.params + (long)slot * a.p_mstride;
    const float n = a.cnt[slot] * (float)a.hw;
    float sc, sh, mean, inv;
    fwd_coef2(a.st1 + (long)slot * NREP * 128, n, prow[a.g1 + c], prow[a.b1 + c], c, sc, sh, mean, inv);
    co[c] = -mean * inv;
    co[64 + c] = inv;
    if (a.h2) {
      fwd_coef2(a.st2 + (long)slot * NREP * 128, n, prow[a.g2 + c], prow[a.b2 + c], c, sc, sh, mean, inv);
      co[128 + c] = -mean * inv;
      co[192 + c] = inv;
    }
  }
  if (threadIdx.x < 3 * 64) acc[threadIdx.x] = 0.f;
  __syncthreads();
  const long base = (long)img * a.hw * C;
  const int n8 = a.hw * C / 8;
  float sd[8], s1[8], s2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) sd[k] = s1[k] = s2[k] = 0.f;
  const int i0 = blockIdx.y * blockDim.x + threadIdx.x;
  const int c0 = (i0 * 8) % C;
  const int stride = gridDim.y * blockDim.x;
  float mi1[8], iv1[8], mi2[8], iv2[8];  // this thread's 8 channels' coefficients in registers
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    mi1[k] = co[c0 + k];
    iv1[k] = co[64 + c0 + k];
    mi2[k] = co[128 + c0 + k];
    iv2[k] = co[192 + c0 + k];
  }
  // two 16-byte chunks per operand in flight per thread and trip (the loop was load-latency bound)
  for (int i = i0; i < n8; i += 2 * stride) {
    const bool two = i + stride < n8;
    uint4 dv[2], hv[2], pv[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const long o = base + (long)(u && two ? i + stride : i) * 8;
      dv[u] = *reinterpret_cast<const uint4*>(a.d + o);
      hv[u] = *reinterpret_cast<const uint4*>(a.h1 + o);
      pv[u] = a.h2 ? *reinterpret_cast<const uint4*>(a.h2 + o) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (u == 1 && !two) break;
      const uint32_t d32[4] = {dv[u].x, dv[u].y, dv[u].z, dv[u].w}, h32[4] = {hv[u].x, hv[u].y, hv[u].z, hv[u].w},
                     p32[4] = {pv[u].x, pv[u].y, pv[u].z, pv[u].w};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float dd = bf2f((bf16_t)((d32[k >> 1] >> (16 * (k & 1))) & 0xffff));
        const float hh = bf2f((bf16_t)((h32[k >> 1] >> (16 * (k & 1))) & 0xffff));
        sd[k] += dd;
        s1[k] += dd * (hh * iv1[k] + mi1[k]);
        if (a.h2) {
          const float pp = bf2f((bf16_t)((p32[k >> 1] >> (16 * (k & 1))) & 0xffff));
          s2[k] += dd * (pp * iv2[k] + mi2[k]);
        }
      }
    }
  }
#ifdef DTF_DETERMINISTIC
  // fixed order: every thread's 8-channel partials to LDS, thread c sums its channel's owners in thread order and
  // stores the image's partial row; bn_bwd_reduce_finish_kernel adds a member's rows in image order (one launch
  // per image: gridDim.y == 1)
  __shared__ float part[3][256][8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    part[0][threadIdx.x][k] = i0 < n8 ? sd[k] : 0.f;
    part[1][threadIdx.x][k] = i0 < n8 ? s1[k] : 0.f;
    part[2][threadIdx.x][k] = i0 < n8 ? s2[k] : 0.f;
  }
  __syncthreads();
  if (threadIdx.x < C) {
    const int c = threadIdx.x, g = C / 8;
    float t0 = 0.f, t1 = 0.f, t2 = 0.f;
    for (int t = c / 8; t < 256; t += g) {
      t0 += part[0][t][c & 7];
      t1 += part[1][t][c & 7];
      t2 += part[2][t][c & 7];
    }
    float* row = a.slab + (long)img * 192;
    row[c] = t0;
    row[64 + c] = t1;
    row[128 + c] = t2;
  }
  (void)acc;
#else
  // lanes l and l ^ (G j) hold the same 8 channels (c0 = 8 (lane % G), G = C / 8): butterfly over them first, so the
  // LDS atomics are 4-way (one per wave) instead of 256 / G-way contended (the contention made this kernel 4x its
  // HBM time)
  const int G = C / 8, lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    for (int o = G; o < 64; o <<= 1) {
      sd[k] += __shfl_xor(sd[k], o, 64);
      s1[k] += __shfl_xor(s1[k], o, 64);
      if (a.h2) s2[k] += __shfl_xor(s2[k], o, 64);
    }
  }
  if (lane < G) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      atomicAdd(&acc[c0 + k], sd[k]);
      atomicAdd(&acc[64 + c0 + k], s1[k]);
      if (a.h2) atomicAdd(&acc[128 + c0 + k], s2[k]);
    }
  }
  __syncthreads();
  const int rep = (blockIdx.x + blockIdx.y) & (NREP - 1);
  if (threadIdx.x < C) {
    const int c = threadIdx.x;
    float* r1 = a.sb1 + (long)slot * NREP * 128 + rep * 128;
    atomicAdd(&r1[c], acc[c]);
    atomicAdd(&r1[64 + c], acc[64 + c]);
    if (a.h2) {
      float* r2 = a.sb2 + (long)slot * NREP * 128 + rep * 128;
      atomicAdd(&r2[c], acc[c]);
      atomicAdd(&r2[64 + c], acc[128 + c]);
    }
  }
#endif
}

// Deterministic build: a member's BN-backward reductions = its images' partial rows (bn_bwd_reduce_kernel) added in
// image order, stored in replica 0 of the member's accumulators (the others stay zero).  grid = members.
__global__ __launch_bounds__(64) void bn_bwd_reduce_finish_kernel(BnEwArgs a, const int* __restrict__ first,
                                                                  const int* __restrict__ slots) {
  const int s = slots[blockIdx.x], f = first[blockIdx.x], n = (int)a.cnt[s];
  const int c = threadIdx.x;
  if (c >= a.C) return;
  float t0 = 0.f, t1 = 0.f, t2 = 0.f;
  for (int i = 0; i < n; ++i) {
    const float* row = a.slab + (long)(f + i) * 192;
    t0 += row[c];
    t1 += row[64 + c];
    t2 += row[128 + c];
  }
  float* r1 = a.sb1 + (long)s * NREP * 128;
  r1[c] += t0;
  r1[64 + c] += t1;
  if (a.h2) {
    float* r2 = a.sb2 + (long)s * NREP * 128;
    r2[c] += t0;
    r2[64 + c] += t2;
  }
}

}  // namespace

DTF_API int dtf_prep_input(const float* x, bf16_t* y, long npix, int c_in, hipStream_t stream) {
  long blocks = (npix + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(prep_input_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, x, y, npix, c_in);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_weight_prep(const float* state, long s_mstride, const int* table, int nconv, const int* slots,
                            int nslots, bf16_t* wf, bf16_t* wd, long w_mstride, float* zbuf, long zn,
                            hipStream_t stream) {
  if (nconv <= 0 || nslots <= 0) return 0;
  hipLaunchKernelGGL(weight_prep_kernel, dim3(nconv, 16, nslots), dim3(256), 0, stream, state, s_mstride, table, slots,
                     wf, wd, w_mstride, zbuf, zn);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_bn_running_update(float* state, long s_mstride, long run_base, const int* table, int nbn,
                                  const float* stats, long stats_bn_stride, const int* slots, int nslots,
                                  const float* cnt, float* grads, long g_mstride, hipStream_t stream) {
  if (nbn <= 0 || nslots <= 0) return 0;
  hipLaunchKernelGGL(bn_running_update_kernel, dim3(nbn, nslots), dim3(64), 0, stream, state, s_mstride, run_base,
                     table, stats, stats_bn_stride, slots, cnt, grads, g_mstride, (const float*)nullptr);
  return DTF_CHECK_LAUNCH();
}

// End of a training step, one launch: BN parameter gradients from the backward reductions (z = 0) and the moving
// mean / variance update from the forward statistics (z = 1).
DTF_API int dtf_bn_step_end(float* state, long s_mstride, long run_base, const int* table, int nbn,
                            const float* stats_fwd, const float* stats_bwd, long stats_bn_stride, const int* slots,
                            int nslots, const float* cnt, float* grads, long g_mstride, hipStream_t stream) {
  if (nbn <= 0 || nslots <= 0) return 0;
  DTF_HOST_CHECK(stats_fwd != nullptr && stats_bwd != nullptr && grads != nullptr);
  hipLaunchKernelGGL(bn_running_update_kernel, dim3(nbn, nslots, 2), dim3(64), 0, stream, state, s_mstride, run_base,
                     table, stats_bwd, stats_bn_stride, slots, cnt, grads, g_mstride, stats_fwd);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_workgen_desc_size() { return (int)sizeof(WorkGenDesc); }

DTF_API int dtf_work_gen(const void* descs, int ndesc, const int* slots, const int* first, int nslots,
                         const float* cnt, hipStream_t stream) {
  if (ndesc <= 0 || nslots <= 0) return 0;
  DTF_HOST_CHECK(descs != nullptr && slots != nullptr && first != nullptr && cnt != nullptr && ndesc <= 65535);
  hipLaunchKernelGGL(work_gen_kernel, dim3(ndesc, nslots), dim3(256), 0, stream,
                     reinterpret_cast<const WorkGenDesc*>(descs), slots, first, cnt, nslots);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_bn_eval_stats(const float* state, long s_mstride, long run_base, const int* table, int nbn,
                              float* stats, long stats_bn_stride, const int* slots, int nslots, const float* cnt,
                              hipStream_t stream) {
  if (nbn <= 0 || nslots <= 0) return 0;
  hipLaunchKernelGGL(bn_eval_stats_kernel, dim3(nbn, nslots), dim3(64), 0, stream, state, s_mstride, run_base, table,
                     stats, stats_bn_stride, slots, cnt);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_bnbwd_args_size() { return (int)sizeof(BnBwdArgs); }
DTF_API int dtf_head_args_size() { return (int)sizeof(HeadArgs); }

DTF_API int dtf_bn_bwd_apply(const BnBwdArgs* a, hipStream_t stream) {
  if (a->nimg <= 0) return 0;
  // split every image over several workgroups when the population batch is small (>= ~2048 WGs in flight)
  const int n8 = a->hw * a->C / 8;
  int split = (int)((2048 + a->nimg - 1) / a->nimg);
  const int max_split = (n8 + 255) / 256;
  if (split > max_split) split = max_split;
  if (split < 1) split = 1;
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3((unsigned)a->nimg, split), dim3(256), 0, stream, *a);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_head(const HeadArgs* a, int nblocks, hipStream_t stream) {
  if (nblocks <= 0) return 0;
  // the kernel's fixed geometry (checked here in every build: a mismatch would read past the image)
  if (a->C != 64 || a->hw % 32 != 0 || a->hw > 32 * HEAD_MAXK || a->ncls > 16 || a->ncls < 1) return -22;
  hipLaunchKernelGGL(head_kernel, dim3(nblocks), dim3(256), 0, stream, *a);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_head_bwd_apply(const bf16_t* x, const float* dfeat, bf16_t* out, const int* img_slot,
                               const float* params, long p_mstride, int gamma_off, int beta_off, const float* st_f,
                               const float* st_b, const float* cnt, int hw, int C, int nimg, hipStream_t stream) {
  if (nimg <= 0) return 0;
  hipLaunchKernelGGL(head_bwd_apply_kernel, dim3(nimg), dim3(256), 0, stream, x, dfeat, out, img_slot, params,
                     p_mstride, gamma_off, beta_off, st_f, st_b, cnt, hw, C);
  return DTF_CHECK_LAUNCH();
}

static int ew_split(const BnEwArgs* a) {
#ifdef DTF_DETERMINISTIC
  if (a->slab != nullptr) return 1;  // bn_bwd_reduce: one workgroup (one partial row) per image
#endif
  const int n8 = a->hw * a->C / 8;
  int split = (int)((2048 + a->nimg - 1) / a->nimg);
  const int max_split = (n8 + 255) / 256;
  if (split > max_split) split = max_split;
  return split < 1 ? 1 : split;
}

DTF_API int dtf_bnew_args_size() { return (int)sizeof(BnEwArgs); }

DTF_API int dtf_bn_add_relu(const BnEwArgs* a, hipStream_t stream) {
  if (a->nimg <= 0) return 0;
  hipLaunchKernelGGL(bn_add_relu_kernel, dim3((unsigned)a->nimg, ew_split(a)), dim3(256), 0, stream, *a);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_bn_bwd_reduce(const BnEwArgs* a, hipStream_t stream) {
  if (a->nimg <= 0) return 0;
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3((unsigned)a->nimg, ew_split(a)), dim3(256), 0, stream, *a);
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_bn_bwd_reduce_finish(const BnEwArgs* a, const int* first, const int* slots, int nslots,
                                     hipStream_t stream) {
#ifdef DTF_DETERMINISTIC
  if (nslots <= 0) return 0;
  DTF_HOST_CHECK(a->slab != nullptr && a->C <= 64);
  hipLaunchKernelGGL(bn_bwd_reduce_finish_kernel, dim3(nslots), dim3(64), 0, stream, *a, first, slots);
  return DTF_CHECK_LAUNCH();
#else
  (void)a, (void)first, (void)slots, (void)nslots, (void)stream;
  return -1;  // release builds reduce with replicated atomics inside bn_bwd_reduce_kernel
#endif
}

DTF_DEBUG_EXPORT(resnet_aux)
