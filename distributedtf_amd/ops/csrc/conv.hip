// Population-batched implicit-GEMM convolutions for the CIFAR ResNet hot path (gfx950).
//
// Tensors are NHWC bf16 with the images of ALL population members packed along N
// (img_slot[n] = member slot of image n), so one launch serves the whole population
// and the grid is >> 256 CUs even at per-member batch 65.  Weights are per member:
// bf16 rows `w + slot*w_mstride + w_off`.
//
// MFMA: v_mfma_f32_16x16x32_bf16, A = weights (16 output channels x 32 k),
// B = activations (32 k x 16 pixels), k = (tap, channel) flattened exactly like the
// OHWI weight layout, so a lane's 8 k-values are 16 contiguous bytes in both LDS
// (NHWC tile) and the weight row.  The C/D fragment (4 consecutive channels of one
// pixel per lane) is stored as one 8-byte packed bf16 write, and a 16-pixel tile
// of a 16-channel layer is a single contiguous 512-byte store.
//
// LDS tiles: [rows][cols][cpad<C>()] bf16 with a zero halo; the pixel pitch keeps the
// ds_read_b128 pixel gathers free of bank conflicts (see cpad).  The producing BatchNorm (+ReLU) of the input is applied
// while the tile is staged (global -> regs -> transform -> LDS), and BN statistics
// of the output are reduced in registers/LDS and added to 8 replicated per-member
// accumulators (cuts same-address atomic contention 8x); consumers sum the
// replicas when they derive their per-channel coefficients.
//
//  conv_fwd   : y = conv(T_in(x)) [+ res]           epilogue: sum(y), sum(y^2)
//  conv_dgrad : dx = conv^T(T_dy(dy)) [+ add]       epilogue: relu-mask by BN(x) + sum(dz), sum(dz*xhat)
//  conv_wgrad : dW += sum_pix T_dy(dy) (x) T_x(x)   operand fragments via ds_read_b64_tr_b16
// T_* in {identity, BN+ReLU (fwd), BN-backward apply A*dz + B*h + C}.
#include "common.h"

#define BN_EPS 1e-5f
// min waves / SIMD the fused backward kernel is register-capped for (C = 16 single-buffered: 3 WGs / CU)
#ifndef DTF_FUSED_SB16
#define DTF_FUSED_SB16 0  // (host allocates the double-buffered size either way: 3 x 46 KB fits the 160 KB LDS)
#endif
#ifndef DTF_FUSED16_WLDS
#define DTF_FUSED16_WLDS 1  // C = 16 fused backward: dgrad weights read from LDS per MFMA instead of held in VGPRs
#endif
#ifndef DTF_TRANSFORM8_PK
#define DTF_TRANSFORM8_PK 1  // strided / generic CIFAR conv staging: packed two-channel BN transforms
#endif
#ifndef DTF_BWD_COEFREG
#define DTF_BWD_COEFREG 1  // conv_bwd_fused<16, 3>: staging + epilogue BN coefficients held in VGPRs
#endif
#ifndef DTF_FWD_COEFREG
#define DTF_FWD_COEFREG 1  // conv_fwd_s1 MODE 1: BN scale / shift of the staged channels held in VGPRs (pop 8 3.078 -> 3.063 ms, profiles/r6_fwd_coefreg_ab.log)
#endif
#ifndef DTF_WGRAD_PF2
#define DTF_WGRAD_PF2 0  // 1: deferred wgrad jobs with tiles prefetched two iterations ahead (conv_wgrad_pf2_body): measured +0.8 % at pop 8, flat at C = 16 only (profiles/r6_wgrad_pf2_ab.log)
#endif
#ifndef DTF_WGRAD_PF2_MAXC
#define DTF_WGRAD_PF2_MAXC 64  // ... for the channel widths up to this
#endif
#ifndef DTF_COEF_SPLIT
#define DTF_COEF_SPLIT 1  // C < 64: wave 0's 64 / C lane groups split the statistic replicas (shuffle-summed)
#endif
#ifndef DTF_COEF_W0
#define DTF_COEF_W0 1
#endif
#ifndef DTF_FUSED16_M3_WAVES
#define DTF_FUSED16_M3_WAVES 2
#endif
#ifndef DTF_FUSED16_M2_WAVES
#define DTF_FUSED16_M2_WAVES 3  // 2: room for register-held coefficients in conv_bwd_fused<16, 2, *> (measured flat: profiles/r6_fused16_m2_waves2_ab.log)
#endif
#define FUSED_WAVES(C, M) ((C) <= 16 ? ((M) != 3 ? DTF_FUSED16_M2_WAVES : DTF_FUSED16_M3_WAVES) : (C) <= 32 ? 2 : 1)
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
#define NREP DTF_NREP
#ifndef DTF_STAMP
#define DTF_STAMP 0  // diagnostic build (tools/stamps.py): per-workgroup s_memrealtime stamps of the fwd_s1 / fused bwd
#endif                // phases; the launch ordinal rides in ConvArgs.cin_real (unused by those kernels)
#if DTF_STAMP
#define STAMP_LAUNCHES 256
#define STAMP_WGS 512
__device__ unsigned long long dtf_stamps[STAMP_LAUNCHES][STAMP_WGS][16];
#define STAMP_DECL unsigned long long st_[16] = {0};
#define STAMP(i) (st_[i] = __builtin_amdgcn_s_memrealtime())
#define STAMP_DRAIN(i) (__builtin_amdgcn_s_waitcnt(0), st_[i] = __builtin_amdgcn_s_memrealtime())
#if DTF_STAMP >= 2  // fine prologue stamps: each drains the loads issued so far (serialises them: read shares)
#define STAMP_FINE(i) STAMP_DRAIN(i)
#else
#define STAMP_FINE(i) ((void)0)
#endif
#define STAMP_FLUSH(row, extra)                                                                        \
  do {                                                                                                 \
    if (threadIdx.x == 0 && (row) >= 0 && (row) < STAMP_LAUNCHES && blockIdx.x < STAMP_WGS) {          \
      st_[7] = (extra);                                                                                \
      for (int i_ = 0; i_ < 16; ++i_) dtf_stamps[row][blockIdx.x][i_] = st_[i_];                        \
    }                                                                                                  \
  } while (0)
#else
#define STAMP_DECL
#define STAMP(i) ((void)0)
#define STAMP_FINE(i) ((void)0)
#define STAMP_DRAIN(i) ((void)0)
#define STAMP_FLUSH(row, extra) ((void)0)
#endif

namespace {

struct ConvArgs {
  const bf16_t* x;    // primary input (fwd: x; dgrad: dy (or dz of the next BN); wgrad: x)
  const bf16_t* x2;   // second input of a BN-backward transform (the BN's forward input h)
  const bf16_t* dy;   // wgrad: dY (or dz)
  const bf16_t* dy2;  // wgrad: BN-backward second input
  bf16_t* y;          // output
  const bf16_t* res;  // fwd: residual to add / dgrad: tensor to add before the mask
  const bf16_t* xm;   // dgrad epilogue: forward input x of the masking BN
  const bf16_t* w;    // bf16 weights (fwd OHWI / dgrad IHWO)
  long w_mstride;
  long w_off;
  float* grads;       // wgrad output (fp32, atomically accumulated)
  long g_mstride;
  long g_off;
  const int* img_slot;
  const int4* work;   // per-WG work item: (img0, nimg, band, slot)
  const float* params;  // fp32 state rows (gamma / beta)
  long p_mstride;
  int in_gamma, in_beta;    // BN applied to the input (fwd) or BN whose backward is applied (dgrad/wgrad dy)
  int ep_gamma, ep_beta;    // BN used by the dgrad epilogue mask
  int x_gamma, x_beta;      // wgrad: BN applied to x
  const float* st_in;       // fwd stats of the input-side BN      [cap][NREP][2][64]
  const float* st_in_b;     // bwd stats of the input-side BN
  const float* st_ep;       // fwd stats of the epilogue BN
  const float* st_x;        // wgrad: fwd stats of x's BN
  float* st_out;            // stats produced by this kernel
  const float* cnt;         // per-slot image count (float)
  int Hi, Wi, Ho, Wo;       // forward input / output spatial dims
  int rows;                 // rows per band (output rows for fwd/wgrad, dx rows for dgrad)
  int cin_real;             // wgrad: real input channels (stem: 3)
  float* slab;              // fused bwd: per-workgroup dW partials (plain stores; reduced by dw_slab_reduce)
  // fused bwd extensions
  const bf16_t* x3;         // MODE_DY 3: residual-stream gradient added after the BN-backward transform
  bf16_t* xout;             // materialise the transformed dY (band interior rows) here (null: don't)
  const float* rslab;       // trailing workgroups (blockIdx >= n_main) reduce these dW slabs of the PREVIOUS
  const int4* rtab;         //   fused launch: rtab[m] = (first wg, n wgs, -, slot) per member
  long r_goff;              //   gradient-row offset of that conv
  int r_c;                  //   its channel count (0: no reduction role)
  int r_nblk;               //   reduce workgroups per member (E / 32)
  int n_main;               // workgroups of the convolution role
  // Uniform populations (every member the same batch, slots 0..n-1 packed in order): the work item of workgroup b
  // is arithmetic -- member b / u_items, iterations [k * u_chunk, ...) of its u_per -- instead of a dependent
  // load of work[b] (one memory round trip less before every address of the kernel).  u_items = 0: use `work`.
  int u_items, u_chunk, u_per, u_pad;
};

__device__ __forceinline__ int4 work_item_at(const ConvArgs& a, int b) {
  if (a.u_items > 0) {
    const int m = b / a.u_items, k = b - m * a.u_items;
    const int it0 = k * a.u_chunk;
    return make_int4(m * a.u_per + it0, min(a.u_chunk, a.u_per - it0), 0, m);
  }
  return a.work[b];
}

__device__ __forceinline__ int4 work_item(const ConvArgs& a) { return work_item_at(a, (int)blockIdx.x); }

// Kernel-argument prologue.  A launch of these latency-bound layers is a chain of dependent memory round trips, and
// hipcc places each kernarg s_load right before its first use -- behind branches and behind the previous
// s_waitcnt -- so a kernel paid 4-6 sequential scalar round trips before its first tile load.  kpin() forces a
// value into SGPRs at the point of the call: calling it for every field the prologue needs, straight after entry,
// issues all their s_loads as one batch behind ONE lgkmcnt wait.
template <typename T>
__device__ __forceinline__ void kpin(T& v) {
  asm volatile("" : "+s"(v));
}
// Pointers are pinned as global-address-space pointers and cast back, so the loads through them stay global_ /
// s_load (not flat_) instructions.
template <typename T>
__device__ __forceinline__ void kpin(T*& p) {
  auto g = (__attribute__((address_space(1))) T*)p;
  asm volatile("" : "+s"(g));
  p = (T*)g;
}

__device__ __forceinline__ const float* stats_row(const float* base, int slot) {
  return base + (long)slot * NREP * 128;
}

// Sum the NREP replicas: returns (sum, sumsq) of channel c.
__device__ __forceinline__ void stats_sum(const float* row, int c, float& s, float& q) {
  s = 0.f;
  q = 0.f;
#pragma unroll
  for (int r = 0; r < NREP; ++r) {
    s += row[r * 128 + c];
    q += row[r * 128 + 64 + c];
  }
}

// Forward BN coefficients: y = x*scale + shift ; also mean / inv-std.
__device__ __forceinline__ void bn_fwd_coef(const float* st, float n, float gamma, float beta, int c, float& scale,
                                            float& shift, float& mean, float& inv) {
  float s, q;
  stats_sum(st, c, s, q);
  mean = s / n;
  float var = fmaxf(q / n - mean * mean, 0.f);
  inv = rsqrtf(var + BN_EPS);
  scale = gamma * inv;
  shift = beta - mean * scale;
}

// Backward BN apply: dh = A*dz + B*h + C  (training-mode BN gradient).
__device__ __forceinline__ void bn_bwd_coef(const float* stf, const float* stb, float n, float gamma, int c, float& A,
                                            float& B, float& C) {
  float scale, shift, mean, inv;
  bn_fwd_coef(stf, n, gamma, 0.f, c, scale, shift, mean, inv);
  float sdz, sdzx;
  stats_sum(stb, c, sdz, sdzx);
  float mdz = sdz / n, mdzx = sdzx / n;
  A = scale;
  B = -scale * inv * mdzx;
  C = -scale * mdz + scale * inv * mean * mdzx;
}

// LDS tiles are [rows][cols][cpad<C>()] bf16: the pixel pitch is picked per channel count so that the
// MFMA operand gathers (ds_read_b128 of 16 consecutive pixels per lane group), the wgrad transposed reads and
// the staging stores hit distinct banks under gfx950's lane grouping; every operand address stays an affine
// function of the pixel index (no swizzle arithmetic in the inner loops).
template <int C>
__host__ __device__ constexpr int cpad() {
  // pixel pitch in bf16: chosen with the gfx950 LDS lane-group banking of ds_read_b128 (4 x 16 lanes) /
  // ds_read_b64_tr_b16 / ds_write_b128 for the tiles' access patterns (tools/lds_banks.py): 16 -> no pad,
  // 32 -> +16, 64 -> +16 (the uniform +8 pad left 2-3-way conflicts on the MFMA operand gathers)
  return C == 16 ? 16 : C == 32 ? 48 : C == 64 ? 80 : C + 8;
}

// LDS row pitch (pixels) of the stage kernels' [RT][WP][CP] tiles (conv_fwd_s1, fused / dual backward).  C = 64
// (W = 8): a 16-pixel MFMA operand gather spans two image rows; with a 16-pixel row pitch the two rows land
// in disjoint bank halves of the ds_read_b128 lane groups (4 instead of 8 cycles per gather, tools/lds_banks.py;
// the extra 6 columns are never staged).  Measured: no step-time change at pop 1 / pop 8 (these kernels wait on
// global memory, not LDS; profiles/r2_wp64_ab.log), so the dense pitch (10) stays the default.
#ifndef DTF_WP64
#define DTF_WP64 10
#endif
template <int C>
__host__ __device__ constexpr int wpitch() {
  return C == 64 ? DTF_WP64 : 512 / C + 2;
}

// Forward (conv_fwd_s1) pitch.  C = 16: the unpadded pitch (16) -- the +8 pad of rounds 2-4 cost 3.6 extra bank
// cycles per ds_read_b128 operand gather (tools/lds_banks.py: 7.6 vs 4.4 cycles, 373 SQ_LDS_BANK_CONFLICT per
// wave); round 5 A/B: pop 1 1.016 -> 1.011 ms, pop 8 equal (profiles/r5_pitch_ab.log).  C = 64 keeps WP = 10
// (DTF_WP64): WP = 16 removes its 4-cycle conflict per gather too but costs LDS (occupancy) and measured +0.5 %.
#ifndef DTF_CPF16
#define DTF_CPF16 16
#endif
template <int C>
__host__ __device__ constexpr int cpad_fwd() {
  return C == 16 ? DTF_CPF16 : cpad<C>();
}

template <int C>
__device__ __forceinline__ int lds_off(int r, int col, int wp, int chunk) {
  return (r * wp + col) * cpad<C>() + (chunk << 3);
}

// Stage a [rows_in][wp][C] tile starting at global row gy0 / col gx0 (halo -> 0).
// MODE 0: copy, 1: relu(x*c0+c1), 2: c0*x + c1*x2 + c2 (BN backward apply).
template <int C, int MODE>
__device__ __forceinline__ void stage_tile(bf16_t* __restrict__ tile, const bf16_t* __restrict__ src,
                                           const bf16_t* __restrict__ src2, int gy0, int rows_in, int gx0, int wp,
                                           int H, int W, const float* __restrict__ coef) {
  constexpr int NCH = C / 8;
  const int total = rows_in * wp * NCH;
  for (int idx = threadIdx.x; idx < total; idx += blockDim.x) {
    const int chunk = idx % NCH;
    const int pc = idx / NCH;
    const int col = pc % wp;
    const int r = pc / wp;
    const int gy = gy0 + r, gx = gx0 + col;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (gy >= 0 && gy < H && gx >= 0 && gx < W) {
      const long off = ((long)gy * W + gx) * C + chunk * 8;
      v = *reinterpret_cast<const uint4*>(src + off);
      if constexpr (MODE != 0) {
        uint4 v2 = make_uint4(0, 0, 0, 0);
        if constexpr (MODE == 2) v2 = *reinterpret_cast<const uint4*>(src2 + off);
        uint32_t w32[4] = {v.x, v.y, v.z, v.w};
        uint32_t h32[4] = {v2.x, v2.y, v2.z, v2.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = chunk * 8 + 2 * j;
          float a0 = bf2f((bf16_t)(w32[j] & 0xffff)), a1 = bf2f((bf16_t)(w32[j] >> 16));
          if constexpr (MODE == 1) {
            a0 = fmaxf(a0 * coef[c] + coef[64 + c], 0.f);
            a1 = fmaxf(a1 * coef[c + 1] + coef[64 + c + 1], 0.f);
          } else {
            float h0 = bf2f((bf16_t)(h32[j] & 0xffff)), h1 = bf2f((bf16_t)(h32[j] >> 16));
            a0 = coef[c] * a0 + coef[64 + c] * h0 + coef[128 + c];
            a1 = coef[c + 1] * a1 + coef[64 + c + 1] * h1 + coef[128 + c + 1];
          }
          w32[j] = pack2bf(a0, a1);
        }
        v = make_uint4(w32[0], w32[1], w32[2], w32[3]);
      }
    }
    *reinterpret_cast<uint4*>(tile + lds_off<C>(r, col, wp, chunk)) = v;
  }
}

// Register-staged tile staging for double buffering.  The tile geometry (rows,
// columns, halo) is identical for every iteration of a workgroup, so each thread's
// chunk -> (tile row, LDS offset, in-row global offset) mapping is computed once
// (TileDesc) and an iteration only adds its first global row: no integer division
// in the steady state.  tile_load issues the 16-byte global loads into registers;
// tile_store applies the transform (BN+ReLU / BN-backward) and writes LDS.
// Chunks beyond MAXC*blockDim fall back to synchronous staging in tile_store.
template <int C, int MAXC>
struct TileDesc {
  int loff[MAXC];  // LDS element offset, -1: slot unused
  int r[MAXC];     // tile row
  int gxo[MAXC];   // gx*C + chunk*8 inside the image row, -1: halo column
  int total, rows_in, gx0, wp;
};

template <int C, int MAXC>
__device__ __forceinline__ void tile_desc_init(TileDesc<C, MAXC>& d, int rows_in, int gx0, int wp, int W) {
  constexpr int NCH = C / 8;
  d.total = rows_in * wp * NCH;
  d.rows_in = rows_in;
  d.gx0 = gx0;
  d.wp = wp;
#pragma unroll
  for (int j = 0; j < MAXC; ++j) {
    const int idx = threadIdx.x + j * blockDim.x;
    d.loff[j] = -1;
    d.r[j] = 0;
    d.gxo[j] = -1;
    if (idx < d.total) {
      const int chunk = idx % NCH;
      const int pc = idx / NCH;
      const int col = pc % wp;
      const int r = pc / wp;
      const int gx = gx0 + col;
      d.loff[j] = lds_off<C>(r, col, wp, chunk);
      d.r[j] = r;
      d.gxo[j] = (gx >= 0 && gx < W) ? gx * C + chunk * 8 : -1;
    }
  }
}

template <int C, int MODE, int MAXC>
struct TileRegs {
  uint4 v[MAXC];
  uint4 v2[MODE == 2 ? MAXC : 1];
  unsigned ok;  // bit j: chunk j is inside the image (else it stages zeros)
};

// Branch-free: every slot issues its load (an out-of-image chunk reads the image's
// first chunk and is zeroed at store time), so the compiler sees a fixed number of
// outstanding loads and can wait for the epilogue operands with a counted vmcnt
// instead of draining this prefetch.
template <int C, int MODE, int MAXC>
__device__ __forceinline__ void tile_load(TileRegs<C, MODE, MAXC>& R, const TileDesc<C, MAXC>& d,
                                          const bf16_t* __restrict__ src, const bf16_t* __restrict__ src2, int gy0,
                                          int H, int W) {
  const long row = (long)W * C;
  R.ok = 0;
#pragma unroll
  for (int j = 0; j < MAXC; ++j) {
    const int gy = gy0 + d.r[j];
    const bool ok = (d.gxo[j] >= 0) & (gy >= 0) & (gy < H);
    const long off = ok ? gy * row + d.gxo[j] : 0;
    R.ok |= (ok ? 1u : 0u) << j;
    R.v[j] = *reinterpret_cast<const uint4*>(src + off);
    if constexpr (MODE == 2) R.v2[j] = *reinterpret_cast<const uint4*>(src2 + off);
  }
}

template <int MODE>
__device__ __forceinline__ uint4 xform8(uint4 v, uint4 v2, int c0, const float* __restrict__ coef);

template <int MODE>
__device__ __forceinline__ uint4 transform8(uint4 v, uint4 v2, int c0, const float* __restrict__ coef) {
  if constexpr (MODE == 0) return v;
  // DTF_TRANSFORM8_PK: the packed two-channel form (v_pk_fma_f32 on 8-byte coefficient pairs, xform8) instead of
  // per-element f32 math and 4-byte coefficient reads
  if constexpr (DTF_TRANSFORM8_PK) return xform8<MODE>(v, v2, c0, coef);
  uint32_t w32[4] = {v.x, v.y, v.z, v.w};
  uint32_t h32[4] = {v2.x, v2.y, v2.z, v2.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = c0 + 2 * j;
    float a0 = lo2f(w32[j]), a1 = hi2f(w32[j]);
    if constexpr (MODE == 1) {
      a0 = fmaxf(a0 * coef[c] + coef[64 + c], 0.f);
      a1 = fmaxf(a1 * coef[c + 1] + coef[64 + c + 1], 0.f);
    } else {
      const float h0 = lo2f(h32[j]), h1 = hi2f(h32[j]);
      a0 = coef[c] * a0 + coef[64 + c] * h0 + coef[128 + c];
      a1 = coef[c + 1] * a1 + coef[64 + c + 1] * h1 + coef[128 + c + 1];
    }
    w32[j] = pack2bf(a0, a1);
  }
  return make_uint4(w32[0], w32[1], w32[2], w32[3]);
}

template <int C, int MODE, int MAXC>
__device__ __forceinline__ void tile_store(bf16_t* __restrict__ tile, const TileRegs<C, MODE, MAXC>& R,
                                           const TileDesc<C, MAXC>& d, const bf16_t* __restrict__ src,
                                           const bf16_t* __restrict__ src2, int gy0, int H, int W,
                                           const float* __restrict__ coef) {
  constexpr int NCH = C / 8;
#pragma unroll
  for (int j = 0; j < MAXC; ++j) {
    if (d.loff[j] >= 0) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if ((R.ok >> j) & 1u) v = transform8<MODE>(R.v[j], MODE == 2 ? R.v2[j] : R.v[j], d.gxo[j] & (C - 1), coef);
      *reinterpret_cast<uint4*>(tile + d.loff[j]) = v;
    }
  }
  for (int idx = threadIdx.x + MAXC * blockDim.x; idx < d.total; idx += blockDim.x) {  // overflow (rare)
    const int chunk = idx % NCH;
    const int pc = idx / NCH;
    const int col = pc % d.wp;
    const int r = pc / d.wp;
    const int gy = gy0 + r, gx = d.gx0 + col;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (gy >= 0 && gy < H && gx >= 0 && gx < W) {
      const long off = ((long)gy * W + gx) * C + chunk * 8;
      uint4 v2 = v;
      v = *reinterpret_cast<const uint4*>(src + off);
      if constexpr (MODE == 2) v2 = *reinterpret_cast<const uint4*>(src2 + off);
      v = transform8<MODE>(v, v2, chunk * 8, coef);
    }
    *reinterpret_cast<uint4*>(tile + lds_off<C>(r, col, d.wp, chunk)) = v;
  }
}

// Per-channel transform coefficients into coef[0..191] for MODE 1 / 2.
template <int C, int MODE>
__device__ __forceinline__ void make_coef(float* coef, const ConvArgs& a, int slot, float n, const float* st_f,
                                          const float* st_b, int g_off, int b_off) {
  if constexpr (MODE == 0) return;
  const int c = threadIdx.x;
  if (c < C) {
    const float* prow = a.params + (long)slot * a.p_mstride;
    if constexpr (MODE == 1) {
      float scale, shift, mean, inv;
      bn_fwd_coef(stats_row(st_f, slot), n, prow[g_off + c], prow[b_off + c], c, scale, shift, mean, inv);
      coef[c] = scale;
      coef[64 + c] = shift;
    } else {
      float A, B, Cc;
      bn_bwd_coef(stats_row(st_f, slot), stats_row(st_b, slot), n, prow[g_off + c], c, A, B, Cc);
      coef[c] = A;
      coef[64 + c] = B;
      coef[128 + c] = Cc;
    }
  }
}

// Two-phase BN coefficients: coef_issue loads the replicated statistics + gamma/beta into registers at the top of a
// kernel (before its tile and weight loads), coef_finish derives the coefficients once they have arrived -- the
// in-order vmcnt wait then covers only the statistics, the tile / weight loads stay in flight behind them.
// MODE 1: forward scale/shift (st_f, gamma, beta); MODE 2/3: backward A, B, C (st_f, st_b, gamma).
// With many replicas (deterministic builds: DTF_NREP = 64, one per workgroup of a member) the loads are summed as
// they are issued (in replica order) instead of being held in registers.
constexpr int CREP = NREP <= 8 ? NREP : 1;
template <int MODE>
struct CoefLd {
  float fs[CREP], fq[CREP], bs[MODE >= 2 ? CREP : 1], bq[MODE >= 2 ? CREP : 1];
  float g, b;
};

template <int C, int MODE>
__device__ __forceinline__ void coef_issue(CoefLd<MODE>& L, const float* params, long p_mstride, int slot,
                                           const float* st_f, const float* st_b, int g_off, int b_off) {
  if constexpr (MODE == 0) return;
  static_assert(C <= 64, "the coefficients' consumers are the threads c < C of wave 0");
#if DTF_COEF_W0
  // only wave 0 loads (its threads c < C are the only consumers): a wave-uniform scalar branch -- the other waves
  // issued 3 x the statistics loads for nothing, all to the same few L2 lines as every other workgroup's
  if (__builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6) != 0) return;
#endif
  // branch-free within the wave: every lane loads (channel threadIdx % C; the copies hit the same lines), so no
  // exec-mask branch makes the compiler consume -- and wait for -- the first statistics before the tile loads
  const int c = (int)threadIdx.x & (C - 1);
#if DTF_COEF_SPLIT
  if constexpr ((CREP == NREP || CREP == 1) && C < 64) {
    // the wave's 64 / C lane groups split the replicas (coef_reduce sums the groups).  Many replicas (CREP = 1,
    // the deterministic build's 64): each group sums its NREP / G replicas in replica order as they arrive -- a
    // fixed order, so the coefficients stay bitwise reproducible -- and a lane issues G x fewer loads (C = 16: 64
    // instead of 256 statistics loads in the prologue of every launch)
    constexpr int G = 64 / C, RJ = NREP / G;
    static_assert(NREP % G == 0, "replicas split evenly over the lane groups");
    const int grp = ((int)threadIdx.x & 63) / C;
    const float* rf = stats_row(st_f, slot) + c + grp * 128;
    if constexpr (CREP == 1) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int j = 0; j < RJ; ++j) {
        a += rf[j * G * 128];
        b += rf[j * G * 128 + 64];
      }
      L.fs[0] = a;
      L.fq[0] = b;
    } else {
#pragma unroll
      for (int j = 0; j < CREP; ++j) {
        L.fs[j] = j < RJ ? rf[j * G * 128] : 0.f;
        L.fq[j] = j < RJ ? rf[j * G * 128 + 64] : 0.f;
      }
    }
    if constexpr (MODE >= 2) {
      const float* rb = stats_row(st_b, slot) + c + grp * 128;
      if constexpr (CREP == 1) {
        float a = 0.f, b = 0.f;
#pragma unroll
        for (int j = 0; j < RJ; ++j) {
          a += rb[j * G * 128];
          b += rb[j * G * 128 + 64];
        }
        L.bs[0] = a;
        L.bq[0] = b;
      } else {
#pragma unroll
        for (int j = 0; j < CREP; ++j) {
          L.bs[j] = j < RJ ? rb[j * G * 128] : 0.f;
          L.bq[j] = j < RJ ? rb[j * G * 128 + 64] : 0.f;
        }
      }
    }
    const float* prow = params + (long)slot * p_mstride;
    L.g = prow[g_off + c];
    if constexpr (MODE == 1) L.b = prow[b_off + c];
    return;
  }
#endif
  {
    const float* rf = stats_row(st_f, slot) + c;
    if constexpr (CREP == NREP) {
#pragma unroll
      for (int r = 0; r < NREP; ++r) {
        L.fs[r] = rf[r * 128];
        L.fq[r] = rf[r * 128 + 64];
      }
    } else {
      L.fs[0] = L.fq[0] = 0.f;
      for (int r = 0; r < NREP; ++r) {
        L.fs[0] += rf[r * 128];
        L.fq[0] += rf[r * 128 + 64];
      }
    }
    if constexpr (MODE >= 2) {
      const float* rb = stats_row(st_b, slot) + c;
      if constexpr (CREP == NREP) {
#pragma unroll
        for (int r = 0; r < NREP; ++r) {
          L.bs[r] = rb[r * 128];
          L.bq[r] = rb[r * 128 + 64];
        }
      } else {
        L.bs[0] = L.bq[0] = 0.f;
        for (int r = 0; r < NREP; ++r) {
          L.bs[0] += rb[r * 128];
          L.bq[0] += rb[r * 128 + 64];
        }
      }
    }
    const float* prow = params + (long)slot * p_mstride;
    L.g = prow[g_off + c];
    if constexpr (MODE == 1) L.b = prow[b_off + c];
  }
}

// DTF_COEF_SPLIT: sum the lane groups' replica partials (called by every lane of wave 0, outside divergent code)
template <int C, int MODE>
__device__ __forceinline__ void coef_reduce(CoefLd<MODE>& L) {
#if DTF_COEF_SPLIT
  if constexpr (MODE != 0 && (CREP == NREP || CREP == 1) && C < 64) {
    float a = 0.f, b = 0.f, d = 0.f, e = 0.f;
#pragma unroll
    for (int j = 0; j < CREP; ++j) {
      a += L.fs[j];
      b += L.fq[j];
      if constexpr (MODE >= 2) {
        d += L.bs[j];
        e += L.bq[j];
      }
    }
#pragma unroll
    for (int off = C; off < 64; off *= 2) {
      a += __shfl_xor(a, off);
      b += __shfl_xor(b, off);
      if constexpr (MODE >= 2) {
        d += __shfl_xor(d, off);
        e += __shfl_xor(e, off);
      }
    }
#pragma unroll
    for (int j = 0; j < CREP; ++j) {
      L.fs[j] = j == 0 ? a : 0.f;
      L.fq[j] = j == 0 ? b : 0.f;
      if constexpr (MODE >= 2) {
        L.bs[j] = j == 0 ? d : 0.f;
        L.bq[j] = j == 0 ? e : 0.f;
      }
    }
  }
#endif
}

// mean / inv-std of the forward statistics in L
template <int MODE>
__device__ __forceinline__ void coef_moments(const CoefLd<MODE>& L, float n, float& mean, float& inv) {
  float s = 0.f, q = 0.f;
#pragma unroll
  for (int r = 0; r < CREP; ++r) {
    s += L.fs[r];
    q += L.fq[r];
  }
  mean = s / n;
  inv = rsqrtf(fmaxf(q / n - mean * mean, 0.f) + BN_EPS);
}

template <int C, int MODE>
__device__ __forceinline__ void coef_finish(float* coef, const CoefLd<MODE>& L, float n) {
  if constexpr (MODE == 0) return;
  const int c = threadIdx.x;
  if (c < C) {
    float mean, inv;
    coef_moments<MODE>(L, n, mean, inv);
    const float scale = L.g * inv;
    if constexpr (MODE == 1) {
      coef[c] = scale;
      coef[64 + c] = L.b - mean * scale;
    } else {
      float sdz = 0.f, sdzx = 0.f;
#pragma unroll
      for (int r = 0; r < CREP; ++r) {
        sdz += L.bs[r];
        sdzx += L.bq[r];
      }
      const float mdz = sdz / n, mdzx = sdzx / n;
      coef[c] = scale;
      coef[64 + c] = -scale * inv * mdzx;
      coef[128 + c] = -scale * mdz + scale * inv * mean * mdzx;
    }
  }
}

__device__ __forceinline__ f32x4_t mfma16(const bf16x8_t& a, const bf16x8_t& b, const f32x4_t& c) {
  return dtf_mfma16(a, b, c);
}

// Reduce per-lane partial channel sums (4 channels per lane, 16 lanes share them)
// into LDS accumulators acc_lds[2][64] (sum, second moment).
__device__ __forceinline__ void reduce_stats_to_lds(float* acc_lds, const float (&s)[4], const float (&q)[4], int ch0,
                                                    int lane) {
  float ss[4], qq[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float a = s[r], b = q[r];
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      a += __shfl_xor(a, o, 64);
      b += __shfl_xor(b, o, 64);
    }
    ss[r] = a;
    qq[r] = b;
  }
#ifdef DTF_DETERMINISTIC
  // waves that share channels add in wave order (the LDS float adds are then order-fixed); callers invoke this
  // with workgroup-uniform control flow
  const int wv = (int)threadIdx.x >> 6;
  for (int w = 0; w < (int)blockDim.x / 64; ++w) {
    if (wv == w && (lane & 15) == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        acc_lds[ch0 + r] += ss[r];
        acc_lds[64 + ch0 + r] += qq[r];
      }
    }
    __syncthreads();
  }
#else
  if ((lane & 15) == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      atomicAdd(&acc_lds[ch0 + r], ss[r]);
      atomicAdd(&acc_lds[64 + ch0 + r], qq[r]);
    }
  }
#endif
}

__device__ __forceinline__ void flush_stats_r(float* st_out, const float* acc_lds, int slot, int nch, int rep) {
  const int t = threadIdx.x;
  if (t < 2 * nch) {
    const int which = t / nch, c = t % nch;
    float* row = st_out + (long)slot * NREP * 128 + (rep & (NREP - 1)) * 128;
    atomicAdd(&row[which * 64 + c], acc_lds[which * 64 + c]);
  }
}

__device__ __forceinline__ void flush_stats(float* st_out, const float* acc_lds, int slot, int nch) {
  flush_stats_r(st_out, acc_lds, slot, nch, (int)blockIdx.x);
}

// Packed-math helpers (v_pk_fma_f32 / v_cvt_pk_bf16_f32 / v_pk_max_i16): two channels per VALU op.
typedef short s16x2_t __attribute__((ext_vector_type(2)));

// (f32x2_t and pk2 -- v_cvt_pk_bf16_f32, or the fp16 pack of the half build -- are in common.h)
__device__ __forceinline__ f32x2_t unpk2(uint32_t w) { return (f32x2_t){lo2f(w), hi2f(w)}; }
// ReLU on two packed bf16: as int16, every negative bf16 (sign bit set) is < 0
__device__ __forceinline__ uint32_t relu_pk2(uint32_t w) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s16x2_t, w), (s16x2_t){0, 0}));
}
__device__ __forceinline__ f32x2_t lds2(const float* p) { return *reinterpret_cast<const f32x2_t*>(p); }

// Activation outputs of the stage kernels are stored write-through (sc1): the line leaves the XCD's L2 while the
// kernel still runs, so the dependent kernel boundary does not first write back megabytes of dirty L2 lines
// (MI355X_MICROARCH.md, price row "boundary": + B / 6 TB/s for B dirty bytes).  The consumer is always the next
// launch, which reads from MALL/HBM either way (its L2 is not coherent with the producer XCD's).
#ifndef DTF_WT_ACT
#define DTF_WT_ACT 1
#endif
typedef __attribute__((address_space(1))) unsigned long long gu64_t;
__device__ __forceinline__ void st_act8(bf16_t* p, uint2 v) {
#if DTF_WT_ACT
  __hip_atomic_store((gu64_t*)p, __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
#else
  *reinterpret_cast<uint2*>(p) = v;
#endif
}

// T(8 channels c0..c0+7): MODE 1 relu(x*coef[c] + coef[64+c]); MODE 2 coef[c]*x + coef[64+c]*h + coef[128+c]
template <int MODE>
__device__ __forceinline__ uint4 xform8(uint4 v, uint4 v2, int c0, const float* __restrict__ coef) {
  if constexpr (MODE == 0) return v;
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
  const uint32_t h[4] = {v2.x, v2.y, v2.z, v2.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = c0 + 2 * j;
    const f32x2_t x = unpk2(w[j]);
    if constexpr (MODE == 1) {
      w[j] = relu_pk2(pk2(x * lds2(coef + c) + lds2(coef + 64 + c)));
    } else {
      w[j] = pk2(x * lds2(coef + c) + unpk2(h[j]) * lds2(coef + 64 + c) + lds2(coef + 128 + c));
    }
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// MODE 2: coef[c]*x + coef[64+c]*h + coef[128+c]; MODE 3: the same + r (residual-stream gradient)
template <int MODE>
__device__ __forceinline__ uint4 xform8r(uint4 v, uint4 v2, uint4 v3, int c0, const float* __restrict__ coef) {
  static_assert(MODE == 2 || MODE == 3, "BN-backward staging only");
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
  const uint32_t h[4] = {v2.x, v2.y, v2.z, v2.w};
  const uint32_t r[4] = {v3.x, v3.y, v3.z, v3.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = c0 + 2 * j;
    f32x2_t t = unpk2(w[j]) * lds2(coef + c) + unpk2(h[j]) * lds2(coef + 64 + c) + lds2(coef + 128 + c);
    if constexpr (MODE == 3) t += unpk2(r[j]);
    w[j] = pk2(t);
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// Compile-time tile geometry for a [RT][WP][C] (+8 pad per pixel) LDS tile of rows gy0..gy0+RT-1 and columns
// -1..W of an H x W x C image.  Each thread owns MAXC 16-byte chunk slots (always the same 8 channels, since
// 256 % (C/8) == 0); per slot: LDS offset, in-band global offset, and three bit masks (column/slot valid,
// top halo row, bottom halo row) so an iteration only adds its band's row offset.  Inactive slots stage zeros
// into pixel 0's pad lanes (never read), keeping load/store branch-free.
template <int C, int RT, int W, int H, int CPV = cpad<C>(), int WPV = W + 2>
struct Stage {
  static constexpr int WD = W + 2, WP = WPV, CP = CPV, NCH = C / 8, ROW = W * C;  // WD staged columns, WP pitch
  static_assert(WP >= WD, "row pitch covers the staged columns");
  static constexpr int TOTAL = RT * WD * NCH, MAXC = (TOTAL + 255) / 256;
  int loff[MAXC];
  int goff[MAXC];
  int roff[MAXC];  // band-interior chunks: offset in an unhaloed [RT-2][W][CP] tile (store_raw)
  unsigned okm, top, bot;
  int c0;
  __device__ __forceinline__ void init() {
    c0 = (threadIdx.x % NCH) * 8;
    okm = top = bot = 0;
#pragma unroll
    for (int j = 0; j < MAXC; ++j) {
      const int idx = threadIdx.x + 256 * j;
      const int pc = idx / NCH, col = pc % WD, r = pc / WD;
      const bool act = idx < TOTAL;
      loff[j] = act ? (r * WP + col) * CP + c0 : RT * WP * CP;  // inactive: the 8-element slack past the tile
      roff[j] = ((r - 1) * W + (col - 1)) * CP + c0;
      goff[j] = (r * ROW + (col - 1) * C + c0) * 2;  // bytes
      if (act && col >= 1 && col <= W) okm |= 1u << j;
      if (r == 0) top |= 1u << j;
      if (r == RT - 1) bot |= 1u << j;
    }
  }
  // first tile row = gy0; rows outside [0, H) are zero
  __device__ __forceinline__ unsigned mask(int gy0) const {
    unsigned m = okm;
    if (gy0 < 0) m &= ~top;
    if (gy0 + RT > H) m &= ~bot;
    return m;
  }
  template <int MODE>
  __device__ __forceinline__ void load(uint4 (&v)[MAXC], uint4 (&v2)[MAXC], unsigned m, const bf16_t* img,
                                       const bf16_t* img2, int gy0) const {
    // byte offsets in 32 bits: uniform base (SGPR) + lane offset -> saddr global loads
    const int rb = gy0 * ROW * 2;
#pragma unroll
    for (int j = 0; j < MAXC; ++j) {
      const uint32_t off = ((m >> j) & 1u) ? (uint32_t)(rb + goff[j]) : 0u;
      v[j] = *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(img) + off);
      if constexpr (MODE >= 2) v2[j] = *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(img2) + off);
    }
  }
  template <int MODE>
  __device__ __forceinline__ void store(bf16_t* buf, const uint4 (&v)[MAXC], const uint4 (&v2)[MAXC], unsigned m,
                                        const float* coef) const {
#pragma unroll
    for (int j = 0; j < MAXC; ++j) {
      uint4 t = make_uint4(0, 0, 0, 0);
      if ((m >> j) & 1u) t = xform8<MODE>(v[j], v2[j], c0, coef);
      *reinterpret_cast<uint4*>(buf + loff[j]) = t;
    }
  }
  // MODE 1 with the thread's 8 scale / shift coefficients in registers (its channels c0..c0+7 are the same for
  // every slot): no LDS coefficient reads per staged band
  __device__ __forceinline__ void load_coef1(float (&sc)[8], float (&sh)[8], const float* coef) const {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      sc[i] = coef[c0 + i];
      sh[i] = coef[64 + c0 + i];
    }
  }
  __device__ __forceinline__ void store1r(bf16_t* buf, const uint4 (&v)[MAXC], unsigned m, const float (&sc)[8],
                                         const float (&sh)[8]) const {
#pragma unroll
    for (int j = 0; j < MAXC; ++j) {
      uint4 t = make_uint4(0, 0, 0, 0);
      if ((m >> j) & 1u) {
        uint32_t w[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
        for (int q = 0; q < 4; ++q)
          w[q] = relu_pk2(pk2(unpk2(w[q]) * (f32x2_t){sc[2 * q], sc[2 * q + 1]} +
                              (f32x2_t){sh[2 * q], sh[2 * q + 1]}));
        t = make_uint4(w[0], w[1], w[2], w[3]);
      }
      *reinterpret_cast<uint4*>(buf + loff[j]) = t;
    }
  }
  // MODE 2 / 3 coefficients of the thread's 8 channels (A, B, C of xform8r) in registers
  __device__ __forceinline__ void load_coef3(float (&ka)[8], float (&kb)[8], float (&kc)[8], const float* coef) const {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      ka[i] = coef[c0 + i];
      kb[i] = coef[64 + c0 + i];
      kc[i] = coef[128 + c0 + i];
    }
  }
  // The untransformed band-interior chunks (tile rows 1..RT-2, image columns) into `raw` ([RT-2][W][CP]).
  __device__ __forceinline__ void store_raw(bf16_t* raw, const uint4 (&v)[MAXC], unsigned m) const {
    const unsigned interior = m & ~top & ~bot;
#pragma unroll
    for (int j = 0; j < MAXC; ++j)
      if ((interior >> j) & 1u) *reinterpret_cast<uint4*>(raw + roff[j]) = v[j];
  }
  // MODE 2 / 3 (BN-backward apply [+ residual v3]) staging that also writes the transformed band-interior
  // chunks (tile rows 1..RT-2, image columns) to `out` (the image base; null: LDS only).
  // (KR: the coefficients come from ka / kb / kc -- load_coef3 -- instead of LDS)
  template <int MODE, bool KR = false>
  __device__ __forceinline__ void store_x(bf16_t* buf, const uint4 (&v)[MAXC], const uint4 (&v2)[MAXC],
                                          const uint4 (&v3)[MAXC], unsigned m, const float* coef, bf16_t* out,
                                          int gy0, const float* ka = nullptr, const float* kb = nullptr,
                                          const float* kc = nullptr) const {
    const unsigned interior = m & ~top & ~bot;
    const int rb = gy0 * ROW * 2;
#if DTF_WT_ACT
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(out, 0, H * ROW * 2, 0x00020000);  // one image
#endif
#pragma unroll
    for (int j = 0; j < MAXC; ++j) {
      uint4 t = make_uint4(0, 0, 0, 0);
      if ((m >> j) & 1u) {
        if constexpr (KR) {
          const uint32_t w[4] = {v[j].x, v[j].y, v[j].z, v[j].w}, h[4] = {v2[j].x, v2[j].y, v2[j].z, v2[j].w},
                         r[4] = {v3[j].x, v3[j].y, v3[j].z, v3[j].w};
          uint32_t o[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            f32x2_t u = unpk2(w[q]) * (f32x2_t){ka[2 * q], ka[2 * q + 1]} +
                        unpk2(h[q]) * (f32x2_t){kb[2 * q], kb[2 * q + 1]} + (f32x2_t){kc[2 * q], kc[2 * q + 1]};
            if constexpr (MODE == 3) u += unpk2(r[q]);
            o[q] = pk2(u);
          }
          t = make_uint4(o[0], o[1], o[2], o[3]);
        } else {
          t = xform8r<MODE>(v[j], v2[j], v3[j], c0, coef);
        }
      }
      *reinterpret_cast<uint4*>(buf + loff[j]) = t;
      if (out != nullptr && ((interior >> j) & 1u)) {
#if DTF_WT_ACT
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, t), rsrc, rb + goff[j], 0, 16);  // sc1
#else
        *reinterpret_cast<uint4*>(reinterpret_cast<char*>(out) + (uint32_t)(rb + goff[j])) = t;
#endif
      }
    }
  }
};

// --------------------------------------------------------------------------------- forward

// Work items are (it0, nit, -, slot): the workgroup processes iterations
// it0 .. it0+nit-1 of the flattened (image, band) sequence of ONE member; weights
// are loaded into registers once, and the next iteration's tile is prefetched
// into registers (tile_load) while the MFMAs of the current one run, then
// written to the other LDS buffer (double buffering).

constexpr int MAXT = 4;  // output tiles per wave per iteration (host-checked)

template <int CIN, int COUT, int S, int K, int MODE_IN, bool RESID, bool STATS>
__global__ __launch_bounds__(256) void conv_fwd_kernel(ConvArgs a) {
  constexpr int NT = COUT / 16;
  constexpr int WPT = 4 / NT;
  constexpr int KTOT = K * K * CIN;
  constexpr int KS = (KTOT + 31) / 32;
  constexpr int P = (K - 1) / 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* coef = reinterpret_cast<float*>(smem);          // 192 floats
  float* acc_lds = coef + 192;                           // 128 floats
  bf16_t* tile0 = reinterpret_cast<bf16_t*>(smem + 1280);

  const int4 wk = a.work[blockIdx.x];
  DTF_WG_CHECK(wk.x >= 0 && wk.y >= 0 && wk.w >= 0 && wk.z >= 0 && a.Hi > 0 && a.Wi > 0 && a.rows > 0);
  const int it0 = wk.x, nit = wk.y, slot = wk.w;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const float n_in = a.cnt[slot] * (float)(a.Hi * a.Wi);
  make_coef<CIN, MODE_IN>(coef, a, slot, n_in, a.st_in, a.st_in_b, a.in_gamma, a.in_beta);
  if (STATS && threadIdx.x < 128) acc_lds[threadIdx.x] = 0.f;

  const int ct = wave % NT;
  bf16x8_t afr[KS];
  {
    const bf16_t* wb = a.w + (long)slot * a.w_mstride + a.w_off + (long)(ct * 16 + (lane & 15)) * KTOT;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int k0 = 32 * s + 8 * (lane >> 4);
      bf16x8_t v = {0, 0, 0, 0, 0, 0, 0, 0};
      if (k0 < KTOT) v = *reinterpret_cast<const bf16x8_t*>(wb + k0);
      afr[s] = v;
    }
  }
  const int rows = a.rows;
  const int bands = a.Ho / rows;
  const int rows_in = (rows - 1) * S + K;
  const int wp = a.Wi + 2 * P;
  const int tsz = (rows_in * wp * cpad<CIN>() + 63) & ~63;
#define TILEBUF(i) (tile0 + ((i) & 1) * tsz)
  const int ntiles = rows * a.Wo / 16;
  const long img_elems = (long)a.Hi * a.Wi * CIN;
  int tapoff[KS];  // per-lane LDS offset of each k-step's tap/channel chunk
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k0 = 32 * s + 8 * (lane >> 4);
    const int tap = k0 / CIN, c0 = k0 % CIN;
    tapoff[s] = ((tap / K) * wp + (tap % K)) * cpad<CIN>() + c0;
  }
  float ssum[4] = {0.f, 0.f, 0.f, 0.f}, ssq[4] = {0.f, 0.f, 0.f, 0.f};
  TileRegs<CIN, MODE_IN, 4> rg;
  TileDesc<CIN, 4> td;
  tile_desc_init<CIN, 4>(td, rows_in, -P, wp, a.Wi);
  __syncthreads();  // coefficients
  {
    const int img = it0 / bands, oy0 = (it0 % bands) * rows;
    tile_load<CIN, MODE_IN, 4>(rg, td, a.x + img * img_elems, nullptr, oy0 * S - P, a.Hi, a.Wi);
    tile_store<CIN, MODE_IN, 4>(TILEBUF(0), rg, td, a.x + img * img_elems, nullptr, oy0 * S - P, a.Hi, a.Wi, coef);
  }
  __syncthreads();
  for (int k = 0; k < nit; ++k) {
    const int it = it0 + k;
    const int img = it / bands, oy0 = (it % bands) * rows;
    const bool more = k + 1 < nit;
    const int nimg_ = (it + 1) / bands, noy0 = ((it + 1) % bands) * rows;
    // epilogue operands of every tile of this iteration first, then the next tile's prefetch:
    // the residual wait is a counted vmcnt that leaves the prefetch in flight
    uint2 rres[MAXT];
    if constexpr (RESID) {
#pragma unroll
      for (int i = 0; i < MAXT; ++i) {
        const int t = min(wave / NT + WPT * i, ntiles - 1);
        const int p = t * 16 + (lane & 15);
        const int oy = p / a.Wo, ox = p % a.Wo;
        rres[i] = *reinterpret_cast<const uint2*>(
            a.res + (((long)img * a.Ho + oy0 + oy) * a.Wo + ox) * COUT + ct * 16 + (lane >> 4) * 4);
      }
    }
    if (more) tile_load<CIN, MODE_IN, 4>(rg, td, a.x + nimg_ * img_elems, nullptr, noy0 * S - P, a.Hi, a.Wi);
    const bf16_t* tile = TILEBUF(k);
#pragma unroll
    for (int i = 0; i < MAXT; ++i) {
      const int t = wave / NT + WPT * i;
      if (t >= ntiles) break;
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
      const int p = t * 16 + (lane & 15);
      const int oy = p / a.Wo, ox = p % a.Wo;
      const int co0 = ct * 16 + (lane >> 4) * 4;
      const long o = (((long)img * a.Ho + oy0 + oy) * a.Wo + ox) * COUT + co0;
      uint2 r = make_uint2(0, 0);
      if constexpr (RESID) r = rres[i];
      const bf16_t* tb = tile + (oy * S * wp + ox * S) * cpad<CIN>();
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        bf16x8_t b = {0, 0, 0, 0, 0, 0, 0, 0};
        if (32 * s + 8 * (lane >> 4) < KTOT) b = *reinterpret_cast<const bf16x8_t*>(tb + tapoff[s]);
        acc = mfma16(afr[s], b, acc);
      }
      float v[4] = {acc[0], acc[1], acc[2], acc[3]};
      if constexpr (RESID) {
        v[0] += bf2f((bf16_t)(r.x & 0xffff));
        v[1] += bf2f((bf16_t)(r.x >> 16));
        v[2] += bf2f((bf16_t)(r.y & 0xffff));
        v[3] += bf2f((bf16_t)(r.y >> 16));
      }
      uint2 pk;
      pk.x = pack2bf(v[0], v[1]);
      pk.y = pack2bf(v[2], v[3]);
      st_act8(a.y + o, pk);
      if constexpr (STATS) {
        const float r0 = bf2f((bf16_t)(pk.x & 0xffff)), r1 = bf2f((bf16_t)(pk.x >> 16));
        const float r2 = bf2f((bf16_t)(pk.y & 0xffff)), r3 = bf2f((bf16_t)(pk.y >> 16));
        ssum[0] += r0; ssq[0] += r0 * r0;
        ssum[1] += r1; ssq[1] += r1 * r1;
        ssum[2] += r2; ssq[2] += r2 * r2;
        ssum[3] += r3; ssq[3] += r3 * r3;
      }
    }
    if (more)
      tile_store<CIN, MODE_IN, 4>(TILEBUF(k + 1), rg, td, a.x + nimg_ * img_elems, nullptr, noy0 * S - P, a.Hi,
                                  a.Wi, coef);
    __syncthreads();
  }
  if constexpr (STATS) {
    reduce_stats_to_lds(acc_lds, ssum, ssq, ct * 16 + (lane >> 4) * 4, lane);
    __syncthreads();
    flush_stats(a.st_out, acc_lds, slot, COUT);
  }
}

// Stride-1 3x3 C->C forward of the CIFAR stages (and the stem, C = 16 padded input) with compile-time
// geometry (W = H = 512/C, 8-row bands), uniform-base + 32-bit lane offsets and packed epilogue math
// (same scheme as conv_bwd_fused_kernel).
// single member's 8x8 C = 64 layer (one image per item) launches 256 workgroups instead of 128.
template <int C, int MODE_IN, bool RESID, int ROWS = 8>
__device__ __forceinline__ void conv_fwd_s1_body(const ConvArgs& a, const int bid, char* smem) {
  constexpr int W = 512 / C, H = W, BANDS = H / ROWS;
  constexpr int NT = C / 16, WPT = 4 / NT;  // NT: output-channel tiles
  constexpr int KTOT = 9 * C, KS = (KTOT + 31) / 32;
  constexpr int CP = cpad_fwd<C>(), RT = ROWS + 2, WP = wpitch<C>();
  constexpr int TSZ = (RT * WP * CP + 8 + 63) & ~63;  // + slack for inactive staging slots
  constexpr int NTILES = ROWS * W / 16;
  constexpr int MT = NTILES / WPT;  // output pixel tiles per wave per iteration
  static_assert(NTILES == WPT * MT && MT <= MAXT, "every wave owns MT output tiles");
  constexpr int ROW = W * C, IMG = H * ROW;
  using St = Stage<C, RT, W, H, CP, WP>;
  constexpr int MAXC = St::MAXC;
  constexpr int LMODE = MODE_IN == 0 ? 0 : 1;
  float* coef = reinterpret_cast<float*>(smem);  // 192 floats
  float* acc_lds = coef + 192;                   // 128 floats
  bf16_t* tile0 = reinterpret_cast<bf16_t*>(smem + 1280);
#define SBUF(i) (tile0 + ((i) & 1) * TSZ)
  STAMP_DECL
  STAMP(0);
  // every kernarg field of the prologue in one s_load batch (kpin)
  int u_items = a.u_items, u_chunk = a.u_chunk, u_per = a.u_per, in_gamma = a.in_gamma, in_beta = a.in_beta;
  const int4* work = a.work;
  const float *params = a.params, *st_in = a.st_in, *cnt = a.cnt;
  long p_mstride = a.p_mstride, w_mstride = a.w_mstride, w_off = a.w_off;
  const bf16_t *xin = a.x, *wgt = a.w, *res = a.res;
  kpin(u_items), kpin(u_chunk), kpin(u_per), kpin(in_gamma), kpin(in_beta), kpin(work), kpin(params), kpin(st_in);
  kpin(cnt), kpin(p_mstride), kpin(w_mstride), kpin(w_off), kpin(xin), kpin(wgt), kpin(res);
  int4 wk;
  if (u_items > 0) {
    const int b = bid, m = b / u_items, k = b - m * u_items, it0_ = k * u_chunk;
    wk = make_int4(m * u_per + it0_, min(u_chunk, u_per - it0_), 0, m);
  } else {
    wk = work[bid];
    wk = make_int4(__builtin_amdgcn_readfirstlane(wk.x), __builtin_amdgcn_readfirstlane(wk.y),
                   __builtin_amdgcn_readfirstlane(wk.z), __builtin_amdgcn_readfirstlane(wk.w));  // uniform (SGPRs)
  }
  DTF_WG_CHECK(wk.x >= 0 && wk.y >= 0 && wk.w >= 0 && wk.z >= 0 && a.Hi > 0 && a.Wi > 0 && a.rows > 0);
  const int it0 = wk.x, nit = wk.y, slot = wk.w;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ct = wave % NT;
  // prologue loads in the order they are consumed: BN statistics -> input tile -> weights
  CoefLd<MODE_IN == 0 ? 0 : 1> cl;
  coef_issue<C, MODE_IN == 0 ? 0 : 1>(cl, params, p_mstride, slot, st_in, nullptr, in_gamma, in_beta);
  const float n_in = cnt[slot] * (float)(H * W);
  St st;
  st.init();
  uint4 tv[MAXC], unused[MAXC];
  unsigned tm;
  {
    const int img = it0 / BANDS, gy0 = (it0 % BANDS) * ROWS - 1;
    tm = st.mask(gy0);
    st.template load<LMODE>(tv, unused, tm, xin + img * IMG, nullptr, gy0);
  }
  bf16x8_t afr[KS];
  {
    const bf16_t* wb = wgt + (long)slot * w_mstride + w_off + (long)(ct * 16 + (lane & 15)) * KTOT;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int k0 = 32 * s + 8 * (lane >> 4);
      bf16x8_t v = {0, 0, 0, 0, 0, 0, 0, 0};
      if (k0 < KTOT) v = *reinterpret_cast<const bf16x8_t*>(wb + k0);
      afr[s] = v;
    }
  }
  coef_reduce<C, MODE_IN == 0 ? 0 : 1>(cl);
  coef_finish<C, MODE_IN == 0 ? 0 : 1>(coef, cl, n_in);
  if (threadIdx.x < 128) acc_lds[threadIdx.x] = 0.f;
  int tapoff[KS];  // k-chunks past KTOT have zero weights and read a valid in-tile address
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k0 = 32 * s + 8 * (lane >> 4);
    const int tap = k0 / C, c0 = k0 % C;
    tapoff[s] = k0 < KTOT ? ((tap / 3) * WP + (tap % 3)) * CP + c0 : 0;
  }
  const int co0 = ct * 16 + (lane >> 4) * 4;
  int tbo[MT];
  uint32_t pofs[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int p = (wave / NT + WPT * i) * 16 + (lane & 15);
    tbo[i] = ((p / W) * WP + p % W) * CP;
    pofs[i] = p * C + co0;
  }
  f32x2_t ssum[2] = {{0.f, 0.f}, {0.f, 0.f}}, ssq[2] = {{0.f, 0.f}, {0.f, 0.f}};
  // residual operands one iteration ahead (software-pipelined: their latency hides behind staging / MFMAs)
  uint2 nres[MT];
  if constexpr (RESID) {
    const long band0 = (long)(it0 / BANDS) * IMG + (it0 % BANDS) * ROWS * ROW;
#pragma unroll
    for (int i = 0; i < MT; ++i) nres[i] = *reinterpret_cast<const uint2*>(res + band0 + pofs[i]);
  }
  __syncthreads();  // coefficients
  STAMP(1);
  // the staging coefficients held in registers for the whole launch (every width stays within its occupancy's VGPR
  // budget: C = 16 / 32 at <= 128 for 4 waves / SIMD, C = 64 at <= 168 for 3)
  constexpr bool CREG = DTF_FWD_COEFREG && LMODE == 1;
  float csc[8], csh[8];
  if constexpr (CREG) {
    st.load_coef1(csc, csh, coef);
    st.store1r(SBUF(0), tv, tm, csc, csh);
  } else {
    st.template store<LMODE>(SBUF(0), tv, unused, tm, coef);
  }
  __syncthreads();
  STAMP(2);
  for (int k = 0; k < nit; ++k) {
    const int it = it0 + k;
    const int img = it / BANDS, r0 = (it % BANDS) * ROWS;
    const bool more = k + 1 < nit;
    const long band = (long)img * IMG + r0 * ROW;
    uint2 rres[MT];
    if constexpr (RESID) {
#pragma unroll
      for (int i = 0; i < MT; ++i) rres[i] = nres[i];
    }
    if (more) {
      const int nimg = (it + 1) / BANDS, ngy0 = ((it + 1) % BANDS) * ROWS - 1;
      tm = st.mask(ngy0);
      st.template load<LMODE>(tv, unused, tm, a.x + nimg * IMG, nullptr, ngy0);
      if constexpr (RESID) {
        const long nband = (long)nimg * IMG + ((it + 1) % BANDS) * ROWS * ROW;
#pragma unroll
        for (int i = 0; i < MT; ++i) nres[i] = *reinterpret_cast<const uint2*>(a.res + nband + pofs[i]);
      }
    }
    const bf16_t* tile = SBUF(k);
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s)
        acc = mfma16(afr[s], *reinterpret_cast<const bf16x8_t*>(tile + tbo[i] + tapoff[s]), acc);
      f32x2_t v0 = {acc[0], acc[1]}, v1 = {acc[2], acc[3]};
      if constexpr (RESID) {
        v0 += unpk2(rres[i].x);
        v1 += unpk2(rres[i].y);
      }
      uint2 pk;
      pk.x = pk2(v0);
      pk.y = pk2(v1);
      st_act8(a.y + band + pofs[i], pk);
      const f32x2_t r0v = unpk2(pk.x), r1v = unpk2(pk.y);
      ssum[0] += r0v;
      ssum[1] += r1v;
      ssq[0] += r0v * r0v;
      ssq[1] += r1v * r1v;
    }
    if (more) {
      if constexpr (CREG)
        st.store1r(SBUF(k + 1), tv, tm, csc, csh);
      else
        st.template store<LMODE>(SBUF(k + 1), tv, unused, tm, coef);
    }
    __syncthreads();
  }
#undef SBUF
  STAMP(3);
  const float s4[4] = {ssum[0].x, ssum[0].y, ssum[1].x, ssum[1].y};
  const float q4[4] = {ssq[0].x, ssq[0].y, ssq[1].x, ssq[1].y};
  reduce_stats_to_lds(acc_lds, s4, q4, co0, lane);
  __syncthreads();
  flush_stats_r(a.st_out, acc_lds, slot, C, bid);
  STAMP_DRAIN(4);
  STAMP_FLUSH(a.cin_real, nit);
}

template <int C, int MODE_IN, bool RESID, int ROWS = 8>
__global__ __launch_bounds__(256) void conv_fwd_s1_kernel(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  conv_fwd_s1_body<C, MODE_IN, RESID, ROWS>(a, (int)blockIdx.x, smem);
}

// ------------------------------------------------------------------ persistent forward segment (small populations)
// A run of conv_fwd_s1 layers of one stage (stem / conv_a / conv_b, the same C and band geometry and the same
// workgroup count) in ONE launch: each workgroup runs its work item of layer l, then a software grid barrier
// replaces the kernel boundary before layer l + 1 (whose BatchNorm prologue needs layer l's complete statistics).
// The barrier: release fence (this workgroup's activation stores / statistic atomics visible at agent scope), one
// arrival atomic on a flat counter, the last arriver resets it and bumps the generation word the others spin on
// (bounded: a barrier that does not complete within ~50 ms counts a failure and ends the kernel -- the step's
// result is then wrong and the host reports it -- instead of hanging the GPU), acquire fence (drops this XCD's
// stale L2 lines of the next layer's inputs).  The host launches it only when every workgroup is co-resident
// (occupancy check in dtf_conv_fwd_s1_persist).  kinds[l]: 0 stem (identity input), 1 BN+ReLU input, 2 + residual.
// fence bits: 1 agent release (else only this wave's counters drained), 2 agent acquire (L2 invalidate).
// bar: [0] generation, [64 + b] arrival flag of workgroup b (generation-stamped: never reset; one bar array per
// persistent segment).  Arrival is a store to the workgroup's own word -- a single arrival counter (512 serialised
// same-address atomics) measured ~8 us per barrier; workgroup 0's first wave polls every flag, then publishes the
// next generation, which the others poll.  (Every workgroup polling all flags itself instead measured slower:
// profiles/r4_persist_ab.log.)
__device__ __forceinline__ bool persist_barrier(unsigned* bar, unsigned nwg, unsigned* fail, int fence) {
  __shared__ int ok;
  __syncthreads();
  const unsigned bid = blockIdx.x;
  const int t = threadIdx.x;
  unsigned g = 0;
  if (t < 64) g = __hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (t == 0) {
    ok = 1;
    // Release: activation stores are write-through (st_act8) and the statistics agent-scope atomics, so completing
    // this workgroup's outstanding memory operations is enough (fence bit 1 adds the agent fence's L2 write-back).
    // Acquire: every buffer a layer reads was first written inside this launch (distinct activation buffers per
    // layer; statistics rows read only after their layer) and the L2 was clean at launch, so no stale line exists
    // (fence bit 2 adds the agent acquire's L2 invalidate).
    if (fence & 1)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    else
      __builtin_amdgcn_s_waitcnt(0);
    __hip_atomic_store(bar + 64 + bid, g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (bid == 0 && t < 64) {
    bool all = false;
    for (int it = 0; it < (1 << 20) && !all; ++it) {
      bool mine = true;
      for (unsigned w = t; w < nwg; w += 64)
        mine = mine && __hip_atomic_load(bar + 64 + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g + 1;
      all = __all(mine);
      if (!all) __builtin_amdgcn_s_sleep(1);
    }
    if (t == 0) {
      if (all) {
        __hip_atomic_store(bar, g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        ok = 0;
        atomicAdd(fail, 1u);
      }
    }
  } else if (t == 0) {
    bool done = false;
    for (int it = 0; it < (1 << 20) && !done; ++it) {
      done = __hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != g;
      if (!done) __builtin_amdgcn_s_sleep(1);
    }
    if (!done) {
      ok = 0;
      atomicAdd(fail, 1u);
    }
  }
  if (t == 0 && (fence & 2)) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  __syncthreads();
  return ok != 0;
}

template <int C, int ROWS>
__global__ __launch_bounds__(256) void conv_fwd_s1_persist_kernel(const ConvArgs* __restrict__ layers,
                                                                  const int* __restrict__ kinds, int nlayers,
                                                                  unsigned* bar, unsigned* fail, int fence) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int bid = (int)blockIdx.x;
  for (int l = 0; l < nlayers; ++l) {
    const int kind = kinds[l];
    if (kind == 0) {
      if constexpr (ROWS == 8) conv_fwd_s1_body<C, 0, false, ROWS>(layers[l], bid, smem);
    } else if (kind == 1) {
      conv_fwd_s1_body<C, 1, false, ROWS>(layers[l], bid, smem);
    } else {
      conv_fwd_s1_body<C, 1, true, ROWS>(layers[l], bid, smem);
    }
    if (l + 1 < nlayers && !persist_barrier(bar, gridDim.x, fail, fence)) return;
  }
}

// ---------------------------------------------------------------------------------- dgrad
// dx[iy,ix,ci] = sum_{ky,kx,co} dy[(iy+P-ky)/S, (ix+P-kx)/S, co] * W[co,ky,kx,ci]
// Weights in IHWO layout: wt[ci][tap][co] (rows of the A operand are ci).
// EPI bit0: add `res` (another dx contribution) before the epilogue;
// EPI bit1: mask by relu(BN_ep(xm)) and accumulate sum(dz), sum(dz*xhat) of BN_ep.
// Bands are over dx rows (forward-input resolution).

template <int CI, int CO, int S, int K, int MODE_IN, int EPI>
__device__ __forceinline__ void conv_dgrad_body(const ConvArgs& a, const int bid, char* smem) {
  // EPI bit2 (ResNet v1): the masking activation is an identity-BN ReLU output -> mask by xm > 0, no stats
  constexpr bool MASK = (EPI & 6) != 0, IDENT = (EPI & 4) != 0, STATS = (EPI & 2) != 0 && !IDENT;
  constexpr int NT = CI / 16;
  constexpr int WPT = 4 / NT;
  constexpr int KTOT = K * K * CO;
  constexpr int KS = (KTOT + 31) / 32;
  constexpr int P = (K - 1) / 2;
  float* coef = reinterpret_cast<float*>(smem);   // input transform (192)
  float* ecoef = coef + 192;                      // epilogue BN: scale, shift, mean, inv (4 x 64)
  float* acc_lds = ecoef + 256;                   // 128
  bf16_t* tile0 = reinterpret_cast<bf16_t*>(smem + 2304);

  const int4 wk = a.work[bid];
  DTF_WG_CHECK(wk.x >= 0 && wk.y >= 0 && wk.w >= 0 && wk.z >= 0 && a.Hi > 0 && a.Wi > 0 && a.rows > 0);
  const int it0 = wk.x, nit = wk.y, slot = wk.w;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // dy lives at the forward-output resolution; the BN transformed on load is the one after this conv.
  make_coef<CO, MODE_IN>(coef, a, slot, a.cnt[slot] * (float)(a.Ho * a.Wo), a.st_in, a.st_in_b, a.in_gamma, a.in_beta);
  if constexpr (MASK) {
    const int c = threadIdx.x;
    if (c < CI) {
      const float* prow = a.params + (long)slot * a.p_mstride;
      float scale = 1.f, shift = 0.f, mean = 0.f, inv = 1.f;
      if constexpr (!IDENT)
        bn_fwd_coef(stats_row(a.st_ep, slot), a.cnt[slot] * (float)(a.Hi * a.Wi), prow[a.ep_gamma + c],
                    prow[a.ep_beta + c], c, scale, shift, mean, inv);
      ecoef[c] = scale;
      ecoef[64 + c] = shift;
      ecoef[128 + c] = mean;
      ecoef[192 + c] = inv;
    }
    if (threadIdx.x < 128) acc_lds[threadIdx.x] = 0.f;
  }
  const int ct = wave % NT;
  bf16x8_t afr[KS];
  {
    const bf16_t* wb = a.w + (long)slot * a.w_mstride + a.w_off + (long)(ct * 16 + (lane & 15)) * KTOT;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int k0 = 32 * s + 8 * (lane >> 4);
      bf16x8_t v = {0, 0, 0, 0, 0, 0, 0, 0};
      if (k0 < KTOT) v = *reinterpret_cast<const bf16x8_t*>(wb + k0);
      afr[s] = v;
    }
  }
  const int rows = a.rows;
  const int bands = a.Hi / rows;
  // dy rows needed by a band starting at iy0: oy in [floor((iy0+P-K+1)/S), floor((iy0+rows-1+P)/S)]
  auto dy_lo = [&](int iy0) {
    const int lo_num = iy0 + P - K + 1;
    return lo_num >= 0 ? lo_num / S : -((-lo_num + S - 1) / S);
  };
  const int rows_t = (S == 1) ? rows + K - 1 : (rows + K + S - 2) / S + 1;  // dy rows per band (host: same)
  const int wp = a.Wo + 2;  // dy cols -1..Wo
  const int tsz = (rows_t * wp * cpad<CO>() + 63) & ~63;
#define TILEBUF(i) (tile0 + ((i) & 1) * tsz)
  const int ntiles = rows * a.Wi / 16;
  const long img_elems = (long)a.Ho * a.Wo * CO;
  // PAR (stride-2 3x3 of the CIFAR stage transitions, Wi = 512 / CI, 8-row bands): tile i of a wave is parity
  // class i -- its 16 pixels share (iy % 2, ix % 2) -- so only the 1-4 taps that reach the class are multiplied
  // (9 of the 36 tap-tiles of a 2 x 2 pixel quad) and the LDS addresses need no per-k-step parity tests
  constexpr bool PAR = S == 2 && K == 3 && (512 / CI) * 8 / 16 == 4 * WPT;
  constexpr int WI = 512 / CI;
  if constexpr (PAR) DTF_WG_CHECK(a.Wi == WI && rows == 8 && MAXT == 4);
  auto par_pix = [&](int i, int iy0_, int& iy_, int& ix_) {
    const int q = (wave / NT) * 16 + (lane & 15), cy = q / (WI / 2), cx = q % (WI / 2);
    iy_ = iy0_ + 2 * cy + (i >> 1);
    ix_ = 2 * cx + (i & 1);
  };
  int tapoff[KS];  // stride 1: LDS offset of (dy row/col shift by the flipped tap, channel chunk)
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k0 = 32 * s + 8 * (lane >> 4);
    const int tap = k0 / CO, c0 = k0 % CO;
    tapoff[s] = -((tap / K) * wp + (tap % K)) * cpad<CO>() + c0;
  }
  float ssum[4] = {0.f, 0.f, 0.f, 0.f}, ssq[4] = {0.f, 0.f, 0.f, 0.f};
  TileRegs<CO, MODE_IN, 4> rg;
  TileDesc<CO, 4> td;
  tile_desc_init<CO, 4>(td, rows_t, -1, wp, a.Wo);
  __syncthreads();
  {
    const int img = it0 / bands, iy0 = (it0 % bands) * rows;
    const bf16_t* x2 = a.x2 ? a.x2 + img * img_elems : nullptr;
    tile_load<CO, MODE_IN, 4>(rg, td, a.x + img * img_elems, x2, dy_lo(iy0), a.Ho, a.Wo);
    tile_store<CO, MODE_IN, 4>(TILEBUF(0), rg, td, a.x + img * img_elems, x2, dy_lo(iy0), a.Ho, a.Wo, coef);
  }
  __syncthreads();
  for (int k = 0; k < nit; ++k) {
    const int it = it0 + k;
    const int img = it / bands, iy0 = (it % bands) * rows;
    const int oy_lo = dy_lo(iy0);
    const bool more = k + 1 < nit;
    const int nimg_ = (it + 1) / bands, niy0 = ((it + 1) % bands) * rows;
    const bf16_t* nx2 = a.x2 ? a.x2 + nimg_ * img_elems : nullptr;
    uint2 rres[MAXT], xres[MAXT];  // epilogue operands, issued before the prefetch (counted vmcnt)
#pragma unroll
    for (int i = 0; i < MAXT; ++i) {
      int py_, px_;
      if constexpr (PAR) {
        par_pix(i, iy0, py_, px_);
      } else {
        const int t = min(wave / NT + WPT * i, ntiles - 1);
        const int p = t * 16 + (lane & 15);
        py_ = iy0 + p / a.Wi;
        px_ = p % a.Wi;
      }
      const long o = (((long)img * a.Hi + py_) * a.Wi + px_) * CI + ct * 16 + (lane >> 4) * 4;
      if constexpr (EPI & 1) rres[i] = *reinterpret_cast<const uint2*>(a.res + o);
      if constexpr (MASK) xres[i] = *reinterpret_cast<const uint2*>(a.xm + o);
    }
    if (more) tile_load<CO, MODE_IN, 4>(rg, td, a.x + nimg_ * img_elems, nx2, dy_lo(niy0), a.Ho, a.Wo);
    const bf16_t* tile = TILEBUF(k);
#pragma unroll
    for (int i = 0; i < MAXT; ++i) {
      const int t = wave / NT + WPT * i;
      if (t >= ntiles) break;
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
      int iy, ix;
      if constexpr (PAR) {
        par_pix(i, iy0, iy, ix);
      } else {
        const int p = t * 16 + (lane & 15);
        iy = iy0 + p / a.Wi;
        ix = p % a.Wi;
      }
      const int ci0 = ct * 16 + (lane >> 4) * 4;
      const long o = (((long)img * a.Hi + iy) * a.Wi + ix) * CI + ci0;
      uint2 rr = make_uint2(0, 0), xr = make_uint2(0, 0);
      if constexpr (EPI & 1) rr = rres[i];
      if constexpr (MASK) xr = xres[i];
      // stride 1: dy(iy+P-ky, ix+P-kx) lives at tile row iy+P-oy_lo-ky, col ix+P+1-kx
      const bf16_t* tb = tile + ((iy + P - oy_lo) * wp + ix + P + 1) * cpad<CO>();
      if constexpr (PAR) {
        // parity class (py, px) = (i >> 1, i & 1): dy(oy, ox) reaches dx(iy, ix) through ky = iy + 1 - 2 oy, so
        // even rows take tap row 1 only and odd rows tap rows 0 and 2 (columns alike): 1, 2, 2 or 4 taps
        constexpr int CJ = CO / 32;
#pragma unroll
        for (int ay = 0; ay < ((i >> 1) ? 2 : 1); ++ay) {
          const int ky = (i >> 1) ? 2 * ay : 1;
#pragma unroll
          for (int ax = 0; ax < ((i & 1) ? 2 : 1); ++ax) {
            const int kx = (i & 1) ? 2 * ax : 1;
            const bf16_t* tp = tile + ((((iy + 1 - ky) >> 1) - oy_lo) * wp + ((ix + 1 - kx) >> 1) + 1) * cpad<CO>() +
                               8 * (lane >> 4);
#pragma unroll
            for (int j = 0; j < CJ; ++j)
              acc = mfma16(afr[(ky * 3 + kx) * CJ + j], *reinterpret_cast<const bf16x8_t*>(tp + 32 * j), acc);
          }
        }
      } else {
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int k0 = 32 * s + 8 * (lane >> 4);
        bf16x8_t b = {0, 0, 0, 0, 0, 0, 0, 0};
        if constexpr (S == 1) {
          if (k0 < KTOT) b = *reinterpret_cast<const bf16x8_t*>(tb + tapoff[s]);
        } else if (k0 < KTOT) {
          const int tap = k0 / CO, c0 = k0 % CO;
          const int ky = tap / K, kx = tap % K;
          const int ty = iy + P - ky, tx = ix + P - kx;
          bool ok = true;
          int oy = ty, ox = tx;
          if constexpr (S > 1) {
            ok = (ty >= 0) && (tx >= 0) && (ty % S == 0) && (tx % S == 0);
            oy = ty / S;
            ox = tx / S;
          }
          const int lr = oy - oy_lo, lc = ox + 1;
          if (ok && lr >= 0 && lr < rows_t && lc >= 0 && lc < wp)
            b = *reinterpret_cast<const bf16x8_t*>(tile + lds_off<CO>(lr, lc, wp, c0 >> 3));
        }
        acc = mfma16(afr[s], b, acc);
      }
      }
      float v[4] = {acc[0], acc[1], acc[2], acc[3]};
      if constexpr (EPI & 1) {
        v[0] += bf2f((bf16_t)(rr.x & 0xffff));
        v[1] += bf2f((bf16_t)(rr.x >> 16));
        v[2] += bf2f((bf16_t)(rr.y & 0xffff));
        v[3] += bf2f((bf16_t)(rr.y >> 16));
      }
      float xv[4] = {0.f, 0.f, 0.f, 0.f};
      if constexpr (MASK) {
        xv[0] = bf2f((bf16_t)(xr.x & 0xffff));
        xv[1] = bf2f((bf16_t)(xr.x >> 16));
        xv[2] = bf2f((bf16_t)(xr.y & 0xffff));
        xv[3] = bf2f((bf16_t)(xr.y >> 16));
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = ci0 + r;
          const float pre = xv[r] * ecoef[c] + ecoef[64 + c];
          v[r] = pre > 0.f ? v[r] : 0.f;
        }
      }
      uint2 pk;
      pk.x = pack2bf(v[0], v[1]);
      pk.y = pack2bf(v[2], v[3]);
      st_act8(a.y + o, pk);
      if constexpr (STATS) {
        const float dz[4] = {bf2f((bf16_t)(pk.x & 0xffff)), bf2f((bf16_t)(pk.x >> 16)), bf2f((bf16_t)(pk.y & 0xffff)),
                             bf2f((bf16_t)(pk.y >> 16))};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = ci0 + r;
          ssum[r] += dz[r];
          ssq[r] += dz[r] * (xv[r] - ecoef[128 + c]) * ecoef[192 + c];
        }
      }
    }
    if (more)
      tile_store<CO, MODE_IN, 4>(TILEBUF(k + 1), rg, td, a.x + nimg_ * img_elems, nx2, dy_lo(niy0), a.Ho, a.Wo,
                                 coef);
    __syncthreads();
  }
  if constexpr (STATS) {
    reduce_stats_to_lds(acc_lds, ssum, ssq, ct * 16 + (lane >> 4) * 4, lane);
    __syncthreads();
    flush_stats_r(a.st_out, acc_lds, slot, CI, bid);
  }
}

// ---------------------------------------------------------------------------------- wgrad
// dW[co][ky][kx][ci] += sum_{pix} dy[pix][co] * x(pix*S + tap - P)[ci]
// GEMM M = co, N = (tap, ci), reduction over the output pixels of the WG's images.
// Both operands are "k = pixel" fragments, read from NHWC LDS tiles with
// ds_read_b64_tr_b16 (4 pixel-rows x 16 channel-columns, delivered column-major).

typedef short s16x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ s16x4_t ds_read_tr(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(p));
}

template <int CI, int CO, int S, int K, int MODE_IN, int EPI>
__global__ __launch_bounds__(256) void conv_dgrad_kernel(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  conv_dgrad_body<CI, CO, S, K, MODE_IN, EPI>(a, (int)blockIdx.x, smem);
}

template <int CIN, int COUT, int S, int K, int MODE_X, int MODE_DY>
__device__ __forceinline__ void conv_wgrad_body(const ConvArgs& a, const int bid, char* smem) {
  constexpr int MT = COUT / 16;
  constexpr int NTN = K * K * CIN / 16;  // n-tiles: (tap, 16-channel chunk)
  constexpr int NJ = (NTN + 3) / 4;
  constexpr int P = (K - 1) / 2;
  float* coef_x = reinterpret_cast<float*>(smem);  // 192
  float* coef_d = coef_x + 192;                   // 192
  bf16_t* xt = reinterpret_cast<bf16_t*>(smem + 1536);

  const int4 wk = a.work[bid];
  DTF_WG_CHECK(wk.x >= 0 && wk.y >= 0 && wk.w >= 0 && wk.z >= 0 && a.Hi > 0 && a.Wi > 0 && a.rows > 0);
  const int it0 = wk.x, nit = wk.y, slot = wk.w;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  make_coef<CIN, MODE_X>(coef_x, a, slot, a.cnt[slot] * (float)(a.Hi * a.Wi), a.st_x, nullptr, a.x_gamma, a.x_beta);
  make_coef<COUT, MODE_DY>(coef_d, a, slot, a.cnt[slot] * (float)(a.Ho * a.Wo), a.st_in, a.st_in_b, a.in_gamma,
                           a.in_beta);
  const int rows = a.rows;
  const int rows_in = (rows - 1) * S + K;
  const int wpx = a.Wi + 2 * P;
  const int xsz = (rows_in * wpx * cpad<CIN>() + 63) & ~63;
  const int dsz = (rows * a.Wo * cpad<COUT>() + 63) & ~63;
#define XBUF(i) (xt + ((i) & 1) * (xsz + dsz))
#define DBUF(i) (xt + xsz + ((i) & 1) * (xsz + dsz))
  const int npix = rows * a.Wo;
  const int bands = a.Ho / rows;

  f32x4_t acc[NJ][MT];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[j][m] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, i = lane & 15, q = i >> 2, p4 = i & 3;
  TileRegs<CIN, MODE_X, 4> rx;
  TileRegs<COUT, MODE_DY, 2> rd;
  TileDesc<CIN, 4> tdx;
  TileDesc<COUT, 2> tdd;
  tile_desc_init<CIN, 4>(tdx, rows_in, -P, wpx, a.Wi);
  tile_desc_init<COUT, 2>(tdd, rows, 0, a.Wo, a.Wo);
  auto src_of = [&](int it, const bf16_t*& xs, const bf16_t*& ds, const bf16_t*& ds2, int& oy0) {
    const int img = (it0 + it) / bands;
    oy0 = ((it0 + it) % bands) * rows;
    xs = a.x + (long)img * a.Hi * a.Wi * CIN;
    const long yo = (long)img * a.Ho * a.Wo * COUT;
    ds = a.dy + yo;
    ds2 = a.dy2 ? a.dy2 + yo : nullptr;
  };
  __syncthreads();  // coefficients visible
  {
    const bf16_t *xs, *ds, *ds2;
    int oy0;
    src_of(0, xs, ds, ds2, oy0);
    tile_load<CIN, MODE_X, 4>(rx, tdx, xs, nullptr, oy0 * S - P, a.Hi, a.Wi);
    tile_load<COUT, MODE_DY, 2>(rd, tdd, ds, ds2, oy0, a.Ho, a.Wo);
    tile_store<CIN, MODE_X, 4>(XBUF(0), rx, tdx, xs, nullptr, oy0 * S - P, a.Hi, a.Wi, coef_x);
    tile_store<COUT, MODE_DY, 2>(DBUF(0), rd, tdd, ds, ds2, oy0, a.Ho, a.Wo, coef_d);
  }
  __syncthreads();
  for (int it = 0; it < nit; ++it) {
    const int cur = it & 1;
    const bf16_t *nxs = nullptr, *nds = nullptr, *nds2 = nullptr;
    int noy0 = 0;
    if (it + 1 < nit) {  // prefetch the next (image, band) into registers
      src_of(it + 1, nxs, nds, nds2, noy0);
      tile_load<CIN, MODE_X, 4>(rx, tdx, nxs, nullptr, noy0 * S - P, a.Hi, a.Wi);
      tile_load<COUT, MODE_DY, 2>(rd, tdd, nds, nds2, noy0, a.Ho, a.Wo);
    }
    const bf16_t* xcur = XBUF(cur);
    const bf16_t* dcur = DBUF(cur);
    // The 32 pixels of a k-step span RSTEP = 32/Wo whole rows (Wo | 32), so each
    // lane's pixel (ya, xa) is (kstep*RSTEP + (8g+q)/Wo, (8g+q)%Wo): all LDS
    // addresses are lane constants plus kstep * increment.
    const int rstep = 32 / a.Wo;
    const int pa = 8 * g + q, pb = pa + 4;
    const int ya = pa / a.Wo, xa = pa % a.Wo, yb = pb / a.Wo, xb = pb % a.Wo;
    const bf16_t* da = dcur + (ya * a.Wo + xa) * cpad<COUT>() + 4 * p4;
    const bf16_t* db = dcur + (yb * a.Wo + xb) * cpad<COUT>() + 4 * p4;
    const bf16_t* xa_ = xcur + (ya * S * wpx + xa * S) * cpad<CIN>() + 4 * p4;
    const bf16_t* xb_ = xcur + (yb * S * wpx + xb * S) * cpad<CIN>() + 4 * p4;
    const int dinc = rstep * a.Wo * cpad<COUT>();
    const int xinc = rstep * S * wpx * cpad<CIN>();
    int boff[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int nt = min(wave + 4 * j, NTN - 1);  // duplicates (nt >= NTN) are computed, never flushed
      const int tap = (nt * 16) / CIN, cb = (nt * 16) % CIN;
      boff[j] = ((tap / K) * wpx + (tap % K)) * cpad<CIN>() + cb;
    }
    const int nk = npix / 32;
    for (int ks = 0; ks < nk; ++ks) {
      bf16x8_t af[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        s16x4_t lo = ds_read_tr(da + ks * dinc + m * 16);
        s16x4_t hi = ds_read_tr(db + ks * dinc + m * 16);
        af[m] = (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
      bf16x8_t bfr[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        s16x4_t lo = ds_read_tr(xa_ + ks * xinc + boff[j]);
        s16x4_t hi = ds_read_tr(xb_ + ks * xinc + boff[j]);
        bfr[j] = (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[j][m] = mfma16(af[m], bfr[j], acc[j][m]);
    }
    if (it + 1 < nit) {
      tile_store<CIN, MODE_X, 4>(XBUF(cur ^ 1), rx, tdx, nxs, nullptr, noy0 * S - P, a.Hi, a.Wi, coef_x);
      tile_store<COUT, MODE_DY, 2>(DBUF(cur ^ 1), rd, tdd, nds, nds2, noy0, a.Ho, a.Wo, coef_d);
    }
    __syncthreads();
  }
  // epilogue: D[co][n] with co = m*16 + 4*(lane>>4) + r, n-col = lane & 15.  With a slab: this workgroup's dense
  // partial dW (every element of [co][tap][ci < cin_real] written once, plain stores), summed in workgroup order by
  // slab_reduce_all_kernel; else fp32 atomics into the gradient row.
  const int KK = K * K;
  const long kel = (long)COUT * KK * a.cin_real;
  float* gb = a.slab ? a.slab + (long)bid * kel : a.grads + (long)slot * a.g_mstride + a.g_off;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int nt = wave + 4 * j;
    if (nt < NTN) {
      const int tap = (nt * 16) / CIN, ci = (nt * 16) % CIN + (lane & 15);
      if (ci < a.cin_real) {
#pragma unroll
        for (int m = 0; m < MT; ++m) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int co = m * 16 + 4 * (lane >> 4) + r;
            const long e = ((long)co * KK + tap) * a.cin_real + ci;
            if (a.slab)
              gb[e] = acc[j][m][r];
            else
              atomicAdd(gb + e, acc[j][m][r]);
          }
        }
      }
    }
  }
}

template <int CIN, int COUT, int S, int K, int MODE_X, int MODE_DY>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  conv_wgrad_body<CIN, COUT, S, K, MODE_X, MODE_DY>(a, (int)blockIdx.x, smem);
}

// Stage transition of the pre-activation ResNet backward (projection block), three independent roles in ONE
// launch, all reading the block output gradient g (and dz2 of conv_a): [0, c.n_main) conv_a (3x3 / 2) wgrad,
// then the projection (1x1 / 2) dgrad (-> pd, added by conv_a's dgrad next), then the projection wgrad.
// Replaces three launches of a latency-bound small population with one.
template <int CI, int CO>
__global__ __launch_bounds__(256) void conv_trans_multi_kernel(ConvArgs c, ConvArgs a, ConvArgs b) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int bx = (int)blockIdx.x;
  if (bx < c.n_main)
    conv_wgrad_body<CI, CO, 2, 3, 1, 2>(c, bx, smem);
  else if (bx < c.n_main + a.n_main)
    conv_dgrad_body<CI, CO, 2, 1, 0, 0>(a, bx - c.n_main, smem);
  else
    conv_wgrad_body<CI, CO, 2, 1, 1, 0>(b, bx - c.n_main - a.n_main, smem);
}

// Dense dW slabs of several wgrad launches (conv_wgrad_kernel with a slab), reduced after the backward in one launch:
// blockIdx.z = job, y = member row of its reduce table (first wg, n wgs, -, slot), x (+ gridDim.x ...) = 32-element
// block; 8 thread groups stride over the member's slabs, an LDS sum in group order (fixed summation order).
struct DenseJob {
  const float* slab;
  const int4* red;
  long g_off;
  int kel;
  int nmem;
};

// One workgroup of the dW slab reduction (see dw_slab_reduce_kernel): 32 slab elements of member row `by`.
// Blocks bx0, bx0 + bstride, ... of 32 slab elements (workgroup-uniform loop: every thread reaches each barrier).
template <int C>
__device__ __forceinline__ void slab_reduce_wg(const float* __restrict__ slab, const int4* __restrict__ red,
                                               float* __restrict__ grads, long g_mstride, long g_off, int bx0, int by,
                                               float* part /* [8][33] */, int bstride) {
  constexpr int MT = C / 16, NTN = 9 * C / 16, NJ = (NTN + 3) / 4, E = NJ * MT * 4 * 256;
  const int el = threadIdx.x & 31, gg = threadIdx.x >> 5;
  const int4 rd = red[by];
  for (int bx = bx0; bx < E / 32; bx += bstride) {
    const int e = bx * 32 + el;
    const float* p = slab + (long)rd.x * E + e;
    float s0 = 0.f, s1 = 0.f;
    int g = gg;
    for (; g + 8 < rd.y; g += 16) {
      s0 += p[(long)g * E];
      s1 += p[(long)(g + 8) * E];
    }
    if (g < rd.y) s0 += p[(long)g * E];
    part[gg * 33 + el] = s0 + s1;
    __syncthreads();
    if (gg == 0) {
      float sum = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) sum += part[i * 33 + el];
      const int r = e & 3, t = (e >> 2) & 255, m = (e >> 10) % MT, j = (e >> 10) / MT;  // slab [j][m][t][r]
      const int wave = t >> 6, lane = t & 63, nt = wave + 4 * j;
      if (nt < NTN) {
        const int tap = (nt * 16) / C, ci = (nt * 16) % C + (lane & 15), co = m * 16 + 4 * (lane >> 4) + r;
        grads[(long)rd.w * g_mstride + g_off + ((long)co * 9 + tap) * C + ci] += sum;
      }
    }
    __syncthreads();  // part is rewritten by the next block
  }
}

// ------------------------------------------------------------------ fused backward
// One launch = dgrad AND wgrad of a stride-1 3x3 C->C conv of the CIFAR stages
// (C = 16/32/64 at W = H = 512/C; 8-row bands), sharing the staged tiles: per
// (image, band) iteration the workgroup stages
//   dY tile  rows r0-1..r0+8, cols -1..W : T_dy(dy)   (plain residual grad, or BN2-backward(dz2, h))
//   X  tile  same geometry               : relu(BN_x(x))  (the conv's forward input activation)
// then computes the dgrad tiles (weights W^T in registers; epilogue: [+ res],
// mask by BN_x(x) > 0, BN_x backward reductions, dz out) and the wgrad k-steps
// (operands from the dY interior and the shifted X tile via ds_read_b64_tr_b16,
// fp32 accumulators across all iterations, one atomic flush at the end).
// All geometry is compile-time, every global address is a wave-uniform base plus
// a 32-bit lane offset fixed for the workgroup, and the elementwise work uses
// packed fp32 / bf16 math: the VALU budget per MFMA is what bounds these
// small-channel layers.
// ROLE (dual backward of small populations, conv_bwd_dual_kernel): 0 = dgrad + wgrad (fused),
// 1 = dgrad only (critical path: no X tile, no wgrad; the transformed dY may be materialised via xout for the
// wgrad), 2 = wgrad only (the wgrad role of a dual launch; no dgrad / stats / xout).
// Body of one workgroup; `bid` = the workgroup's index within its role (work item, stats replica, dW slab row).
template <int C, int MODE_DY, int EPI, int ROLE, int ROWS = 8>
__device__ __forceinline__ void conv_bwd_body(const ConvArgs& a, const int bid, char* smem) {
  constexpr bool DG = ROLE != 2, WG = ROLE != 1;
  static_assert(ROWS == 8 || ROLE == 1, "half-image bands: dgrad role only");
  constexpr int W = 512 / C, H = W, BANDS = H / ROWS;
  constexpr int NT = C / 16;           // dgrad output-channel tiles
  constexpr int WPT = 4 / NT;
  constexpr int KTOT = 9 * C;
  constexpr int KS = (KTOT + 31) / 32;
  constexpr int MT = C / 16;           // wgrad co tiles
  constexpr int NTN = 9 * C / 16;      // wgrad (tap, ci) tiles
  constexpr int NJ = (NTN + 3) / 4;
  constexpr int CP = cpad<C>(), RT = ROWS + 2, WP = wpitch<C>();
  constexpr int TSZ = (RT * WP * CP + 8 + 63) & ~63;  // + slack for inactive staging slots
  constexpr int NTILES = ROWS * W / 16;
  constexpr int MTD = NTILES / WPT;  // dgrad tiles per wave (MAXT for 8-row bands)
  static_assert(NTILES == WPT * MTD && MTD <= MAXT, "every wave owns MTD dgrad tiles");
  constexpr int ROW = W * C, IMG = H * ROW;
  constexpr int NK = ROWS * W / 32, RSTEP = 32 / W, KINC = RSTEP * WP * CP;
  using St = Stage<C, RT, W, H, CP, WP>;
  constexpr int MAXC = St::MAXC;
  float* coef_d = reinterpret_cast<float*>(smem);  // dy transform (192)
  float* ecoef = coef_d + 192;                     // x BN: scale, shift, -mean*inv, inv (256)
  float* acc_lds = ecoef + 256;                    // 128
  bf16_t* t0 = reinterpret_cast<bf16_t*>(smem + 2304);
  // SB: single-buffered tiles (one extra barrier per iteration) so that C = 16 fits 3 workgroups per CU in LDS
  constexpr bool SB = DTF_FUSED_SB16 && C == 16 && MODE_DY != 3 && ROLE == 0;
  constexpr int BSTR = WG ? 2 * TSZ : TSZ;  // dgrad-only: dY tiles only
#define FDBUF(i) (t0 + (SB ? 0 : ((i) & 1) * BSTR))
#define FXBUF(i) (t0 + TSZ + (SB ? 0 : ((i) & 1) * BSTR))
  // raw (untransformed) x of the band interior, for the dgrad epilogue's mask / x-hat: read from LDS instead of
  // re-reading x from global memory (double-buffered like the tiles)
  // (C <= 32 keeps the global re-read: the extra LDS would cost its 2nd WG per CU)
  constexpr bool RAWX = ROLE == 0 && C >= 64;
  constexpr int RAWSZ = ROWS * W * CP;
#define FXRAW(i) (t0 + 4 * TSZ + ((i) & 1) * RAWSZ)
  STAMP_DECL
  STAMP(0);
  // every kernarg field of the body in one s_load batch (kpin): one scalar round trip before the first load
  const bf16_t* k_x = a.x;
  const bf16_t* k_x2 = a.x2;
  const bf16_t* k_x3 = a.x3;
  const bf16_t* k_xm = a.xm;
  const bf16_t* k_w = a.w;
  const bf16_t* k_res = a.res;
  bf16_t* k_xout = a.xout;
  bf16_t* k_y = a.y;
  const float* k_st_in = a.st_in;
  const float* k_st_in_b = a.st_in_b;
  const float* k_st_ep = a.st_ep;
  const float* k_params = a.params;
  const float* k_cnt = a.cnt;
  float* k_st_out = a.st_out;
  float* k_slab = a.slab;
  float* k_grads = a.grads;
  const int4* k_work = a.work;
  long k_w_mstride = a.w_mstride;
  long k_w_off = a.w_off;
  int k_in_gamma = a.in_gamma;
  int k_in_beta = a.in_beta;
  int k_ep_gamma = a.ep_gamma;
  int k_ep_beta = a.ep_beta;
  long k_p_mstride = a.p_mstride;
  long k_g_mstride = a.g_mstride;
  long k_g_off = a.g_off;
  int k_u_items = a.u_items;
  int k_u_chunk = a.u_chunk;
  int k_u_per = a.u_per;
  kpin(k_x); kpin(k_x2); kpin(k_x3); kpin(k_xm); kpin(k_w); kpin(k_res); kpin(k_xout); kpin(k_y); kpin(k_st_in); kpin(k_st_in_b); kpin(k_st_ep); kpin(k_params); kpin(k_cnt); kpin(k_st_out); kpin(k_slab); kpin(k_grads); kpin(k_work);
  kpin(k_w_mstride); kpin(k_w_off); kpin(k_in_gamma); kpin(k_in_beta); kpin(k_ep_gamma); kpin(k_ep_beta); kpin(k_p_mstride); kpin(k_g_mstride); kpin(k_g_off); kpin(k_u_items); kpin(k_u_chunk); kpin(k_u_per);
  int4 wk;
  if (k_u_items > 0) {
    const int m = bid / k_u_items, kk = bid - m * k_u_items, it0_ = kk * k_u_chunk;
    wk = make_int4(m * k_u_per + it0_, min(k_u_chunk, k_u_per - it0_), 0, m);
  } else {
    wk = k_work[bid];
    wk = make_int4(__builtin_amdgcn_readfirstlane(wk.x), __builtin_amdgcn_readfirstlane(wk.y),
                   __builtin_amdgcn_readfirstlane(wk.z), __builtin_amdgcn_readfirstlane(wk.w));  // uniform (SGPRs)
  }
  DTF_WG_CHECK(wk.x >= 0 && wk.y >= 0 && wk.w >= 0 && wk.z >= 0 && a.Hi > 0 && a.Wi > 0 && a.rows > 0);
  const int it0 = wk.x, nit = wk.y, slot = wk.w;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ct = wave % NT;
  STAMP_FINE(8);
  // prologue loads in the order they are consumed: BN statistics (dY transform, x BN) -> tiles -> weights
  CoefLd<MODE_DY == 0 ? 0 : 2> cld;
  coef_issue<C, MODE_DY == 0 ? 0 : 2>(cld, k_params, k_p_mstride, slot, k_st_in, k_st_in_b, k_in_gamma, k_in_beta);
  // EPI bit 8 (v1 chain): the statistics' x-hat comes from x3 = the BN input h of the NEXT BN in the backward (the
  // previous block's BN_b), normalised with that BN's batch statistics (st_ep); the mask stays the identity BN
  static_assert(!(EPI & 8) || ((EPI & 2) && MODE_DY != 3 && ROLE != 2), "EPI 8: identity mask, x3 free, dgrad");
  CoefLd<1> cle;
  if constexpr (!(EPI & 2) || (EPI & 8))
    coef_issue<C, 1>(cle, k_params, k_p_mstride, slot, k_st_ep, nullptr, k_ep_gamma, k_ep_beta);
  const float n_hw = k_cnt[slot] * (float)(H * W);
  STAMP_FINE(9);
  St st;
  st.init();
  // MODE_DY 3: dY = BN-backward(x, x2) + x3; with xout the transformed band interior is also written out
  constexpr bool XSTORE = MODE_DY >= 2;
  uint4 dv[MAXC], dv2[MAXC], dv3[MAXC], xv_[MAXC], unused[MAXC];  // dv3: MODE_DY 3 only
  unsigned dm, xm;
  int cimg = it0 / BANDS, cgy0 = (it0 % BANDS) * ROWS - 1;  // image / first tile row of the staged tile
  {
    dm = xm = st.mask(cgy0);
    st.template load<MODE_DY == 3 ? 2 : MODE_DY>(dv, dv2, dm, k_x + cimg * IMG, k_x2 + cimg * IMG, cgy0);
    if constexpr (MODE_DY == 3) st.template load<0>(dv3, unused, dm, k_x3 + cimg * IMG, nullptr, cgy0);
    if constexpr (WG) st.template load<1>(xv_, unused, xm, k_xm + cimg * IMG, nullptr, cgy0);
  }
  STAMP_FINE(10);
  // WLDS (C = 16: all four waves share the 16 x 144 weights): the weights are staged once into LDS rows of
  // WLP elements (zero past KTOT) and read per MFMA, freeing the 20 VGPRs of afr for the pipelines
  constexpr bool WLDS = DTF_FUSED16_WLDS && DG && C == 16 && ROLE == 0;
  constexpr int WLP = 32 * KS + 8;
  bf16_t* wl = t0 + 4 * TSZ;  // after the (double-buffered) dY / X tiles
  bf16x8_t afr[WLDS ? 1 : KS];
  uint4 wst[2];
  if constexpr (WLDS) {
    // 16 rows x (KS * 4) 16-byte chunks = 320 chunks: threads 0..255 + 0..63
    const bf16_t* wb = k_w + (long)slot * k_w_mstride + k_w_off;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int idx = (int)threadIdx.x + 256 * j, r = idx / (KS * 4), k0 = (idx % (KS * 4)) * 8;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (idx < 16 * KS * 4 && k0 < KTOT) v = *reinterpret_cast<const uint4*>(wb + (long)r * KTOT + k0);
      wst[j] = v;
    }
  } else if constexpr (DG) {
    const bf16_t* wb = k_w + (long)slot * k_w_mstride + k_w_off + (long)(ct * 16 + (lane & 15)) * KTOT;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int k0 = 32 * s + 8 * (lane >> 4);
      bf16x8_t v = {0, 0, 0, 0, 0, 0, 0, 0};
      if (k0 < KTOT) v = *reinterpret_cast<const bf16x8_t*>(wb + k0);
      afr[s] = v;
    }
  }
  STAMP_FINE(12);
  coef_reduce<C, MODE_DY == 0 ? 0 : 2>(cld);
  if constexpr (!(EPI & 2) || (EPI & 8)) coef_reduce<C, 1>(cle);
  coef_finish<C, MODE_DY == 0 ? 0 : 2>(coef_d, cld, n_hw);
  STAMP_FINE(13);
  {
    const int c = threadIdx.x;
    if (c < C) {
      float scale = 1.f, shift = 0.f, mean = 0.f, inv = 1.f;  // EPI bit1: identity BN (v1 block input)
      if constexpr (!(EPI & 2)) {
        coef_moments<1>(cle, n_hw, mean, inv);
        scale = cle.g * inv;
        shift = cle.b - mean * scale;
      } else if constexpr ((EPI & 8) != 0) {
        coef_moments<1>(cle, n_hw, mean, inv);  // x-hat of x3 only; the mask keeps scale 1, shift 0
      }
      ecoef[c] = scale;
      ecoef[64 + c] = shift;
      ecoef[128 + c] = -mean * inv;
      ecoef[192 + c] = inv;
    }
    if (threadIdx.x < 128) acc_lds[threadIdx.x] = 0.f;
  }
  if constexpr (WLDS) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int idx = (int)threadIdx.x + 256 * j, r = idx / (KS * 4), k0 = (idx % (KS * 4)) * 8;
      if (idx < 16 * KS * 4) *reinterpret_cast<uint4*>(wl + r * WLP + k0) = wst[j];
    }
  }
  STAMP_FINE(11);
  // dgrad lane constants; k-chunks past KTOT have zero weights and read a valid in-tile address
  int tapoff[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k0 = 32 * s + 8 * (lane >> 4);
    const int tap = k0 / C, c0 = k0 % C;
    tapoff[s] = k0 < KTOT ? -((tap / 3) * WP + (tap % 3)) * CP + c0 : 0;
  }
  const int ci0 = ct * 16 + (lane >> 4) * 4;
  int tbo[MTD], rpo[MTD];
  uint32_t pofs[MTD];
#pragma unroll
  for (int i = 0; i < MTD; ++i) {
    const int p = (wave / NT + WPT * i) * 16 + (lane & 15);
    tbo[i] = ((p / W + 2) * WP + p % W + 2) * CP;
    pofs[i] = p * C + ci0;
    rpo[i] = p * CP + ci0;
  }
  // wgrad lane constants (pixel rows 8g+q and +4 of each 32-pixel k-step)
  const int g = lane >> 4, q = (lane & 15) >> 2, p4 = lane & 3;
  const int pa = 8 * g + q, pb = pa + 4;
  const int da_off = ((pa / W + 1) * WP + pa % W + 1) * CP + 4 * p4;
  const int db_off = ((pb / W + 1) * WP + pb % W + 1) * CP + 4 * p4;
  const int xa_off = ((pa / W) * WP + pa % W) * CP + 4 * p4, xb_off = ((pb / W) * WP + pb % W) * CP + 4 * p4;
  int boff[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int nt = min(wave + 4 * j, NTN - 1);  // duplicates (nt >= NTN) are computed, never flushed
    const int tap = (nt * 16) / C, cb = (nt * 16) % C;
    boff[j] = ((tap / 3) * WP + (tap % 3)) * CP + cb;
  }
  f32x4_t wacc[NJ][MT];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int m = 0; m < MT; ++m) wacc[j][m] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  f32x2_t ssum[2] = {{0.f, 0.f}, {0.f, 0.f}}, ssq[2] = {{0.f, 0.f}, {0.f, 0.f}};
  // dgrad epilogue operands from global memory one iteration ahead (software-pipelined)
  uint2 nres[MTD], nxres[MTD], nhres[MTD];
  auto epi_load = [&](int it_) {
    const long b_ = (long)(it_ / BANDS) * IMG + (it_ % BANDS) * ROWS * ROW;
#pragma unroll
    for (int i = 0; i < MTD; ++i) {
      if constexpr (EPI & 1) nres[i] = *reinterpret_cast<const uint2*>(k_res + b_ + pofs[i]);
      if constexpr (!RAWX) nxres[i] = *reinterpret_cast<const uint2*>(k_xm + b_ + pofs[i]);
      if constexpr ((EPI & 8) != 0) nhres[i] = *reinterpret_cast<const uint2*>(k_x3 + b_ + pofs[i]);
    }
  };
  if constexpr (DG) epi_load(it0);

  __syncthreads();  // coefficients
  STAMP(1);
  // Coefficients of the thread's channels held in registers for the whole launch instead of re-read from LDS per
  // band, where the VGPR budget of the launch's occupancy has room: KREG_D the dY staging transform (BN-backward
  // [+ residual]), KREG_X the x staging (BN + ReLU), KREG_E the dgrad epilogue's mask / x-hat coefficients.
  // C = 16 fused with MODE_DY 3 (2 waves / SIMD: 176 -> 222 VGPRs); the dgrad-only role (2 waves / SIMD) at every C,
  // its epilogue set up to C = 32 (C = 64 would pass 256); the deferred wgrad role's staging sets at every C
  // (conv_wgrad_all: <64, 32> runs one wave per SIMD anyway, <16, 16> is LDS-bound at 3 workgroups per CU)
  constexpr bool KREG_F = DTF_BWD_COEFREG && C == 16 && ROLE == 0 && (MODE_DY == 3 || (MODE_DY == 2 && DTF_FUSED16_M2_WAVES == 2));
  constexpr bool KREG_D = KREG_F || (DTF_BWD_COEFREG && ROLE != 0 && XSTORE);
  constexpr bool KREG_X = KREG_F || (DTF_BWD_COEFREG && ROLE == 2);
  constexpr bool KREG_E = KREG_F || (DTF_BWD_COEFREG && ROLE == 1 && C <= 32);
  float ka[KREG_D ? 8 : 1], kb[KREG_D ? 8 : 1], kc[KREG_D ? 8 : 1], xsc[KREG_X ? 8 : 1], xsh[KREG_X ? 8 : 1];
  if constexpr (KREG_D) st.load_coef3(ka, kb, kc, coef_d);
  if constexpr (KREG_X) st.load_coef1(xsc, xsh, ecoef);
  if constexpr (XSTORE)  // (the wgrad role stages the same transform but never writes xout)
    st.template store_x<MODE_DY == 3 ? 3 : 2, KREG_D>(FDBUF(0), dv, dv2, dv3, dm, coef_d,
                                                      (DG && k_xout) ? k_xout + cimg * IMG : nullptr, cgy0, ka, kb,
                                                      kc);
  else
    st.template store<MODE_DY>(FDBUF(0), dv, dv2, dm, coef_d);
  if constexpr (KREG_X)
    st.store1r(FXBUF(0), xv_, xm, xsc, xsh);
  else if constexpr (WG)
    st.template store<1>(FXBUF(0), xv_, unused, xm, ecoef);
  if constexpr (RAWX) st.store_raw(FXRAW(0), xv_, xm);
  f32x2_t esc0, esc1, esh0, esh1, enm0, enm1, eiv0, eiv1;
  if constexpr (KREG_E) {
    esc0 = lds2(ecoef + ci0), esc1 = lds2(ecoef + ci0 + 2);
    esh0 = lds2(ecoef + 64 + ci0), esh1 = lds2(ecoef + 64 + ci0 + 2);
    enm0 = lds2(ecoef + 128 + ci0), enm1 = lds2(ecoef + 128 + ci0 + 2);
    eiv0 = lds2(ecoef + 192 + ci0), eiv1 = lds2(ecoef + 192 + ci0 + 2);
  }
  __syncthreads();
  STAMP(2);
  for (int k = 0; k < nit; ++k) {
    const int it = it0 + k;
    const int img = it / BANDS, r0 = (it % BANDS) * ROWS;
    const bool more = k + 1 < nit;
    const long band = (long)img * IMG + r0 * ROW;
    // epilogue operands before the prefetch (counted vmcnt)
    uint2 rres[MTD], xres[MTD], hres[MTD];
    if constexpr (DG) {
#pragma unroll
    for (int i = 0; i < MTD; ++i) {
      if constexpr (EPI & 1) rres[i] = nres[i];
      if constexpr ((EPI & 8) != 0) hres[i] = nhres[i];
      if constexpr (RAWX)
        xres[i] = *reinterpret_cast<const uint2*>(FXRAW(k) + rpo[i]);
      else
        xres[i] = nxres[i];
    }
    }
    if (more) {
      cimg = (it + 1) / BANDS;
      cgy0 = ((it + 1) % BANDS) * ROWS - 1;
      dm = xm = st.mask(cgy0);
      st.template load<MODE_DY == 3 ? 2 : MODE_DY>(dv, dv2, dm, k_x + cimg * IMG, k_x2 + cimg * IMG, cgy0);
      if constexpr (MODE_DY == 3) st.template load<0>(dv3, unused, dm, k_x3 + cimg * IMG, nullptr, cgy0);
      if constexpr (WG) st.template load<1>(xv_, unused, xm, k_xm + cimg * IMG, nullptr, cgy0);
      if constexpr (DG) epi_load(it + 1);
    }
    const bf16_t* dcur = FDBUF(k);
    const bf16_t* xcur = FXBUF(k);
    // ---- dgrad (KREG_E: the epilogue coefficients are loop-invariant registers, read before the loop)
    const f32x2_t sc0 = KREG_E ? esc0 : lds2(ecoef + ci0), sc1 = KREG_E ? esc1 : lds2(ecoef + ci0 + 2);
    const f32x2_t sh0 = KREG_E ? esh0 : lds2(ecoef + 64 + ci0), sh1 = KREG_E ? esh1 : lds2(ecoef + 64 + ci0 + 2);
    const f32x2_t nm0 = KREG_E ? enm0 : lds2(ecoef + 128 + ci0), nm1 = KREG_E ? enm1 : lds2(ecoef + 128 + ci0 + 2);
    const f32x2_t iv0 = KREG_E ? eiv0 : lds2(ecoef + 192 + ci0), iv1 = KREG_E ? eiv1 : lds2(ecoef + 192 + ci0 + 2);
    if constexpr (DG) {
#pragma unroll
    for (int i = 0; i < MTD; ++i) {
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        bf16x8_t wa;
        if constexpr (WLDS)
          wa = *reinterpret_cast<const bf16x8_t*>(wl + (lane & 15) * WLP + 32 * s + 8 * (lane >> 4));
        else
          wa = afr[s];
        acc = mfma16(wa, *reinterpret_cast<const bf16x8_t*>(dcur + tbo[i] + tapoff[s]), acc);
      }
      f32x2_t v0 = {acc[0], acc[1]}, v1 = {acc[2], acc[3]};
      if constexpr (EPI & 1) {
        v0 += unpk2(rres[i].x);
        v1 += unpk2(rres[i].y);
      }
      const f32x2_t x0 = unpk2(xres[i].x), x1 = unpk2(xres[i].y);
      const f32x2_t pre0 = x0 * sc0 + sh0, pre1 = x1 * sc1 + sh1;
      v0.x = pre0.x > 0.f ? v0.x : 0.f;
      v0.y = pre0.y > 0.f ? v0.y : 0.f;
      v1.x = pre1.x > 0.f ? v1.x : 0.f;
      v1.y = pre1.y > 0.f ? v1.y : 0.f;
      uint2 pk;
      pk.x = pk2(v0);
      pk.y = pk2(v1);
      st_act8(k_y + band + pofs[i], pk);
      const f32x2_t dz0 = unpk2(pk.x), dz1 = unpk2(pk.y);
      ssum[0] += dz0;
      ssum[1] += dz1;
      if constexpr ((EPI & 8) != 0) {  // x-hat of the chained BN's input x3
        ssq[0] += dz0 * (unpk2(hres[i].x) * iv0 + nm0);
        ssq[1] += dz1 * (unpk2(hres[i].y) * iv1 + nm1);
      } else {
        ssq[0] += dz0 * (x0 * iv0 + nm0);
        ssq[1] += dz1 * (x1 * iv1 + nm1);
      }
    }
    }
    // ---- wgrad
    if constexpr (WG) {
#pragma unroll
    for (int ks = 0; ks < NK; ++ks) {
      bf16x8_t af[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        s16x4_t lo = ds_read_tr(dcur + da_off + ks * KINC + m * 16);
        s16x4_t hi = ds_read_tr(dcur + db_off + ks * KINC + m * 16);
        af[m] = (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
      bf16x8_t bfr[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        s16x4_t lo = ds_read_tr(xcur + xa_off + ks * KINC + boff[j]);
        s16x4_t hi = ds_read_tr(xcur + xb_off + ks * KINC + boff[j]);
        bfr[j] = (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int m = 0; m < MT; ++m) wacc[j][m] = mfma16(af[m], bfr[j], wacc[j][m]);
    }
    }
    if (more) {
      if constexpr (SB) __syncthreads();  // every wave is done with the current tiles
      if constexpr (XSTORE)
        st.template store_x<MODE_DY == 3 ? 3 : 2, KREG_D>(FDBUF(k + 1), dv, dv2, dv3, dm, coef_d,
                                                          (DG && k_xout) ? k_xout + cimg * IMG : nullptr, cgy0, ka,
                                                          kb, kc);
      else
        st.template store<MODE_DY>(FDBUF(k + 1), dv, dv2, dm, coef_d);
      if constexpr (KREG_X)
        st.store1r(FXBUF(k + 1), xv_, xm, xsc, xsh);
      else if constexpr (WG)
        st.template store<1>(FXBUF(k + 1), xv_, unused, xm, ecoef);
      if constexpr (RAWX) st.store_raw(FXRAW(k + 1), xv_, xm);
    }
    __syncthreads();
  }
#undef FDBUF
#undef FXBUF
#undef FXRAW
  STAMP(3);
  if constexpr (DG) {
    const float s4[4] = {ssum[0].x, ssum[0].y, ssum[1].x, ssum[1].y};
    const float q4[4] = {ssq[0].x, ssq[0].y, ssq[1].x, ssq[1].y};
    reduce_stats_to_lds(acc_lds, s4, q4, ci0, lane);
    __syncthreads();
  }
  if constexpr (DG && (!(EPI & 2) || (EPI & 8))) flush_stats_r(k_st_out, acc_lds, slot, C, bid);
  STAMP(4);
  if constexpr (!WG) {
    STAMP_DRAIN(5);
    STAMP_FLUSH(a.cin_real, nit);
    return;
  }
  if (k_slab) {
    // partial-sum slab [wg][j][m][256 threads][4]: one 16-byte store per lane per accumulator tile (a 1 KB
    // row per wave instruction; the store tail is issue-bound); dw_slab_reduce sums a member's slabs
    f32x4_t* sb = reinterpret_cast<f32x4_t*>(k_slab + (long)bid * (NJ * MT * 4 * 256)) + threadIdx.x;
    {
      // write-through (sc1) buffer stores: the slab does not sit dirty in L2 at the kernel boundary
      const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(k_slab + (long)bid * (NJ * MT * 4 * 256), 0,
                                                         NJ * MT * 4 * 256 * 4, 0x00020000);
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int m = 0; m < MT; ++m)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, wacc[j][m]), rsrc,
                                                 (((j * MT + m) * 256) + (int)threadIdx.x) * 16, 0, 16);
    }
    STAMP_DRAIN(5);
    STAMP_FLUSH(a.cin_real, nit);
    return;
  }
  float* gb = k_grads + (long)slot * k_g_mstride + k_g_off;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int nt = wave + 4 * j;
    if (nt < NTN) {
      const int tap = (nt * 16) / C, ci = (nt * 16) % C + (lane & 15);
#pragma unroll
      for (int m = 0; m < MT; ++m) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = m * 16 + 4 * (lane >> 4) + r;
          atomicAdd(gb + ((long)co * 9 + tap) * C + ci, wacc[j][m][r]);
        }
      }
    }
  }
  STAMP_DRAIN(5);
  STAMP_FLUSH(a.cin_real, nit);
}

// Weight-gradient role with the input tiles prefetched TWO (image, band) iterations ahead (two register sets; the
// loop unrolled by two so each set is a compile-time array).  Same operands, staging transforms, MFMA order and slab
// layout as conv_bwd_body<C, MODE_DY, 0, 2> -- bitwise the same partials -- for the deferred jobs of
// conv_wgrad_all_kernel: one round of staging loads in flight behind the MFMAs was not enough to cover the L2 /
// MALL latency of these 1-2-workgroups-per-CU launches (C = 64: ~1 TB/s of traffic, 3x its MFMA + HBM floor).
template <int C, int MODE_DY>
__device__ __forceinline__ void conv_wgrad_pf2_body(const ConvArgs& a, const int bid, char* smem) {
  static_assert(MODE_DY == 0 || MODE_DY == 2, "deferred wgrad jobs: plain dY or BN-backward(dz, h)");
  constexpr int ROWS = 8, W = 512 / C, H = W, BANDS = H / ROWS;
  constexpr int MT = C / 16, NTN = 9 * C / 16, NJ = (NTN + 3) / 4;
  constexpr int CP = cpad<C>(), RT = ROWS + 2, WP = wpitch<C>();
  constexpr int TSZ = (RT * WP * CP + 8 + 63) & ~63;
  constexpr int IMG = H * W * C;
  constexpr int NK = ROWS * W / 32, RSTEP = 32 / W, KINC = RSTEP * WP * CP;
  using St = Stage<C, RT, W, H, CP, WP>;
  constexpr int MAXC = St::MAXC;
  float* coef_d = reinterpret_cast<float*>(smem);
  float* ecoef = coef_d + 192;
  bf16_t* t0 = reinterpret_cast<bf16_t*>(smem + 2304);
#define PDBUF(i) (t0 + ((i) & 1) * 2 * TSZ)
#define PXBUF(i) (t0 + TSZ + ((i) & 1) * 2 * TSZ)
  const bf16_t* k_x = a.x;
  const bf16_t* k_x2 = a.x2;
  const bf16_t* k_xm = a.xm;
  const float* k_st_in = a.st_in;
  const float* k_st_in_b = a.st_in_b;
  const float* k_st_ep = a.st_ep;
  const float* k_params = a.params;
  const float* k_cnt = a.cnt;
  float* k_slab = a.slab;
  float* k_grads = a.grads;
  const int4* k_work = a.work;
  int k_in_gamma = a.in_gamma, k_in_beta = a.in_beta, k_ep_gamma = a.ep_gamma, k_ep_beta = a.ep_beta;
  long k_p_mstride = a.p_mstride, k_g_mstride = a.g_mstride, k_g_off = a.g_off;
  int k_u_items = a.u_items, k_u_chunk = a.u_chunk, k_u_per = a.u_per;
  kpin(k_x); kpin(k_x2); kpin(k_xm); kpin(k_st_in); kpin(k_st_in_b); kpin(k_st_ep); kpin(k_params); kpin(k_cnt);
  kpin(k_slab); kpin(k_grads); kpin(k_work); kpin(k_in_gamma); kpin(k_in_beta); kpin(k_ep_gamma); kpin(k_ep_beta);
  kpin(k_p_mstride); kpin(k_g_mstride); kpin(k_g_off); kpin(k_u_items); kpin(k_u_chunk); kpin(k_u_per);
  int4 wk;
  if (k_u_items > 0) {
    const int m = bid / k_u_items, kk = bid - m * k_u_items, it0_ = kk * k_u_chunk;
    wk = make_int4(m * k_u_per + it0_, min(k_u_chunk, k_u_per - it0_), 0, m);
  } else {
    wk = k_work[bid];
    wk = make_int4(__builtin_amdgcn_readfirstlane(wk.x), __builtin_amdgcn_readfirstlane(wk.y),
                   __builtin_amdgcn_readfirstlane(wk.z), __builtin_amdgcn_readfirstlane(wk.w));
  }
  DTF_WG_CHECK(wk.x >= 0 && wk.y >= 0 && wk.w >= 0 && wk.z >= 0 && a.Hi > 0 && a.Wi > 0 && a.rows > 0);
  const int it0 = wk.x, nit = wk.y, slot = wk.w;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  CoefLd<MODE_DY == 0 ? 0 : 2> cld;
  coef_issue<C, MODE_DY == 0 ? 0 : 2>(cld, k_params, k_p_mstride, slot, k_st_in, k_st_in_b, k_in_gamma, k_in_beta);
  CoefLd<1> cle;
  coef_issue<C, 1>(cle, k_params, k_p_mstride, slot, k_st_ep, nullptr, k_ep_gamma, k_ep_beta);
  const float n_hw = k_cnt[slot] * (float)(H * W);
  St st;
  st.init();
  // two register sets: set A holds the even iterations' tiles, set B the odd ones
  uint4 dA[MAXC], d2A[MAXC], xA[MAXC], dB[MAXC], d2B[MAXC], xB[MAXC], unused[MAXC];
  unsigned mA = 0, mB = 0;
  int gA = 0, gB = 0;  // first tile row of the staged band (for the staging masks)
  auto issue = [&](int it, uint4 (&d)[MAXC], uint4 (&d2)[MAXC], uint4 (&xv)[MAXC], unsigned& m, int& gy0) {
    const int img = it / BANDS;
    gy0 = (it % BANDS) * ROWS - 1;
    m = st.mask(gy0);
    st.template load<MODE_DY>(d, d2, m, k_x + img * IMG, k_x2 + img * IMG, gy0);
    st.template load<1>(xv, unused, m, k_xm + img * IMG, nullptr, gy0);
  };
  auto put = [&](int k, const uint4 (&d)[MAXC], const uint4 (&d2)[MAXC], const uint4 (&xv)[MAXC], unsigned m,
                 int gy0) {
    if constexpr (MODE_DY >= 2)
      st.template store_x<2>(PDBUF(k), d, d2, unused, m, coef_d, nullptr, gy0);
    else
      st.template store<MODE_DY>(PDBUF(k), d, d2, m, coef_d);
    st.template store<1>(PXBUF(k), xv, unused, m, ecoef);
  };
  issue(it0, dA, d2A, xA, mA, gA);
  if (nit > 1) issue(it0 + 1, dB, d2B, xB, mB, gB);
  coef_reduce<C, MODE_DY == 0 ? 0 : 2>(cld);
  coef_reduce<C, 1>(cle);
  coef_finish<C, MODE_DY == 0 ? 0 : 2>(coef_d, cld, n_hw);
  if (threadIdx.x < C) {
    float mean, inv;
    coef_moments<1>(cle, n_hw, mean, inv);
    const float scale = cle.g * inv;
    ecoef[threadIdx.x] = scale;
    ecoef[64 + threadIdx.x] = cle.b - mean * scale;
  }
  const int g = lane >> 4, q = (lane & 15) >> 2, p4 = lane & 3;
  const int pa = 8 * g + q, pb = pa + 4;
  const int da_off = ((pa / W + 1) * WP + pa % W + 1) * CP + 4 * p4;
  const int db_off = ((pb / W + 1) * WP + pb % W + 1) * CP + 4 * p4;
  const int xa_off = ((pa / W) * WP + pa % W) * CP + 4 * p4, xb_off = ((pb / W) * WP + pb % W) * CP + 4 * p4;
  int boff[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int nt = min(wave + 4 * j, NTN - 1);
    const int tap = (nt * 16) / C, cb = (nt * 16) % C;
    boff[j] = ((tap / 3) * WP + (tap % 3)) * CP + cb;
  }
  f32x4_t wacc[NJ][MT];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int m = 0; m < MT; ++m) wacc[j][m] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  __syncthreads();  // coefficients
  put(0, dA, d2A, xA, mA, gA);
  __syncthreads();
  auto mfmas = [&](int k) {
    const bf16_t* dcur = PDBUF(k);
    const bf16_t* xcur = PXBUF(k);
#pragma unroll
    for (int ks = 0; ks < NK; ++ks) {
      bf16x8_t af[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        s16x4_t lo = ds_read_tr(dcur + da_off + ks * KINC + m * 16);
        s16x4_t hi = ds_read_tr(dcur + db_off + ks * KINC + m * 16);
        af[m] = (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
      bf16x8_t bfr[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        s16x4_t lo = ds_read_tr(xcur + xa_off + ks * KINC + boff[j]);
        s16x4_t hi = ds_read_tr(xcur + xb_off + ks * KINC + boff[j]);
        bfr[j] = (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int m = 0; m < MT; ++m) wacc[j][m] = mfma16(af[m], bfr[j], wacc[j][m]);
    }
  };
  // iteration k: tiles of k + 1 sit in the other register set (loaded an iteration ago), k + 2 is issued into the set
  // that held k (already in LDS)
  for (int k = 0; k < nit; k += 2) {
    if (k + 2 < nit) issue(it0 + k + 2, dA, d2A, xA, mA, gA);
    mfmas(k);
    if (k + 1 < nit) put(k + 1, dB, d2B, xB, mB, gB);
    __syncthreads();
    if (k + 1 >= nit) break;
    if (k + 3 < nit) issue(it0 + k + 3, dB, d2B, xB, mB, gB);
    mfmas(k + 1);
    if (k + 2 < nit) put(k + 2, dA, d2A, xA, mA, gA);
    __syncthreads();
  }
#undef PDBUF
#undef PXBUF
  if (k_slab) {
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(k_slab + (long)bid * (NJ * MT * 4 * 256), 0,
                                                       NJ * MT * 4 * 256 * 4, 0x00020000);
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int m = 0; m < MT; ++m)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, wacc[j][m]), rsrc,
                                               (((j * MT + m) * 256) + (int)threadIdx.x) * 16, 0, 16);
    return;
  }
  float* gb = k_grads + (long)slot * k_g_mstride + k_g_off;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int nt = wave + 4 * j;
    if (nt < NTN) {
      const int tap = (nt * 16) / C, ci = (nt * 16) % C + (lane & 15);
#pragma unroll
      for (int m = 0; m < MT; ++m) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = m * 16 + 4 * (lane >> 4) + r;
          atomicAdd(gb + ((long)co * 9 + tap) * C + ci, wacc[j][m][r]);
        }
      }
    }
  }
}

// Trailing workgroups of a backward launch: dW slab reduction of the PREVIOUS launch (r = index among them).
__device__ __forceinline__ void trailing_reduce(const ConvArgs& a, int r, char* smem) {
  float* part = reinterpret_cast<float*>(smem);
  // r_nblk reduce workgroups per member, each looping over every r_nblk-th block of 32 slab elements
  const int bx = r % a.r_nblk, by = r / a.r_nblk;
  if (a.r_c == 16) slab_reduce_wg<16>(a.rslab, a.rtab, a.grads, a.g_mstride, a.r_goff, bx, by, part, a.r_nblk);
  else if (a.r_c == 32) slab_reduce_wg<32>(a.rslab, a.rtab, a.grads, a.g_mstride, a.r_goff, bx, by, part, a.r_nblk);
  else if (a.r_c == 64) slab_reduce_wg<64>(a.rslab, a.rtab, a.grads, a.g_mstride, a.r_goff, bx, by, part, a.r_nblk);
}

template <int C, int MODE_DY, int EPI>
__global__ __launch_bounds__(256, FUSED_WAVES(C, MODE_DY)) void conv_bwd_fused_kernel(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if ((int)blockIdx.x >= a.n_main) {
    trailing_reduce(a, (int)blockIdx.x - a.n_main, smem);
    return;
  }
  conv_bwd_body<C, MODE_DY, EPI, 0>(a, (int)blockIdx.x, smem);
}

// Dual backward (engine/hip_resnet.py _conv_bwd_dual): ONE launch whose workgroups take
// different roles of the same layer -- [0, a.n_main): dgrad role (args a: staging, dgrad MFMAs, mask / stats
// epilogue, dz out); [a.n_main, + b.n_main): wgrad role (args b: its own work split over the same (image, band)
// iterations, the same dY / X staging, wgrad MFMAs, dW slab); then the trailing slab reduction of the previous
// launch (a.r_*).  The two roles run side by side on different CUs, so the layer costs max(dgrad, wgrad) instead
// of their sum while a small population leaves most CUs idle.
template <int C, int MODE_DY, int EPI>
__global__ __launch_bounds__(256, FUSED_WAVES(C, MODE_DY)) void conv_bwd_dual_kernel(ConvArgs a, ConvArgs b) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int bx = (int)blockIdx.x;
  int na = a.n_main, nb = b.n_main;
  kpin(na), kpin(nb);  // both role bounds in one scalar round trip
  if (bx < na) {
    conv_bwd_body<C, MODE_DY, EPI, 1>(a, bx, smem);
  } else if (bx < na + nb) {
    conv_bwd_body<C, MODE_DY, EPI & 2, 2>(b, bx - a.n_main, smem);
  } else {
    trailing_reduce(a, bx - a.n_main - b.n_main, smem);
  }
}

// dgrad role alone (the backward launch of a layer whose wgrad is deferred to conv_wgrad_all_kernel): without the
// wgrad role's accumulators the kernel fits two waves per SIMD (the dual kernel is register-capped at one).
template <int C, int MODE_DY, int EPI, int ROWS = 8>
__global__ __launch_bounds__(256, 2) void conv_bwd_dg_kernel(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  conv_bwd_body<C, MODE_DY, EPI, 1, ROWS>(a, (int)blockIdx.x, smem);
}

// Deferred weight gradients (engine/hip_resnet.py): the backward launches of a deferred layer run only their dgrad
// role (the critical path: every layer waits for the previous one's BatchNorm statistics), and the wgrad work of
// all those layers runs afterwards as wide launches (conv_wgrad_all_kernel) -- hundreds of independent workgroups
// instead of a wgrad role that stretched every latency-bound backward launch.  jobs[j]: the wgrad-role arguments
// of layer j (dY / x operands kept alive for the whole backward, own dW slab).
// The deferred wgrad jobs of the channel widths CA and CB (both dY modes) in ONE launch: map[block] = (job,
// workgroup index, C, mode); the jobs of different layers / widths overlap instead of each launch draining its own
// tail.  <64, 32> (register-heavy, one wave per SIMD) and <16, 16> (kept apart: it runs at several waves per SIMD).
template <int CA, int CB>
__global__ __launch_bounds__(256, 1) void conv_wgrad_all_kernel(const ConvArgs* __restrict__ jobs,
                                                                const int4* __restrict__ map) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int4 m = map[blockIdx.x];
  const int j = __builtin_amdgcn_readfirstlane(m.x), bid = __builtin_amdgcn_readfirstlane(m.y);
  const int c = __builtin_amdgcn_readfirstlane(m.z), mode = __builtin_amdgcn_readfirstlane(m.w);
  // (the <64, 32> kernel runs one wave per SIMD either way: 300 VGPRs one-ahead, 502 with the two C = 64 register
  // sets; <16, 16> stays LDS-bound at 3 workgroups per CU: 108 -> 140 VGPRs)
  if (c == CA) {
    if constexpr (DTF_WGRAD_PF2 && CA <= DTF_WGRAD_PF2_MAXC) {
      if (mode == 0) conv_wgrad_pf2_body<CA, 0>(jobs[j], bid, smem); else conv_wgrad_pf2_body<CA, 2>(jobs[j], bid, smem);
    } else {
      if (mode == 0) conv_bwd_body<CA, 0, 0, 2>(jobs[j], bid, smem); else conv_bwd_body<CA, 2, 0, 2>(jobs[j], bid, smem);
    }
  } else if constexpr (CB != CA) {
    if constexpr (DTF_WGRAD_PF2 && CB <= DTF_WGRAD_PF2_MAXC) {
      if (mode == 0) conv_wgrad_pf2_body<CB, 0>(jobs[j], bid, smem); else conv_wgrad_pf2_body<CB, 2>(jobs[j], bid, smem);
    } else {
      if (mode == 0) conv_bwd_body<CB, 0, 0, 2>(jobs[j], bid, smem); else conv_bwd_body<CB, 2, 0, 2>(jobs[j], bid, smem);
    }
  }
}

// Sum of one member's per-workgroup dW slabs (written by conv_bwd_fused_kernel) into its gradient row.
// grid (E/32, members), 256 threads = 32 slab elements x 8 workgroup groups (each thread strides over the
// member's slabs, then an LDS reduction across the 8 groups); red[y] = (first wg, n wgs, -, slot).  Element
// e of a slab is (j, m, r, thread) -> dW[co][tap][ci] with the MFMA C/D lane mapping of the fused kernel;
// duplicate tiles (nt >= NTN) are skipped.
template <int C>
__global__ __launch_bounds__(256) void dw_slab_reduce_kernel(const float* __restrict__ slab,
                                                             const int4* __restrict__ red, float* __restrict__ grads,
                                                             long g_mstride, long g_off) {
  __shared__ float part[8 * 33];
  slab_reduce_wg<C>(slab, red, grads, g_mstride, g_off, blockIdx.x, blockIdx.y, part, gridDim.x);
}

// Slab reduction job (slab_reduce_all_kernel): the dW slabs of one deferred layer
// blockIdx.z = layer, y = member row of that layer's reduce table, x = 32-element block.
struct SlabJob {
  const float* slab;
  const int4* red;
  long g_off;
  int nmem;
  int pad;
};

// Every deferred dW reduction of a step in ONE launch (x = block of 256 slab elements, y = member row of the job's
// reduce table, z = job).  z < nsj: a conv slab job (channel width C in SlabJob.pad): thread t reads elements
// 4*(t%64)..+3 (float4) of every 4th slab starting at t/64, four loads in flight; the partial sums meet in LDS and
// thread t finishes element t (fixed summation order).  Else dense job z - nsj: 32 elements x 8 slab groups per
// block, LDS reduction across the groups.  Blocks past a job's extent exit (workgroup-uniform).
__global__ __launch_bounds__(256) void slab_reduce_all_kernel(const SlabJob* __restrict__ sjobs, int nsj,
                                                              const DenseJob* __restrict__ djobs,
                                                              float* __restrict__ grads, long g_mstride) {
  __shared__ float4 part4[4][64];
  if ((int)blockIdx.z < nsj) {
    SlabJob j = sjobs[blockIdx.z];
    kpin(j.slab), kpin(j.red);
    const int C = j.pad, MT = C / 16, NTN = 9 * C / 16, NJ = (NTN + 3) / 4, E = NJ * MT * 4 * 256;
    if ((int)blockIdx.y >= j.nmem || (int)blockIdx.x * 256 >= E) return;
    const int4 rd = j.red[blockIdx.y];
    const int q = threadIdx.x & 63, gg = threadIdx.x >> 6;
    const long E4 = E / 4;
    // a block walks every gridDim.x-th 256-element chunk of the job (the host caps gridDim.x: one chunk per block
    // made 20k blocks of 8 KB each at pop 8 -- launch-bound); the per-element summation order is unchanged
    for (int xb = blockIdx.x; xb * 256 < E; xb += gridDim.x) {
      const int e0 = xb * 256;
      const float4* p = reinterpret_cast<const float4*>(j.slab + (long)rd.x * E + e0) + q;
      float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0, s2 = s0, s3 = s0;
      int g = gg;
      for (; g + 12 < rd.y; g += 16) {
        const float4 a0 = p[(long)g * E4], a1 = p[(long)(g + 4) * E4], a2 = p[(long)(g + 8) * E4],
                     a3 = p[(long)(g + 12) * E4];
        s0.x += a0.x; s0.y += a0.y; s0.z += a0.z; s0.w += a0.w;
        s1.x += a1.x; s1.y += a1.y; s1.z += a1.z; s1.w += a1.w;
        s2.x += a2.x; s2.y += a2.y; s2.z += a2.z; s2.w += a2.w;
        s3.x += a3.x; s3.y += a3.y; s3.z += a3.z; s3.w += a3.w;
      }
      for (; g < rd.y; g += 4) {
        const float4 a0 = p[(long)g * E4];
        s0.x += a0.x; s0.y += a0.y; s0.z += a0.z; s0.w += a0.w;
      }
      part4[gg][q] = make_float4((s0.x + s1.x) + (s2.x + s3.x), (s0.y + s1.y) + (s2.y + s3.y),
                                 (s0.z + s1.z) + (s2.z + s3.z), (s0.w + s1.w) + (s2.w + s3.w));
      __syncthreads();
      const float* pf = reinterpret_cast<const float*>(part4);
      const int t0 = threadIdx.x;
      const float sum = (pf[t0] + pf[256 + t0]) + (pf[512 + t0] + pf[768 + t0]);
      const int e = e0 + t0;
      const int r = e & 3, t = (e >> 2) & 255, m = (e >> 10) % MT, jj = (e >> 10) / MT;  // slab [j][m][t][r]
      const int wave = t >> 6, lane = t & 63, nt = wave + 4 * jj;
      if (nt < NTN) {
        const int tap = (nt * 16) / C, ci = (nt * 16) % C + (lane & 15), co = m * 16 + 4 * (lane >> 4) + r;
        grads[(long)rd.w * g_mstride + j.g_off + ((long)co * 9 + tap) * C + ci] += sum;
      }
      __syncthreads();  // part4 is rewritten by the next chunk
    }
    return;
  }
  float* part = reinterpret_cast<float*>(part4);  // [8][33]
  DenseJob j = djobs[blockIdx.z - nsj];
  kpin(j.slab), kpin(j.red);
  if ((int)blockIdx.y >= j.nmem) return;
  const int el = threadIdx.x & 31, gg = threadIdx.x >> 5;
  const int4 rd = j.red[blockIdx.y];
  for (int bx = blockIdx.x; bx * 32 < j.kel; bx += gridDim.x) {
    const int e = bx * 32 + el;
    const bool ok = e < j.kel;
    // four slab loads in flight per thread and trip (the 2-deep chain left this latency-bound at small
    // populations: 128 slabs per member of the standalone wgrad launches)
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int g = gg;
    const float* sp = j.slab + (long)rd.x * j.kel + (ok ? e : 0);
    for (; g + 24 < rd.y; g += 32) {
      const float a0 = sp[(long)g * j.kel], a1 = sp[(long)(g + 8) * j.kel], a2 = sp[(long)(g + 16) * j.kel],
                  a3 = sp[(long)(g + 24) * j.kel];
      s0 += a0;
      s1 += a1;
      s2 += a2;
      s3 += a3;
    }
    for (; g < rd.y; g += 8) s0 += sp[(long)g * j.kel];
    part[gg * 33 + el] = ok ? (s0 + s1) + (s2 + s3) : 0.f;
    __syncthreads();
    if (gg == 0 && ok) {
      float sum = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) sum += part[i * 33 + el];
      grads[(long)rd.w * g_mstride + j.g_off + e] += sum;
    }
    __syncthreads();
  }
}

template <typename KernelT>
int launch(KernelT k, int nblocks, size_t lds, hipStream_t st, const ConvArgs& a) {
  if (nblocks <= 0) return 0;
  DTF_HOST_CHECK(lds <= 160 * 1024);
  DTF_HOST_CHECK(a.work != nullptr);
  DTF_HOST_CHECK(DTF_ALIGNED16(a.x) && DTF_ALIGNED16(a.w) && DTF_ALIGNED16(a.y) && DTF_ALIGNED16(a.dy));
  DTF_HOST_CHECK(a.Hi > 0 && a.Wi > 0 && a.Ho > 0 && a.Wo > 0 && a.rows > 0 && a.Ho <= a.Hi);
  hipLaunchKernelGGL(k, dim3(nblocks), dim3(256), lds, st, a);
  return DTF_CHECK_LAUNCH();
}

}  // namespace

// ------------------------------------------------------------------------------ dispatch
// cfg: CIN, COUT, S, K and the mode flags select one instantiation.

#define FWD_CASE(CI, CO, S, K, M, R, ST)                                                             \
  if (cin == CI && cout == CO && s == S && k == K && mode == M && resid == R && stats == ST)         \
    return launch(conv_fwd_kernel<CI, CO, S, K, M, R, ST>, nblocks, lds, stream, *args);

#define DGRAD_CASE(CI, CO, S, K, M, E)                                                               \
  if (cin == CI && cout == CO && s == S && k == K && mode == M && epi == E)                          \
    return launch(conv_dgrad_kernel<CI, CO, S, K, M, E>, nblocks, lds, stream, *args);

#define WGRAD_CASE(CI, CO, S, K, MX, MD)                                                             \
  if (cin == CI && cout == CO && s == S && k == K && mode_x == MX && mode_dy == MD)                  \
    return launch(conv_wgrad_kernel<CI, CO, S, K, MX, MD>, nblocks, lds, stream, *args);

// rows: band height (8; 4: half-image bands for C = 64, twice the workgroups of one member; C = 32 measured slower)
DTF_API int dtf_conv_fwd_s1(const ConvArgs* args, int c, int mode, int resid, int rows, int nblocks, int lds,
                            hipStream_t stream) {
  DTF_HOST_CHECK(args->rows == rows);
  if (rows == 4) {
    if (c == 64 && mode == 1 && resid == 0) return launch(conv_fwd_s1_kernel<64, 1, false, 4>, nblocks, lds, stream, *args);
    if (c == 64 && mode == 1 && resid == 1) return launch(conv_fwd_s1_kernel<64, 1, true, 4>, nblocks, lds, stream, *args);
    return -1;
  }
#define S1_CASE(CC, M, R) \
  if (c == CC && mode == M && resid == R) return launch(conv_fwd_s1_kernel<CC, M, R>, nblocks, lds, stream, *args);
  S1_CASE(16, 0, false)  // stem (input padded to 16 channels); v1 conv_a (identity input)
  S1_CASE(32, 0, false)
  S1_CASE(64, 0, false)
  S1_CASE(16, 1, false)
  S1_CASE(16, 1, true)
  S1_CASE(32, 1, false)
  S1_CASE(32, 1, true)
  S1_CASE(64, 1, false)
  S1_CASE(64, 1, true)
#undef S1_CASE
  return -1;
}

// Persistent forward segment (conv_fwd_s1_persist_kernel): layers = device ConvArgs table, kinds[l] as above.
// check_only: return 1 if nblocks workgroups of this instantiation are co-resident on the device (0 otherwise)
// without launching.  Returns -3 (no launch) when they are not: the caller must not rely on the barrier then.
DTF_API int dtf_conv_fwd_s1_persist(const ConvArgs* layers, const int* kinds, int nlayers, int c, int rows,
                                    int nblocks, int lds, unsigned* bar, unsigned* fail, int fence,
                                    int check_only, hipStream_t stream) {
  if (nblocks <= 0 || nlayers <= 0) return 0;
  DTF_HOST_CHECK(lds <= 160 * 1024);
  auto go = [&](auto kern) -> int {
    int per_cu = 0, dev = 0, ncu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, lds) != hipSuccess) return -3;
    if (hipGetDevice(&dev) != hipSuccess) return -3;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return -3;
    if ((long)per_cu * ncu < nblocks) return check_only ? 0 : -3;
    if (check_only) return 1;
    hipLaunchKernelGGL(kern, dim3(nblocks), dim3(256), lds, stream, layers, kinds, nlayers, bar, fail, fence);
    return DTF_CHECK_LAUNCH();
  };
  if (rows == 8 && c == 16) return go(conv_fwd_s1_persist_kernel<16, 8>);
  if (rows == 8 && c == 32) return go(conv_fwd_s1_persist_kernel<32, 8>);
  if (rows == 8 && c == 64) return go(conv_fwd_s1_persist_kernel<64, 8>);
  if (rows == 4 && c == 64) return go(conv_fwd_s1_persist_kernel<64, 4>);
  return -1;
}

DTF_API int dtf_dw_slab_reduce(const float* slab, const int4* red, int nmembers, float* grads, long g_mstride,
                               long g_off, int c, hipStream_t stream) {
  if (nmembers <= 0) return 0;
#define RED_CASE(CC)                                                                                        \
  if (c == CC) {                                                                                            \
    constexpr int E = ((9 * CC / 16 + 3) / 4) * (CC / 16) * 4 * 256;                                         \
    hipLaunchKernelGGL(dw_slab_reduce_kernel<CC>, dim3(E / 32, nmembers), dim3(256), 0, stream, slab, red, \
                       grads, g_mstride, g_off);                                                            \
    return DTF_CHECK_LAUNCH();                                                                              \
  }
  RED_CASE(16)
  RED_CASE(32)
  RED_CASE(64)
#undef RED_CASE
  return -1;
}

DTF_API int dtf_slab_job_size() { return (int)sizeof(SlabJob); }
DTF_API int dtf_dense_job_size() { return (int)sizeof(DenseJob); }

DTF_API int dtf_slab_reduce_all(const void* sjobs, int nsj, const void* djobs, int ndj, int max_members, int max_blocks,
                                float* grads, long g_mstride, hipStream_t stream) {
  if (nsj + ndj <= 0 || max_members <= 0 || max_blocks <= 0) return 0;
  DTF_HOST_CHECK((nsj == 0 || sjobs != nullptr) && (ndj == 0 || djobs != nullptr) && nsj + ndj <= 65535);
  hipLaunchKernelGGL(slab_reduce_all_kernel, dim3(max_blocks, max_members, nsj + ndj), dim3(256), 0, stream,
                     reinterpret_cast<const SlabJob*>(sjobs), nsj, reinterpret_cast<const DenseJob*>(djobs), grads,
                     g_mstride);
  return DTF_CHECK_LAUNCH();
}

DTF_DEBUG_EXPORT(conv)

// Diagnostic stamp buffer (DTF_STAMP builds): [launch row][workgroup][8] u64; returns -1 in normal builds.
DTF_API int dtf_stamp_read(void* dst, long bytes) {
#if DTF_STAMP
  if (bytes > (long)sizeof(dtf_stamps)) bytes = (long)sizeof(dtf_stamps);
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(dtf_stamps), bytes);
#else
  (void)dst;
  (void)bytes;
  return -1;
#endif
}

DTF_API int dtf_conv_args_size() { return (int)sizeof(ConvArgs); }

// conv_trans_multi_kernel: c = conv_a wgrad (3x3 s2), a = projection dgrad (1x1 s2), b = projection wgrad
DTF_API int dtf_conv_trans_multi(const ConvArgs* c, const ConvArgs* a, const ConvArgs* b, int ci, int co, int nblocks,
                                 int lds, hipStream_t stream) {
  DTF_HOST_CHECK(c->work != nullptr && a->work != nullptr && b->work != nullptr);
  DTF_HOST_CHECK(nblocks == c->n_main + a->n_main + b->n_main && lds <= 160 * 1024);
  if (nblocks <= 0) return 0;
#define TM_CASE(CI_, CO_)                                                                                   \
  if (ci == CI_ && co == CO_) {                                                                           \
    hipLaunchKernelGGL((conv_trans_multi_kernel<CI_, CO_>), dim3(nblocks), dim3(256), lds, stream, *c, *a, *b); \
    return DTF_CHECK_LAUNCH();                                                                            \
  }
  TM_CASE(16, 32)
  TM_CASE(32, 64)
#undef TM_CASE
  return -1;
}
// LDS row pitch of the stage kernels (the host sizes their dynamic LDS with it)
// compile-time knobs the host plan must agree with (engine/hip_resnet.py reads these, not its environment)
DTF_API int dtf_fused16_wlds() { return DTF_FUSED16_WLDS; }
DTF_API int dtf_fused16_m3_waves() { return DTF_FUSED16_M3_WAVES; }
DTF_API int dtf_fused16_m2_waves() { return DTF_FUSED16_M2_WAVES; }

DTF_API int dtf_cpad_fwd(int c) { return c == 16 ? cpad_fwd<16>() : c == 32 ? cpad_fwd<32>() : c == 64 ? cpad_fwd<64>() : -1; }
DTF_API int dtf_wpitch(int c) { return c == 16 ? wpitch<16>() : c == 32 ? wpitch<32>() : c == 64 ? wpitch<64>() : -1; }

DTF_API int dtf_conv_fwd(const ConvArgs* args, int cin, int cout, int s, int k, int mode, int resid, int stats,
                         int nblocks, int lds, hipStream_t stream) {
  // stem (input padded to 16 channels, no input BN)
  FWD_CASE(16, 16, 1, 3, 0, false, true)
  // stage convs: conv_a (BN1+ReLU on the block input), conv_b (BN2+ReLU, + residual)
  FWD_CASE(16, 16, 1, 3, 1, false, true)
  FWD_CASE(16, 16, 1, 3, 1, true, true)
  FWD_CASE(32, 32, 1, 3, 1, false, true)
  FWD_CASE(32, 32, 1, 3, 1, true, true)
  FWD_CASE(64, 64, 1, 3, 1, false, true)
  FWD_CASE(64, 64, 1, 3, 1, true, true)
  FWD_CASE(16, 32, 2, 3, 1, false, true)
  FWD_CASE(32, 64, 2, 3, 1, false, true)
  // projection shortcuts (1x1, on the pre-activated block input; no stats)
  FWD_CASE(16, 16, 1, 1, 1, false, false)
  FWD_CASE(16, 32, 2, 1, 1, false, false)
  FWD_CASE(32, 64, 2, 1, 1, false, false)
  // ResNet v1: convs read the (post-ReLU) block input directly and feed a BN (stats)
  FWD_CASE(16, 32, 2, 3, 0, false, true)
  FWD_CASE(32, 64, 2, 3, 0, false, true)
  FWD_CASE(16, 16, 1, 1, 0, false, true)
  FWD_CASE(16, 32, 2, 1, 0, false, true)
  FWD_CASE(32, 64, 2, 1, 0, false, true)
  FWD_CASE(32, 32, 1, 3, 0, false, true)
  FWD_CASE(64, 64, 1, 3, 0, false, true)
  return -1;
}

DTF_API int dtf_conv_dgrad(const ConvArgs* args, int cin, int cout, int s, int k, int mode, int epi, int nblocks,
                           int lds, hipStream_t stream) {
  // conv_b dgrad: dy = residual-stream grad (plain), epilogue: mask by BN2(h) + stats
  DGRAD_CASE(16, 16, 1, 3, 0, 2)
  DGRAD_CASE(32, 32, 1, 3, 0, 2)
  DGRAD_CASE(64, 64, 1, 3, 0, 2)
  // conv_a dgrad: dy = BN2-backward(dz2, h); epilogue: [+ proj dgrad] mask by BN1(x) + stats
  DGRAD_CASE(16, 16, 1, 3, 2, 2)
  DGRAD_CASE(32, 32, 1, 3, 2, 2)
  DGRAD_CASE(64, 64, 1, 3, 2, 2)
  DGRAD_CASE(16, 16, 1, 3, 2, 3)
  DGRAD_CASE(16, 32, 2, 3, 2, 3)
  DGRAD_CASE(32, 64, 2, 3, 2, 3)
  // projection dgrad (1x1): plain dy, plain output (added by the conv_a dgrad epilogue)
  DGRAD_CASE(16, 16, 1, 1, 0, 0)
  DGRAD_CASE(16, 32, 2, 1, 0, 0)
  DGRAD_CASE(32, 64, 2, 1, 0, 0)
  // ResNet v1: projection dgrad of BN_p-backward(dpre, hp); conv_a with identity mask (+ shortcut grad)
  DGRAD_CASE(16, 16, 1, 1, 2, 0)
  DGRAD_CASE(16, 32, 2, 1, 2, 0)
  DGRAD_CASE(32, 64, 2, 1, 2, 0)
  DGRAD_CASE(16, 32, 2, 3, 2, 5)
  DGRAD_CASE(32, 64, 2, 3, 2, 5)
  DGRAD_CASE(16, 16, 1, 3, 2, 5)
  DGRAD_CASE(16, 16, 1, 3, 2, 4)
  DGRAD_CASE(32, 32, 1, 3, 2, 4)
  DGRAD_CASE(64, 64, 1, 3, 2, 4)
  return -1;
}

#define FUSED_CASE(CC, M, E)                                                                          \
  if (c == CC && mode_dy == M && epi == E)                                                           \
    return launch(conv_bwd_fused_kernel<CC, M, E>, nblocks, lds, stream, *args);

DTF_API int dtf_conv_bwd_fused(const ConvArgs* args, int c, int mode_dy, int epi, int nblocks, int lds,
                               hipStream_t stream) {
  FUSED_CASE(16, 0, 0)  // conv_b: dy = residual grad, x = h (BN2)
  FUSED_CASE(32, 0, 0)
  FUSED_CASE(64, 0, 0)
  FUSED_CASE(16, 3, 0)  // conv_b with the previous block's BN1-backward + residual folded into the dY staging
  FUSED_CASE(32, 3, 0)
  FUSED_CASE(64, 3, 0)
  FUSED_CASE(16, 2, 0)  // conv_a: dy = BN2-backward(dz2, h), x = block input (BN1)
  FUSED_CASE(32, 2, 0)
  FUSED_CASE(64, 2, 0)
  FUSED_CASE(16, 2, 1)  // conv_a of the first block (+ stride-1 projection dgrad)
  FUSED_CASE(16, 2, 3)  // v1 conv_a: identity-BN block input (+ shortcut grad)
  FUSED_CASE(32, 2, 3)
  FUSED_CASE(64, 2, 3)
  FUSED_CASE(16, 2, 11)  // v1 conv_a + the previous block's BN_b backward sums (x-hat of x3) in the epilogue
  FUSED_CASE(32, 2, 11)
  FUSED_CASE(64, 2, 11)
  return -1;
}

DTF_API int dtf_conv_bwd_dual(const ConvArgs* a, const ConvArgs* b, int c, int mode_dy, int epi, int nblocks, int lds,
                              hipStream_t stream) {
  if (nblocks <= 0) return 0;
  DTF_HOST_CHECK(lds <= 160 * 1024);
  DTF_HOST_CHECK(a->work != nullptr && b->work != nullptr && a->n_main >= 0 && b->n_main >= 0);
  DTF_HOST_CHECK(nblocks >= a->n_main + b->n_main);
#define DUAL_CASE(CC, M, E)                                                                                  \
  if (c == CC && mode_dy == M && epi == E) {                                                                \
    hipLaunchKernelGGL((conv_bwd_dual_kernel<CC, M, E>), dim3(nblocks), dim3(256), lds, stream, *a, *b);    \
    return DTF_CHECK_LAUNCH();                                                                              \
  }
  DUAL_CASE(16, 0, 0) DUAL_CASE(32, 0, 0) DUAL_CASE(64, 0, 0)
  DUAL_CASE(16, 3, 0) DUAL_CASE(32, 3, 0) DUAL_CASE(64, 3, 0)
  DUAL_CASE(16, 2, 0) DUAL_CASE(32, 2, 0) DUAL_CASE(64, 2, 0)
  DUAL_CASE(16, 2, 1)
#undef DUAL_CASE
  return -1;
}

// rows: band height (8; 4: half-image bands for C = 64, twice the workgroups of one member; C = 32 measured slower)
DTF_API int dtf_conv_bwd_dg(const ConvArgs* a, int c, int mode_dy, int epi, int rows, int nblocks, int lds,
                            hipStream_t stream) {
  if (nblocks <= 0) return 0;
  DTF_HOST_CHECK(lds <= 160 * 1024);
  DTF_HOST_CHECK(a->work != nullptr && nblocks == a->n_main && a->rows == rows);
  if (rows == 4) {
#define DG4_CASE(CC, M)                                                                                      \
    if (c == CC && mode_dy == M && epi == 0) {                                                              \
      hipLaunchKernelGGL((conv_bwd_dg_kernel<CC, M, 0, 4>), dim3(nblocks), dim3(256), lds, stream, *a);     \
      return DTF_CHECK_LAUNCH();                                                                            \
    }
    DG4_CASE(64, 0) DG4_CASE(64, 2) DG4_CASE(64, 3)
#undef DG4_CASE
    return -1;
  }
#define DG_CASE(CC, M, E)                                                                                    \
  if (c == CC && mode_dy == M && epi == E) {                                                                \
    hipLaunchKernelGGL((conv_bwd_dg_kernel<CC, M, E>), dim3(nblocks), dim3(256), lds, stream, *a);          \
    return DTF_CHECK_LAUNCH();                                                                              \
  }
  DG_CASE(16, 0, 0) DG_CASE(32, 0, 0) DG_CASE(64, 0, 0)
  DG_CASE(16, 3, 0) DG_CASE(32, 3, 0) DG_CASE(64, 3, 0)
  DG_CASE(16, 2, 0) DG_CASE(32, 2, 0) DG_CASE(64, 2, 0)
  DG_CASE(16, 2, 1)
#undef DG_CASE
  return -1;
}

// cset 0: widths 64 and 32; 1: width 16
DTF_API int dtf_conv_wgrad_all(const void* jobs, const void* map, int nblocks, int cset, int lds, hipStream_t stream) {
  if (nblocks <= 0) return 0;
  DTF_HOST_CHECK(jobs != nullptr && map != nullptr && lds <= 160 * 1024 && (cset == 0 || cset == 1));
  if (cset == 0)
    hipLaunchKernelGGL((conv_wgrad_all_kernel<64, 32>), dim3(nblocks), dim3(256), lds, stream,
                       reinterpret_cast<const ConvArgs*>(jobs), reinterpret_cast<const int4*>(map));
  else
    hipLaunchKernelGGL((conv_wgrad_all_kernel<16, 16>), dim3(nblocks), dim3(256), lds, stream,
                       reinterpret_cast<const ConvArgs*>(jobs), reinterpret_cast<const int4*>(map));
  return DTF_CHECK_LAUNCH();
}

DTF_API int dtf_conv_wgrad(const ConvArgs* args, int cin, int cout, int s, int k, int mode_x, int mode_dy,
                           int nblocks, int lds, hipStream_t stream) {
  WGRAD_CASE(16, 16, 1, 3, 0, 0)  // stem (x = padded image)
  WGRAD_CASE(16, 16, 1, 3, 1, 0)  // conv_b: x = h (BN2+ReLU), dy = residual grad
  WGRAD_CASE(32, 32, 1, 3, 1, 0)
  WGRAD_CASE(64, 64, 1, 3, 1, 0)
  WGRAD_CASE(16, 16, 1, 3, 1, 2)  // conv_a: x = block input (BN1+ReLU), dy = BN2-backward(dz2, h)
  WGRAD_CASE(32, 32, 1, 3, 1, 2)
  WGRAD_CASE(64, 64, 1, 3, 1, 2)
  WGRAD_CASE(16, 32, 2, 3, 1, 2)
  WGRAD_CASE(32, 64, 2, 3, 1, 2)
  WGRAD_CASE(16, 16, 1, 1, 1, 0)  // projections: x = BN1+ReLU(block input), dy = residual grad
  WGRAD_CASE(16, 32, 2, 1, 1, 0)
  WGRAD_CASE(32, 64, 2, 1, 1, 0)
  // ResNet v1: x = block input (identity), dy = BN-backward(dpre, h) (stem, projections, conv_a)
  WGRAD_CASE(16, 16, 1, 3, 0, 2)
  WGRAD_CASE(16, 16, 1, 1, 0, 2)
  WGRAD_CASE(16, 32, 2, 1, 0, 2)
  WGRAD_CASE(32, 64, 2, 1, 0, 2)
  WGRAD_CASE(16, 32, 2, 3, 0, 2)
  WGRAD_CASE(32, 64, 2, 3, 0, 2)
  WGRAD_CASE(32, 32, 1, 3, 0, 2)
  WGRAD_CASE(64, 64, 1, 3, 0, 2)
  return -1;
}
