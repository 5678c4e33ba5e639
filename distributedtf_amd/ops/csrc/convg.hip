// Generic population-batched NHWC implicit-GEMM convolution for large-channel ResNets (gfx950).
//
// Used by the ImageNet-shape ResNet-50 path (stem 7x7/2, bottleneck 1x1 / 3x3 convs, C = 64..2048),
// where the CIFAR kernels' compile-time small-channel geometry does not apply.  All layouts are NHWC bf16
// with the images of every member packed along N; weights are per member bf16 rows.
//
//  convg_fwd  : out[p][o] = sum_{tap,i} W[o][tap][i] * T_in(src)[gather(p, tap)][i]
//               GEMM rows = output channels (A = weights, ds_read_b128 from LDS [rows][32+8]),
//               cols = output pixels (B = gathered activations), v_mfma_f32_16x16x32_bf16.
//               One kernel serves the forward conv (gather = p*S + tap - P) and the data gradient
//               (weights flipped/transposed; stride 1: same gather with P' = K-1-P; stride 2: "transposed"
//               gather q = p + tap - P', valid iff q % S == 0, then q / S).
//               T_in: identity | BN+ReLU (fwd prologue) | BN-backward apply A*dz + B*h + C (dgrad prologue).
//               Epilogue: [+ residual], [mask by BN(xm)+ReLU > 0], bf16 store, per-channel sum / second
//               moment (BN forward statistics, or sum(dz) / sum(dz*xhat) for the BN backward); the fp32 tile is
//               staged through LDS so residual / mask loads and stores are whole 16-byte row segments.
//               Tiles: TC (64 | 128) output channels x TP (128 | 256) pixels, k depth BK (32 | 64) per stage.
//  convg_wgrad: dW[o][tap][i] += sum_p T_dy(dy)[p][o] * T_x(x)[p*S + tap - P][i], split over pixel ranges,
//               both operands "k = pixel" fragments via ds_read_b64_tr_b16 from K-major LDS tiles, fp32
//               atomics into the member's gradient row (64- or 128-row tiles x 128 columns).
//  convg_wgrad_wide: the same for plain operands with wide column tiles (x 288 for 3x3, x 256 for 1x1,
//               one 64 x 416 tile for the 7x7 stem) -- more MFMA work per k-step and per staged dy tile.
// Every gather is branch-free (ld16: a masked-off lane reads a zero vector), so a thread's loads stay in flight
// together.  tools/imagenet_roofline.py prices each launch of the step against its HBM / MFMA floor.
// Per-member BN coefficients are precomputed by bn_finalize (convg_aux.hip) into [cap][4][CMAX] tables and
// staged into LDS per workgroup (a workgroup's pixels always belong to one member).
#include "common.h"

namespace {

typedef short s16x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4_t mfma16(const bf16x8_t& a, const bf16x8_t& b, const f32x4_t& c) {
  return dtf_mfma16(a, b, c);
}

__device__ __forceinline__ s16x4_t ds_read_tr(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(p));
}

// k-major operand tiles read with ds_read_b64_tr_b16 (weight gradients): lane (g = lane >> 4, q = (lane & 15) >> 2)
// reads k rows 8g + q and 8g + 4 + q.  With a row pitch of 4 (mod 64) dwords, rows r and r + 1 overlap in 4 of
// their 8 banks and rows 8 apart coincide: every read 2-way (4 cycles per instruction instead of 2; PMC: 5.8k bank
// conflict cycles per wave in convg_wgrad_wide_kernel).  The k order inside a 32-deep tile is free as long as both
// operands use the same one, so tile row kperm(k) holds k: the 8 rows a 32-lane half reads (k 8g + {0..3},
// 8g + 8 + {0..3}, or their +4 partners) land on 8 even (or odd) rows, whose segments tile the 64 banks for the
// pitches used here (4 or 20 mod 64 dwords; tools/lds_banks.py).  Reads: rows 8g + 2q (k 8g + q) and 8g + 2q + 1.
#ifndef CG_WG_KPERM
#define CG_WG_KPERM 1
#endif
__device__ __forceinline__ int kperm(int k) {
  return CG_WG_KPERM ? ((k & ~7) | ((k & 3) << 1) | ((k >> 2) & 1)) : k;
}
__device__ __forceinline__ int ktr_lo(int g, int q) { return CG_WG_KPERM ? 8 * g + 2 * q : 8 * g + q; }
__device__ __forceinline__ int ktr_hi(int g, int q) { return CG_WG_KPERM ? 8 * g + 2 * q + 1 : 8 * g + 4 + q; }

// Branch-free predicated 16-byte load: a masked-off lane reads a zero vector in global memory.  A conditional load
// makes hipcc branch around it and wait vmcnt(0) per element, which serialises a thread's gathers (PMC before
// the change: 5-12 VALU per MFMA in these kernels).
__device__ uint4 g_zero16 = {0u, 0u, 0u, 0u};  // what a masked-off lane loads (never written; not const: a const
// __device__ variable lives in the constant address space, and a select with it made every gather a flat_load)

typedef unsigned int u32x4v_t __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4v_t guint4_t;
__device__ __forceinline__ uint4 ld16(const bf16_t* base, long off, bool ok) {
  // a pointer select (2 VALU), not `ok ? load : 0` (hipcc turns that into a branch) nor a value mask (4 VALU).
  // Both arms are GLOBAL-address-space pointers: a select between a generic pointer and a __device__ variable is a
  // generic pointer, i.e. a flat_load -- which also counts in lgkmcnt, so every LDS-read wait of the k-loop
  // drained the whole global prefetch behind it
  guint4_t* p = ok ? (guint4_t*)(base + off) : (guint4_t*)&g_zero16;
  return __builtin_bit_cast(uint4, *p);
}

typedef unsigned int u32x2v_t __attribute__((ext_vector_type(2)));
typedef const __attribute__((address_space(1))) u32x2v_t guint2_t;
__device__ __forceinline__ uint2 ld8(const bf16_t* base, long off, bool ok) {  // 8-byte form of ld16
  guint2_t* p = ok ? (guint2_t*)(base + off) : (guint2_t*)&g_zero16;
  return __builtin_bit_cast(uint2, *p);
}

// relu(x * sc + sh) of 8 bf16 channels (BN + ReLU applied while an operand is staged: the folded forward)
__device__ __forceinline__ uint4 bnrelu8(uint4 v, const float (&sc)[8], const float (&sh)[8]) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t r[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float lo = fmaxf(lo2f(w[q]) * sc[2 * q] + sh[2 * q], 0.f);
    const float hi = fmaxf(hi2f(w[q]) * sc[2 * q + 1] + sh[2 * q + 1], 0.f);
    r[q] = pack2bf(lo, hi);
  }
  return make_uint4(r[0], r[1], r[2], r[3]);
}

struct CgArgs {
  const bf16_t* x;    // gathered operand (fwd: input activations; dgrad: output gradient; wgrad: input)
  const bf16_t* x2;   // second input of a BN-backward transform
  const bf16_t* dy;   // wgrad: output-side operand
  const bf16_t* dy2;  // wgrad: BN-backward second input of dy
  const bf16_t* w;    // bf16 weights [rows][K] per member
  long w_mstride, w_off;
  bf16_t* y;          // output NHWC
  const bf16_t* res;  // residual added in the epilogue
  const bf16_t* xm;   // epilogue mask source
  dtf_acc_t* grads;   // wgrad output rows (deterministic build: int64 fixed-point accumulators, common.h)
  long g_mstride, g_off;
  const float* c_in;  // transform coefficients of the gathered operand [cap][4][cmax]
  const float* c_dy;  // wgrad: transform coefficients of dy
  const float* c_ep;  // epilogue mask BN: scale, shift, mean, inv [cap][4][cmax]
  dtf_acc_t* st_out;  // per-channel sums [cap][2][cmax] (atomics)
  const int4* work;   // fwd: (slot, p0, p1, o0); wgrad: (slot, p0, p1, o0 | n0 << 16 (in 8-col units))
  int Hi, Wi, Ci;     // gathered tensor geometry
  int Ho, Wo, Co;     // output geometry (Co = GEMM rows)
  int kh, kw, stride, pad;
  int cmax;
  int log2ci;
  int cin_real;       // wgrad: real input channels of a channel-padded operand (stem: 3 of 8); 0 = Ci
  int flags;          // convg_t3 forward: bit 0 keeps the LDS-staged weights (A/B of the direct fragment loads)
  const bf16_t* x3;   // MODE 3: residual-stream gradient added by the gathered operand's BN-backward transform
  bf16_t* xout;       // MODE 3: the transformed gathered operand written out (1x1 stride-1 data gradient, co tile 0)
};


#ifndef CG_WIDE_P1
#define CG_WIDE_P1 1  // wide 1x1 weight gradients: stride-1 table-free addressing (convg_wgrad_wide_kernel P1)
#endif
#ifndef CG_EPI_AHEAD
#define CG_EPI_AHEAD 1  // generic epilogue: the next part's residual / mask loads issued while a part is processed
#endif
// Epilogue shared by the forward / data-gradient kernels: the fp32 accumulator tile (wave grid WRN x 4/WRN of
// (TC/WRN) x (TP/(4/WRN)) per wave) goes through LDS (cst, NHALF passes), then [+ residual], [mask by BN(xm)+ReLU],
// bf16 store and per-channel statistics.
// stage(h): writes staging part h (pixel rows [h * TP / NHALF, (h + 1) * TP / NHALF) of the tile) into cst as
// [pixel][channel] fp32 rows of pitch TC + 4 (the MFMA-shape-specific half; convg_epilogue below for 16x16 tiles,
// convg_epilogue32 for 32x32 ones)
template <int TC, int EPI, bool TRANS, int TP, int NHALF, bool AHEAD, class StageFn>
__device__ __forceinline__ void convg_epilogue_impl(const CgArgs& a, StageFn&& stage, float* cst,
                                                    dtf_acc_t (&acc_lds)[2][TC], int slot, int o0, int p0, int p1,
                                                    int HWo, int GW, int py, int px) {
  const int tid = threadIdx.x, lane = tid & 63;
  // ---- epilogue through LDS: the fp32 tile is staged as [pixel][channel] rows (the k loop ended with a barrier,
  // so the operand buffers are free), then every thread owns one 16-byte channel chunk of a pixel row: the
  // residual / mask loads and the bf16 store are whole contiguous row segments (TC * 2 bytes per pixel) instead
  // of 8-byte pieces of 16 pixel rows per wave instruction
  constexpr int CH = TC / 8;     // 16-byte channel chunks per pixel row
  constexpr int PPP = 256 / CH;  // pixel rows per pass of the workgroup
  const int ch = tid % CH, pr = tid / CH;
  const int oc = o0 + 8 * ch;
  const bool cok = oc < a.Co;  // Co % 8 == 0 (host check)
  float esc[8], esh[8], emu[8], eiv[8];
  if constexpr (EPI & 2) {
    const float* ep = a.c_ep + (long)slot * 4 * a.cmax + (cok ? oc : 0);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float4 u0 = *reinterpret_cast<const float4*>(ep + 4 * h);
      const float4 u1 = *reinterpret_cast<const float4*>(ep + a.cmax + 4 * h);
      const float4 u2 = *reinterpret_cast<const float4*>(ep + 2 * a.cmax + 4 * h);
      const float4 u3 = *reinterpret_cast<const float4*>(ep + 3 * a.cmax + 4 * h);
      esc[4 * h] = u0.x; esc[4 * h + 1] = u0.y; esc[4 * h + 2] = u0.z; esc[4 * h + 3] = u0.w;
      esh[4 * h] = u1.x; esh[4 * h + 1] = u1.y; esh[4 * h + 2] = u1.z; esh[4 * h + 3] = u1.w;
      emu[4 * h] = u2.x; emu[4 * h + 1] = u2.y; emu[4 * h + 2] = u2.z; emu[4 * h + 3] = u2.w;
      eiv[4 * h] = u3.x; eiv[4 * h + 1] = u3.y; eiv[4 * h + 2] = u3.z; eiv[4 * h + 3] = u3.w;
    }
  }
  float ss[8], sq[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) ss[i] = sq[i] = 0.f;
  constexpr int CPF = TC + 4;
  // all residual / mask rows of a part are loaded before the first store (the stores may alias them for the
  // compiler), so a thread keeps NPASS 16-byte loads in flight instead of one per pass; part 0's are issued before
  // the accumulator staging and its barrier (their latency overlaps that LDS traffic), and with CG_EPI_AHEAD part
  // h + 1's while part h is processed (two register sets)
  constexpr int NPASS = TP / NHALF / PPP;
  // (two sets only where they fit: one epilogue operand, and not in the register-bound t3 kernels -- AHEAD)
  constexpr int NB = (CG_EPI_AHEAD && AHEAD && NHALF > 1 && (EPI & 3) != 3) ? 2 : 1;
  long orow_[NB][NPASS];
  uint4 rrv_[NB][NPASS], xrv_[NB][NPASS];
  auto issue = [&](int h, long (&orow)[NPASS], uint4 (&rrv)[NPASS], uint4 (&xrv)[NPASS]) {
#pragma unroll
    for (int it = 0; it < NPASS; ++it) {
      const int p = p0 + h * (TP / NHALF) + pr + PPP * it;
      long pf = p;  // output pixel (full resolution)
      if constexpr (TRANS) {
        const int img = p / HWo, rem = p - img * HWo, qy = rem / GW, qx = rem - qy * GW;
        pf = ((long)img * a.Ho + 2 * qy + py) * a.Wo + 2 * qx + px;
      }
      orow[it] = (p < p1 && cok) ? pf * a.Co + oc : -1;
      rrv[it] = xrv[it] = make_uint4(0, 0, 0, 0);
      if constexpr ((EPI & 8) != 0) {
        // EPI bit 8: the residual is a stride-2 1x1 projection's data gradient stored compact, [N][Ho/2][Wo/2][Co]
        // (it is zero at every odd row / column of the full-resolution output): read it at even (y, x) only
        static_assert(!TRANS && (EPI & 1), "compact residual: full-grid output, residual add");
        const int img = p / HWo, rem = p - img * HWo, y = rem / GW, x = rem - y * GW;
        const bool ev = orow[it] >= 0 && ((y | x) & 1) == 0;
        const long ro = (((long)img * (a.Ho >> 1) + (y >> 1)) * (a.Wo >> 1) + (x >> 1)) * a.Co + oc;
        rrv[it] = ld16(a.res, ro, ev);
      } else if constexpr (EPI & 1) {
        rrv[it] = ld16(a.res, orow[it], orow[it] >= 0);
      }
      if constexpr (EPI & 2) xrv[it] = ld16(a.xm, orow[it], orow[it] >= 0);
    }
  };
#pragma unroll
  for (int h = 0; h < NHALF; ++h) {
    const int b = NB == 2 ? (h & 1) : 0;
    if (NB == 1 || h == 0) issue(h, orow_[b], rrv_[b], xrv_[b]);
    if (h > 0) __syncthreads();  // the previous part's rows have been read
    stage(h);
    __syncthreads();
    if (NB == 2 && h + 1 < NHALF) issue(h + 1, orow_[b ^ 1], rrv_[b ^ 1], xrv_[b ^ 1]);
    const long (&orow)[NPASS] = orow_[b];
    const uint4 (&rrv)[NPASS] = rrv_[b];
    const uint4 (&xrv)[NPASS] = xrv_[b];
#pragma unroll
  for (int it = 0; it < NPASS; ++it) {
    const int pl = pr + PPP * it;  // staged row
    if (orow[it] < 0) continue;
    const long o = orow[it];
    const float4 c0 = *reinterpret_cast<const float4*>(cst + pl * CPF + 8 * ch);
    const float4 c1 = *reinterpret_cast<const float4*>(cst + pl * CPF + 8 * ch + 4);
    float v[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
    const uint4 rr = rrv[it], xr = xrv[it];
    const uint32_t r32[4] = {rr.x, rr.y, rr.z, rr.w}, x32[4] = {xr.x, xr.y, xr.z, xr.w};
    float xv[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      xv[2 * q] = lo2f(x32[q]);
      xv[2 * q + 1] = hi2f(x32[q]);
      if constexpr (EPI & 1) {
        v[2 * q] += lo2f(r32[q]);
        v[2 * q + 1] += hi2f(r32[q]);
      }
    }
    if constexpr (EPI & 2) {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = (xv[i] * esc[i] + esh[i] > 0.f) ? v[i] : 0.f;
    }
    uint32_t pk[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) pk[q] = pack2bf(v[2 * q], v[2 * q + 1]);
    *reinterpret_cast<uint4*>(a.y + o) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
    if constexpr (EPI & 4) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float r0 = lo2f(pk[q]), r1 = hi2f(pk[q]);
        ss[2 * q] += r0;
        ss[2 * q + 1] += r1;
        if constexpr (EPI & 2) {
          sq[2 * q] += r0 * (xv[2 * q] - emu[2 * q]) * eiv[2 * q];
          sq[2 * q + 1] += r1 * (xv[2 * q + 1] - emu[2 * q + 1]) * eiv[2 * q + 1];
        } else {
          sq[2 * q] += r0 * r0;
          sq[2 * q + 1] += r1 * r1;
        }
      }
    }
  }
  }
  if constexpr (EPI & 4) {
    // lanes l, l + CH, l + 2 CH, .. of a wave hold the same channel chunk: butterfly over them, then one LDS
    // atomic per wave and channel, one global atomic per workgroup and channel
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float s_ = ss[i], q_ = sq[i];
#pragma unroll
      for (int o = CH; o < 64; o <<= 1) {
        s_ += __shfl_xor(s_, o, 64);
        q_ += __shfl_xor(q_, o, 64);
      }
      if (lane < CH && cok) {
        // forward statistics (y, y^2) or BN-backward sums (dz, dz*xhat): fixed-point scales of the deterministic build
        constexpr int FX = (EPI & 2) ? DTF_FX_GRAD : DTF_FX_STAT;
        dtf_acc_add(&acc_lds[0][8 * ch + i], s_, FX, slot);
        dtf_acc_add(&acc_lds[1][8 * ch + i], q_, FX, slot);
      }
    }
    __syncthreads();
    if (tid < TC && o0 + tid < a.Co) {
      dtf_acc_t* st = a.st_out + (long)slot * 2 * a.cmax;
      dtf_acc_addw(st + o0 + tid, acc_lds[0][tid]);
      dtf_acc_addw(st + a.cmax + o0 + tid, acc_lds[1][tid]);
    }
  }
}

template <int TC, int EPI, bool TRANS, int TP, int WRN, int NHALF, bool AHEAD = true>
__device__ __forceinline__ void convg_epilogue(const CgArgs& a, f32x4_t (&acc)[TC / WRN / 16][TP / (4 / WRN) / 16],
                                               float* cst, dtf_acc_t (&acc_lds)[2][TC], int slot, int o0, int p0, int p1,
                                               int HWo, int GW, int py, int px) {
  constexpr int PW = TP / (4 / WRN), NTP = PW / 16, MT = TC / WRN / 16;
  constexpr int CPF = TC + 4;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = wave % WRN, wc = wave / WRN;
  auto stage = [&](int h) {
#pragma unroll
    for (int n = 0; n < NTP; ++n) {
      const int pl = wc * PW + 16 * n - h * (TP / NHALF);  // staged row of this 16-pixel tile (wave-uniform)
      if (NHALF == 1 || (pl >= 0 && pl < TP / NHALF)) {
#pragma unroll
        for (int m = 0; m < MT; ++m)
          *reinterpret_cast<f32x4_t*>(cst + (pl + (lane & 15)) * CPF + wr * (TC / WRN) + 16 * m + 4 * (lane >> 4)) =
              acc[m][n];
      }
    }
  };
  convg_epilogue_impl<TC, EPI, TRANS, TP, NHALF, AHEAD>(a, stage, cst, acc_lds, slot, o0, p0, p1, HWo, GW, py, px);
}

// 32x32 accumulator tiles (v_mfma_f32_32x32x16_bf16): register r of lane l holds D[row 8 (r >> 2) + 4 (l >> 5) +
// (r & 3)][col l & 31] -- each group of 4 registers is 4 consecutive output channels of one pixel (one float4)
template <int TC, int EPI, bool TRANS, int TP, int WRN, int NHALF>
__device__ __forceinline__ void convg_epilogue32(const CgArgs& a, f32x16_t (&acc)[TC / WRN / 32][TP / (4 / WRN) / 32],
                                                 float* cst, dtf_acc_t (&acc_lds)[2][TC], int slot, int o0, int p0,
                                                 int p1, int HWo, int GW, int py, int px) {
  constexpr int PW = TP / (4 / WRN), NT2 = PW / 32, MT2 = TC / WRN / 32;
  constexpr int CPF = TC + 4;
  static_assert((TP / NHALF) % 32 == 0, "32-pixel tiles must not straddle staging parts");
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = wave % WRN, wc = wave / WRN;
  auto stage = [&](int h) {
#pragma unroll
    for (int n = 0; n < NT2; ++n) {
      const int pl = wc * PW + 32 * n - h * (TP / NHALF);
      if (NHALF == 1 || (pl >= 0 && pl < TP / NHALF)) {
#pragma unroll
        for (int m = 0; m < MT2; ++m)
#pragma unroll
          for (int g = 0; g < 4; ++g)
            *reinterpret_cast<f32x4_t*>(cst + (pl + (lane & 31)) * CPF + wr * (TC / WRN) + 32 * m + 8 * g +
                                        4 * (lane >> 5)) =
                (f32x4_t){acc[m][n][4 * g], acc[m][n][4 * g + 1], acc[m][n][4 * g + 2], acc[m][n][4 * g + 3]};
      }
    }
  };
  convg_epilogue_impl<TC, EPI, TRANS, TP, NHALF, true>(a, stage, cst, acc_lds, slot, o0, p0, p1, HWo, GW, py, px);
}

// Register-direct epilogue of the 16x16 accumulator tiles (no residual, TRANS = false): lane l of a wave holds, per
// (m, n) tile, 4 consecutive output channels (rows 4 (l >> 4) .. + 3) of pixel l & 15 -- packed to 4 bf16 and stored
// as one 8-byte piece (the 4 lanes of a pixel write 32 contiguous bytes; the wave's MT m-tiles complete 128-byte
// lines back to back).  No LDS staging, hence none of the staged epilogue's 2 barriers per part (NHALF parts): the
// convg_t3 stamps (tools/t3_bench.py --stamps) put that epilogue at 7 us of a 33 us k loop (forward, 28 x 28) and
// 14 us (data gradient with the ReLU mask).  EPI bit 1: mask by BN(xm) + ReLU > 0 (xm loads issued together up
// front); bit 2: per-channel statistics of the stored bf16 values, summed over the lane's pixels in registers, then
// over the 16 pixel lanes by xor shuffles, one LDS add per wave and channel, one global add per workgroup and channel.
// EPI bit 0: + residual (loaded like xm).  TRANS: the pixel index is on the parity-class grid (GW wide, HWo per
// image) of output parity (py, px), as in convg_epilogue_impl.
template <int TC, int EPI, int TP, int WRN, bool TRANS = false>
__device__ __forceinline__ void convg_epilogue_regs(const CgArgs& a, f32x4_t (&acc)[TC / WRN / 16][TP / (4 / WRN) / 16],
                                                    dtf_acc_t (&acc_lds)[2][TC], int slot, int o0, int p0, int p1,
                                                    int HWo = 0, int GW = 0, int py = 0, int px = 0) {
  static_assert(!(EPI & 8), "the compact projection residual is read by the LDS-staged epilogue only");
  constexpr int PW = TP / (4 / WRN), NTP = PW / 16, MT = TC / WRN / 16;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wr = wave % WRN, wc = wave / WRN;
  const int cb = wr * (TC / WRN) + 4 * (lane >> 4);  // tile channel of register 0, m-tile 0
  long prow[NTP];
#pragma unroll
  for (int n = 0; n < NTP; ++n) {
    const int p = p0 + wc * PW + 16 * n + (lane & 15);
    long pf = p;
    if constexpr (TRANS) {
      const int img = p / HWo, rem = p - img * HWo, qy = rem / GW, qx = rem - qy * GW;
      pf = ((long)img * a.Ho + 2 * qy + py) * a.Wo + 2 * qx + px;
    }
    prow[n] = p < p1 ? pf * a.Co : -1;
  }
  uint2 xr[(EPI & 2) ? MT : 1][(EPI & 2) ? NTP : 1];
  uint2 rr[(EPI & 1) ? MT : 1][(EPI & 1) ? NTP : 1];
  if constexpr ((EPI & 3) != 0) {
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int n = 0; n < NTP; ++n) {
        const int oc = o0 + cb + 16 * m;
        const bool ok = prow[n] >= 0 && oc < a.Co;
        if constexpr (EPI & 2) xr[m][n] = ld8(a.xm, prow[n] + oc, ok);
        if constexpr (EPI & 1) rr[m][n] = ld8(a.res, prow[n] + oc, ok);
      }
  }
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int oc = o0 + cb + 16 * m;
    const bool cok = oc < a.Co;
    float esc[4], esh[4], emu[4], eiv[4];
    if constexpr (EPI & 2) {
      const float* ep = a.c_ep + (long)slot * 4 * a.cmax + (cok ? oc : 0);
      const float4 u0 = *reinterpret_cast<const float4*>(ep);
      const float4 u1 = *reinterpret_cast<const float4*>(ep + a.cmax);
      const float4 u2 = *reinterpret_cast<const float4*>(ep + 2 * a.cmax);
      const float4 u3 = *reinterpret_cast<const float4*>(ep + 3 * a.cmax);
      esc[0] = u0.x; esc[1] = u0.y; esc[2] = u0.z; esc[3] = u0.w;
      esh[0] = u1.x; esh[1] = u1.y; esh[2] = u1.z; esh[3] = u1.w;
      emu[0] = u2.x; emu[1] = u2.y; emu[2] = u2.z; emu[3] = u2.w;
      eiv[0] = u3.x; eiv[1] = u3.y; eiv[2] = u3.z; eiv[3] = u3.w;
    }
    float ss[4] = {0.f, 0.f, 0.f, 0.f}, sq[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int n = 0; n < NTP; ++n) {
      const bool ok = prow[n] >= 0 && cok;
      float v[4] = {acc[m][n][0], acc[m][n][1], acc[m][n][2], acc[m][n][3]};
      float xv[4] = {0.f, 0.f, 0.f, 0.f};
      if constexpr (EPI & 1) {
        const uint2 r2 = rr[m][n];
        v[0] += lo2f(r2.x); v[1] += hi2f(r2.x); v[2] += lo2f(r2.y); v[3] += hi2f(r2.y);
      }
      if constexpr (EPI & 2) {
        const uint2 x2 = xr[m][n];
        xv[0] = lo2f(x2.x); xv[1] = hi2f(x2.x); xv[2] = lo2f(x2.y); xv[3] = hi2f(x2.y);
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = (xv[i] * esc[i] + esh[i] > 0.f) ? v[i] : 0.f;
      }
      const uint32_t k0 = pack2bf(v[0], v[1]), k1 = pack2bf(v[2], v[3]);
      if (ok) *reinterpret_cast<uint2*>(a.y + prow[n] + oc) = make_uint2(k0, k1);
      if constexpr (EPI & 4) {
        const float r[4] = {lo2f(k0), hi2f(k0), lo2f(k1), hi2f(k1)};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float ri = ok ? r[i] : 0.f;
          ss[i] += ri;
          if constexpr (EPI & 2)
            sq[i] += ri * (xv[i] - emu[i]) * eiv[i];
          else
            sq[i] += ri * ri;
        }
      }
    }
    if constexpr (EPI & 4) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float s_ = ss[i], q_ = sq[i];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          s_ += __shfl_xor(s_, o, 64);
          q_ += __shfl_xor(q_, o, 64);
        }
        if ((lane & 15) == 0 && cok) {
          constexpr int FX = (EPI & 2) ? DTF_FX_GRAD : DTF_FX_STAT;
          dtf_acc_add(&acc_lds[0][cb + 16 * m + i], s_, FX, slot);
          dtf_acc_add(&acc_lds[1][cb + 16 * m + i], q_, FX, slot);
        }
      }
    }
  }
  if constexpr (EPI & 4) {
    __syncthreads();
    if (tid < TC && o0 + tid < a.Co) {
      dtf_acc_t* st = a.st_out + (long)slot * 2 * a.cmax;
      dtf_acc_addw(st + o0 + tid, acc_lds[0][tid]);
      dtf_acc_addw(st + a.cmax + o0 + tid, acc_lds[1][tid]);
    }
  }
}

// ---------------------------------------------------------------------------------------------- fwd / dgrad
// MODE: 0 identity, 1 relu(x*s + t), 2 A*x + B*x2 + C, 3 A*x + B*x2 + C + x3 also stored to xout (the BN-backward
// apply of the next block's input gradient done by its consumer: a stride-1 1x1 data gradient whose single co tile
// gathers each element once).   EPI: bit0 residual, bit1 mask, bit2 stats (fwd: y, y^2;
// with bit1: dz, dz*xhat).  TRANS: transposed (dgrad, stride > 1) gather.
// AKM (data gradient): the A operand (rows = dx channels i, k = (tap', dy channel o)) is read straight from the
// FORWARD weight layout W[o][tap][i] (k-major: 8 consecutive i per 16-byte load, fragments via
// ds_read_b64_tr_b16), so no transposed weight copy exists.
// BK: k depth per LDS stage (32 or 64).  BK = 64 halves the barriers and fragment-read restarts per MFMA and doubles
// the bytes in flight per load batch; it needs Ci >= 64 on the incremental (one tap per k-step) gather path.
// TP: pixels per workgroup tile.  128: 2 x 2 waves of (TC/2 rows x 64 pixels); 256: with TC = 64 1 x 4 waves of
// 64 x 64 (twice the MFMA work per k-step and wave of the 32 x 64 wave tile a 64-row conv gets otherwise), with
// TC = 128 2 x 2 waves of 64 x 128 (32 MFMAs per wave and k-step; the epilogue is staged in 64-pixel quarters).
// M32: v_mfma_f32_32x32x16_bf16 tiles (a wave's TC/WRN x PW block as 32 x 32 MFMA tiles: half the MFMA
// instructions of the 16x16x32 form for the same fragment reads; plain-A (non-AKM) forward only)
#ifndef CG_XF_VEC
#define CG_XF_VEC 1  // generic kernel: BN transform coefficients of a k-step read as 16-byte LDS rows (else per element)
#endif
#ifndef CG_EPI_REGS
#define CG_EPI_REGS 0  // generic kernel: register-direct epilogue (convg_epilogue_regs) for the 16x16 tiles
#endif
template <int TC, int MODE, int EPI, bool TRANS, bool AKM = false, int BK = 32, int TP = 128, bool M32 = false>
__global__ __launch_bounds__(256) void convg_fwd_kernel(CgArgs a) {
  static_assert(TP == 128 || TP == 256, "pixel tile");
  static_assert(!M32 || (!AKM && (TC / ((TP == 256 && TC == 64) ? 1 : 2)) % 32 == 0), "32x32 tiles: plain A");
  // wave grid: TC = 64 x TP = 256 -> 1 x 4 waves of 64 x 64; else 2 x 2 waves of (TC/2) x (TP/2)
  constexpr int WRN = (TP == 256 && TC == 64) ? 1 : 2;
  constexpr int PW = TP / (4 / WRN), NTP = PW / 16;  // pixels per wave, MFMA pixel tiles per wave
  constexpr int RP = BK + 8;        // [rows][BK] tile pitch (+16 B)
  constexpr int CPR = BK / 8;       // 16-byte chunks per tile row
  constexpr int RPT = 256 / CPR;    // tile rows covered per pass of the workgroup
  constexpr int NJ = TP / RPT;      // B (pixel) rows per thread
  constexpr int KPA = TC + 8;       // [BK][TC] k-major A tile pitch
  constexpr int MT = TC / WRN / 16;  // MFMA row tiles per wave (wave covers TC/WRN rows)
  constexpr int SA = (TC * RP > BK * KPA) ? TC * RP : BK * KPA;
  constexpr int CPF = TC + 4;  // epilogue staging row pitch (floats; 16-byte rows, conflict-free float4 stores)
  // bf16 elements: operand buffers | fp32 epilogue staging of the whole tile; when the staging would exceed the
  // operand buffers (BK = 32) the tile is staged in two 64-pixel halves so LDS (and occupancy) stays the same
  constexpr int SOPS = 2 * SA + 2 * TP * RP, SEPI_FULL = 2 * TP * CPF;
  constexpr int NHALF = SOPS >= SEPI_FULL ? 1 : (2 * SOPS >= SEPI_FULL ? 2 : 4), SEPI = SEPI_FULL / NHALF;
  __shared__ __attribute__((aligned(16))) bf16_t smem_[SOPS > SEPI ? SOPS : SEPI];
  bf16_t (*sa)[SA] = reinterpret_cast<bf16_t (*)[SA]>(smem_);
  bf16_t (*sb)[TP * RP] = reinterpret_cast<bf16_t (*)[TP * RP]>(smem_ + 2 * SA);
  extern __shared__ __attribute__((aligned(16))) float dyn[];  // transform coefficients: MODE 1: 2*Ci, MODE 2/3: 3*Ci
  __shared__ dtf_acc_t acc_lds[2][TC];
  const int4 wk = a.work[blockIdx.x];
  DTF_WG_CHECK(wk.x >= 0 && wk.y >= 0 && wk.z >= wk.y);
  const int slot = wk.x, p0 = wk.y, p1 = wk.z;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wr = wave % WRN, wc = wave / WRN;
  const int Ci = a.Ci, Kfull = a.kh * a.kw * Ci;
  // TRANS (stride-2 data gradient): the workgroup covers one output parity class (py, px); pixels are indexed on
  // the class grid (= the gathered dy grid) and only the taps with (parity + tap - pad) even contribute:
  // ky = ky0, ky0 + 2, ..  -> K = nky * nkx * Ci instead of kh * kw * Ci with 3/4 of the products zero.
  int o0 = wk.w, py = 0, px = 0, ky0 = 0, kx0 = 0, nky = a.kh, nkx = a.kw;
  if constexpr (TRANS) {
    o0 = wk.w & 0xffff;
    py = (wk.w >> 17) & 1;
    px = (wk.w >> 16) & 1;
    ky0 = (a.pad - py) & 1;
    kx0 = (a.pad - px) & 1;
    nky = (a.kh - ky0 + 1) >> 1;
    nkx = (a.kw - kx0 + 1) >> 1;
  }
  const int K = nky * nkx * Ci;
  if constexpr (MODE != 0) {
    const float* cb = a.c_in + (long)slot * 4 * a.cmax;
    for (int i = tid; i < Ci; i += 256) {
      dyn[i] = cb[i];
      dyn[Ci + i] = cb[a.cmax + i];
      if constexpr (MODE >= 2) dyn[2 * Ci + i] = cb[2 * a.cmax + i];
    }
  }
  for (int i = tid; i < 2 * TC; i += 256) (&acc_lds[0][0])[i] = 0;
  // per-thread B rows (pixels): r = tid / CPR + RPT j, chunk c = tid % CPR
  const int cB = tid % CPR, rB = tid / CPR;
  int pix_img[NJ], pix_y[NJ], pix_x[NJ];
  bool pix_ok[NJ];
  const int GH = TRANS ? a.Hi : a.Ho, GW = TRANS ? a.Wi : a.Wo;  // pixel grid of the work items
  const int HWo = GH * GW;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int p = p0 + rB + RPT * j;
    pix_ok[j] = p < p1;
    const int pp = pix_ok[j] ? p : p0;
    pix_img[j] = pp / HWo;
    const int rem = pp - pix_img[j] * HWo;
    pix_y[j] = rem / GW;
    pix_x[j] = rem - pix_y[j] * GW;
  }
  const bf16_t* wbase = a.w + (long)slot * a.w_mstride + a.w_off;
  const long img_elems = (long)a.Hi * a.Wi * Ci;
  // gather position of this thread's chunk: for Ci >= BK a BK-wide k-step lies inside one tap, so the tap
  // indices (ty, tx) along the (possibly parity-strided) tap grid and ci advance incrementally (no division in the
  // loop); Ci < BK (the channel-padded stem) decomposes k per step
  const bool inc = Ci >= BK;
  const int kstep = TRANS ? 2 : 1;
  int g_ty = 0, g_tx = 0, g_ci = 8 * cB;
  if (!inc) {  // stem: first tap of this thread's chunk
    const int tap = (8 * cB) >> a.log2ci;
    g_ty = tap / a.kw;
    g_tx = tap - g_ty * a.kw;
  }
  int cur_ky = 0, cur_kx = 0, cur_ci = 0;  // position of this thread's chunk in the current k-step
  int cur_ty = 0, cur_tx = 0;              // the same as indices into the tap grid (ky = ky0 + kstep * ty)
  // Per-pixel gather origin, hoisted out of the k loop: tap (ty, tx) of pixel j reads row y0 + ty, column x0 + tx
  // of the gathered image (forward: y0 = y*S - P; stride-2 data gradient: the class-grid origin), valid iff bit
  // ty of rmask and bit tx of cmask are set; pbase = element offset of (img, y0, x0) (may be negative: only used
  // when valid).  A k-step then costs one mask test and one add per pixel.
  long pbase[NJ];
  unsigned rmask[NJ], cmask[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    int y0, x0;
    if constexpr (TRANS) {  // class pixel (2*qy + py): dy row (py + ky - pad) / 2 + qy (even numerator)
      y0 = pix_y[j] + ((py + ky0 - a.pad) >> 1);
      x0 = pix_x[j] + ((px + kx0 - a.pad) >> 1);
    } else {
      y0 = pix_y[j] * a.stride - a.pad;
      x0 = pix_x[j] * a.stride - a.pad;
    }
    unsigned rm = 0, cm = 0;
    for (int t = 0; t < nky; ++t) rm |= (unsigned)(y0 + t >= 0 && y0 + t < a.Hi) << t;
    for (int t = 0; t < nkx; ++t) cm |= (unsigned)(x0 + t >= 0 && x0 + t < a.Wi) << t;
    rmask[j] = pix_ok[j] ? rm : 0u;
    cmask[j] = cm;
    pbase[j] = (long)pix_img[j] * img_elems + ((long)y0 * a.Wi + x0) * Ci;
  }
  auto next_pos = [&](int k0) {
    if (inc) {
      cur_ty = g_ty;
      cur_tx = g_tx;
      cur_ky = ky0 + kstep * g_ty;
      cur_kx = kx0 + kstep * g_tx;
      cur_ci = g_ci;
      g_ci += BK;
      if (g_ci >= Ci) {
        g_ci -= Ci;
        if (++g_tx >= nkx) {
          g_tx = 0;
          ++g_ty;
        }
      }
    } else {  // Ci < BK only occurs for the (non-transposed) channel-padded stem
      // this thread's chunk keeps its channel offset; its tap advances by BK / Ci per k-step (kept as (ky, kx)
      // incrementally: no integer division by kw in the loop)
      cur_ci = g_ci & (Ci - 1);
      cur_ky = g_ty;
      cur_kx = g_tx;
      cur_ty = cur_ky;
      cur_tx = cur_kx;
      g_tx += BK >> a.log2ci;
      while (g_tx >= a.kw) {
        g_tx -= a.kw;
        ++g_ty;
      }
    }
  };
  static_assert(MODE != 3 || (AKM && !TRANS), "MODE 3: stride-1 data gradient");
  constexpr int NJ3 = MODE == 3 ? NJ : 1;
  // MODE 3: xout is written by the co-tile-0 workgroups only (with one tile, every element exactly once)
  bf16_t* const xo = (MODE == 3 && wk.w == 0) ? a.xout : nullptr;
  const bool has3 = MODE == 3 && a.x3 != nullptr;
  auto load_b = [&](int k0, uint4 (&v)[NJ], uint4 (&v2)[NJ], uint4 (&v3)[NJ3], int& cch, int& tof, unsigned& okb) {
    const int k = k0 + 8 * cB;
    const int ty = cur_ty, tx = cur_tx, ci0 = cur_ci;
    const int toff = (ty * a.Wi + tx) * Ci + ci0;
    cch = ci0;
    tof = toff;
    okb = 0;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const bool ok = ((rmask[j] >> ty) & (cmask[j] >> tx) & 1u) && k < K;
      const long off = pbase[j] + toff;
      v[j] = ld16(a.x, off, ok);
      v2[j] = make_uint4(0, 0, 0, 0);
      if constexpr (MODE >= 2) v2[j] = ld16(a.x2, off, ok);
      if constexpr (MODE == 3) v3[j] = ld16(a.x3, off, ok && has3);  // (no x3: a projection block's g)
      okb |= (unsigned)ok << j;  // unset: zero padding (stays zero after the transform)
    }
  };
  auto xform_store = [&](bf16_t* dst, const uint4 (&v)[NJ], const uint4 (&v2)[NJ], const uint4 (&v3)[NJ3], int cch,
                         int tof, unsigned okb) {
    // this thread's 8 channels cch..cch+7 are the same for all NJ chunks of the k-step: their coefficients are read
    // once per k-step as 16-byte LDS rows (CG_XF_VEC; the element-wise form issued 2-3 scalar LDS reads per element)
    float ca[8], cb[8], cc[8];
    if constexpr (MODE != 0) {
#if CG_XF_VEC
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float4 a4 = *reinterpret_cast<const float4*>(dyn + cch + 4 * h);
        const float4 b4 = *reinterpret_cast<const float4*>(dyn + Ci + cch + 4 * h);
        ca[4 * h] = a4.x, ca[4 * h + 1] = a4.y, ca[4 * h + 2] = a4.z, ca[4 * h + 3] = a4.w;
        cb[4 * h] = b4.x, cb[4 * h + 1] = b4.y, cb[4 * h + 2] = b4.z, cb[4 * h + 3] = b4.w;
        if constexpr (MODE >= 2) {
          const float4 c4 = *reinterpret_cast<const float4*>(dyn + 2 * Ci + cch + 4 * h);
          cc[4 * h] = c4.x, cc[4 * h + 1] = c4.y, cc[4 * h + 2] = c4.z, cc[4 * h + 3] = c4.w;
        }
      }
#else
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        ca[e] = dyn[cch + e];
        cb[e] = dyn[Ci + cch + e];
        if constexpr (MODE >= 2) cc[e] = dyn[2 * Ci + cch + e];
      }
#endif
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      uint4 t = v[j];
      if (!((okb >> j) & 1u)) {
        t = make_uint4(0, 0, 0, 0);
      } else if constexpr (MODE != 0) {
        uint32_t w32[4] = {t.x, t.y, t.z, t.w};
        const uint32_t h32[4] = {v2[j].x, v2[j].y, v2[j].z, v2[j].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float x0 = lo2f(w32[q]), x1 = hi2f(w32[q]);
          if constexpr (MODE == 1) {
            x0 = fmaxf(x0 * ca[2 * q] + cb[2 * q], 0.f);
            x1 = fmaxf(x1 * ca[2 * q + 1] + cb[2 * q + 1], 0.f);
          } else {
            const float h0 = lo2f(h32[q]), h1 = hi2f(h32[q]);
            x0 = ca[2 * q] * x0 + cb[2 * q] * h0 + cc[2 * q];
            x1 = ca[2 * q + 1] * x1 + cb[2 * q + 1] * h1 + cc[2 * q + 1];
            if constexpr (MODE == 3) {  // (the order of cg_ew_apply_cf_kernel: A dz + B h + C + add)
              const uint32_t r32 = q == 0 ? v3[j].x : q == 1 ? v3[j].y : q == 2 ? v3[j].z : v3[j].w;
              x0 += lo2f(r32);
              x1 += hi2f(r32);
            }
          }
          w32[q] = pack2bf(x0, x1);
        }
        t = make_uint4(w32[0], w32[1], w32[2], w32[3]);
        if constexpr (MODE == 3)
          if (xo != nullptr) *reinterpret_cast<uint4*>(xo + pbase[j] + tof) = t;
      }
      *reinterpret_cast<uint4*>(dst + (rB + RPT * j) * RP + 8 * cB) = t;
    }
  };
  // A (weights): rows o0 + r, r = tid / CPR + RPT j (j < TC / RPT); AKM: k rows kr = tid / ACH + (256 / ACH) j
  constexpr int AJ = TC * BK / 2048;
  constexpr int ACH = TC / 8;  // AKM: 8-row chunks per k row
  auto load_a = [&](int k0, uint4 (&v)[AJ]) {
    const int k = k0 + 8 * cB;
    if constexpr (AKM) {
      // all BK k of a step share one tap (Ci >= BK)
      const int kk = a.kh * a.kw;
      const int tapf = kk - 1 - (cur_ky * a.kw + cur_kx);  // forward tap of the flipped tap'
      const int obase = cur_ci - 8 * cB;                     // first dy channel of this k step
#pragma unroll
      for (int j = 0; j < AJ; ++j) {
        const int kr = tid / ACH + (256 / ACH) * j, ch = tid % ACH;
        const int oc = obase + kr;
        v[j] = ld16(wbase, ((long)oc * kk + tapf) * a.Co + o0 + 8 * ch, k0 + kr < K && o0 + 8 * ch < a.Co);
      }
    } else {
      const int kcol = TRANS ? (cur_ky * a.kw + cur_kx) * Ci + cur_ci : k;  // column in the full [o][K] row
#pragma unroll
      for (int j = 0; j < AJ; ++j) {
        const int r = rB + RPT * j;
        v[j] = ld16(wbase, (long)(o0 + r) * Kfull + kcol, o0 + r < a.Co && k < K);
      }
    }
  };
  auto store_a = [&](bf16_t* dst, const uint4 (&v)[AJ]) {
#pragma unroll
    for (int j = 0; j < AJ; ++j) {
      if constexpr (AKM)
        *reinterpret_cast<uint4*>(dst + kperm(tid / ACH + (256 / ACH) * j) * KPA + 8 * (tid % ACH)) = v[j];
      else
        *reinterpret_cast<uint4*>(dst + (rB + RPT * j) * RP + 8 * cB) = v[j];
    }
  };
  constexpr int MT2 = M32 ? MT / 2 : 1, NT2 = M32 ? NTP / 2 : 1;
  f32x4_t acc[M32 ? 1 : MT][M32 ? 1 : NTP];
  f32x16_t acc32[MT2][NT2];
  if constexpr (M32) {
#pragma unroll
    for (int m = 0; m < MT2; ++m)
#pragma unroll
      for (int n = 0; n < NT2; ++n)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc32[m][n][r] = 0.f;
  } else {
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int n = 0; n < NTP; ++n) acc[m][n] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  }
  __syncthreads();  // coefficients in LDS
  const int nk = (K + BK - 1) / BK;
  uint4 ra[AJ], rb[NJ], rb2[NJ], rb3[NJ3];
  int cch, tof;
  unsigned okb;
  next_pos(0);
  load_a(0, ra);
  load_b(0, rb, rb2, rb3, cch, tof, okb);
  store_a(sa[0], ra);
  xform_store(sb[0], rb, rb2, rb3, cch, tof, okb);
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    const int cur = ks & 1;
    const bool more = ks + 1 < nk;
    int ncch = 0, ntof = 0;
    if (more) {
      next_pos(BK * (ks + 1));
      load_a(BK * (ks + 1), ra);
      load_b(BK * (ks + 1), rb, rb2, rb3, ncch, ntof, okb);
    }
    if constexpr (M32) {
      // lane l: A row (l & 31), B pixel (l & 31), k = 16 s + 8 (l >> 5) .. + 7 of each 16-deep half step s
#pragma unroll
      for (int s2 = 0; s2 < BK / 16; ++s2) {
        bf16x8_t fa[MT2], fb[NT2];
#pragma unroll
        for (int m = 0; m < MT2; ++m)
          fa[m] = *reinterpret_cast<const bf16x8_t*>(sa[cur] + (wr * (TC / WRN) + 32 * m + (lane & 31)) * RP +
                                                     16 * s2 + 8 * (lane >> 5));
#pragma unroll
        for (int n = 0; n < NT2; ++n)
          fb[n] = *reinterpret_cast<const bf16x8_t*>(sb[cur] + (wc * PW + 32 * n + (lane & 31)) * RP + 16 * s2 +
                                                     8 * (lane >> 5));
#pragma unroll
        for (int m = 0; m < MT2; ++m)
#pragma unroll
          for (int n = 0; n < NT2; ++n) acc32[m][n] = dtf_mfma32(fa[m], fb[n], acc32[m][n]);
      }
    } else
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8_t fa[MT], fb[NTP];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        if constexpr (AKM) {
          const int g = lane >> 4, q = (lane & 15) >> 2, p4 = lane & 3;
          const int rb_ = wr * (TC / WRN) + 16 * m + 4 * p4;
          const s16x4_t lo = ds_read_tr(sa[cur] + (32 * kk + ktr_lo(g, q)) * KPA + rb_);
          const s16x4_t hi = ds_read_tr(sa[cur] + (32 * kk + ktr_hi(g, q)) * KPA + rb_);
          fa[m] = (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        } else {
          fa[m] = *reinterpret_cast<const bf16x8_t*>(sa[cur] + (wr * (TC / WRN) + 16 * m + (lane & 15)) * RP +
                                                     32 * kk + 8 * (lane >> 4));
        }
      }
#pragma unroll
      for (int n = 0; n < NTP; ++n)
        fb[n] = *reinterpret_cast<const bf16x8_t*>(sb[cur] + (wc * PW + 16 * n + (lane & 15)) * RP + 32 * kk +
                                                   8 * (lane >> 4));
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NTP; ++n) acc[m][n] = mfma16(fa[m], fb[n], acc[m][n]);
    }
    if (more) {
      store_a(sa[cur ^ 1], ra);
      xform_store(sb[cur ^ 1], rb, rb2, rb3, ncch, ntof, okb);
    }
    __syncthreads();
  }
  if constexpr (M32)
    convg_epilogue32<TC, EPI, TRANS, TP, WRN, NHALF>(a, acc32, reinterpret_cast<float*>(smem_), acc_lds, slot, o0, p0,
                                                      p1, HWo, GW, py, px);
  else if constexpr (CG_EPI_REGS)
    convg_epilogue_regs<TC, EPI, TP, WRN, TRANS>(a, acc, acc_lds, slot, o0, p0, p1, HWo, GW, py, px);
  else
    convg_epilogue<TC, EPI, TRANS, TP, WRN, NHALF>(a, acc, reinterpret_cast<float*>(smem_), acc_lds, slot, o0, p0, p1,
                                                    HWo, GW, py, px);
}

// ------------------------------------------------------------------------ stride-1 3x3: LDS-resident input rows
// The generic kernel above gathers every (tap, channel-chunk) k-step of B from global memory: a 3x3 conv re-reads
// each input row 9 times through L1 and spends 5-14 VALU per MFMA on per-tap gather addressing
// (profiles/r2_s3_pmc_imagenet_after.txt).  Here a work item is R whole rows of one image (TP >= R*W pixels); for
// each BK-channel chunk the (R+2) x (W+2) halo tile is staged in LDS ONCE (loads issued a whole chunk -- 9 k-steps
// -- ahead) and the 9 taps read their B fragments from it at a constant offset.  A (weights) is staged per k-step
// as in the generic kernel (AKM: data gradient straight from the forward layout, taps flipped).
// k order: chunk c outer, tap t inner.  Forward: A columns t*Ci + c*BK; gathered rows y + t/3 - 1, x + t%3 - 1.
template <int TP, int TC, int SOPS>
__host__ __device__ constexpr int t3_nhalf() {
  // smallest split of the fp32 epilogue staging (TP * (TC + 4) floats) that fits the operand buffers, with whole
  // 16-pixel tiles and whole workgroup passes (256 / (TC / 8) pixel rows) per part
  for (int n = 1; n <= TP / 16; ++n) {
    if (TP % n != 0 || (TP / n) % 16 != 0 || (TP / n) % (2048 / TC) != 0) continue;
    if (2 * TP * (TC + 4) / n <= SOPS) return n;
  }
  return -1;
}

#ifndef T3_DIRECT_A
#define T3_DIRECT_A 1  // forward t3: A fragments loaded directly from the weight rows (no LDS staging of A)
#endif
#ifndef T3_EPI_REGS
#define T3_EPI_REGS 0  // 1: register-direct epilogue (convg_epilogue_regs) instead of the LDS-staged one
#endif
#ifndef T3_EPI_LDS
// epilogue staging budget (bf16 elements; 0: the operand buffers' size).  30000 (59 KB, still 2 workgroups per CU)
// stages the 28 / 14-wide tiles in 2 parts instead of 7: data gradient 429 -> 404 us (28), 334 -> 316 us (14), the
// forward unchanged (tools/t3_bench.py, profiles/r5_t3_epilogue.log)
#define T3_EPI_LDS 30000
#endif
#ifndef T3_A_AHEAD
#define T3_A_AHEAD 1  // ... that many k-steps ahead (2: a 3-set register ring, measured flat: profiles/r5_imagenet_stem_ahead_ab.log)
#endif
#ifndef DTF_STAMP
#define DTF_STAMP 0
#endif
#if DTF_STAMP  // diagnostic build (tools/t3_bench.py --stamps): per-workgroup phase stamps of convg_t3_kernel
#define T3_STAMP_WGS 8192
__device__ unsigned long long dtf_t3_stamps[T3_STAMP_WGS][8];
#define T3_STAMP_DECL unsigned long long st_[8] = {0};
#define T3_STAMP(i) (st_[i] = __builtin_amdgcn_s_memrealtime())
#define T3_STAMP_FLUSH()                                                                  \
  do {                                                                                    \
    __builtin_amdgcn_s_waitcnt(0);                                                        \
    st_[4] = __builtin_amdgcn_s_memrealtime();                                            \
    unsigned hw_, xcc_;                                                                   \
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_));                     \
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_));                   \
    st_[5] = hw_;                                                                         \
    st_[6] = xcc_;                                                                        \
    if (threadIdx.x == 0 && blockIdx.x < T3_STAMP_WGS)                                    \
      for (int i_ = 0; i_ < 8; ++i_) dtf_t3_stamps[blockIdx.x][i_] = st_[i_];              \
  } while (0)
#else
#define T3_STAMP_DECL
#define T3_STAMP(i) ((void)0)
#define T3_STAMP_FLUSH() ((void)0)
#endif

// XF: the staged input rows get BN + ReLU (coefficients c_in: scale / shift of the input's BN) -- the folded forward
template <int TC, int EPI, bool AKM, int W, int R, int TP, int WRN, bool XF = false>
__global__ __launch_bounds__(256, 2) void convg_t3_kernel(CgArgs a) {
  constexpr int BK = 32;
  constexpr int PW = TP / (4 / WRN), NTP = PW / 16, MT = TC / WRN / 16;
  static_assert(PW % 16 == 0 && TP >= R * W && W % R == 0, "pixel tile: whole rows, bands divide the image");
  constexpr int RP = BK + 16;  // A row / staged-pixel pitch (bf16; 96 B = 6 bank quads per pixel)
  constexpr int CPR = BK / 8, RPT = 256 / CPR;
  constexpr int KPA = TC + 8;
  constexpr int SA = (TC * RP > BK * KPA) ? TC * RP : BK * KPA;
  // staged tile: RT rows x WS columns (halo), LDS row pitch WT = W + 8 pixels, pixel pitch 96 B: every B fragment
  // read (ds_read_b128: its lane groups are {0-3,12-15,20-27}, {4-11,16-19,28-31}, .. -- pixel i with k-chunk j
  // against pixels i' with chunk j + 1) hits 16 distinct bank quads for every tap offset and for fragments that
  // wrap to the next image row (the former 80 B / W + 16 pitches were 2-way: 1,193-4,432 conflicts per wave,
  // profiles/r3_pmc_imagenet_t3.txt; exhaustive check over tap offsets / fragment starts in tools/t3_bank_check.py)
  constexpr int WS = W + 2, WT = W + 8, RT = R + 2, NBP = RT * WS;
  constexpr int NBC = NBP * CPR, MAXB = (NBC + 255) / 256;
  constexpr int SBT = RT * WT * RP + 8;  // + slack for the inactive staging slots
  constexpr int SOPS = 2 * SA + SBT;
  constexpr int NHALF = t3_nhalf<TP, TC, (T3_EPI_LDS > SOPS ? T3_EPI_LDS : SOPS)>();
  static_assert(NHALF > 0, "epilogue staging split");
  constexpr int SEPI = 2 * TP * (TC + 4) / NHALF;
  __shared__ __attribute__((aligned(16))) bf16_t smem_[SOPS > SEPI ? SOPS : SEPI];
  __shared__ dtf_acc_t acc_lds[2][TC];
  bf16_t (*sa)[SA] = reinterpret_cast<bf16_t (*)[SA]>(smem_);
  bf16_t* sbt = smem_ + 2 * SA;
  T3_STAMP_DECL
  T3_STAMP(0);
  const int4 wk = a.work[blockIdx.x];
  DTF_WG_CHECK(wk.x >= 0 && wk.y >= 0 && wk.z > wk.y && wk.z - wk.y <= R * W && a.Wi == W && a.Hi % R == 0);
  const int slot = wk.x, p0 = wk.y, p1 = wk.z, o0 = wk.w;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wr = wave % WRN, wc = wave / WRN;
  const int Ci = a.Ci, H = a.Hi;
  const int img = p0 / (H * W), y0 = (p0 - img * H * W) / W;
  for (int i = tid; i < 2 * TC; i += 256) (&acc_lds[0][0])[i] = 0;
  // B staging slots: chunk idx = tid + 256 j -> staged pixel (r, col), 8-channel piece c8
  const bf16_t* xb = a.x + (long)img * H * W * Ci;
  int bl[MAXB], bg[MAXB];
  unsigned bok = 0;
#pragma unroll
  for (int j = 0; j < MAXB; ++j) {
    const int idx = tid + 256 * j;
    const int pix = idx / CPR, c8 = idx % CPR, r = pix / WS, col = pix % WS;
    const int gy = y0 - 1 + r, gx = col - 1;
    const bool ok = idx < NBC && gy >= 0 && gy < H && gx >= 0 && gx < W;
    bl[j] = idx < NBC ? (r * WT + col) * RP + 8 * c8 : RT * WT * RP;
    bg[j] = ok ? (gy * W + gx) * Ci + 8 * c8 : 0;
    bok |= (unsigned)ok << j;
  }
  // XF: the input BN's scale / shift of every channel in LDS (Ci <= 512), read at staging time (held in registers
  // across the 9 k-steps of a chunk they made the kernel spill)
  __shared__ float xcf[XF ? 2 * 512 : 1];
  if constexpr (XF) {
    const float* cb = a.c_in + (long)slot * 4 * a.cmax;
    for (int i = tid; i < Ci; i += 256) {
      xcf[i] = cb[i];
      xcf[512 + i] = cb[a.cmax + i];
    }
    __syncthreads();  // the first staging (before the k loop's first barrier) reads them
  }
  int cur_c = 0;  // XF: channel chunk of the rows last loaded by load_b
  auto load_b = [&](int c, uint4 (&v)[MAXB]) {
#pragma unroll
    for (int j = 0; j < MAXB; ++j) v[j] = ld16(xb, bg[j] + c * BK, (bok >> j) & 1u);
    cur_c = c;
  };
  auto store_b = [&](const uint4 (&v)[MAXB]) {
    float sc[8], sh[8];
    if constexpr (XF) {
      const int c0 = cur_c * BK + 8 * (tid % CPR);  // the same 8 channels for every slot j of this thread
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        sc[k] = xcf[c0 + k];
        sh[k] = xcf[512 + c0 + k];
      }
    }
#pragma unroll
    for (int j = 0; j < MAXB; ++j) {
      uint4 t = v[j];
      if constexpr (XF) t = ((bok >> j) & 1u) ? bnrelu8(t, sc, sh) : make_uint4(0, 0, 0, 0);  // halo stays 0
      *reinterpret_cast<uint4*>(sbt + bl[j]) = t;
    }
  };
  // A (weights), one k-step = (chunk c, tap t)
  const bf16_t* wbase = a.w + (long)slot * a.w_mstride + a.w_off;
  constexpr int AJ = TC * BK / 2048, ACH = TC / 8;
  const int cB = tid % CPR, rB = tid / CPR;
  auto load_a = [&](int c, int t, uint4 (&v)[AJ]) {
    if constexpr (AKM) {  // rows of the k-major tile: dy channels c*BK + kr of forward tap 8 - t
#pragma unroll
      for (int j = 0; j < AJ; ++j) {
        const int kr = tid / ACH + (256 / ACH) * j, ch = tid % ACH;
        v[j] = ld16(wbase, ((long)(c * BK + kr) * 9 + (8 - t)) * a.Co + o0 + 8 * ch, o0 + 8 * ch < a.Co);
      }
    } else {
#pragma unroll
      for (int j = 0; j < AJ; ++j) {
        const int r = rB + RPT * j;
        v[j] = ld16(wbase, (long)(o0 + r) * 9 * Ci + t * Ci + c * BK + 8 * cB, o0 + r < a.Co);
      }
    }
  };
  auto store_a = [&](bf16_t* dst, const uint4 (&v)[AJ]) {
#pragma unroll
    for (int j = 0; j < AJ; ++j) {
      if constexpr (AKM)
        *reinterpret_cast<uint4*>(dst + kperm(tid / ACH + (256 / ACH) * j) * KPA + 8 * (tid % ACH)) = v[j];
      else
        *reinterpret_cast<uint4*>(dst + (rB + RPT * j) * RP + 8 * cB) = v[j];
    }
  };
  // this lane's B fragment rows: pixel p = wc * PW + 16 n + lane % 16 of the tile -> staged pixel (y, x)
  int bpo[NTP];
#pragma unroll
  for (int n = 0; n < NTP; ++n) {
    int p = wc * PW + 16 * n + (lane & 15);
    p = p < R * W ? p : 0;  // padding pixels (discarded by the epilogue) read pixel 0
    bpo[n] = ((p / W) * WT + p % W) * RP + 8 * (lane >> 4);
  }
  f32x4_t acc[MT][NTP];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NTP; ++n) acc[m][n] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  const int nch = Ci / BK, nk = 9 * nch;
  // (the 64-channel 56-wide instance keeps LDS-staged A: its 28 accumulator tiles plus two fragment sets spill)
  if (!AKM && T3_DIRECT_A && TC == 128 && !(a.flags & 1)) {
    // Forward: A fragments straight from the OHWI weight rows (lane: row o, 8 consecutive channels of one tap = one
    // 16-byte load) into registers one k-step ahead -- no LDS staging of A, so no barrier per k-step: the workgroup
    // synchronises only when the next channel chunk's input rows replace the staged tile (every 9 k-steps)
    uint4 rb[MAXB];
    load_b(0, rb);
    store_b(rb);
    const int orow0 = o0 + wr * (TC / WRN) + (lane & 15);
    const bf16_t* wl = wbase + (long)orow0 * 9 * Ci + 8 * (lane >> 4);
    auto load_fa = [&](int c_, int t_, bf16x8_t (&f)[MT]) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
        f[m] = __builtin_bit_cast(bf16x8_t, ld16(wl, (long)16 * m * 9 * Ci + t_ * Ci + c_ * BK, orow0 + 16 * m < a.Co));
    };
    // A fragments T3_A_AHEAD k-steps ahead (2: a register ring of three sets -- one k-step of 28 MFMAs is ~450
    // cycles per wave, less than an L2-hit round trip of the weight rows)
    bf16x8_t fa[MT], fan[MT], fan2[MT];
    load_fa(0, 0, fa);
    if (T3_A_AHEAD > 1 && nk > 1) load_fa(0, 1, fan);  // k-step 1 = (chunk 0, tap 1)
    __syncthreads();
    int c = 0, t = 0;
    for (int ks = 0; ks < nk; ++ks) {
      const bool more = ks + 1 < nk;
      if constexpr (T3_A_AHEAD > 1) {
        if (ks + 2 < nk) {  // k-step ks + 2 = (chunk, tap) two taps on
          const int t2 = t + 2 > 8 ? t + 2 - 9 : t + 2, c2 = t + 2 > 8 ? c + 1 : c;
          load_fa(c2, t2, fan2);
        }
      } else if (more) {
        load_fa(t == 8 ? c + 1 : c, t == 8 ? 0 : t + 1, fan);
      }
      if (t == 0 && c + 1 < nch) load_b(c + 1, rb);  // next chunk's rows: 9 k-steps of latency cover
      const int tapo = ((t / 3) * WT + t % 3) * RP;
      bf16x8_t fb[NTP];
#pragma unroll
      for (int n = 0; n < NTP; ++n) fb[n] = *reinterpret_cast<const bf16x8_t*>(sbt + bpo[n] + tapo);
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NTP; ++n) acc[m][n] = mfma16(fa[m], fb[n], acc[m][n]);
      if (t == 8 && more) {  // chunk boundary: every wave is done with the staged rows
        __syncthreads();
        store_b(rb);
        __syncthreads();
      }
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        fa[m] = fan[m];
        if constexpr (T3_A_AHEAD > 1) fan[m] = fan2[m];
      }
      if (++t == 9) {
        t = 0;
        ++c;
      }
    }
    if constexpr (T3_EPI_REGS) {
      convg_epilogue_regs<TC, EPI, TP, WRN>(a, acc, acc_lds, slot, o0, p0, p1);
    } else {
      __syncthreads();  // the epilogue reuses the operand LDS
      convg_epilogue<TC, EPI, false, TP, WRN, NHALF, false>(a, acc, reinterpret_cast<float*>(smem_), acc_lds, slot, o0, p0,
                                                     p1, 0, 0, 0, 0);
    }
    return;
  }
  // A (weights) is prefetched one k-step ahead (a two-deep register ring, loop unrolled by two, measured the same:
  // profiles/r3_imagenet_t3_ab.log); the input rows of the next channel chunk a whole chunk (9 k-steps) ahead
  uint4 ra[AJ], rb[MAXB];
  load_b(0, rb);
  load_a(0, 0, ra);
  store_b(rb);
  store_a(sa[0], ra);
  __syncthreads();
  T3_STAMP(1);
  int c = 0, t = 0;
  for (int ks = 0; ks < nk; ++ks) {
    const bool more = ks + 1 < nk;
    bf16_t* sa_cur = sa[ks & 1];
    if (more) load_a(t == 8 ? c + 1 : c, t == 8 ? 0 : t + 1, ra);
    if (t == 0 && c + 1 < nch) load_b(c + 1, rb);  // next chunk's rows: 9 k-steps of latency cover
    const int tapo = ((t / 3) * WT + t % 3) * RP;
    bf16x8_t fa[MT], fb[NTP];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      if constexpr (AKM) {
        const int g = lane >> 4, q = (lane & 15) >> 2, p4 = lane & 3;
        const int rb_ = wr * (TC / WRN) + 16 * m + 4 * p4;
        const s16x4_t lo = ds_read_tr(sa_cur + ktr_lo(g, q) * KPA + rb_);
        const s16x4_t hi = ds_read_tr(sa_cur + ktr_hi(g, q) * KPA + rb_);
        fa[m] = (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      } else {
        fa[m] = *reinterpret_cast<const bf16x8_t*>(sa_cur + (wr * (TC / WRN) + 16 * m + (lane & 15)) * RP +
                                                   8 * (lane >> 4));
      }
    }
#pragma unroll
    for (int n = 0; n < NTP; ++n) fb[n] = *reinterpret_cast<const bf16x8_t*>(sbt + bpo[n] + tapo);
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int n = 0; n < NTP; ++n) acc[m][n] = mfma16(fa[m], fb[n], acc[m][n]);
    if (more) {
      if (t == 8) {  // chunk boundary: every wave is done with the staged rows
        __syncthreads();
        store_b(rb);
      }
      store_a(sa[(ks & 1) ^ 1], ra);
    }
    __syncthreads();
    if (++t == 9) {
      t = 0;
      ++c;
    }
  }
  T3_STAMP(2);
  if constexpr (T3_EPI_REGS)
    convg_epilogue_regs<TC, EPI, TP, WRN>(a, acc, acc_lds, slot, o0, p0, p1);
  else
    convg_epilogue<TC, EPI, false, TP, WRN, NHALF, false>(a, acc, reinterpret_cast<float*>(smem_), acc_lds, slot, o0, p0,
                                                   p1, 0, 0, 0, 0);
  T3_STAMP(3);
  T3_STAMP_FLUSH();
}

// ---------------------------------------------------------------------------------------------- wgrad
// Tile: 128 output channels (rows) x 128 (tap, ci) columns, k = PK output pixels per step (32 or 64).
constexpr int WT = 128;
constexpr int KP = WT + 8;

// WO: output-channel rows per tile (128: 2 x 2 waves of 64 x 64; 64: 1 x 4 waves of 64 x 32, for Co = 64 layers
// whose 128-row tile would be half padding)
// occupancy matters more than anything else here (the k-step loads are latency-bound): ask for 4 workgroups per
// CU (<= 128 registers); measured: the 140-register build at 3 per CU, and a prefetch-2 build at 2 per CU, slower
template <int MODE_X, int MODE_DY, int PK = 32, int WO = 128, bool P1 = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PK == 32 ? 4 : 2))) void convg_wgrad_kernel(CgArgs a) {
  constexpr int NJ = PK / 16;  // pixel rows per thread per k-step
  constexpr int WRN = WO / 64, WCN = 4 / WRN;  // wave grid (rows x columns)
  constexpr int CWW = WT / WCN, NTN = CWW / 16;  // columns per wave, MFMA column tiles per wave
  __shared__ __attribute__((aligned(16))) bf16_t sd[2][PK * KP];
  __shared__ __attribute__((aligned(16))) bf16_t sx[2][PK * KP];
  extern __shared__ float dyn[];  // x coefficients (2*Ci) then dy coefficients (3*Co)
  const int4 wk = a.work[blockIdx.x];
  DTF_WG_CHECK(wk.x >= 0 && wk.y >= 0 && wk.z >= wk.y);
  const int slot = wk.x, p0 = wk.y, p1 = wk.z, o0 = wk.w & 0xffff, n0 = (wk.w >> 16) * 8;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wr = wave % WRN, wc = wave / WRN;
  const int Ci = a.Ci, Co = a.Co, K = a.kh * a.kw * Ci;
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
    for (int i = tid; i < Co; i += 256) {
      cd[i] = cb[i];
      cd[Co + i] = cb[a.cmax + i];
      if constexpr (MODE_DY == 2) cd[2 * Co + i] = cb[2 * a.cmax + i];
    }
  }
  // loads: k-row = tid >> 4 (+16 for j = 1), 8-wide column chunk = tid & 15
  const int kr = tid >> 4, cc = tid & 15;
  const int HWo = a.Ho * a.Wo;
  const long img_x = (long)a.Hi * a.Wi * Ci;
  // x column chunk -> (tap, ci0), fixed for the workgroup
  const int xcol = n0 + 8 * cc;
  const int xtap = xcol >> a.log2ci, xci = xcol & (Ci - 1);
  const int xky = xtap / a.kw, xkx = xtap - xky * a.kw;
  const bool xcol_ok = xcol < K;
  const int dcol = o0 + 8 * cc;
  const bool dcol_ok = dcol < Co && 8 * cc < WO;
  const float r_hw = 1.0f / (float)HWo, r_w = 1.0f / (float)a.Wo;
  auto divmod = [](int n, int d, float rd, int& q, int& r) {  // exact for n < 2^24
    q = (int)((float)n * rd);
    r = n - q * d;
    if (r < 0) {
      --q;
      r += d;
    } else if (r >= d) {
      ++q;
      r -= d;
    }
  };
  // Pixel table of a k-step (PK output pixels), computed by the first PK threads one k-step ahead and shared
  // through LDS (every pixel used to be decomposed by all 16 column-chunk threads of its row):
  // {dy element offset, x image base, oy*S - P, ox*S - P}; an out-of-range pixel gets oy*S - P = -2^30.
  __shared__ int4 pinfo[2][PK];
  auto make_pinfo = [&](int pk0) {
    if (tid < PK) {
      const int p = pk0 + tid;
      int4 inf = make_int4(0, 0, -(1 << 30), 0);
      if (p < p1) {
        int img, rem, oy, ox;
        divmod(p, HWo, r_hw, img, rem);
        divmod(rem, a.Wo, r_w, oy, ox);
        inf = make_int4((int)((unsigned)p * (unsigned)Co), (int)((unsigned)img * (unsigned)img_x),
                        oy * a.stride - a.pad, ox * a.stride - a.pad);
      }
      pinfo[(pk0 - p0) / PK & 1][tid] = inf;
    }
  };
  // P1 (stride-1 1x1 conv, x pixel = dy pixel): base offsets advanced by a wave-uniform k-step stride instead of
  // the per-k-step pixel table (as convg_wgrad_wide_kernel P1)
  const long dbase = (long)(p0 + kr) * Co + dcol, xbase = (long)(p0 + kr) * Ci + xci;
  auto load = [&](int pk0, uint4 (&dv)[NJ], uint4 (&dv2)[NJ], uint4 (&xv)[NJ], unsigned& okm) {
    okm = 0;
    if constexpr (P1) {
      const long dk = (long)(pk0 - p0) * Co, xk = (long)(pk0 - p0) * Ci;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const bool pin = pk0 + kr + 16 * j < p1;
        const bool dok = pin && dcol_ok, xok = pin && xcol_ok;
        const long dofs = dbase + dk + (long)(16 * j) * Co;
        dv[j] = ld16(a.dy, dofs, dok);
        dv2[j] = make_uint4(0, 0, 0, 0);
        if constexpr (MODE_DY == 2) dv2[j] = ld16(a.dy2, dofs, dok);
        xv[j] = ld16(a.x, xbase + xk + (long)(16 * j) * Ci, xok);
        okm |= ((unsigned)dok << j) | (((unsigned)xok << NJ) << j);
      }
      return;
    }
    const int par = (pk0 - p0) / PK & 1;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int4 inf = pinfo[par][kr + 16 * j];
      const bool pin = inf.z > -(1 << 29);
      dv2[j] = make_uint4(0, 0, 0, 0);
      const bool dok = pin && dcol_ok;
      dv[j] = ld16(a.dy, (long)(unsigned)inf.x + dcol, dok);
      if constexpr (MODE_DY == 2) dv2[j] = ld16(a.dy2, (long)(unsigned)inf.x + dcol, dok);
      okm |= (unsigned)dok << j;
      const int gy = inf.z + xky, gx = inf.w + xkx;
      const bool xok = pin && xcol_ok && gy >= 0 && gy < a.Hi && gx >= 0 && gx < a.Wi;
      xv[j] = ld16(a.x, (long)(unsigned)inf.y + (unsigned)((gy * a.Wi + gx) * Ci + xci), xok);
      okm |= ((unsigned)xok << NJ) << j;
    }
  };
  auto store = [&](bf16_t* d, bf16_t* xx, const uint4 (&dv)[NJ], const uint4 (&dv2)[NJ], const uint4 (&xv)[NJ],
                   unsigned okm) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      uint4 t = dv[j];
      if (MODE_DY != 0 && ((okm >> j) & 1u)) {
        uint32_t w32[4] = {t.x, t.y, t.z, t.w};
        const uint32_t h32[4] = {dv2[j].x, dv2[j].y, dv2[j].z, dv2[j].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int c = dcol + 2 * q;
          float x0 = lo2f(w32[q]), x1 = hi2f(w32[q]);
          if constexpr (MODE_DY == 1) {
            x0 = fmaxf(x0 * cd[c] + cd[Co + c], 0.f);
            x1 = fmaxf(x1 * cd[c + 1] + cd[Co + c + 1], 0.f);
          } else {
            const float h0 = lo2f(h32[q]), h1 = hi2f(h32[q]);
            x0 = cd[c] * x0 + cd[Co + c] * h0 + cd[2 * Co + c];
            x1 = cd[c + 1] * x1 + cd[Co + c + 1] * h1 + cd[2 * Co + c + 1];
          }
          w32[q] = pack2bf(x0, x1);
        }
        t = make_uint4(w32[0], w32[1], w32[2], w32[3]);
      }
      *reinterpret_cast<uint4*>(d + kperm(kr + 16 * j) * KP + 8 * cc) = t;
      uint4 u = xv[j];
      if (MODE_X == 1 && ((okm >> (NJ + j)) & 1u)) {
        uint32_t w32[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int c = xci + 2 * q;
          const float x0 = lo2f(w32[q]), x1 = hi2f(w32[q]);
          w32[q] = pack2bf(fmaxf(x0 * cx[c] + cx[Ci + c], 0.f), fmaxf(x1 * cx[c + 1] + cx[Ci + c + 1], 0.f));
        }
        u = make_uint4(w32[0], w32[1], w32[2], w32[3]);
      }
      *reinterpret_cast<uint4*>(xx + kperm(kr + 16 * j) * KP + 8 * cc) = u;
    }
  };
  f32x4_t acc[4][NTN];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < NTN; ++n) acc[m][n] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  // (A two-register-stage variant -- loads of k-step ks + 2 in flight while ks computes -- measured slower:
  // 22.5 -> 27.3 ms of wgrad per pop-8 ResNet-50 step, occupancy 3 -> 2; profiles/r2_s3_imagenet_wgrad_pf2.log)
  const int nk = (p1 - p0 + PK - 1) / PK;
  if constexpr (!P1) {
    make_pinfo(p0);
    if (nk > 1) make_pinfo(p0 + PK);
  }
  __syncthreads();  // coefficients + the first two pixel tables
  uint4 dv[NJ], dv2[NJ], xv[NJ];
  unsigned okm;
  load(p0, dv, dv2, xv, okm);
  store(sd[0], sx[0], dv, dv2, xv, okm);
  __syncthreads();
  const int g = lane >> 4, q = (lane & 15) >> 2, p4 = lane & 3;
  for (int ks = 0; ks < nk; ++ks) {
    const int cur = ks & 1;
    const bool more = ks + 1 < nk;
    if (more) load(p0 + PK * (ks + 1), dv, dv2, xv, okm);
    // table of k-step ks + 2 into the slot k-step ks read (its readers passed the previous barrier)
    if constexpr (!P1)
      if (ks + 2 < nk) make_pinfo(p0 + PK * (ks + 2));
#pragma unroll
    for (int kk = 0; kk < PK / 32; ++kk) {
      bf16x8_t fa[4], fb[NTN];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int cb = wr * 64 + 16 * m + 4 * p4;
        const s16x4_t lo = ds_read_tr(sd[cur] + (32 * kk + ktr_lo(g, q)) * KP + cb);
        const s16x4_t hi = ds_read_tr(sd[cur] + (32 * kk + ktr_hi(g, q)) * KP + cb);
        fa[m] = (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int n = 0; n < NTN; ++n) {
        const int cb = wc * CWW + 16 * n + 4 * p4;
        const s16x4_t lo = ds_read_tr(sx[cur] + (32 * kk + ktr_lo(g, q)) * KP + cb);
        const s16x4_t hi = ds_read_tr(sx[cur] + (32 * kk + ktr_hi(g, q)) * KP + cb);
        fb[n] = (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < NTN; ++n) acc[m][n] = mfma16(fa[m], fb[n], acc[m][n]);
    }
    if (more) store(sd[cur ^ 1], sx[cur ^ 1], dv, dv2, xv, okm);
    __syncthreads();
  }
  // D: lane holds column n = lane & 15 ((tap, ci) index), rows (o) 4*(lane>>4) + r
  dtf_acc_t* gr = a.grads + (long)slot * a.g_mstride + a.g_off;
  const int cr = a.cin_real > 0 ? a.cin_real : Ci;
  const int Kr = a.kh * a.kw * cr;
#pragma unroll
  for (int n = 0; n < NTN; ++n) {
    const int col = n0 + wc * CWW + 16 * n + (lane & 15);
    const int tap = col >> a.log2ci, ci = col & (Ci - 1);
    if (col >= K || ci >= cr) continue;
    const int colr = tap * cr + ci;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = o0 + wr * 64 + 16 * m + 4 * (lane >> 4) + r;
        if (o < Co) dtf_acc_add(gr + (long)o * Kr + colr, acc[m][n][r], DTF_FX_GRAD, slot);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------- wide wgrad
// Weight gradient of a 3x3 conv (plain operands, the default non-folded path) with WIDE column tiles: 64 output
// channels x 288 (tap, ci) columns per workgroup (K = 9 * Ci is a multiple of 576 for Ci % 64 == 0), 2 x 2 waves of
// 32 x 144 (18 MFMAs per wave and 32-pixel k-step instead of the 8 of a 64 x 128 tile): the per-k-step cost --
// pixel table, dy / x gathers, LDS writes, the barrier -- is paid for 2.25x the MFMA work, and the dy tile is staged
// once per 288 instead of 128 columns.

// WWO = 64 (Co = 64) or 128 output-channel rows per tile: 2 x 2 waves of (WWO/2) x 144 -- the 128-row form reads
// each B fragment for 4 instead of 2 MFMAs (the 64-row one is LDS-read-bound: 22 tr-reads per 18 MFMAs)
// WWT: columns per tile, 288 (3x3 convs: K = 9 Ci), 256 (1x1 convs with Ci % 256 == 0) or 416 (the 7x7 stem:
// 49 taps x 8 channels, one tile).
// MX 1: x operand = relu(BN(x)) applied while staging (c_in scale / shift per channel, staged in LDS; the folded
// forward keeps no materialised BN+ReLU output)
template <int WWO, int WWT, int MX = 0, bool P1 = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WWO == 64 ? 3 : 2))) void convg_wgrad_wide_kernel(CgArgs a) {
  constexpr int WWOP = WWO + 8, MTW = WWO / 32, DJ = WWO / 64, WWP = WWT + 8;
  constexpr int WXC = 32 * (WWT / 8);  // x chunks (8 columns) per k-step
  constexpr int WXJ = (WXC + 255) / 256;
  __shared__ __attribute__((aligned(16))) bf16_t sd[2][32 * WWOP];
  __shared__ __attribute__((aligned(16))) bf16_t sx[2][32 * WWP];
  __shared__ int4 pinfo[2][32];
  extern __shared__ float xcoef[];  // MX 1: scale [Ci] | shift [Ci]
  const int4 wk = a.work[blockIdx.x];
  DTF_WG_CHECK(wk.x >= 0 && wk.y >= 0 && wk.z >= wk.y);
  const int slot = wk.x, p0 = wk.y, p1 = wk.z, o0 = wk.w & 0xffff, n0 = (wk.w >> 16) * 8;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wr = wave & 1, wc = wave >> 1;
  const int Ci = a.Ci, Co = a.Co, K = a.kh * a.kw * Ci;
  if constexpr (MX == 1) {
    const float* cb = a.c_in + (long)slot * 4 * a.cmax;
    for (int i = tid; i < Ci; i += 256) {
      xcoef[i] = cb[i];
      xcoef[Ci + i] = cb[a.cmax + i];
    }
  }
  const int HWo = a.Ho * a.Wo;
  const long img_x = (long)a.Hi * a.Wi * Ci;
  // dy: DJ 16-byte chunks per thread and k-step (row (tid + 256 j) / (WWO / 8), 8 channels)
  int drow[DJ], dch[DJ];
  bool dok[DJ];
#pragma unroll
  for (int j = 0; j < DJ; ++j) {
    const int c = tid + 256 * j;
    drow[j] = c / (WWO / 8);
    dch[j] = 8 * (c % (WWO / 8));
    dok[j] = o0 + dch[j] < Co;
  }
  // x: chunks c = tid + 256 j of the [32 rows][36 chunks] k-step tile; (row, tap, ci) fixed for the workgroup
  int xrow[WXJ], xky[WXJ], xkx[WXJ], xoff[WXJ];
  bool xok[WXJ];
#pragma unroll
  for (int j = 0; j < WXJ; ++j) {
    const int c = tid + 256 * j;
    const int r = c / (WWT / 8), ch = c - r * (WWT / 8);
    const int col = n0 + 8 * ch;
    const int tap = col >> a.log2ci, ci = col & (Ci - 1);
    xrow[j] = r;
    xky[j] = tap / a.kw;
    xkx[j] = tap - xky[j] * a.kw;
    xoff[j] = kperm(r & 31) * WWP + 8 * ch;  // LDS element offset in the k-step tile (tile row kperm(pixel))
    xok[j] = c < WXC && col < K;
    xoff[j] += ci << 16;         // ci in the high half (unpacked at use)
  }
  const float r_hw = 1.0f / (float)HWo, r_w = 1.0f / (float)a.Wo;
  auto divmod = [](int n, int d, float rd, int& q, int& r) {  // exact for n < 2^24
    q = (int)((float)n * rd);
    r = n - q * d;
    if (r < 0) {
      --q;
      r += d;
    } else if (r >= d) {
      ++q;
      r -= d;
    }
  };
  auto make_pinfo = [&](int pk0) {
    if (tid < 32) {
      const int p = pk0 + tid;
      int4 inf = make_int4(0, 0, -(1 << 30), 0);
      if (p < p1) {
        int img, rem, oy, ox;
        divmod(p, HWo, r_hw, img, rem);
        divmod(rem, a.Wo, r_w, oy, ox);
        inf = make_int4((int)((unsigned)p * (unsigned)Co), (int)((unsigned)img * (unsigned)img_x),
                        oy * a.stride - a.pad, ox * a.stride - a.pad);
      }
      pinfo[(pk0 - p0) / 32 & 1][tid] = inf;
    }
  };
  bool xval[WXJ];  // MX 1: the chunk of xv holds real pixels (not padding)
  // P1 (stride-1 1x1 conv: the x pixel of a k row IS its dy pixel): per-thread base offsets advanced by a
  // wave-uniform k-step stride -- no per-k-step pixel table (make_pinfo's divides, an LDS int4 read per chunk) and
  // no bounds arithmetic beyond the item's pixel range
  long dbase[P1 ? DJ : 1], xbase[P1 ? WXJ : 1];
  if constexpr (P1) {
#pragma unroll
    for (int j = 0; j < DJ; ++j) dbase[j] = (long)(p0 + drow[j]) * Co + o0 + dch[j];
#pragma unroll
    for (int j = 0; j < WXJ; ++j) xbase[j] = (long)(p0 + xrow[j]) * Ci + (xoff[j] >> 16);
  }
  auto load = [&](int pk0, uint4 (&dv)[DJ], uint4 (&xv)[WXJ]) {
    if constexpr (P1) {
      const long dk = (long)(pk0 - p0) * Co, xk = (long)(pk0 - p0) * Ci;
#pragma unroll
      for (int j = 0; j < DJ; ++j) dv[j] = ld16(a.dy, dbase[j] + dk, pk0 + drow[j] < p1 && dok[j]);
#pragma unroll
      for (int j = 0; j < WXJ; ++j) {
        const bool ok = xok[j] && pk0 + xrow[j] < p1;
        xv[j] = ld16(a.x, xbase[j] + xk, ok);
        xval[j] = ok;
      }
      return;
    }
    const int par = (pk0 - p0) / 32 & 1;
#pragma unroll
    for (int j = 0; j < DJ; ++j) {
      const int4 di = pinfo[par][drow[j]];
      dv[j] = ld16(a.dy, (long)(unsigned)di.x + o0 + dch[j], di.z > -(1 << 29) && dok[j]);
    }
#pragma unroll
    for (int j = 0; j < WXJ; ++j) {
      const int4 inf = pinfo[par][xrow[j] & 31];
      const int gy = inf.z + xky[j], gx = inf.w + xkx[j];
      const bool ok = xok[j] && inf.z > -(1 << 29) && gy >= 0 && gy < a.Hi && gx >= 0 && gx < a.Wi;
      xv[j] = ld16(a.x, (long)(unsigned)inf.y + (unsigned)((gy * a.Wi + gx) * Ci + (xoff[j] >> 16)), ok);
      xval[j] = ok;
    }
  };
  // MX 1: the BN scale / shift of chunk j's 8 channels.  When 256 is a multiple of the chunks per tile row
  // (WWT = 256: the 1x1 tiles), every chunk j of a thread sits in the same column, so its 16 coefficients are read
  // from LDS once for the whole kernel (XCOL) instead of 4 16-byte reads per chunk and k-step -- as many LDS reads
  // as the k-step's MFMA operand fetches
  constexpr bool XCOL = MX == 1 && (256 % (WWT / 8)) == 0;
  float xsc[XCOL ? 8 : 1], xsh[XCOL ? 8 : 1];
  auto coef8 = [&](int c0, float (&sc)[8], float (&sh)[8]) {
    const float4 s0 = *reinterpret_cast<const float4*>(xcoef + c0), s1 = *reinterpret_cast<const float4*>(xcoef + c0 + 4);
    const float4 h0 = *reinterpret_cast<const float4*>(xcoef + Ci + c0),
                 h1 = *reinterpret_cast<const float4*>(xcoef + Ci + c0 + 4);
    sc[0] = s0.x; sc[1] = s0.y; sc[2] = s0.z; sc[3] = s0.w; sc[4] = s1.x; sc[5] = s1.y; sc[6] = s1.z; sc[7] = s1.w;
    sh[0] = h0.x; sh[1] = h0.y; sh[2] = h0.z; sh[3] = h0.w; sh[4] = h1.x; sh[5] = h1.y; sh[6] = h1.z; sh[7] = h1.w;
  };
  auto store = [&](bf16_t* d, bf16_t* xx, const uint4 (&dv)[DJ], const uint4 (&xv)[WXJ]) {
#pragma unroll
    for (int j = 0; j < DJ; ++j) *reinterpret_cast<uint4*>(d + kperm(drow[j]) * WWOP + dch[j]) = dv[j];
#pragma unroll
    for (int j = 0; j < WXJ; ++j) {
      if (tid + 256 * j >= WXC) continue;
      uint4 t = xv[j];
      if constexpr (MX == 1) {
        // a padding / out-of-range chunk (loaded as zeros) must stay zero after the transform
        if constexpr (XCOL) {
          t = xval[j] ? bnrelu8(t, xsc, xsh) : make_uint4(0, 0, 0, 0);
        } else {
          float sc[8], sh[8];
          coef8(xoff[j] >> 16, sc, sh);
          t = xval[j] ? bnrelu8(t, sc, sh) : make_uint4(0, 0, 0, 0);
        }
      }
      *reinterpret_cast<uint4*>(xx + (xoff[j] & 0xffff)) = t;
    }
  };
  constexpr int NTN = WWT / 2 / 16;  // 9 column tiles per wave
  f32x4_t acc[MTW][NTN];
#pragma unroll
  for (int m = 0; m < MTW; ++m)
#pragma unroll
    for (int n = 0; n < NTN; ++n) acc[m][n] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  const int nk = (p1 - p0 + 31) / 32;
  if constexpr (!P1) {
    make_pinfo(p0);
    if (nk > 1) make_pinfo(p0 + 32);
  }
  __syncthreads();
  if constexpr (XCOL) coef8(xoff[0] >> 16, xsc, xsh);  // (the xcoef rows are visible after the barrier above)
  uint4 dv[DJ], xv[WXJ];
  load(p0, dv, xv);
  store(sd[0], sx[0], dv, xv);
  __syncthreads();
  const int g = lane >> 4, q = (lane & 15) >> 2, p4 = lane & 3;
  for (int ks = 0; ks < nk; ++ks) {
    const int cur = ks & 1;
    const bool more = ks + 1 < nk;
    if (more) load(p0 + 32 * (ks + 1), dv, xv);
    if constexpr (!P1)
      if (ks + 2 < nk) make_pinfo(p0 + 32 * (ks + 2));
    bf16x8_t fa[MTW];
#pragma unroll
    for (int m = 0; m < MTW; ++m) {
      const int cb = wr * (WWO / 2) + 16 * m + 4 * p4;
      const s16x4_t lo = ds_read_tr(sd[cur] + ktr_lo(g, q) * WWOP + cb);
      const s16x4_t hi = ds_read_tr(sd[cur] + ktr_hi(g, q) * WWOP + cb);
      fa[m] = (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
#pragma unroll
    for (int n = 0; n < NTN; ++n) {
      const int cb = wc * (WWT / 2) + 16 * n + 4 * p4;
      const s16x4_t lo = ds_read_tr(sx[cur] + ktr_lo(g, q) * WWP + cb);
      const s16x4_t hi = ds_read_tr(sx[cur] + ktr_hi(g, q) * WWP + cb);
      const bf16x8_t fb = (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
      for (int m = 0; m < MTW; ++m) acc[m][n] = mfma16(fa[m], fb, acc[m][n]);
    }
    if (more) store(sd[cur ^ 1], sx[cur ^ 1], dv, xv);
    __syncthreads();
  }
  dtf_acc_t* gr = a.grads + (long)slot * a.g_mstride + a.g_off;
  // real input channels of a channel-padded operand (stem); cin_real = -3: the space-to-depth stem (4x4 taps over
  // 2x2 blocks of a 3-channel image): column (tap', (2 dy + dx) * 3 + c) is weight (2a + dy - 1, 2b + dx - 1, c) of
  // the 7x7 kernel (cg_weight_prep s2d); each 7x7x3 weight is reached from exactly one column
  const bool s2d = a.cin_real == -3;
  const int cr = a.cin_real > 0 ? a.cin_real : (s2d ? 3 : Ci);
  const int Kr = s2d ? 49 * 3 : a.kh * a.kw * cr;
#pragma unroll
  for (int n = 0; n < NTN; ++n) {
    const int col0 = n0 + wc * (WWT / 2) + 16 * n + (lane & 15);
    const int ci_ = col0 & (Ci - 1);
    int col;
    if (s2d) {
      const int tap = col0 >> a.log2ci, q = ci_ / 3, c = ci_ - 3 * q;
      const int ky = 2 * (tap >> 2) + (q >> 1) - 1, kx = 2 * (tap & 3) + (q & 1) - 1;
      if (col0 >= K || q >= 4 || ky < 0 || ky > 6 || kx < 0 || kx > 6) continue;
      col = (ky * 7 + kx) * 3 + c;
    } else {
      if (col0 >= K || ci_ >= cr) continue;
      col = (col0 >> a.log2ci) * cr + ci_;
    }
#pragma unroll
    for (int m = 0; m < MTW; ++m) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = o0 + wr * (WWO / 2) + 16 * m + 4 * (lane >> 4) + r;
        if (o < Co) dtf_acc_add(gr + (long)o * Kr + col, acc[m][n][r], DTF_FX_GRAD, slot);
      }
    }
  }
}

// ----------------------------------------------------------------------------------------- row-band wgrad
// Weight gradient of a stride-1 3x3 conv (plain operands) from LDS-resident row bands.  The wide kernel above
// gathers its x operand per 32-pixel k-step as 288 (tap, ci) columns -- every input element is fetched once per tap
// (9x) plus per-column addressing VALU, and with a 64-row tile (Co = 64) that traffic feeds only 18 MFMAs per wave
// (311 B per MFMA; the stage-1 3x3 weight gradients ran at 4.6x their MFMA floor).  Here a workgroup stages ONE
// band of R image rows: dy [R*W pixels][64 co] and the input halo [(R+2)][(W+2)][32 ci], and all 9 taps read their
// B fragments from the halo at a constant offset (ds_read_b64_tr_b16 along the pixels), so x is fetched ~1.5x
// (halo) instead of 9x.  Tile: 64 co x (9 taps x 32 ci) = 288 columns, 2 x 2 waves of 32 x 144 (18 MFMAs per wave
// and k-step); the next band is prefetched into registers while the current one runs.
// work: (slot, first band, end band, o0 | ci-chunk << 16); band b = image b / (H / R), rows (b % (H / R)) * R ..
// Pixels past R * W in the last k-step (W = 28: 196 of 224) stage zero dY rows and contribute nothing.
// KT x KT taps, BKC input channels per column tile, PAD rows / columns before the image: <W, R, 3, 32, 1> for the
// 3x3 convs; <112, 2, 4, 16, 2> for the space-to-depth stem (4x4 over 16 block channels, cin_real = -3: columns
// remapped onto the 7x7x3 kernel as in the wide kernel)
// MX 1: x operand = relu(BN(x)) applied while the halo is staged (c_in scale / shift; padding stays zero) -- the
// selectively folded forward (hip_imagenet.py CG_FOLD2) keeps no materialised relu(BN2(h1))
template <int W, int R, int KT = 3, int BKC = 32, int PAD = 1, int MX = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void convg_wgrad_t3_kernel(CgArgs a) {
  constexpr int WO = 64, HPC = BKC / 16;  // HPC: 16-channel column tiles per tap
  constexpr int NPV = R * W, NKS = (NPV + 31) / 32, NPX = NKS * 32;
  constexpr int WOP = WO + 8;            // dY tile pitch (bf16)
  constexpr int CP = BKC + 8;            // halo pixel pitch (bf16)
  constexpr int WS = W + KT - 1, RT = R + KT - 1;  // halo columns / rows
  constexpr int NCT = KT * KT * HPC;     // column tiles of the workgroup (9 x 2 = 18; 16 x 1 = 16)
  constexpr int MTW = WO / 32, NTW = NCT / 2;  // A tiles per wave (32 rows), B column tiles per wave
  constexpr int DCH = NPX * WO / 8, DJ = (DCH + 255) / 256;
  constexpr int XCH = RT * WS * (BKC / 8), XJ = (XCH + 255) / 256;
  __shared__ __attribute__((aligned(16))) bf16_t sd[NPX * WOP];
  __shared__ __attribute__((aligned(16))) bf16_t sx[RT * WS * CP + 8];
  __shared__ float xcf[MX ? 2 * BKC : 1];
  const int4 wk = a.work[blockIdx.x];
  DTF_WG_CHECK(wk.x >= 0 && wk.y >= 0 && wk.z > wk.y && a.Wi == W && a.Wo == W && a.Ho == a.Hi && a.Hi % R == 0 &&
               a.kh == KT && a.pad == PAD);
  const int slot = wk.x, b0 = wk.y, b1 = wk.z, o0 = wk.w & 0xffff, cc = wk.w >> 16;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wr = wave & 1, wc = wave >> 1;
  const int Ci = a.Ci, Co = a.Co, H = a.Hi, BPI = H / R;
  if constexpr (MX == 1) {
    if (tid < BKC) {
      const float* cb = a.c_in + (long)slot * 4 * a.cmax + cc * BKC;
      xcf[tid] = cb[tid];
      xcf[BKC + tid] = cb[a.cmax + tid];
    }
    __syncthreads();
  }
  // dY slots: chunk q = tid + 256 j -> band pixel q / 8, channels 8 (q % 8)
  int dpx[DJ], dch[DJ];
  unsigned dok = 0;
#pragma unroll
  for (int j = 0; j < DJ; ++j) {
    const int q = tid + 256 * j;
    dpx[j] = q / (WO / 8);
    dch[j] = 8 * (q % (WO / 8));
    dok |= (unsigned)(q < DCH && dpx[j] < NPV && o0 + dch[j] < Co) << j;
  }
  // halo slots: chunk q = tid + 256 j -> halo pixel (hr, hc), 8-channel piece c8
  int xhr[XJ], xhc[XJ], xc8[XJ];
#pragma unroll
  for (int j = 0; j < XJ; ++j) {
    const int q = tid + 256 * j, hp = q / (BKC / 8);
    xc8[j] = q < XCH ? 8 * (q % (BKC / 8)) : 0;
    xhr[j] = q < XCH ? hp / WS : RT;  // RT: inactive slot (never valid, stores into the slack)
    xhc[j] = hp % WS;
  }
  uint4 dv[DJ], xv[XJ];
  unsigned xok = 0;
  auto load = [&](int band) {
    const int img = band / BPI, y0 = (band - img * BPI) * R;
    const long dbase = ((long)img * H + y0) * W * Co + o0;
#pragma unroll
    for (int j = 0; j < DJ; ++j) dv[j] = ld16(a.dy, dbase + (long)dpx[j] * Co + dch[j], (dok >> j) & 1u);
    xok = 0;
    const long xbase = (long)img * H * W * Ci + cc * BKC;
#pragma unroll
    for (int j = 0; j < XJ; ++j) {
      const int gy = y0 - PAD + xhr[j], gx = xhc[j] - PAD;
      const bool ok = xhr[j] < RT && gy >= 0 && gy < H && gx >= 0 && gx < W;
      xv[j] = ld16(a.x, xbase + ((long)gy * W + gx) * Ci + xc8[j], ok);
      xok |= (unsigned)ok << j;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int j = 0; j < DJ; ++j) {
      const int q = tid + 256 * j;
      if (q < DCH) *reinterpret_cast<uint4*>(sd + dpx[j] * WOP + dch[j]) = (dok >> j) & 1u ? dv[j] : make_uint4(0, 0, 0, 0);
    }
    float sc[8], sh[8];
    if constexpr (MX == 1) {
      const int c0 = xc8[0];  // the same 8 channels for every slot of this thread (256 % (BKC / 8) == 0)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        sc[k] = xcf[c0 + k];
        sh[k] = xcf[BKC + c0 + k];
      }
    }
#pragma unroll
    for (int j = 0; j < XJ; ++j) {
      const int off = xhr[j] < RT ? (xhr[j] * WS + xhc[j]) * CP + xc8[j] : RT * WS * CP;
      uint4 t = (xok >> j) & 1u ? xv[j] : make_uint4(0, 0, 0, 0);
      if constexpr (MX == 1) t = (xok >> j) & 1u ? bnrelu8(t, sc, sh) : t;
      *reinterpret_cast<uint4*>(sx + off) = t;
    }
  };
  // fragment lanes: g = lane / 16 (8 k-rows), q = k-row within the quad, p4 = 4-column piece
  const int g = lane >> 4, q = (lane & 15) >> 2, p4 = lane & 3;
  f32x4_t acc[MTW][NTW];
#pragma unroll
  for (int m = 0; m < MTW; ++m)
#pragma unroll
    for (int n = 0; n < NTW; ++n) acc[m][n] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  load(b0);
  store();
  __syncthreads();
  for (int b = b0; b < b1; ++b) {
    const bool more = b + 1 < b1;
    if (more) load(b + 1);
#pragma unroll 1
    for (int ks = 0; ks < NKS; ++ks) {
      // this lane's two k-rows (band pixels); kperm order: the 8 pixels a 32-lane half reads are 2 apart, which
      // spreads both the dY rows and the halo pixels over distinct banks
      const int pa = ks * 32 + ktr_lo(g, q), pb = ks * 32 + ktr_hi(g, q);
      bf16x8_t fa[MTW];
#pragma unroll
      for (int m = 0; m < MTW; ++m) {
        const int cb = wr * (WO / 2) + 16 * m + 4 * p4;
        const s16x4_t lo = ds_read_tr(sd + pa * WOP + cb);
        const s16x4_t hi = ds_read_tr(sd + pb * WOP + cb);
        fa[m] = (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
      const int qa = pa < NPV ? pa : 0, qb = pb < NPV ? pb : 0;  // padding pixels (zero dY) read pixel 0
      const int ha = ((qa / W) * WS + qa % W) * CP + 4 * p4, hb = ((qb / W) * WS + qb % W) * CP + 4 * p4;
#pragma unroll
      for (int n = 0; n < NTW; ++n) {
        const int j = NTW * wc + n, t = j / HPC;  // column tile j = (tap t, 16-channel piece j % HPC)
        const int toff = ((t / KT) * WS + t % KT) * CP + 16 * (j % HPC);
        const s16x4_t lo = ds_read_tr(sx + ha + toff);
        const s16x4_t hi = ds_read_tr(sx + hb + toff);
        const bf16x8_t fb = (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int m = 0; m < MTW; ++m) acc[m][n] = mfma16(fa[m], fb, acc[m][n]);
      }
    }
    __syncthreads();
    if (more) {
      store();
      __syncthreads();
    }
  }
  // D: lane holds column (lane & 15) of tile (tap, piece), rows 4 (lane >> 4) + r
  dtf_acc_t* gr = a.grads + (long)slot * a.g_mstride + a.g_off;
  const bool s2d = a.cin_real == -3;
#pragma unroll
  for (int n = 0; n < NTW; ++n) {
    const int j = NTW * wc + n, t = j / HPC;
    const int ci = cc * BKC + 16 * (j % HPC) + (lane & 15);
    long col = (long)t * Ci + ci;
    int Kr = KT * KT * Ci;
    if (s2d) {  // (tap', (2 dy + dx) * 3 + c) -> weight (2a + dy - 1, 2b + dx - 1, c) of the 7x7x3 kernel
      const int qd = ci / 3, c = ci - 3 * qd;
      const int ky = 2 * (t / KT) + (qd >> 1) - 1, kx = 2 * (t % KT) + (qd & 1) - 1;
      if (qd >= 4 || ky < 0 || ky > 6 || kx < 0 || kx > 6) continue;
      col = (ky * 7 + kx) * 3 + c;
      Kr = 49 * 3;
    }
#pragma unroll
    for (int m = 0; m < MTW; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = o0 + wr * (WO / 2) + 16 * m + 4 * (lane >> 4) + r;
        if (o < Co) dtf_acc_add(gr + (long)o * Kr + col, acc[m][n][r], DTF_FX_GRAD, slot);
      }
  }
}

// ------------------------------------------------------------------------------------ s2d stem forward
#ifndef STEM_LDS_OUT
#define STEM_LDS_OUT 1
#endif
// The space-to-depth stem (4x4/1 over 2x2 blocks of the image, 16 channels, pad 2 before / 1 after, Co = 64) from
// LDS-resident row bands: a workgroup keeps the whole 64 x 256 weight tile in registers (wave w: output channels
// 16 w .. 16 w + 15, 8 k-steps of 2 taps x 16 channels), stages a band of R output rows' input halo
// [(R + 3) x (W + 3) x 16] once and reads every tap's B fragment from it; the next band's halo is prefetched into
// registers.  Each input element is fetched ~1.3x (halo) instead of 16x (the generic gather: one k-step = 2 taps).
// EPI 4: per-channel sum / sum of squares of the bf16 outputs (the v1 stem's BatchNorm) into st_out.
// work: (slot, first band, end band, -); band b = image b / (H / R), rows (b % (H / R)) * R ..
template <int W, int R, int EPI>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void convg_stem_s2d_kernel(CgArgs a) {
  constexpr int CI = 16, KT = 4, PAD = 2, CO = 64, KS = KT * KT * CI / 32;
  constexpr int NPV = R * W, NPT = (NPV + 15) / 16;  // pixels per band, 16-pixel tiles
  constexpr int CP = CI + 8, WS = W + KT - 1, RT = R + KT - 1;
  constexpr int XCH = RT * WS * (CI / 8), XJ = (XCH + 255) / 256;
  __shared__ __attribute__((aligned(16))) bf16_t sx[RT * WS * CP + 8];
  // STEM_LDS_OUT: the band's outputs are staged as [pixel][64 + 8] rows and stored as whole 128-byte pixel rows
  // (each wave's fragments are 4-channel / 8-byte pieces, 32 bytes per pixel -- partial lines)
  // rows of 64 channels (128 B), 16-byte chunk c of pixel p at chunk c ^ (p & 7): the fragment writes (8-byte pieces,
  // 16 pixels) and the row reads (8 pixels x 8 chunks per wave) spread over all banks (tools/lds_banks.py model:
  // reads 4 cycles per instruction instead of 8 with a padded 72-element row)
  constexpr int OP = CO;
  __shared__ __attribute__((aligned(16))) bf16_t so[STEM_LDS_OUT ? NPT * 16 * OP : 8];
  __shared__ dtf_acc_t acc_lds[2][CO];
  const int4 wk = a.work[blockIdx.x];
  DTF_WG_CHECK(wk.x >= 0 && wk.y >= 0 && wk.z > wk.y && a.Wi == W && a.Wo == W && a.Ci == CI && a.Co == CO &&
               a.Hi % R == 0);
  const int slot = wk.x, b0 = wk.y, b1 = wk.z;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int H = a.Hi, BPI = H / R;
  if (tid < 2 * CO) (&acc_lds[0][0])[tid] = 0;
  // weights: lane = output channel 16 wave + (lane & 15), k = 32 s + 8 (lane >> 4) .. + 7
  bf16x8_t afr[KS];
  {
    const bf16_t* wr = a.w + (long)slot * a.w_mstride + a.w_off + (long)(16 * wave + (lane & 15)) * (KS * 32);
#pragma unroll
    for (int s_ = 0; s_ < KS; ++s_)
      afr[s_] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(wr + 32 * s_ + 8 * (lane >> 4)));
  }
  // B fragment: lane = pixel (lane & 15) of the tile; k chunk (lane >> 4) = tap 2 s + (lane >> 5), channels
  // 8 ((lane >> 4) & 1) .. + 7
  int tapo[KS];
#pragma unroll
  for (int s_ = 0; s_ < KS; ++s_) {
    const int t = 2 * s_ + (lane >> 5);
    tapo[s_] = ((t / KT) * WS + t % KT) * CP + 8 * ((lane >> 4) & 1);
  }
  int xhr[XJ], xhc[XJ], xc8[XJ];
#pragma unroll
  for (int j = 0; j < XJ; ++j) {
    const int q = tid + 256 * j, hp = q / (CI / 8);
    xc8[j] = 8 * (q % (CI / 8));
    xhr[j] = q < XCH ? hp / WS : RT;
    xhc[j] = hp % WS;
  }
  uint4 xv[XJ];
  unsigned xok = 0;
  auto load = [&](int band) {
    const int img = band / BPI, y0 = (band - img * BPI) * R;
    const long xbase = (long)img * H * W * CI;
    xok = 0;
#pragma unroll
    for (int j = 0; j < XJ; ++j) {
      const int gy = y0 - PAD + xhr[j], gx = xhc[j] - PAD;
      const bool ok = xhr[j] < RT && gy >= 0 && gy < H && gx >= 0 && gx < W;
      xv[j] = ld16(a.x, xbase + ((long)gy * W + gx) * CI + xc8[j], ok);
      xok |= (unsigned)ok << j;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int j = 0; j < XJ; ++j) {
      const int off = xhr[j] < RT ? (xhr[j] * WS + xhc[j]) * CP + xc8[j] : RT * WS * CP;
      *reinterpret_cast<uint4*>(sx + off) = (xok >> j) & 1u ? xv[j] : make_uint4(0, 0, 0, 0);
    }
  };
  const int co0 = 16 * wave + 4 * (lane >> 4);
  float ss[4] = {0.f, 0.f, 0.f, 0.f}, sq[4] = {0.f, 0.f, 0.f, 0.f};
  load(b0);
  store();
  __syncthreads();
  for (int b = b0; b < b1; ++b) {
    const bool more = b + 1 < b1;
    if (more) load(b + 1);
    const int img = b / BPI, y0 = (b - img * BPI) * R;
    bf16_t* yb = a.y + (((long)img * H + y0) * W) * CO + co0;
#pragma unroll 2
    for (int n = 0; n < NPT; ++n) {
      const int p = 16 * n + (lane & 15);
      const int pc = p < NPV ? p : 0;
      const int bo = ((pc / W) * WS + pc % W) * CP;
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s_ = 0; s_ < KS; ++s_)
        acc = mfma16(afr[s_], *reinterpret_cast<const bf16x8_t*>(sx + bo + tapo[s_]), acc);
      // D: lane holds channels co0 .. co0 + 3 of pixel 16 n + (lane & 15)
      const uint32_t lo = pack2bf(acc[0], acc[1]), hi = pack2bf(acc[2], acc[3]);
      if (p < NPV) {
        if constexpr (STEM_LDS_OUT)
          *reinterpret_cast<uint2*>(so + p * OP + (((co0 >> 3) ^ (p & 7)) << 3) + (co0 & 7)) = make_uint2(lo, hi);
        else
          *reinterpret_cast<uint2*>(yb + (long)p * CO) = make_uint2(lo, hi);
        if constexpr (EPI & 4) {
          const float r[4] = {lo2f(lo), hi2f(lo), lo2f(hi), hi2f(hi)};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            ss[i] += r[i];
            sq[i] += r[i] * r[i];
          }
        }
      }
    }
    __syncthreads();
    if constexpr (STEM_LDS_OUT) {  // whole pixel rows: chunk q = tid + 256 j -> pixel q / 8, channels 8 (q % 8)
      bf16_t* yrow = a.y + (((long)img * H + y0) * W) * CO;
#pragma unroll
      for (int j = 0; j < (NPV * 8 + 255) / 256; ++j) {
        const int q = tid + 256 * j, px = q >> 3, c8 = 8 * (q & 7);
        if (px < NPV)
          *reinterpret_cast<uint4*>(yrow + (long)px * CO + c8) =
              *reinterpret_cast<const uint4*>(so + px * OP + (((q & 7) ^ (px & 7)) << 3));
      }
    }
    if (more) {
      store();
      __syncthreads();
    }
  }
  if constexpr (EPI & 4) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float s_ = ss[i], q_ = sq[i];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {  // the 16 lanes of a (lane >> 4) group hold the same 4 channels
        s_ += __shfl_xor(s_, o, 64);
        q_ += __shfl_xor(q_, o, 64);
      }
      if ((lane & 15) == 0) {
        dtf_acc_add(&acc_lds[0][co0 + i], s_, DTF_FX_STAT, slot);
        dtf_acc_add(&acc_lds[1][co0 + i], q_, DTF_FX_STAT, slot);
      }
    }
    __syncthreads();
    if (tid < CO) {
      dtf_acc_t* st = a.st_out + (long)slot * 2 * a.cmax;
      dtf_acc_addw(st + tid, acc_lds[0][tid]);
      dtf_acc_addw(st + a.cmax + tid, acc_lds[1][tid]);
    }
  }
}

}  // namespace

DTF_API int dtf_cg_args_size() { return (int)sizeof(CgArgs); }

// flags: tc (64 | 128), mode (0..2), epi (0..7), trans: bit0 transposed gather, bit1 A operand k-major from the
// forward weight layout (data gradient), bit2 BK = 64 (k depth per LDS stage; else 32), bit3 256-pixel tiles (tc 64)
DTF_API int dtf_convg_fwd(const CgArgs* a, int tc, int mode, int epi, int trans, int nwork, hipStream_t stream) {
  const int akm = (trans >> 1) & 1;
  const int bk64 = (trans >> 2) & 1;
  const int tp256 = (trans >> 3) & 1;  // 256-pixel tiles (tc = 64, BK = 32)
  const int m32 = (trans >> 4) & 1;    // 32x32x16 MFMA tiles (plain-A forward, tc = 128, 256-pixel tiles)
  if (m32 && (akm || !tp256 || tc != 128)) return -2;
  if (tp256 && bk64) return -2;
  trans &= 1;
  if (nwork <= 0) return 0;
  if ((a->Ci & (a->Ci - 1)) != 0 || a->Ci < 8 || (a->Co & 7) != 0) return -2;
  // the incremental one-tap-per-k-step gather of the dgrad (AKM / transposed) path needs Ci >= BK
  if ((akm || trans) && a->Ci < (bk64 ? 64 : 32)) return -2;
  const size_t dyn = (size_t)(mode == 0 ? 0 : (mode == 1 ? 2 : 3)) * a->Ci * sizeof(float);
  dim3 grid(nwork), block(256);
#define CG_CASE(TC_, M_, E_, T_, AK_)                                                                      \
  if (tc == TC_ && mode == M_ && epi == E_ && trans == T_ && akm == AK_) {                                 \
    if (m32)                                                                                               \
      hipLaunchKernelGGL((convg_fwd_kernel<TC_, M_, E_, T_, AK_, 32, 256, (TC_ == 128 && !AK_)>), grid, block, dyn, \
                         stream, *a);                                                                      \
    else if (tp256)                                                                                        \
      hipLaunchKernelGGL((convg_fwd_kernel<TC_, M_, E_, T_, AK_, 32, 256>), grid, block, dyn, stream, *a); \
    else if (bk64)                                                                                         \
      hipLaunchKernelGGL((convg_fwd_kernel<TC_, M_, E_, T_, AK_, 64>), grid, block, dyn, stream, *a);     \
    else                                                                                                   \
      hipLaunchKernelGGL((convg_fwd_kernel<TC_, M_, E_, T_, AK_, 32>), grid, block, dyn, stream, *a);     \
    return DTF_CHECK_LAUNCH();                                                                             \
  }
#define CG_ALL_TC(M_, E_, T_, AK_) CG_CASE(64, M_, E_, T_, AK_) CG_CASE(128, M_, E_, T_, AK_)
  // forward: identity (stem / v1) or BN+ReLU prologue; stats epilogue; optional residual
  CG_ALL_TC(0, 4, false, 0)
  CG_ALL_TC(0, 5, false, 0)
  CG_ALL_TC(0, 7, false, 0)
  CG_ALL_TC(1, 4, false, 0)
  CG_ALL_TC(1, 0, false, 0)
  CG_ALL_TC(1, 5, false, 0)
  CG_ALL_TC(1, 1, false, 0)
  CG_ALL_TC(0, 0, false, 0)
  // dgrad (A operand k-major from the forward layout): dy plain or BN-backward prologue; [+res] mask + stats
  // epilogue, or plain
  CG_ALL_TC(0, 6, false, 1)
  CG_ALL_TC(2, 6, false, 1)
  CG_ALL_TC(3, 6, false, 1)  // v2 bottleneck conv3: dy = the next block's BN1-backward apply, also stored (xout)
  CG_ALL_TC(2, 7, false, 1)
  CG_ALL_TC(0, 7, false, 1)
  CG_ALL_TC(0, 15, false, 1)  // + the compact stride-2 projection gradient (v2 bottleneck conv1 of a stage's first block)
  CG_ALL_TC(0, 0, false, 1)
  CG_ALL_TC(2, 0, false, 1)
  CG_ALL_TC(0, 3, false, 1)  // v1 bottleneck conv1: + shortcut gradient, masked by the block input's ReLU
  CG_ALL_TC(0, 6, true, 1)
  CG_ALL_TC(2, 6, true, 1)
  CG_ALL_TC(2, 7, true, 1)
  CG_ALL_TC(0, 7, true, 1)
  CG_ALL_TC(0, 0, true, 1)
  CG_ALL_TC(2, 0, true, 1)
#undef CG_ALL_TC
#undef CG_CASE
  return -1;
}

DTF_API int dtf_t3_stamp_read(void* dst, long bytes) {
#if DTF_STAMP
  if (bytes > (long)sizeof(dtf_t3_stamps)) bytes = sizeof(dtf_t3_stamps);
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(dtf_t3_stamps), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -3;
#else
  (void)dst;
  (void)bytes;
  return -1;
#endif
}

// Stride-1 3x3 conv / data gradient with LDS-resident input rows (convg_t3_kernel).  w: image width (56: 8-row
// tiles of 448 pixels, 64-channel tiles; 28: 7 rows, 14: whole 14-row images, 224-pixel tiles of 128 channels);
// epi 4 (forward, statistics) or 6 (data gradient: mask + statistics, akm = 1).
// mode 1 (forward only): BN + ReLU of the input applied while its rows are staged (c_in), the folded forward
DTF_API int dtf_convg_t3(const CgArgs* a, int tc, int epi, int akm, int w, int nwork, int mode, hipStream_t stream) {
  if (nwork <= 0) return 0;
  if (a->kh != 3 || a->kw != 3 || a->stride != 1 || a->pad != 1 || a->Wi != w || a->Hi != w || a->Ho != w ||
      a->Ci % 32 != 0 || (a->Co & 7) != 0)
    return -2;
  dim3 grid(nwork), block(256);
#define T3_CASE(TC_, E_, AK_, W_, R_, TP_, WRN_)                                                              \
  if (tc == TC_ && epi == E_ && akm == AK_ && w == W_ && mode == 0) {                                       \
    hipLaunchKernelGGL((convg_t3_kernel<TC_, E_, AK_, W_, R_, TP_, WRN_>), grid, block, 0, stream, *a);     \
    return DTF_CHECK_LAUNCH();                                                                              \
  }                                                                                                         \
  if (tc == TC_ && epi == E_ && akm == AK_ && w == W_ && mode == 1 && !AK_) {                               \
    hipLaunchKernelGGL((convg_t3_kernel<TC_, E_, AK_, W_, R_, TP_, WRN_, !AK_>), grid, block, 0, stream, *a); \
    return DTF_CHECK_LAUNCH();                                                                              \
  }
#define T3_GEO(E_, AK_) T3_CASE(64, E_, AK_, 56, 8, 448, 1) T3_CASE(128, E_, AK_, 28, 7, 224, 2) \
  T3_CASE(128, E_, AK_, 14, 14, 224, 2)
  T3_GEO(4, false)
  T3_GEO(6, true)
#undef T3_GEO
#undef T3_CASE
  return -1;
}

// mode_dy bit 2 (value 4): 64 pixels per k-step (else 32); bit 3 (value 8): 64-row tiles (Co = 64 layers)
DTF_API int dtf_convg_wgrad(const CgArgs* a, int mode_x, int mode_dy, int nwork, hipStream_t stream) {
  const int pk64 = (mode_dy >> 2) & 1, wo64 = (mode_dy >> 3) & 1;
  mode_dy &= 3;
  if (nwork <= 0) return 0;
  if ((a->Ci & (a->Ci - 1)) != 0 || a->Ci < 8 || (a->Co & 7) != 0) return -2;
  const size_t dyn = (size_t)(2 * a->Ci + 3 * a->Co) * sizeof(float);
  dim3 grid(nwork), block(256);
  const bool p1x1 = CG_WIDE_P1 && a->kh == 1 && a->kw == 1 && a->stride == 1 && a->pad == 0 && a->Hi == a->Ho &&
                    a->Wi == a->Wo && a->cin_real == a->Ci;
#define WG_CASE(MX, MD)                                                                     \
  if (mode_x == MX && mode_dy == MD) {                                                      \
    if (p1x1 && !pk64 && !wo64)                                                             \
      hipLaunchKernelGGL((convg_wgrad_kernel<MX, MD, 32, 128, true>), grid, block, dyn, stream, *a); \
    else if (pk64 && wo64)                                                                  \
      hipLaunchKernelGGL((convg_wgrad_kernel<MX, MD, 64, 64>), grid, block, dyn, stream, *a); \
    else if (pk64)                                                                          \
      hipLaunchKernelGGL((convg_wgrad_kernel<MX, MD, 64>), grid, block, dyn, stream, *a);   \
    else if (wo64)                                                                          \
      hipLaunchKernelGGL((convg_wgrad_kernel<MX, MD, 32, 64>), grid, block, dyn, stream, *a); \
    else                                                                                    \
      hipLaunchKernelGGL((convg_wgrad_kernel<MX, MD, 32>), grid, block, dyn, stream, *a);   \
    return DTF_CHECK_LAUNCH();                                                              \
  }
  WG_CASE(0, 0)
  WG_CASE(1, 0)
  WG_CASE(1, 2)
  WG_CASE(0, 2)
#undef WG_CASE
  return -1;
}

// wide-column weight gradient with plain operands (work: (slot, p0, p1, o0 | n0/8 << 16)): wo x 288 tiles for 3x3
// convs, wo x 256 for 1x1 convs with Ci % 256 == 0
// mode_x 1: x operand relu(BN(x)) applied while staging (c_in), 3x3 / 1x1 tiles only
DTF_API int dtf_convg_wgrad_wide(const CgArgs* a, int wo, int wt, int nwork, int mode_x, hipStream_t stream) {
  if (nwork <= 0) return 0;
  const int K = a->kh * a->kw * a->Ci;
  if ((a->Ci & (a->Ci - 1)) != 0 || a->Ci < 8 || (a->Co & 7) != 0) return -2;
  if (wt != 416 && ((a->Ci < 64 && a->cin_real != -3) || K % wt != 0)) return -2;  // -3: the s2d stem (16 ch)
  if (mode_x != 0 && (mode_x != 1 || wt == 416 || a->Ci > 4096)) return -2;
  const size_t dyn = mode_x ? (size_t)2 * a->Ci * sizeof(float) : 0;
  // a stride-1 1x1 conv (x pixel = dy pixel): the table-free P1 addressing (CG_WIDE_P1)
  const bool p1x1 = CG_WIDE_P1 && a->kh == 1 && a->kw == 1 && a->stride == 1 && a->pad == 0 && a->Hi == a->Ho &&
                    a->Wi == a->Wo && a->cin_real == a->Ci;
#define WW_CASE(WO_, WT_)                                                                                     \
  if (wo == WO_ && wt == WT_) {                                                                               \
    if (mode_x)                                                                                               \
      hipLaunchKernelGGL((convg_wgrad_wide_kernel<WO_, WT_, 1>), dim3(nwork), dim3(256), dyn, stream, *a);    \
    else                                                                                                      \
      hipLaunchKernelGGL((convg_wgrad_wide_kernel<WO_, WT_>), dim3(nwork), dim3(256), 0, stream, *a);         \
    return DTF_CHECK_LAUNCH();                                                                                \
  }
#define WW_CASE_P1(WO_)                                                                                           \
  if (p1x1 && wo == WO_ && wt == 256) {                                                                           \
    if (mode_x)                                                                                                   \
      hipLaunchKernelGGL((convg_wgrad_wide_kernel<WO_, 256, 1, true>), dim3(nwork), dim3(256), dyn, stream, *a);  \
    else                                                                                                          \
      hipLaunchKernelGGL((convg_wgrad_wide_kernel<WO_, 256, 0, true>), dim3(nwork), dim3(256), 0, stream, *a);    \
    return DTF_CHECK_LAUNCH();                                                                                    \
  }
  WW_CASE_P1(128) WW_CASE_P1(64)
  WW_CASE(128, 288) WW_CASE(64, 288) WW_CASE(128, 256) WW_CASE(64, 256)
#undef WW_CASE
#undef WW_CASE_P1
  if (wo == 64 && wt == 416 && mode_x == 0) {  // the 7x7 stem: 49 taps x 8 (3 real) channels in one tile
    hipLaunchKernelGGL((convg_wgrad_wide_kernel<64, 416>), dim3(nwork), dim3(256), 0, stream, *a);
    return DTF_CHECK_LAUNCH();
  }
  return -2;
}

// stride-1 3x3 weight gradient from row bands (convg_wgrad_t3_kernel): W = image width, R = rows per band
DTF_API int dtf_convg_wgrad_t3(const CgArgs* a, int W, int R, int nwork, int mode_x, hipStream_t stream) {
  if (nwork <= 0) return 0;
  const bool stem = a->cin_real == -3;  // the space-to-depth stem: 4x4 taps over 16 block channels, pad 2
  if (a->stride != 1 || a->Co % 8 || a->Wi != W || a->Hi % R ||
      (stem ? (a->kh != 4 || a->kw != 4 || a->pad != 2 || a->Ci != 16)
            : (a->kh != 3 || a->kw != 3 || a->pad != 1 || a->Ci % 32)))
    return -2;
  if (stem && W == 112 && R == 2) {
    hipLaunchKernelGGL((convg_wgrad_t3_kernel<112, 2, 4, 16, 2>), dim3(nwork), dim3(256), 0, stream, *a);
    return DTF_CHECK_LAUNCH();
  }
  if (stem) return -1;
  if (mode_x != 0 && (mode_x != 1 || stem)) return -2;
#define WT3_CASE(W_, R_)                                                                                    \
  if (W == W_ && R == R_) {                                                                                 \
    if (mode_x)                                                                                             \
      hipLaunchKernelGGL((convg_wgrad_t3_kernel<W_, R_, 3, 32, 1, 1>), dim3(nwork), dim3(256), 0, stream, *a); \
    else                                                                                                    \
      hipLaunchKernelGGL((convg_wgrad_t3_kernel<W_, R_>), dim3(nwork), dim3(256), 0, stream, *a);           \
    return DTF_CHECK_LAUNCH();                                                                              \
  }
  WT3_CASE(56, 4) WT3_CASE(28, 7) WT3_CASE(14, 14)
#undef WT3_CASE
  return -1;
}

// the space-to-depth stem forward from row bands (convg_stem_s2d_kernel): W = 112 (224 images), R = 2 rows per band
DTF_API int dtf_convg_stem_s2d(const CgArgs* a, int W, int R, int epi, int nwork, hipStream_t stream) {
  if (nwork <= 0) return 0;
  if (a->Ci != 16 || a->Co != 64 || a->kh != 4 || a->kw != 4 || a->pad != 2 || a->stride != 1 || a->Wi != W ||
      a->Wo != W || a->Hi % R)
    return -2;
  if (W == 112 && R == 2 && epi == 0) {
    hipLaunchKernelGGL((convg_stem_s2d_kernel<112, 2, 0>), dim3(nwork), dim3(256), 0, stream, *a);
    return DTF_CHECK_LAUNCH();
  }
  if (W == 112 && R == 2 && epi == 4) {
    hipLaunchKernelGGL((convg_stem_s2d_kernel<112, 2, 4>), dim3(nwork), dim3(256), 0, stream, *a);
    return DTF_CHECK_LAUNCH();
  }
  return -1;
}

DTF_DEBUG_EXPORT(convg)
DTF_POISON_EXPORT(convg)
