// Grouped bf16 GEMM with fp32 accumulation on v_mfma_f32_16x16x32_bf16 (gfx950).
//
// One launch runs a list of independent GEMMs ("groups", one per population member: each member has its
// own weights and its own row count) -- C_g = A_g . B_g with
//   A_g : M x K, stored row-major [M][K] (A_KM = 0) or K-major [K][M] (A_KM = 1)
//   B_g : K x N, stored [N][K] (B_KM = 0, i.e. the "NT" weight layout) or K-major [K][N] (B_KM = 1)
//   C_g : [M][N] row-major; OUT 0 = fp32 store, 1 = bf16 store, 2 = fp32 accumulate (C += AB)
// Work item = (group, m0, n0): a 64x64 C tile, 4 waves in 2x2, each wave 32x32 = 2x2 MFMA tiles.
// K-steps of 32 are double buffered: the next step's global loads are issued into registers before the
// current step's MFMAs, then written to the other LDS buffer.
//   [rows][K] operands -> LDS [64][32+8]  (ds_read_b128 fragments, 16-byte pad per row)
//   [K][rows] operands -> LDS [32][64+8]  (k = row fragments via ds_read_b64_tr_b16)
// Requirements (checked by the host wrapper): ld* % 8 == 0; K % 32 == 0 for non-K-major operands;
// M (N) % 8 == 0 where the operand is K-major.  Out-of-range rows / k are zero-filled.
#include "common.h"

namespace {

typedef short s16x4_t __attribute__((ext_vector_type(4)));

struct GemmGroup {
  long a_off, b_off, c_off;
  int M, N, K, Ms;  // Ms > 0: store only rows < Ms (operands may be padded past the real row count)
};

struct GemmArgs {
  const bf16_t* A;
  const bf16_t* B;
  void* C;
  long lda, ldb, ldc;
  const GemmGroup* groups;
  const int4* work;  // (group, m0, n0, 0)
};

__device__ __forceinline__ f32x4_t mfma16(const bf16x8_t& a, const bf16x8_t& b, const f32x4_t& c) {
  return dtf_mfma16(a, b, c);
}

__device__ __forceinline__ s16x4_t ds_read_tr(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(p));
}

constexpr int RP = 40;  // [rows][K] tile pitch
constexpr int KP = 72;  // [K][rows] tile pitch
constexpr int TILE_ELEMS = 64 * RP > 32 * KP ? 64 * RP : 32 * KP;  // 2560

// Global -> register stage of one 64-row x 32-k operand tile (one uint4 per thread).
template <bool KM>
__device__ __forceinline__ uint4 load_tile(const bf16_t* base, long ld, int r0, int rows, int k0, int K, int tid) {
  if constexpr (!KM) {
    const int r = tid >> 2, c = tid & 3;
    if (r0 + r < rows) return *reinterpret_cast<const uint4*>(base + (long)(r0 + r) * ld + k0 + 8 * c);
  } else {
    const int k = tid >> 3, c = tid & 7;
    if (k0 + k < K && r0 + 8 * c < rows) return *reinterpret_cast<const uint4*>(base + (long)(k0 + k) * ld + r0 + 8 * c);
  }
  return make_uint4(0, 0, 0, 0);
}

template <bool KM>
__device__ __forceinline__ void store_tile(bf16_t* lds, uint4 v, int tid) {
  if constexpr (!KM) {
    *reinterpret_cast<uint4*>(lds + (tid >> 2) * RP + 8 * (tid & 3)) = v;
  } else {
    *reinterpret_cast<uint4*>(lds + (tid >> 3) * KP + 8 * (tid & 7)) = v;
  }
}

// MFMA operand fragment for rows rb..rb+15 (lane row = lane & 15, k = 8*(lane>>4)..+7).
template <bool KM>
__device__ __forceinline__ bf16x8_t frag(const bf16_t* lds, int rb, int lane) {
  if constexpr (!KM) {
    return *reinterpret_cast<const bf16x8_t*>(lds + (rb + (lane & 15)) * RP + 8 * (lane >> 4));
  } else {
    const int g = lane >> 4, q = (lane & 15) >> 2, p4 = lane & 3;
    const s16x4_t lo = ds_read_tr(lds + (8 * g + q) * KP + rb + 4 * p4);
    const s16x4_t hi = ds_read_tr(lds + (8 * g + 4 + q) * KP + rb + 4 * p4);
    return (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  }
}

template <bool A_KM, bool B_KM, int OUT>
__global__ __launch_bounds__(256) void gemm_bf16_kernel(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t sa[2][TILE_ELEMS];
  __shared__ __attribute__((aligned(16))) bf16_t sb[2][TILE_ELEMS];
  const int4 wk = a.work[blockIdx.x];
  DTF_WG_CHECK(wk.x >= 0 && wk.y >= 0 && wk.z >= 0);
  const GemmGroup gp = a.groups[wk.x];
  const int m0 = wk.y, n0 = wk.z;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave & 1, wn = wave >> 1;
  const bf16_t* A = a.A + gp.a_off;
  const bf16_t* B = a.B + gp.b_off;
  const int nk = (gp.K + 31) / 32;
  f32x4_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jn = 0; jn < 2; ++jn) acc[i][jn] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  uint4 ra = load_tile<A_KM>(A, a.lda, m0, gp.M, 0, gp.K, tid);
  uint4 rb = load_tile<B_KM>(B, a.ldb, n0, gp.N, 0, gp.K, tid);
  store_tile<A_KM>(sa[0], ra, tid);
  store_tile<B_KM>(sb[0], rb, tid);
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    const int cur = ks & 1;
    if (ks + 1 < nk) {
      ra = load_tile<A_KM>(A, a.lda, m0, gp.M, 32 * (ks + 1), gp.K, tid);
      rb = load_tile<B_KM>(B, a.ldb, n0, gp.N, 32 * (ks + 1), gp.K, tid);
    }
    bf16x8_t fa[2], fb[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) fa[i] = frag<A_KM>(sa[cur], 32 * wm + 16 * i, lane);
#pragma unroll
    for (int jn = 0; jn < 2; ++jn) fb[jn] = frag<B_KM>(sb[cur], 32 * wn + 16 * jn, lane);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jn = 0; jn < 2; ++jn) acc[i][jn] = mfma16(fa[i], fb[jn], acc[i][jn]);
    if (ks + 1 < nk) {
      store_tile<A_KM>(sa[cur ^ 1], ra, tid);
      store_tile<B_KM>(sb[cur ^ 1], rb, tid);
    }
    __syncthreads();
  }
  // D fragment: lane holds column n = lane & 15, rows m = 4*(lane>>4) + r
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jn = 0; jn < 2; ++jn) {
      const int n = n0 + 32 * wn + 16 * jn + (lane & 15);
      if (n >= gp.N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + 32 * wm + 16 * i + 4 * (lane >> 4) + r;
        if (m >= (gp.Ms > 0 ? gp.Ms : gp.M)) continue;
        const long o = gp.c_off + (long)m * a.ldc + n;
        if constexpr (OUT == 0) {
          reinterpret_cast<float*>(a.C)[o] = acc[i][jn][r];
        } else if constexpr (OUT == 1) {
          reinterpret_cast<bf16_t*>(a.C)[o] = f2bf(acc[i][jn][r]);
        } else {
          reinterpret_cast<float*>(a.C)[o] += acc[i][jn][r];
        }
      }
    }
}

}  // namespace

DTF_API int dtf_gemm_args_size() { return (int)sizeof(GemmArgs); }
DTF_API int dtf_gemm_group_size() { return (int)sizeof(GemmGroup); }

// mode = A_KM | (B_KM << 1) | (OUT << 2)
DTF_API int dtf_gemm_bf16(const GemmArgs* a, int mode, int nwork, hipStream_t stream) {
  if (nwork <= 0) return 0;
  dim3 grid(nwork), block(256);
#define DTF_GEMM_CASE(AK, BK, O)                                                     \
  case (AK) | ((BK) << 1) | ((O) << 2):                                              \
    hipLaunchKernelGGL((gemm_bf16_kernel<AK, BK, O>), grid, block, 0, stream, *a);   \
    break;
  switch (mode) {
    DTF_GEMM_CASE(0, 0, 0)
    DTF_GEMM_CASE(0, 0, 1)
    DTF_GEMM_CASE(0, 0, 2)
    DTF_GEMM_CASE(0, 1, 0)
    DTF_GEMM_CASE(0, 1, 1)
    DTF_GEMM_CASE(0, 1, 2)
    DTF_GEMM_CASE(1, 1, 0)
    DTF_GEMM_CASE(1, 1, 1)
    DTF_GEMM_CASE(1, 1, 2)
    DTF_GEMM_CASE(1, 0, 0)
    DTF_GEMM_CASE(1, 0, 1)
    DTF_GEMM_CASE(1, 0, 2)
    default:
      return -1;
  }
#undef DTF_GEMM_CASE
  return DTF_CHECK_LAUNCH();
}

DTF_DEBUG_EXPORT(gemm)
