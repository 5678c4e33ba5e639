// Per-launch floor of a dependent kernel chain replayed from a hipGraph (diagnostic, tools/gpu_chain_floor.sh).
//
// The ResNet step at one member per GPU is ~130 dependent launches of 256 workgroups; this measures what a launch
// costs before any convolution arithmetic: an empty launch, a large kernarg struct, a 16-B-per-thread read of the
// previous launch's output + write, the BatchNorm-statistics pattern (every workgroup reads the same replicated
// accumulators first, adds its partial sums atomically at the end), and a 4x larger payload.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/chain_floor tools/chain_floor.hip && /tmp/chain_floor
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

struct Big {  // the size of the conv kernels' ConvArgs (~0.4 KB)
  const uint4* in;
  uint4* out;
  float* st;
  const float* st_in;
  long pad[44];
  int per_thread;
  int mode;
};

__global__ __launch_bounds__(256) void k_empty(int) {}

__global__ __launch_bounds__(256) void k_bigarg(Big a) {
  long s = 0;
#pragma unroll
  for (int i = 0; i < 44; ++i) s += a.pad[i];
  if (s == 12345 && threadIdx.x == 0) a.out[0] = make_uint4(1, 1, 1, 1);
}

// mode bit0: read stats first (coefficients), bit1: atomically add partial stats at the end; PT 16-B chunks per thread
__device__ unsigned long long g_st[128][1024][2];  // per launch ordinal, per workgroup: start, end (plain stores)

template <int PT>
__device__ void body(const Big& a, float* coef, float* acc, int t);

template <int PT>
__global__ __launch_bounds__(256) void k_chain(Big a) {
  __shared__ float coef[128];
  __shared__ float acc[128];
  const int t = threadIdx.x;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (a.mode & 4) {  // loads only
    const uint4 v = a.in[(long)blockIdx.x * 256 + t];
    if (v.x == 0x12345678u) a.out[0] = v;
  } else if (a.mode & 8) {  // stores only
    a.out[(long)blockIdx.x * 256 + t] = make_uint4(t, 0, 0, 0);
  } else {
    body<PT>(a, coef, acc, t);
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (t == 0) {
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    g_st[a.pad[0] & 127][blockIdx.x & 1023][0] = t0;
    g_st[a.pad[0] & 127][blockIdx.x & 1023][1] = t1;
  }
}

template <int PT>
__device__ void body(const Big& a, float* coef, float* acc, int t) {
  if (a.mode & 1) {
    if (t < 128) {
      float s = 0.f;
#pragma unroll
      for (int r = 0; r < 8; ++r) s += a.st_in[r * 128 + t];
      coef[t] = s * 1e-9f + 1.f;
    }
  } else if (t < 128) {
    coef[t] = 1.f;
  }
  if (t < 128) acc[t] = 0.f;
  uint4 v[PT];
  const long base = ((long)blockIdx.x * 256 + t) * PT;
#pragma unroll
  for (int i = 0; i < PT; ++i) v[i] = a.in[base + i];
  __syncthreads();
  float part = 0.f;
#pragma unroll
  for (int i = 0; i < PT; ++i) {
      uint4 w = v[i];
      w.x = __float_as_uint(__uint_as_float(w.x) * coef[t & 127]);
      part += __uint_as_float(w.x);
      a.out[base + i] = w;
    }
  if (a.mode & 2) {
    atomicAdd(&acc[t & 127], part);
    __syncthreads();
    if (t < 128) atomicAdd(&a.st[(blockIdx.x & 7) * 128 + t], acc[t]);
  }
}

int main() {
  const int NK = 128, REPS = 200, NWG = 256;
  uint4 *b0, *b1;
  float *st0, *st1;
  CHECK(hipMalloc(&b0, 64 << 20));
  CHECK(hipMalloc(&b1, 64 << 20));
  CHECK(hipMalloc(&st0, 1 << 20));
  CHECK(hipMalloc(&st1, 1 << 20));
  CHECK(hipMemset(b0, 0, 64 << 20));
  CHECK(hipMemset(b1, 0, 64 << 20));
  CHECK(hipMemset(st0, 0, 1 << 20));
  CHECK(hipMemset(st1, 0, 1 << 20));
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  const char* names[] = {"empty (tiny kernarg)", "empty, 0.4 KB kernarg read", "1 MB read+write",
                         "1 MB + BN stats read", "1 MB + stats read + atomic flush", "4 MB + stats + atomics",
                         "1 WG/CU x 4: 1024 WG, 1 MB + stats + atomics", "1 MB loads only", "1 MB stores only",
                         "1 MB read+write, eager launches (no graph)"};
  for (int variant = 0; variant < 10; ++variant) {
    const bool eager = variant == 9;
    auto enqueue = [&]() {
      for (int k = 0; k < NK; ++k) {
        Big a = {};
        a.in = (k & 1) ? b1 : b0;
        a.out = (k & 1) ? b0 : b1;
        a.st = (k & 1) ? st0 : st1;
        a.st_in = (k & 1) ? st1 : st0;
        a.per_thread = 1;
        a.pad[0] = k;
        int nwg = NWG;
        switch (variant) {
          case 0: k_empty<<<NWG, 256, 0, s>>>(k); continue;
          case 1: k_bigarg<<<NWG, 256, 0, s>>>(a); continue;
          case 2: a.mode = 0; break;
          case 3: a.mode = 1; break;
          case 4: a.mode = 3; break;
          case 5: a.mode = 3; a.per_thread = 4; break;
          case 6: a.mode = 3; nwg = 4 * NWG; break;
          case 7: a.mode = 4; break;
          case 8: a.mode = 8; break;
          case 9: a.mode = 0; break;
        }
        if (a.per_thread == 4)
          k_chain<4><<<nwg, 256, 0, s>>>(a);
        else
          k_chain<1><<<nwg, 256, 0, s>>>(a);
      }
    };
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    if (!eager) {
      CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
      enqueue();
      CHECK(hipStreamEndCapture(s, &g));
      CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    }
    auto run = [&]() {
      if (eager)
        enqueue();
      else
        CHECK(hipGraphLaunch(ge, s));
    };
    for (int w = 0; w < 300; ++w) run();  // >= 0.5 s: clocks ramped up
    CHECK(hipStreamSynchronize(s));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipEventRecord(e0, s));
    for (int r = 0; r < REPS; ++r) run();
    CHECK(hipEventRecord(e1, s));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-48s %6.2f us/launch", names[variant], 1000.f * ms / (REPS * NK));
    if (variant >= 2) {  // one more run with stamps: kernel execution span vs launch gap, mean workgroup duration
      static unsigned long long st[128][1024][2];
      run();
      CHECK(hipStreamSynchronize(s));
      CHECK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_st), sizeof(st)));
      const int nwg = variant == 6 ? 1024 : 256;
      double busy = 0, gap = 0, wgd = 0;
      unsigned long long prev_end = 0;
      for (int k = 0; k < NK; ++k) {
        unsigned long long mn = ~0ull, mx = 0;
        double d = 0;
        for (int b = 0; b < nwg; ++b) {
          mn = st[k][b][0] < mn ? st[k][b][0] : mn;
          mx = st[k][b][1] > mx ? st[k][b][1] : mx;
          d += (st[k][b][1] - st[k][b][0]) * 0.01;
        }
        busy += (mx - mn) * 0.01;
        wgd += d / nwg;
        if (k) gap += ((double)mn - (double)prev_end) * 0.01;
        prev_end = mx;
      }
      printf("   span %.2f us (mean WG %.2f us), end->next start %.2f us", busy / NK, wgd / NK, gap / (NK - 1));
      if (variant == 2) {  // start offsets of launch 64's workgroups, by blockIdx % 8
        unsigned long long mn = ~0ull;
        for (int b = 0; b < nwg; ++b) mn = st[64][b][0] < mn ? st[64][b][0] : mn;
        printf("\n   launch 64 start offsets (us) by blockIdx%%8:");
        for (int x = 0; x < 8; ++x) {
          printf("\n     x%d:", x);
          for (int b = x; b < nwg; b += 8) printf(" %.1f", (st[64][b][0] - mn) * 0.01);
        }
      }
    }
    printf("\n");
    if (!eager) {
      CHECK(hipGraphExecDestroy(ge));
      CHECK(hipGraphDestroy(g));
    }
  }
  return 0;
}
