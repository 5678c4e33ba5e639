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
  unsigned* ticket;     // last-arriver finalize: arrival counter of this launch's statistics
  float* coef_out;      // ... the finalized coefficients it writes
  const float* coef_in; // ... the coefficients the previous launch finalized
  long pad[41];
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
  if (a.mode & 32) {  // coefficients finalized by the previous launch's last arriver: one load per channel
    if (t < 128) coef[t] = __hip_atomic_load(a.coef_in + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1.f;
  } else if (a.mode & 1) {
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
  if (a.mode & 16) {  // producer-side finalize: the last-arriving workgroup sums the replicas into coefficients
    __shared__ int last;
    __syncthreads();  // every wave's statistic atomics are issued
    if (t == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      const unsigned tk = atomicAdd(a.ticket, 1u);  // returning: the arrival order
      last = tk == gridDim.x - 1;
    }
    __syncthreads();
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      if (t < 128) {
        float s = 0.f;
#pragma unroll
        for (int r = 0; r < 8; ++r) s += __hip_atomic_load(a.st + r * 128 + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(a.coef_out + t, s * 1e-12f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (t == 0) __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Persistent variant: NPH phases of the "1 MB + stats read + atomic flush" body in ONE launch of nwg workgroups (one
// per CU), separated by a software grid barrier instead of a kernel boundary.  xcd = 0: one flat arrival counter;
// xcd = 1: hierarchical (per-XCC counter, the XCC's last arriver then arrives at the top counter).  Spins are bounded
// (a broken barrier ends the kernel instead of hanging the GPU; *fail counts such exits).
__device__ unsigned long long g_ph[2][1024];  // phase 0 start / last phase end per workgroup
__device__ __forceinline__ bool spin_until_changed(unsigned* gen, unsigned g) {
  for (long it = 0; it < (1L << 16); ++it) {  // ~0.1 s: far above any real barrier wait
    if (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != g) return true;
    __builtin_amdgcn_s_sleep(1);
  }
  return false;
}

__device__ bool grid_barrier(unsigned* bar, int nwg, int xcd, unsigned* fail) {
  // bar: [0] top counter, [1] generation, [2..9] per-XCC counters; XCC of this workgroup from the hardware register
  __shared__ int ok;
  __syncthreads();
  if (threadIdx.x == 0) {
    ok = 1;
    const unsigned g = __hip_atomic_load(bar + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bool top = true;
    if (xcd) {
      const int xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11)) & 7;  // HW_REG_XCC_ID bits 0..2
      const unsigned per = nwg / 8;
      const unsigned tk = atomicAdd(bar + 2 + xcc, 1u);
      top = tk == per - 1;
      if (top) __hip_atomic_store(bar + 2 + xcc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (top) {
      const unsigned want = xcd ? 8u : (unsigned)nwg;
      const unsigned tk = atomicAdd(bar, 1u);
      if (tk == want - 1) {
        __hip_atomic_store(bar, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(bar + 1, g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else if (!spin_until_changed(bar + 1, g)) {
        ok = 0;
      }
    } else if (!spin_until_changed(bar + 1, g)) {
      ok = 0;
    }
    if (!ok) atomicAdd(fail, 1u);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
  return ok;
}

__global__ __launch_bounds__(256) void k_persist(Big a, int nph, int xcd, unsigned* bar, unsigned* fail,
                                                 const uint4* b0, uint4* b1, float* s0, float* s1) {
  __shared__ float coef[128];
  __shared__ float acc[128];
  const int t = threadIdx.x;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int k = 0; k < nph; ++k) {
    Big p = a;
    p.in = (k & 1) ? reinterpret_cast<const uint4*>(b1) : b0;
    p.out = (k & 1) ? const_cast<uint4*>(b0) : b1;
    p.st = (k & 1) ? s0 : s1;
    p.st_in = (k & 1) ? s1 : s0;
    body<1>(p, coef, acc, t);
    __builtin_amdgcn_s_waitcnt(0);
    if (!grid_barrier(bar, gridDim.x, xcd, fail)) break;  // a broken barrier ends the kernel (bounded)
  }
  if (t == 0) {
    g_ph[0][blockIdx.x & 1023] = t0;
    g_ph[1][blockIdx.x & 1023] = __builtin_amdgcn_s_memrealtime();
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
  unsigned *ticket, *bar, *fail;
  float *coef0, *coef1;
  CHECK(hipMalloc(&ticket, 4096));
  CHECK(hipMalloc(&bar, 4096));
  CHECK(hipMalloc(&fail, 4096));
  CHECK(hipMalloc(&coef0, 4096));
  CHECK(hipMalloc(&coef1, 4096));
  CHECK(hipMemset(ticket, 0, 4096));
  CHECK(hipMemset(bar, 0, 4096));
  CHECK(hipMemset(fail, 0, 4096));
  CHECK(hipMemset(coef0, 0, 4096));
  CHECK(hipMemset(coef1, 0, 4096));
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  const char* names[] = {"empty (tiny kernarg)", "empty, 0.4 KB kernarg read", "1 MB read+write",
                         "1 MB + BN stats read", "1 MB + stats read + atomic flush", "4 MB + stats + atomics",
                         "1 WG/CU x 4: 1024 WG, 1 MB + stats + atomics", "1 MB loads only", "1 MB stores only",
                         "1 MB read+write, eager launches (no graph)",
                         "1 MB + atomics + last-arriver finalize (ticket)",
                         "persistent: flat grid barrier per phase",
                         "persistent: XCD-hierarchical barrier per phase"};
  for (int variant = 0; variant < 13; ++variant) {
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
        a.ticket = ticket + (k & 1) * 64;
        a.coef_out = (k & 1) ? coef1 : coef0;
        a.coef_in = (k & 1) ? coef0 : coef1;
        int nwg = NWG;
        if (variant >= 11) {  // one persistent launch holds all NK phases
          if (k == 0) {
            a.mode = 3;
            k_persist<<<NWG, 256, 0, s>>>(a, NK, variant == 12, bar, fail, b0, b1, st0, st1);
          }
          continue;
        }
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
          case 10: a.mode = 2 | 16 | 32; break;
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
    if (variant >= 11) {  // one checked run first: a persistent kernel with a broken barrier must not be replayed
      run();
      CHECK(hipStreamSynchronize(s));
      unsigned nf = 0;
      CHECK(hipMemcpy(&nf, fail, 4, hipMemcpyDeviceToHost));
      if (nf) {
        printf("%-48s barrier timeouts on the first run (%u): stopping\n", names[variant], nf);
        return 2;
      }
    }
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
    if (variant >= 11) {
      unsigned nf = 0;
      CHECK(hipMemcpy(&nf, fail, 4, hipMemcpyDeviceToHost));
      printf("   (per phase; barrier timeouts: %u)\n", nf);
      if (nf) return 2;  // a broken barrier: stop here
      continue;
    }
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
