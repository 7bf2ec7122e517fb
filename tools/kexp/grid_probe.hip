// Item 6 probe: what a persistent 3-phase apply could save on a cache-resident grid.
//
//   which = 0: R grid barriers and nothing else, in one cooperative launch of `wgs` workgroups of
//              TB threads: the cost of one barrier.
//   which = 1: three streaming sweeps (in -> t, t -> u, u -> out; 16-byte lanes) as three launches.
//   which = 2: the same three sweeps in ONE cooperative launch with a grid barrier between them.
//   which = 3 / 4: as 0 / 2 with the two-level barrier (8 group counters, then one top counter).
//   which = 10..13: as 0 with the fences taken apart (none, acquire only, release only, both).
//   which = 14: as 2 with barrier 13 (one release fence, relaxed spin, one acquire fence).
//
// The barrier is a generation counter: one thread per workgroup adds to `count` with a vector
// global atomic; the last arriver resets it and bumps `gen`; the others spin on `gen` with
// device-coherent loads.  Everything stays in vector memory instructions.
#include <hip/hip_runtime.h>

#include <cstdint>

typedef double dv2 __attribute__((ext_vector_type(2)));

struct Bar {
  unsigned count;
  unsigned gen;
};

__device__ __forceinline__ void grid_barrier(Bar* b, unsigned nwg) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned g = __hip_atomic_load(&b->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __atomic_thread_fence(__ATOMIC_RELEASE);
    const unsigned arrived = __hip_atomic_fetch_add(&b->count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (arrived == nwg - 1) {
      __hip_atomic_store(&b->count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(&b->gen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      while (__hip_atomic_load(&b->gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) __builtin_amdgcn_s_sleep(1);
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
  }
  __syncthreads();
}

// Two-level variant: workgroups count on one of 8 group counters (blockIdx % 8, 256 bytes
// apart), the last of each group on the top counter; everyone spins on the generation word.
struct Bar2 {
  unsigned grp[8][64];
  unsigned top;
  unsigned pad[63];
  unsigned gen;
};

__device__ __forceinline__ void grid_barrier2(Bar2* b, unsigned nwg) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned g = blockIdx.x & 7;
    const unsigned gsize = nwg / 8 + (g < nwg % 8 ? 1u : 0u);
    const unsigned ng = nwg < 8 ? nwg : 8;
    const unsigned gen = __hip_atomic_load(&b->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __atomic_thread_fence(__ATOMIC_RELEASE);
    if (__hip_atomic_fetch_add(&b->grp[g][0], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gsize - 1) {
      __hip_atomic_store(&b->grp[g][0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__hip_atomic_fetch_add(&b->top, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == ng - 1) {
        __hip_atomic_store(&b->top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(&b->gen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    while (__hip_atomic_load(&b->gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == gen) __builtin_amdgcn_s_sleep(2);
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
  }
  __syncthreads();
}

// Decomposition of the barrier's cost (no data is exchanged, so correctness does not matter):
// FENCE 0 = relaxed atomics only, 1 = acquire side only (L2 invalidate), 2 = release side only
// (L2 write-back), 3 = both (as grid_barrier).
template <int FENCE>
__device__ __forceinline__ void grid_barrier_f(Bar* b, unsigned nwg) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned g = __hip_atomic_load(&b->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (FENCE & 2) __atomic_thread_fence(__ATOMIC_RELEASE);
    const unsigned arrived = __hip_atomic_fetch_add(&b->count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (arrived == nwg - 1) {
      __hip_atomic_store(&b->count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(&b->gen, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      while (__hip_atomic_load(&b->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) __builtin_amdgcn_s_sleep(1);
    }
    if (FENCE & 1) __atomic_thread_fence(__ATOMIC_ACQUIRE);
  }
  __syncthreads();
}

template <int TB, int FENCE>
__global__ void __launch_bounds__(TB) k_barriers_f(Bar* b, int rounds) {
  for (int r = 0; r < rounds; ++r) grid_barrier_f<FENCE>(b, gridDim.x);
}

template <int TB>
__global__ void __launch_bounds__(TB) k_barriers2(Bar2* b, int rounds) {
  for (int r = 0; r < rounds; ++r) grid_barrier2(b, gridDim.x);
}

template <int TB>
__global__ void __launch_bounds__(TB) k_barriers(Bar* b, int rounds) {
  for (int r = 0; r < rounds; ++r) grid_barrier(b, gridDim.x);
}

template <int TB>
__device__ __forceinline__ void sweep(const dv2* __restrict__ in, dv2* __restrict__ out, long n) {
  const long stride = (long)gridDim.x * TB;
  for (long i = (long)blockIdx.x * TB + threadIdx.x; i < n; i += stride) out[i] = in[i];
}

template <int TB>
__global__ void __launch_bounds__(TB) k_sweep(const dv2* __restrict__ in, dv2* __restrict__ out, long n) {
  sweep<TB>(in, out, n);
}

template <int TB>
__global__ void __launch_bounds__(TB) k_three(const dv2* in, dv2* t, dv2* u, dv2* out, long n, Bar* b) {
  sweep<TB>(in, t, n);
  grid_barrier(b, gridDim.x);
  sweep<TB>(t, u, n);
  grid_barrier(b, gridDim.x);
  sweep<TB>(u, out, n);
}

template <int TB>
__global__ void __launch_bounds__(TB) k_three2(const dv2* in, dv2* t, dv2* u, dv2* out, long n, Bar2* b) {
  sweep<TB>(in, t, n);
  grid_barrier2(b, gridDim.x);
  sweep<TB>(t, u, n);
  grid_barrier2(b, gridDim.x);
  sweep<TB>(u, out, n);
}

template <int TB>
__global__ void __launch_bounds__(TB) k_three_f(const dv2* in, dv2* t, dv2* u, dv2* out, long n, Bar* b) {
  sweep<TB>(in, t, n);
  grid_barrier_f<3>(b, gridDim.x);
  sweep<TB>(t, u, n);
  grid_barrier_f<3>(b, gridDim.x);
  sweep<TB>(u, out, n);
}

template <int TB>
static int run(int which, int wgs, int rounds, const dv2* in, dv2* t, dv2* u, dv2* out, long n, int iters,
               float* ms) {
  Bar* b = nullptr;
  if (hipMalloc(&b, sizeof(Bar2)) != hipSuccess) return 1;
  hipMemset(b, 0, sizeof(Bar2));
  Bar2* b2 = (Bar2*)b;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto once = [&]() -> hipError_t {
    if (which == 0) {
      void* args[] = {&b, &rounds};
      return hipLaunchCooperativeKernel((const void*)k_barriers<TB>, dim3(wgs), dim3(TB), args, 0, 0);
    }
    if (which >= 10 && which <= 13) {
      void* args[] = {&b, &rounds};
      const void* f = which == 10 ? (const void*)k_barriers_f<TB, 0>
                    : which == 11 ? (const void*)k_barriers_f<TB, 1>
                    : which == 12 ? (const void*)k_barriers_f<TB, 2> : (const void*)k_barriers_f<TB, 3>;
      return hipLaunchCooperativeKernel(f, dim3(wgs), dim3(TB), args, 0, 0);
    }
    if (which == 14) {
      void* args[] = {&in, &t, &u, &out, &n, &b};
      return hipLaunchCooperativeKernel((const void*)k_three_f<TB>, dim3(wgs), dim3(TB), args, 0, 0);
    }
    if (which == 3) {
      void* args[] = {&b2, &rounds};
      return hipLaunchCooperativeKernel((const void*)k_barriers2<TB>, dim3(wgs), dim3(TB), args, 0, 0);
    }
    if (which == 4) {
      void* args[] = {&in, &t, &u, &out, &n, &b2};
      return hipLaunchCooperativeKernel((const void*)k_three2<TB>, dim3(wgs), dim3(TB), args, 0, 0);
    }
    if (which == 1) {
      hipLaunchKernelGGL(k_sweep<TB>, dim3(wgs), dim3(TB), 0, 0, in, t, n);
      hipLaunchKernelGGL(k_sweep<TB>, dim3(wgs), dim3(TB), 0, 0, (const dv2*)t, u, n);
      hipLaunchKernelGGL(k_sweep<TB>, dim3(wgs), dim3(TB), 0, 0, (const dv2*)u, out, n);
      return hipGetLastError();
    }
    void* args[] = {&in, &t, &u, &out, &n, &b};
    return hipLaunchCooperativeKernel((const void*)k_three<TB>, dim3(wgs), dim3(TB), args, 0, 0);
  };
  for (int i = 0; i < 20; ++i)
    if (once() != hipSuccess) return 2;
  hipEventRecord(e0, 0);
  for (int i = 0; i < iters; ++i) once();
  hipEventRecord(e1, 0);
  if (hipEventSynchronize(e1) != hipSuccess) return 3;
  hipEventElapsedTime(ms, e0, e1);
  *ms /= iters;
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  hipFree(b);
  return hipGetLastError() == hipSuccess ? 0 : 4;
}

extern "C" int grid_probe(int which, int tb, int wgs, int rounds, const void* in, void* t, void* u, void* out, long n,
                          int iters, float* ms) {
  const dv2* a = (const dv2*)in;
  if (tb == 256) return run<256>(which, wgs, rounds, a, (dv2*)t, (dv2*)u, (dv2*)out, n, iters, ms);
  if (tb == 1024) return run<1024>(which, wgs, rounds, a, (dv2*)t, (dv2*)u, (dv2*)out, n, iters, ms);
  return 9;
}

// the largest cooperative grid: workgroups per CU the occupancy calculator allows for TB threads
extern "C" int grid_probe_max_wgs(int which, int tb, int* per_cu) {
  const void* f = which == 0 ? (tb == 256 ? (const void*)k_barriers<256> : (const void*)k_barriers<1024>)
                             : (tb == 256 ? (const void*)k_three<256> : (const void*)k_three<1024>);
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, f, tb, 0) == hipSuccess ? 0 : 1;
}
