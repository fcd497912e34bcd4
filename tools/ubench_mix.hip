// Mixed read + write streaming ceilings, round 3 (diagnostic, not part of the library).  Which plain kernel
// shape moves the most HBM bytes when it reads its input once and writes W output bytes per input byte, the
// newline index's mix (uint16 index: VCF W ~0.025, CSV W ~0.056; uint32 / uint64 forms 0.05-0.22)?
//   A  the library's dp_stream_rw today: per 16 KiB wave range, 16 loads, then that range's stores
//   B  the same, software-pipelined: two 8 KiB buffers, the next buffer's loads issued before the stores
//   C  writes batched per workgroup: every wave reads its range as in B; one 16-range step's output (the
//      workgroup's 16 ranges) goes out as one contiguous run, all 16 waves storing it together after a
//      workgroup barrier (the scan's output of one unit is one contiguous run too)
//   D  like C, with the run's stores issued before the next step's loads are waited on
//   E  like D, storing every 4th step the last 4 steps' runs (bigger write bursts)
//   F  like D, storing the previous step's run (writes one step behind the reads)
// Total (read + write) bytes / kernel time, best of `reps`, HIP events.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_mix tools/ubench_mix.hip && ./tools/ubench_mix [GiB]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

constexpr int kRange = 16384;
constexpr int kRows = kRange / 1024;
constexpr int kHalf = kRows / 2;

__device__ __forceinline__ uint4 ld(const uint4* p) {
  uint4 v;
  v.x = __builtin_nontemporal_load(&p->x);
  v.y = __builtin_nontemporal_load(&p->y);
  v.z = __builtin_nontemporal_load(&p->z);
  v.w = __builtin_nontemporal_load(&p->w);
  return v;
}
__device__ __forceinline__ void st(uint4* p, uint4 v) {
  __builtin_nontemporal_store(v.x, &p->x);
  __builtin_nontemporal_store(v.y, &p->y);
  __builtin_nontemporal_store(v.z, &p->z);
  __builtin_nontemporal_store(v.w, &p->w);
}
// 16-byte output elements of range r: [e(r), e(r + 1)), e(r) = r * wq16 / 65536 (wq16 = W * 65536 * 1024)
__device__ __forceinline__ uint64_t e_of(uint64_t r, uint64_t wq16) { return (r * wq16) >> 16; }

template <int V>
__global__ void __launch_bounds__(1024) mix_kernel(const uint4* __restrict__ in, uint64_t nranges,
                                                   uint4* __restrict__ out, uint64_t wq16, unsigned* sink) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  uint32_t acc = 0;
  if constexpr (V == 0) {
    const uint64_t nwaves = (uint64_t)gridDim.x * 16;
    for (uint64_t r = (uint64_t)blockIdx.x * 16 + wave; r < nranges; r += nwaves) {
      const uint4* p = in + r * (kRange / 16) + lane;
      uint4 v[kRows];
#pragma unroll
      for (int i = 0; i < kRows; ++i) v[i] = ld(p + i * 64);
      uint32_t x = 0;
#pragma unroll
      for (int i = 0; i < kRows; ++i) x ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
      acc ^= x;
      if (out)
        for (uint64_t e = e_of(r, wq16) + lane; e < e_of(r + 1, wq16); e += 64) st(out + e, uint4{x, (uint32_t)e, (uint32_t)r, acc});
    }
  } else if constexpr (V == 1) {
    const uint64_t nwaves = (uint64_t)gridDim.x * 16;
    uint64_t r = (uint64_t)blockIdx.x * 16 + wave;
    if (r >= nranges) return;
    uint4 a[kHalf], b[kHalf];
    const uint4* p = in + r * (kRange / 16) + lane;
#pragma unroll
    for (int i = 0; i < kHalf; ++i) a[i] = ld(p + i * 64);
#pragma unroll
    for (int i = 0; i < kHalf; ++i) b[i] = ld(p + (kHalf + i) * 64);
    for (;;) {
      const uint64_t rn = r + nwaves;
      const uint4* pn = in + (rn < nranges ? rn : r) * (kRange / 16) + lane;
      uint32_t x = 0;
#pragma unroll
      for (int i = 0; i < kHalf; ++i) x ^= a[i].x ^ a[i].y ^ a[i].z ^ a[i].w;
#pragma unroll
      for (int i = 0; i < kHalf; ++i) a[i] = ld(pn + i * 64);
#pragma unroll
      for (int i = 0; i < kHalf; ++i) x ^= b[i].x ^ b[i].y ^ b[i].z ^ b[i].w;
      acc ^= x;
      if (out)
        for (uint64_t e = e_of(r, wq16) + lane; e < e_of(r + 1, wq16); e += 64) st(out + e, uint4{x, (uint32_t)e, (uint32_t)r, acc});
#pragma unroll
      for (int i = 0; i < kHalf; ++i) b[i] = ld(pn + (kHalf + i) * 64);
      if (rn >= nranges) break;
      r = rn;
    }
#pragma unroll
    for (int i = 0; i < kHalf; ++i) acc ^= a[i].x ^ b[i].y;
  } else {
    // groups of 16 consecutive ranges per workgroup step; group g = blockIdx.x + k * gridDim.x
    const uint64_t ngroups = (nranges + 15) / 16;
    uint64_t g = blockIdx.x;
    if (g >= ngroups) return;
    uint64_t r = g * 16 + wave;
    uint4 a[kHalf], b[kHalf];
    const uint4* p = in + (r < nranges ? r : 0) * (kRange / 16) + lane;
#pragma unroll
    for (int i = 0; i < kHalf; ++i) a[i] = ld(p + i * 64);
#pragma unroll
    for (int i = 0; i < kHalf; ++i) b[i] = ld(p + (kHalf + i) * 64);
    __shared__ uint32_t s_x[16];
    for (;;) {
      const uint64_t gn = g + gridDim.x;
      const uint64_t rn = gn * 16 + wave;
      const uint4* pn = in + (rn < nranges ? rn : (r < nranges ? r : 0)) * (kRange / 16) + lane;
      uint32_t x = 0;
#pragma unroll
      for (int i = 0; i < kHalf; ++i) x ^= a[i].x ^ a[i].y ^ a[i].z ^ a[i].w;
#pragma unroll
      for (int i = 0; i < kHalf; ++i) a[i] = ld(pn + i * 64);
#pragma unroll
      for (int i = 0; i < kHalf; ++i) x ^= b[i].x ^ b[i].y ^ b[i].z ^ b[i].w;
      acc ^= x;
      if constexpr (V >= 3) {
#pragma unroll
        for (int i = 0; i < kHalf; ++i) b[i] = ld(pn + (kHalf + i) * 64);
      }
      if (lane == 0) s_x[wave] = x;
      __syncthreads();
      // V 2/3: this step's group; V 4: every 4th step, the last 4 steps' groups (one run of 4 groups, strided
      // by the grid: 4 separate runs); V 5: the previous step's group (stores one step behind the reads)
      const bool go = V == 4 ? (((g - blockIdx.x) / gridDim.x) % 4 == 3 || gn >= ngroups) : (V == 5 ? g >= gridDim.x + blockIdx.x || gn >= ngroups : true);
      if (out && go) {
        const int nb = V == 4 ? 4 : (V == 5 && gn >= ngroups && g >= gridDim.x ? 2 : 1);
        for (int k = 0; k < nb; ++k) {
          const uint64_t gg = V == 5 ? (gn >= ngroups && k == 1 ? g : g - gridDim.x) : g - (uint64_t)k * gridDim.x;
          if (gg > g || (V == 5 && gg >= ngroups)) continue;
          const uint64_t e0 = e_of(gg * 16, wq16), e1 = e_of(gg * 16 + 16 < nranges ? gg * 16 + 16 : nranges, wq16);
          const uint32_t xx = s_x[threadIdx.x & 15];
          for (uint64_t e = e0 + threadIdx.x; e < e1; e += 1024) st(out + e, uint4{xx, (uint32_t)e, (uint32_t)gg, acc});
        }
      }
      if constexpr (V == 2) {
#pragma unroll
        for (int i = 0; i < kHalf; ++i) b[i] = ld(pn + (kHalf + i) * 64);
      }
      __syncthreads();
      if (gn >= ngroups) break;
      g = gn;
      r = rn;
    }
#pragma unroll
    for (int i = 0; i < kHalf; ++i) acc ^= a[i].x ^ b[i].y;
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;
}

template <int V>
float run(const uint4* in, uint64_t nranges, uint4* out, uint64_t wq16, unsigned* sink, int grid, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float best = 1e30f;
  for (int i = 0; i < reps; ++i) {
    hipEventRecord(a, 0);
    hipLaunchKernelGGL(mix_kernel<V>, dim3(grid), dim3(1024), 0, 0, in, nranges, out, wq16, sink);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  hipEventDestroy(a);
  hipEventDestroy(b);
  return best;
}

int main(int argc, char** argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 4.0;
  const uint64_t bytes = (uint64_t)(gib * (1ull << 30));
  const uint64_t nranges = bytes / kRange;
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int grid = prop.multiProcessorCount;
  uint4 *in, *out;
  unsigned* sink;
  if (hipMalloc(&in, bytes) != hipSuccess || hipMalloc(&out, bytes / 4 + (1 << 20)) != hipSuccess ||
      hipMalloc(&sink, 64) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  hipMemset(in, 0x41, bytes);
  hipMemset(out, 0, bytes / 4);
  hipDeviceSynchronize();
  const double ws[] = {0.0, 0.025, 0.056, 0.10, 0.224};
  for (double w : ws) {
    const uint64_t wq16 = (uint64_t)(w * 65536.0 * 1024.0);   // 16-byte elements per range x 65536
    const uint64_t wbytes = (nranges * wq16 >> 16) * 16;
    float t[6];
    t[0] = run<0>(in, nranges, w > 0 ? out : nullptr, wq16, sink, grid, 8);
    t[1] = run<1>(in, nranges, w > 0 ? out : nullptr, wq16, sink, grid, 8);
    t[2] = run<2>(in, nranges, w > 0 ? out : nullptr, wq16, sink, grid, 8);
    t[3] = run<3>(in, nranges, w > 0 ? out : nullptr, wq16, sink, grid, 8);
    t[4] = run<4>(in, nranges, w > 0 ? out : nullptr, wq16, sink, grid, 8);
    t[5] = run<5>(in, nranges, w > 0 ? out : nullptr, wq16, sink, grid, 8);
    for (int v = 0; v < 6; ++v)
      printf("{\"variant\": \"%c\", \"write_per_read\": %.3f, \"us\": %.1f, \"read_TBps\": %.3f, \"total_TBps\": %.3f}\n",
             'A' + v, w, t[v] * 1e3, bytes / (t[v] * 1e-3) / 1e12, (bytes + wbytes) / (t[v] * 1e-3) / 1e12);
  }
  return 0;
}
