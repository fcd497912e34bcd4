// Mixed read + write streaming ceiling (diagnostic, not part of the library): the HBM rate of a kernel
// that reads its input once in the scan's geometry (one 1024-thread workgroup per CU, 16 KiB per wave
// range, 16-byte non-temporal lane loads) and writes W output bytes per input byte as contiguous
// non-temporal 16-byte lane stores, range by range (like the DELIM index's uint64 offsets: CSV W = 0.224,
// VCF W = 0.10, FASTA W = 0.004).  Reports total (read + write) bytes / kernel time.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_rw tools/ubench_rw.hip && ./tools/ubench_rw
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kRange = 16384;       // bytes per wave range
constexpr int kRows = kRange / 1024;

// stores with an explicit cache policy (gfx950 global_store_dwordx4 modifiers)
typedef unsigned v4u_t __attribute__((ext_vector_type(4)));
#define POLICY_STORE(NAME, POL)                                                                              \
  __device__ __forceinline__ void NAME(uint4* p, uint4 v) {                                                  \
    const v4u_t w = {v.x, v.y, v.z, v.w};                                                                    \
    asm volatile("global_store_dwordx4 %0, %1, off " POL :: "v"((uint64_t)p), "v"(w) : "memory");           \
  }
POLICY_STORE(st_plain, "")
POLICY_STORE(st_nt, "nt")
POLICY_STORE(st_sc1, "sc1")
POLICY_STORE(st_sc0sc1, "sc0 sc1")
POLICY_STORE(st_sc1nt, "sc1 nt")
POLICY_STORE(st_sc0sc1nt, "sc0 sc1 nt")
POLICY_STORE(st_sc0nt, "sc0 nt")

template <int POL>
__global__ void __launch_bounds__(1024) pol_kernel(const uint4* __restrict__ in, uint64_t nranges,
                                                   uint4* __restrict__ out, double w16, unsigned* sink) {
  const int lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  uint32_t acc = 0;
  for (uint64_t r = wave; r < nranges; r += nwaves) {
    const uint4* p = in + r * (kRange / 16) + lane;
    uint4 v[kRows];
#pragma unroll
    for (int i = 0; i < kRows; ++i) {
      v[i].x = __builtin_nontemporal_load(&p[i * 64].x);
      v[i].y = __builtin_nontemporal_load(&p[i * 64].y);
      v[i].z = __builtin_nontemporal_load(&p[i * 64].z);
      v[i].w = __builtin_nontemporal_load(&p[i * 64].w);
    }
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < kRows; ++i) x ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
    acc ^= x;
    const uint64_t e0 = (uint64_t)((double)r * w16), e1 = (uint64_t)((double)(r + 1) * w16);
    for (uint64_t e = e0 + lane; e < e1; e += 64) {
      const uint4 o = {x, (uint32_t)e, (uint32_t)r, acc};
      switch (POL) {
        case 0: st_plain(out + e, o); break;
        case 1: st_nt(out + e, o); break;
        case 2: st_sc1(out + e, o); break;
        case 3: st_sc0sc1(out + e, o); break;
        case 4: st_sc1nt(out + e, o); break;
        case 5: st_sc0sc1nt(out + e, o); break;
        default: st_sc0nt(out + e, o); break;
      }
    }
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;
}

// B consecutive ranges per wave step: their outputs form one contiguous run written after the B ranges
template <bool NT, int B>
__global__ void __launch_bounds__(1024) rw_kernel(const uint4* __restrict__ in, uint64_t nranges,
                                                  uint4* __restrict__ out, double w16, unsigned* sink) {
  const int lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  uint32_t acc = 0;
  for (uint64_t r0 = wave * B; r0 < nranges; r0 += nwaves * B) {
    uint32_t x = 0;
    for (int b = 0; b < B && r0 + b < nranges; ++b) {
      const uint4* p = in + (r0 + b) * (kRange / 16) + lane;
      uint4 v[kRows];
#pragma unroll
      for (int i = 0; i < kRows; ++i) {
        v[i].x = __builtin_nontemporal_load(&p[i * 64].x);
        v[i].y = __builtin_nontemporal_load(&p[i * 64].y);
        v[i].z = __builtin_nontemporal_load(&p[i * 64].z);
        v[i].w = __builtin_nontemporal_load(&p[i * 64].w);
      }
#pragma unroll
      for (int i = 0; i < kRows; ++i) x ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
    }
    acc ^= x;
    const uint64_t r1 = r0 + B < nranges ? r0 + B : nranges;
    const uint64_t e0 = (uint64_t)((double)r0 * w16), e1 = (uint64_t)((double)r1 * w16);
    for (uint64_t e = e0 + lane; e < e1; e += 64) {
      const uint4 o = {x, (uint32_t)e, (uint32_t)r0, acc};
      if (NT) {
        __builtin_nontemporal_store(o.x, &out[e].x);
        __builtin_nontemporal_store(o.y, &out[e].y);
        __builtin_nontemporal_store(o.z, &out[e].z);
        __builtin_nontemporal_store(o.w, &out[e].w);
      } else {
        out[e] = o;
      }
    }
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;
}

typedef void (*kfn)(const uint4*, uint64_t, uint4*, double, unsigned*);

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const uint64_t n = 4ull << 30;
  uint4 *in, *out;
  unsigned* sink;
  hipMalloc(&in, n);
  hipMalloc(&out, n / 2);
  hipMalloc(&sink, 64);
  hipMemset(in, 7, n);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const double ws[] = {0.10, 0.224};
  struct { const char* n; kfn f; int b; } ks[] = {{"nt_b1", rw_kernel<true, 1>, 1}, {"st_b1", rw_kernel<false, 1>, 1},
                                                   {"nt_b4", rw_kernel<true, 4>, 4}, {"nt_b16", rw_kernel<true, 16>, 16},
                                                   {"asm_plain", pol_kernel<0>, 1}, {"asm_nt", pol_kernel<1>, 1},
                                                   {"asm_sc1", pol_kernel<2>, 1}, {"asm_sc0sc1", pol_kernel<3>, 1},
                                                   {"asm_sc1nt", pol_kernel<4>, 1}, {"asm_sc0sc1nt", pol_kernel<5>, 1},
                                                   {"asm_sc0nt", pol_kernel<6>, 1}};
  for (auto& k : ks) {
    for (double w : ws) {
      const double w16 = w * kRange / 16.0;   // output 16-byte elements per range
      for (int warm = 0; warm < 2; ++warm)
        hipLaunchKernelGGL(k.f, dim3(cus), dim3(1024), 0, 0, in, n / kRange, out, w16, sink);
      const int reps = 10;
      hipEventRecord(e0);
      for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL(k.f, dim3(cus), dim3(1024), 0, 0, in, n / kRange, out, w16, sink);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double s = ms / 1e3 / reps;
      const double wb = (double)(uint64_t)((double)(n / kRange) * w16) * 16.0;
      printf("{\"kernel\": \"%s\", \"write_per_read\": %.3f, \"kernel_us\": %.1f, \"read_TBps\": %.3f, \"total_TBps\": %.3f}\n",
             k.n, w, s * 1e6, n / s / 1e12, (n + wb) / s / 1e12);
    }
  }
  return 0;
}
