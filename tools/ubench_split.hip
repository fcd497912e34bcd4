// Round 6 probe (diagnostic, not part of the library): is the newline kernels' placement-dependent slow mode the
// loading waves' own stores sharing their in-order vmcnt, or read/write interference in the memory system?
// Several separately allocated input buffers, every variant over each of them in turn, same process:
//   r16   read only, 16 loading waves per 1024-thread workgroup, a group of 16 consecutive 16 KiB ranges per step
//   r15   read only, 15 loading waves (groups of 15 ranges), wave 15 only takes the barriers
//   rw16  the library's stream_rw_kernel shape: 16 loading waves, the step's output run stored by all 1024 threads
//   rw15  15 loading waves storing the run themselves (960 threads), wave 15 idle
//   sw15  15 loading waves; wave 15 alone stores the run (no loading wave ever has a store in its vmcnt)
// If the slow buffers of rw16 / rw15 are fast under sw15, it is the shared counter; if sw15 is slow on the same
// buffers, it is the memory system.  HIP events per launch, median of `reps`.
//   hipcc --offload-arch=gfx950 -O3 -Wno-unused-result -Wno-unused-value -o tools/ubench_split tools/ubench_split.hip
//   ./tools/ubench_split [GiB per buffer=4] [buffers=6] [write bytes per read byte=0.025] [reps=5] [variants]
//                        [output buffers=1] [allocation per input buffer: d / c, e.g. dcdc]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <vector>

constexpr int kRange = 16384;
constexpr int kHalf = kRange / 2048;   // 8 rows of 1 KiB per half range

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
// 16-byte output elements of range r: [e(r), e(r + 1)), e(r) = r * wq16 >> 16
__host__ __device__ __forceinline__ uint64_t e_of(uint64_t r, uint64_t wq16) { return (r * wq16) >> 16; }

// W loading waves per group; STORE: 0 none, 1 loading waves store, 2 wave 15 stores; SWAP: a wave reads its
// range's second half first when (group ^ wave) is odd; NOBAR: no barrier per step (read only: free-running waves)
// BURST: the runs of BURST consecutive steps stored together, after every BURST-th step (and the last)
// SEQ: workgroup b takes groups [b K, (b + 1) K) in order (each CU walks its own contiguous region: 256 regions
// in flight across the buffer) instead of b, b + grid, ... (the grid walks one 64 MiB window)
template <int W, int STORE, bool SWAP = false, bool NOBAR = false, int BURST = 1, bool SEQ = false>
__global__ void __launch_bounds__(1024) split_kernel(const uint4* __restrict__ in, uint64_t nranges,
                                                     uint4* __restrict__ out, uint64_t wq16, unsigned* sink) {
  __shared__ uint32_t s_x[2][16];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const bool loader = wave < W;
  const uint64_t ngroups_all = (nranges + W - 1) / W;
  const uint64_t K = (ngroups_all + gridDim.x - 1) / gridDim.x;
  const uint64_t gstep = SEQ ? 1 : gridDim.x;
  const uint64_t ngroups = SEQ ? ((blockIdx.x + 1) * K < ngroups_all ? (blockIdx.x + 1) * K : ngroups_all) : ngroups_all;
  uint64_t g = SEQ ? blockIdx.x * K : blockIdx.x;
  if (g >= ngroups) return;
  uint32_t acc = 0;
  uint4 a[kHalf], b[kHalf];
  auto ptr = [&](uint64_t gg) {
    const uint64_t r = gg * W + (uint64_t)(loader ? wave : 0);
    const uint64_t sw = SWAP && ((gg ^ (uint64_t)wave) & 1ull) ? kHalf * 64 : 0;
    return in + (r < nranges ? r : 0ull) * (kRange / 16) + lane + sw;
  };
  // (SWAP) the half read second sits at -kHalf rows from the pointer instead of +kHalf
  auto other = [&](uint64_t gg) -> int64_t {
    return SWAP && ((gg ^ (uint64_t)wave) & 1ull) ? -(int64_t)kHalf * 64 : (int64_t)kHalf * 64;
  };
  if (loader) {
    const uint4* p = ptr(g);
#pragma unroll
    for (int i = 0; i < kHalf; ++i) a[i] = ld(p + i * 64);
#pragma unroll
    for (int i = 0; i < kHalf; ++i) b[i] = ld(p + other(g) + i * 64);
  }
  for (uint32_t k = 0;; ++k) {
    const uint64_t gn = g + gstep;
    const uint32_t par = k & 1u;
    if (loader) {
      const uint64_t gq = gn < ngroups ? gn : g;
      const uint4* pn = ptr(gq);
      uint32_t x = 0;
#pragma unroll
      for (int i = 0; i < kHalf; ++i) x ^= a[i].x ^ a[i].y ^ a[i].z ^ a[i].w;
#pragma unroll
      for (int i = 0; i < kHalf; ++i) a[i] = ld(pn + i * 64);
#pragma unroll
      for (int i = 0; i < kHalf; ++i) x ^= b[i].x ^ b[i].y ^ b[i].z ^ b[i].w;
#pragma unroll
      for (int i = 0; i < kHalf; ++i) b[i] = ld(pn + other(gq) + i * 64);
      acc ^= x;
      if (lane == 0) s_x[par][wave] = x;
    }
    if (!NOBAR) __syncthreads();
    const bool flush = BURST == 1 || k % BURST == BURST - 1 || gn >= ngroups;
    for (int j = 0; flush && j < BURST; ++j) {
      const uint64_t back = (uint64_t)(BURST == 1 ? 0 : (gn >= ngroups ? k % BURST : BURST - 1) - j);
      if ((int64_t)back < 0 || back * gstep > g) continue;
      const uint64_t gg = g - back * gstep;
      const uint64_t r0 = gg * W, r1 = r0 + W < nranges ? r0 + W : nranges;
      const uint64_t e0 = e_of(r0, wq16), e1 = e_of(r1, wq16);
      if (STORE == 1 && loader) {
        const uint32_t xx = s_x[par][threadIdx.x % W];
        for (uint64_t e = e0 + threadIdx.x; e < e1; e += 64 * W) st(out + e, uint4{xx, (uint32_t)e, (uint32_t)gg, acc});
      } else if (STORE == 2 && !loader) {
        const uint32_t xx = s_x[par][lane % W];
        for (uint64_t e = e0 + lane; e < e1; e += 64) st(out + e, uint4{xx, (uint32_t)e, (uint32_t)gg, acc});
      }
    }
    if (STORE == 1) __syncthreads();   // (the library's stream_rw shape: the run's stores between two barriers)
    if (gn >= ngroups) break;
    g = gn;
  }
  if (loader) {
#pragma unroll
    for (int i = 0; i < kHalf; ++i) acc ^= a[i].x ^ b[i].y;
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;
}

// The rw16 shape with buffer loads of cache policy LP (the aux bits: 1 sc0, 2 nt, 16 sc1) and stores of policy SP
// (0 plain, 1 non-temporal); wq16 == 0: read only
template <int LP, int SP, int H = kHalf>
__global__ void __launch_bounds__(1024) pol_kernel(const uint4* __restrict__ in, uint64_t nranges,
                                                   uint4* __restrict__ out, uint64_t wq16, unsigned* sink) {
  __shared__ uint32_t s_x[16];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const uint64_t ngroups = (nranges * kRange / (2 * H * 1024) + 15) / 16;
  uint64_t g = blockIdx.x;
  if (g >= ngroups) return;
  uint32_t acc = 0;
  typedef __attribute__((ext_vector_type(4))) unsigned v4;
  v4 a[H], b[H];
  constexpr int R = 2 * H * 1024;   // range bytes
  const uint64_t nr = nranges * kRange / R;      // ranges of R bytes
  auto rsrc = [&](uint64_t gg) {
    const uint64_t r = gg * 16 + (uint64_t)wave;
    return __builtin_amdgcn_make_buffer_rsrc((void*)(in + (r < nr ? r : 0ull) * (R / 16)), 0, R, 0x00020000);
  };
  {
    auto rs = rsrc(g);
#pragma unroll
    for (int i = 0; i < H; ++i) a[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (lane + i * 64) * 16, 0, LP);
#pragma unroll
    for (int i = 0; i < H; ++i) b[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (lane + (H + i) * 64) * 16, 0, LP);
  }
  for (;;) {
    const uint64_t gn = g + gridDim.x;
    auto rs = rsrc(gn < ngroups ? gn : g);
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < H; ++i) x ^= a[i][0] ^ a[i][1] ^ a[i][2] ^ a[i][3];
#pragma unroll
    for (int i = 0; i < H; ++i) a[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (lane + i * 64) * 16, 0, LP);
#pragma unroll
    for (int i = 0; i < H; ++i) x ^= b[i][0] ^ b[i][1] ^ b[i][2] ^ b[i][3];
#pragma unroll
    for (int i = 0; i < H; ++i) b[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (lane + (H + i) * 64) * 16, 0, LP);
    acc ^= x;
    if (wq16) {
      if (lane == 0) s_x[wave] = x;
      __syncthreads();
      // output elements in 16 KiB-range units, as the other variants
      const uint64_t r0 = g * 16 * R / kRange, r1x = (g * 16 + 16) * R / kRange, r1 = r1x < nranges ? r1x : nranges;
      const uint64_t e0 = e_of(r0, wq16), e1 = e_of(r1, wq16);
      const uint32_t xx = s_x[threadIdx.x & 15];
      for (uint64_t e = e0 + threadIdx.x; e < e1; e += 1024) {
        if (SP) st(out + e, uint4{xx, (uint32_t)e, (uint32_t)g, acc});
        else out[e] = uint4{xx, (uint32_t)e, (uint32_t)g, acc};
      }
    }
    __syncthreads();
    if (gn >= ngroups) break;
    g = gn;
  }
#pragma unroll
  for (int i = 0; i < H; ++i) acc ^= a[i][0] ^ b[i][1];
  if (acc == 0x9E3779B9u) sink[0] = acc;
}

struct Variant {
  const char* name;
  void (*k)(const uint4*, uint64_t, uint4*, uint64_t, unsigned*);
  bool writes;
};

// VMM-composed input buffers (kinds 'v' and 'p'): physical chunks of UB_CHUNK_MIB (default 512) mapped into one
// reserved VA range.  'p' probes each candidate chunk first (read-only vs read-while-writing time over the chunk,
// through a temporary mapping) and keeps the fast ones; the slow candidates are held until the buffer is built.
// (Round 6: 'v' works -- 4 GiB buffers of 512 MiB chunks read-while-write in 679-757 us, mixtures like large
// hipMalloc buffers.  'p' probing through temporary mappings crashed in the host runtime at 4 GiB; it now probes
// each chunk in place, at its final offset, and unmaps a slow one.)
static hipMemAllocationProp vmm_prop() {
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  return prop;
}

static bool vmm_map(void* va, uint64_t off, uint64_t n, hipMemGenericAllocationHandle_t h) {
  if (hipMemMap((char*)va + off, n, 0, h, 0) != hipSuccess) return false;
  hipMemAccessDesc acc = {};
  acc.location = vmm_prop().location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  return hipMemSetAccess((char*)va + off, n, &acc, 1) == hipSuccess;
}

template <class KR, class KW>
static float chunk_ratio(void* va, uint64_t n, uint4* out, uint64_t wq16, unsigned* sink, int grid, KR kr, KW kw) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float t[2] = {0, 0};
  for (int rep = 0; rep < 3; ++rep)
    for (int v = 0; v < 2; ++v) {
      hipEventRecord(a, 0);
      if (v == 0) hipLaunchKernelGGL(kr, dim3(grid), dim3(1024), 0, 0, (const uint4*)va, n / kRange, nullptr, 0ull, sink);
      else hipLaunchKernelGGL(kw, dim3(grid), dim3(1024), 0, 0, (const uint4*)va, n / kRange, out, wq16, sink);
      hipEventRecord(b, 0);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (rep > 0) t[v] += ms;
    }
  hipEventDestroy(a);
  hipEventDestroy(b);
  return t[1] / t[0];
}

int main(int argc, char** argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 4.0;
  const int nbuf = argc > 2 ? atoi(argv[2]) : 6;
  const double w = argc > 3 ? atof(argv[3]) : 0.025;
  const int reps = argc > 4 ? atoi(argv[4]) : 5;
  const uint64_t bytes = (uint64_t)(gib * (1ull << 30));
  const uint64_t nranges = bytes / kRange;
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int grid = prop.multiProcessorCount;
  // argv[7]: per input buffer its allocation, d = hipMalloc, c = hipExtMallocWithFlags(hipDeviceMallocContiguous)
  const char* kinds = argc > 7 ? argv[7] : "";
  std::vector<uint4*> bufs(nbuf);
  // argv[6]: output buffers (default 1); with more, every (input, output) pair is timed for each variant
  const int nout = argc > 6 ? atoi(argv[6]) : 1;
  std::vector<uint4*> outs(nout);
  unsigned* sink;
  const uint64_t wq16 = (uint64_t)(w * 65536.0 * 1024.0);
  const uint64_t wbytes = e_of(nranges, wq16) * 16;
  for (int o = 0; o < nout; ++o) {
    if (hipMalloc(&outs[o], wbytes + (1 << 20)) != hipSuccess) {
      printf("alloc failed\n");
      return 1;
    }
    hipMemset(outs[o], 0, wbytes);
  }
  if (hipMalloc(&sink, 64) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  const uint64_t chunk = (uint64_t)(getenv("UB_CHUNK_MIB") ? atoi(getenv("UB_CHUNK_MIB")) : 512) << 20;
  const double slow = getenv("UB_SLOW") ? atof(getenv("UB_SLOW")) : 1.125;
  for (int i = 0; i < nbuf; ++i) {
    const char k = i < (int)strlen(kinds) ? kinds[i] : 'd';
    hipError_t e = hipSuccess;
    if (k == 'v' || k == 'p') {
      if (bytes % chunk) {
        printf("size not a multiple of the chunk\n");
        return 1;
      }
      void* va = nullptr;
      const hipMemAllocationProp prop = vmm_prop();
      size_t gran = 0;
      hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum);
      int vmm = 0;
      hipDeviceGetAttribute(&vmm, hipDeviceAttributeVirtualMemoryManagementSupported, 0);
      fprintf(stderr, "vmm supported %d granularity %zu\n", vmm, gran);
      if (!vmm || hipMemAddressReserve(&va, bytes, 0, nullptr, 0) != hipSuccess) {
        printf("reserve failed\n");
        return 1;
      }
      std::vector<hipMemGenericAllocationHandle_t> held;
      std::vector<float> ratios;
      uint64_t off = 0;
      int tries = 0;
      while (off < bytes) {
        hipMemGenericAllocationHandle_t h;
        if (hipMemCreate(&h, chunk, &prop, 0) != hipSuccess) {
          printf("create failed after %d tries\n", tries);
          return 1;
        }
        ++tries;
        fprintf(stderr, "chunk %d created\n", tries);
        bool keep = true;
        if (k == 'p') {
          // probe the chunk in place (mapped at its final offset); a slow one is unmapped and held
          if (!vmm_map(va, off, chunk, h)) {
            printf("map failed\n");
            return 1;
          }
          hipMemset((char*)va + off, 0x41, chunk);
          const float r = chunk_ratio((char*)va + off, chunk, outs[0], wq16, sink, grid, split_kernel<16, 0>,
                                      split_kernel<16, 1>);
          ratios.push_back(r);
          hipDeviceSynchronize();
          keep = r <= slow || tries > 4 * (int)(bytes / chunk);
          if (keep) {
            off += chunk;
          } else {
            hipMemUnmap((char*)va + off, chunk);
            held.push_back(h);
          }
          continue;
        }
        if (keep) {
          fprintf(stderr, "map at %llu\n", (unsigned long long)off);
          if (!vmm_map(va, off, chunk, h)) {
            printf("map failed\n");
            return 1;
          }
          off += chunk;
        } else {
          held.push_back(h);
        }
      }
      for (auto h : held) hipMemRelease(h);
      bufs[i] = (uint4*)va;
      fprintf(stderr, "buffer %d mapped\n", i);
      if (k == 'p') {
        printf("{\"buffer\": %d, \"chunk_ratios\": [", i);
        for (size_t j = 0; j < ratios.size(); ++j) printf("%s%.3f", j ? ", " : "", ratios[j]);
        printf("]}\n");
      }
    } else {
      e = k == 'c' ? hipExtMallocWithFlags((void**)&bufs[i], bytes, hipDeviceMallocContiguous) : hipMalloc(&bufs[i], bytes);
    }
    if (e != hipSuccess) {
      printf("alloc %c failed\n", k);
      return 1;
    }
    hipMemset(bufs[i], 0x41 + i, bytes);
  }
  hipDeviceSynchronize();
  const Variant all[] = {{"r16", split_kernel<16, 0>, false},  {"r15", split_kernel<15, 0>, false},
                         {"rw16", split_kernel<16, 1>, true},  {"rw15", split_kernel<15, 1>, true},
                         {"sw15", split_kernel<15, 2>, true},  {"r14", split_kernel<14, 0>, false},
                         {"r12", split_kernel<12, 0>, false},  {"r16swap", split_kernel<16, 0, true>, false},
                         {"r16free", split_kernel<16, 0, false, true>, false},
                         {"r15free", split_kernel<15, 0, false, true>, false},
                         {"rw16swap", split_kernel<16, 1, true>, true},
                         {"rw16b2", split_kernel<16, 1, false, false, 2>, true},
                         {"rw16b4", split_kernel<16, 1, false, false, 4>, true},
                         {"rw16b8", split_kernel<16, 1, false, false, 8>, true},
                         {"rw16b16", split_kernel<16, 1, false, false, 16>, true},
                         {"sw15b4", split_kernel<15, 2, false, false, 4>, true},
                         {"r16seq", split_kernel<16, 0, false, false, 1, true>, false},
                         {"rw16seq", split_kernel<16, 1, false, false, 1, true>, true},
                         // buffer loads by cache policy (n: nt, p: plain, s1: sc1, s01: sc0 sc1, s01n: sc0 sc1 nt),
                         // stores non-temporal (n) or plain (p); "r" read only
                         {"rbn", pol_kernel<2, 1>, false},   {"rbp", pol_kernel<0, 1>, false},
                         {"rbs1", pol_kernel<16, 1>, false}, {"rbs01", pol_kernel<17, 1>, false},
                         {"rbn_n", pol_kernel<2, 1>, true},  {"rbp_n", pol_kernel<0, 1>, true},
                         {"rbs1_n", pol_kernel<16, 1>, true}, {"rbs01_n", pol_kernel<17, 1>, true},
                         {"rbs01n_n", pol_kernel<19, 1>, true}, {"rbn_p", pol_kernel<2, 0>, true},
                         {"rbp_p", pol_kernel<0, 0>, true},
                         // rows of 1 KiB per half range (in flight per wave: H to 2H KiB)
                         {"rbn4", pol_kernel<2, 1, 4>, false},   {"rbn12", pol_kernel<2, 1, 12>, false},
                         {"rbn_n4", pol_kernel<2, 1, 4>, true},  {"rbn_n12", pol_kernel<2, 1, 12>, true},
                         {"rbn_n16", pol_kernel<2, 1, 16>, true}, {"rbn16", pol_kernel<2, 1, 16>, false}};
  // argv[5]: a comma list of variant names (default: the first five)
  std::vector<Variant> vs;
  const char* pick = argc > 5 ? argv[5] : "r16,r15,rw16,rw15,sw15";
  for (const Variant& v : all) {
    const char* f = strstr(pick, v.name);
    const size_t n = strlen(v.name);
    // whole names only
    while (f && !((f == pick || f[-1] == ',') && (f[n] == ',' || f[n] == 0))) f = strstr(f + 1, v.name);
    if (f) vs.push_back(v);
  }
  const int nv = (int)vs.size();
  std::vector<std::vector<float>> t(nbuf * nv * nout);
  hipEvent_t ea, eb;
  hipEventCreate(&ea);
  hipEventCreate(&eb);
  for (int rep = 0; rep < reps + 1; ++rep)
    for (int i = 0; i < nbuf; ++i)
      for (int o = 0; o < nout; ++o)
      for (int v = 0; v < nv; ++v) {
        hipEventRecord(ea, 0);
        hipLaunchKernelGGL(vs[v].k, dim3(grid), dim3(1024), 0, 0, bufs[i], nranges, vs[v].writes ? outs[o] : nullptr,
                           vs[v].writes ? wq16 : 0ull, sink);
        hipEventRecord(eb, 0);
        hipEventSynchronize(eb);
        float ms;
        hipEventElapsedTime(&ms, ea, eb);
        if (rep > 0) t[(i * nout + o) * nv + v].push_back(ms * 1e3f);   // rep 0: warm-up
      }
  for (int i = 0; i < nbuf; ++i)
  for (int o = 0; o < nout; ++o) {
    printf("{\"buffer\": %d, \"alloc\": \"%c\", \"out\": %d, \"addr_gib\": %.2f, \"out_gib\": %.3f, \"write_per_read\": %.3f", i,
           i < (int)strlen(kinds) ? kinds[i] : 'd', o, (double)(uintptr_t)bufs[i] / (1ull << 30),
           (double)(uintptr_t)outs[o] / (1ull << 30), w);
    for (int v = 0; v < nv; ++v) {
      auto& s = t[(i * nout + o) * nv + v];
      std::sort(s.begin(), s.end());
      printf(", \"%s\": %.1f", vs[v].name, s[s.size() / 2]);
    }
    printf("}\n");
  }
  return 0;
}
