// VALU issue-rate micro-benchmark (diagnostic, not part of the library): relative throughput of the
// instructions the byte classifier can use, measured against v_add_u32 on the same launch geometry
// (4 waves per SIMD, 8 independent chains).
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_valu tools/ubench_valu.hip && ./tools/ubench_valu
#include <hip/hip_runtime.h>
#include <stdio.h>

#define BODY8(INS)                                                                                   \
  asm volatile(INS : "+v"(a0) : "v"(b), "v"(c)); asm volatile(INS : "+v"(a1) : "v"(b), "v"(c));   \
  asm volatile(INS : "+v"(a2) : "v"(b), "v"(c)); asm volatile(INS : "+v"(a3) : "v"(b), "v"(c));   \
  asm volatile(INS : "+v"(a4) : "v"(b), "v"(c)); asm volatile(INS : "+v"(a5) : "v"(b), "v"(c));   \
  asm volatile(INS : "+v"(a6) : "v"(b), "v"(c)); asm volatile(INS : "+v"(a7) : "v"(b), "v"(c));

#define KERNEL(NAME, INS)                                                                            \
  __global__ void __launch_bounds__(1024) NAME(unsigned* out, int iters) {                           \
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,      \
             a6 = a0 + 6, a7 = a0 + 7;                                                               \
    unsigned b = 0x01020304u ^ threadIdx.x, c = 0x80808080u;                                         \
    for (int i = 0; i < iters; ++i) { BODY8(INS) BODY8(INS) }                                        \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;             \
  }

KERNEL(k_add, "v_add_u32 %0, %0, %1")
KERNEL(k_xad, "v_xad_u32 %0, %0, %1, %2")
KERNEL(k_bfi, "v_bfi_b32 %0, %0, %1, %2")
KERNEL(k_or3, "v_or3_b32 %0, %0, %1, %2")
KERNEL(k_dot4, "v_dot4_u32_u8 %0, %0, %1, %2")
KERNEL(k_mul24, "v_mul_u32_u24 %0, %0, %1")
KERNEL(k_mullo, "v_mul_lo_u32 %0, %0, %1")
KERNEL(k_lshlor, "v_lshl_or_b32 %0, %0, 3, %1")
KERNEL(k_alignbit, "v_alignbit_b32 %0, %0, %1, 7")
KERNEL(k_bcnt, "v_bcnt_u32_b32 %0, %0, %1")
KERNEL(k_perm, "v_perm_b32 %0, %0, %1, %2")
KERNEL(k_ffbl, "v_ffbl_b32 %0, %0")
KERNEL(k_add_e64, "v_add_u32_e64 %0, %0, %1")
KERNEL(k_and_lit, "v_and_b32 %0, 0x7f7f7f7f, %0")
KERNEL(k_xor, "v_xor_b32 %0, %1, %0")
KERNEL(k_lshr, "v_lshrrev_b32 %0, 7, %0")
KERNEL(k_add_lit, "v_add_u32 %0, 0x7f7f7f7f, %0")
KERNEL(k_add3, "v_add3_u32 %0, %0, %1, %2")
KERNEL(k_mbcnt, "v_mbcnt_lo_u32_b32 %0, %0, %1")
KERNEL(k_and_or, "v_and_or_b32 %0, %0, %1, %2")

typedef void (*kfn)(unsigned*, int);

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  unsigned* out;
  hipMalloc(&out, (size_t)cus * 1024 * 4);
  const int iters = 20000;
  struct { const char* n; kfn f; } ks[] = {{"v_add_u32", k_add}, {"v_xad_u32", k_xad}, {"v_bfi_b32", k_bfi},
                                           {"v_or3_b32", k_or3}, {"v_dot4_u32_u8", k_dot4},
                                           {"v_mul_u32_u24", k_mul24}, {"v_mul_lo_u32", k_mullo},
                                           {"v_lshl_or_b32", k_lshlor}, {"v_alignbit_b32", k_alignbit},
                                           {"v_bcnt_u32_b32", k_bcnt}, {"v_perm_b32", k_perm},
                                           {"v_ffbl_b32", k_ffbl},
                                           {"v_add_u32_e64", k_add_e64}, {"v_and_b32 lit", k_and_lit},
                                           {"v_xor_b32", k_xor}, {"v_lshrrev_b32", k_lshr}, {"v_add_u32 lit", k_add_lit},
                                           {"v_add3_u32", k_add3}, {"v_mbcnt_lo", k_mbcnt}, {"v_and_or_b32", k_and_or}};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  double base = 0;
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.f, dim3(cus), dim3(1024), 0, 0, out, 100);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k.f, dim3(cus), dim3(1024), 0, 0, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    // wave-instructions per SIMD: 4 waves x iters x 16
    const double per_simd = 4.0 * iters * 16;
    const double ns = ms * 1e6 / per_simd;
    if (base == 0) base = ns;
    printf("%-16s %7.3f ns per wave-instruction per SIMD  (x%.2f of v_add_u32)\n", k.n, ns, ns / base);
  }
  return 0;
}
