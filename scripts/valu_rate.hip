// Measures the chip-wide issue rate of the integer VALU instructions the sweep
// kernel is built from (gfx950), to ground the roofline peak of DESIGN.md §5.
//   hipcc --offload-arch=gfx950 -O3 scripts/valu_rate.hip -o /tmp/valu_rate && /tmp/valu_rate
// Each lane runs 8 independent dependency chains of one instruction (inline
// asm, so the compiler cannot fold them); rate = lane-instructions / second.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHAIN8(INS)                                                                                          \
  asm volatile(INS : "+v"(a0) : "v"(k)); asm volatile(INS : "+v"(a1) : "v"(k));                             \
  asm volatile(INS : "+v"(a2) : "v"(k)); asm volatile(INS : "+v"(a3) : "v"(k));                             \
  asm volatile(INS : "+v"(a4) : "v"(k)); asm volatile(INS : "+v"(a5) : "v"(k));                             \
  asm volatile(INS : "+v"(a6) : "v"(k)); asm volatile(INS : "+v"(a7) : "v"(k));

#define KERNEL(NAME, INS)                                                                                    \
  __global__ void __launch_bounds__(256) NAME(unsigned* out, unsigned iters, unsigned seed) {               \
    unsigned a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,     \
             a6 = a0 + 6, a7 = a0 + 7, k = seed * 3u + 1u;                                                  \
    for (unsigned i = 0; i < iters; ++i) {                                                                   \
      CHAIN8(INS) CHAIN8(INS)                                                                                \
    }                                                                                                        \
    unsigned s = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                                                     \
    if (s == 0x12345678u) out[blockIdx.x] = s;                                                               \
  }

KERNEL(k_add_u32, "v_add_u32 %0, %0, %1")
KERNEL(k_pk_min_u16, "v_pk_min_u16 %0, %0, %1")
KERNEL(k_pk_add_u16, "v_pk_add_u16 %0, %0, %1")
KERNEL(k_dot2_u32_u16, "v_dot2_u32_u16 %0, %1, %1, %0")
KERNEL(k_perm_b32, "v_perm_b32 %0, %0, %1, %1")
KERNEL(k_lshl_add_u32, "v_lshl_add_u32 %0, %0, 3, %1")
KERNEL(k_mul_lo_u32, "v_mul_lo_u32 %0, %0, %1")
KERNEL(k_mul_u32_u24, "v_mul_u32_u24 %0, %0, %1")
KERNEL(k_fma_f32, "v_fma_f32 %0, %0, %1, %1")
KERNEL(k_rcp_f32, "v_rcp_f32 %0, %0")

typedef void (*kfn)(unsigned*, unsigned, unsigned);

int main() {
  struct { const char* name; kfn f; } ks[] = {
      {"v_add_u32", k_add_u32},       {"v_pk_min_u16", k_pk_min_u16},   {"v_pk_add_u16", k_pk_add_u16},
      {"v_dot2_u32_u16", k_dot2_u32_u16}, {"v_perm_b32", k_perm_b32},   {"v_lshl_add_u32", k_lshl_add_u32},
      {"v_mul_lo_u32", k_mul_lo_u32}, {"v_mul_u32_u24", k_mul_u32_u24}, {"v_fma_f32", k_fma_f32},
      {"v_rcp_f32", k_rcp_f32}};
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const unsigned cus = prop.multiProcessorCount;
  const unsigned blocks = cus * 8, threads = 256, iters = 4096;  // 8 waves per SIMD
  unsigned* out;
  hipMalloc(&out, blocks * sizeof(unsigned));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  printf("{\"cus\": %u, \"clock_khz\": %d, \"waves_per_simd\": 8, \"rates\": {", cus, prop.clockRate);
  for (unsigned i = 0; i < sizeof(ks) / sizeof(ks[0]); ++i) {
    hipLaunchKernelGGL(ks[i].f, dim3(blocks), dim3(threads), 0, 0, out, 16u, 1u);  // warm-up
    hipEventRecord(e0);
    hipLaunchKernelGGL(ks[i].f, dim3(blocks), dim3(threads), 0, 0, out, iters, 1u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double lane_ops = (double)blocks * threads * iters * 16.0;
    const double rate = lane_ops / (ms * 1e-3);
    // lanes per clock per SIMD at the nominal clock
    const double per_simd_clk = rate / (cus * 4.0) / (prop.clockRate * 1e3);
    printf("%s\"%s\": {\"Tlane_ops_s\": %.2f, \"lanes_per_simd_clk\": %.1f}", i ? ", " : "", ks[i].name, rate / 1e12,
           per_simd_clk);
  }
  printf("}}\n");
  hipFree(out);
  return 0;
}
