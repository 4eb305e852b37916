// Front-end (instruction issue) probe for gfx950: the same integer add in
// different encodings, and at different waves per SIMD.  If the VOP3 (8-byte)
// and literal (8-byte) forms run at half the rate of the 4-byte VOP2 form, the
// limit is instruction bytes, not VALU lanes.
//   hipcc --offload-arch=gfx950 -O3 scripts/issue_rate.hip -o /tmp/issue_rate && /tmp/issue_rate
#include <hip/hip_runtime.h>
#include <cstdio>

#define C8(INS)                                                                                          \
  asm volatile(INS : "+v"(a0) : "v"(k)); asm volatile(INS : "+v"(a1) : "v"(k));                         \
  asm volatile(INS : "+v"(a2) : "v"(k)); asm volatile(INS : "+v"(a3) : "v"(k));                         \
  asm volatile(INS : "+v"(a4) : "v"(k)); asm volatile(INS : "+v"(a5) : "v"(k));                         \
  asm volatile(INS : "+v"(a6) : "v"(k)); asm volatile(INS : "+v"(a7) : "v"(k));

#define KERNEL(NAME, INS)                                                                                \
  __global__ void __launch_bounds__(256) NAME(unsigned* out, unsigned iters, unsigned seed) {           \
    unsigned a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, \
             a6 = a0 + 6, a7 = a0 + 7, k = seed * 3u + 1u;                                              \
    for (unsigned i = 0; i < iters; ++i) {                                                               \
      C8(INS) C8(INS) C8(INS) C8(INS)                                                                    \
    }                                                                                                    \
    unsigned s = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                                                 \
    if (s == 0x12345678u) out[blockIdx.x] = s;                                                           \
  }

KERNEL(k_add_e32, "v_add_u32_e32 %0, %0, %1")          // 4 B
KERNEL(k_add_e64, "v_add_u32_e64 %0, %0, %1")          // 8 B, same op
KERNEL(k_add_lit, "v_add_u32_e32 %0, 0x12345, %0")     // 4 B + 4 B literal
KERNEL(k_pk_add, "v_pk_add_u16 %0, %0, %1")            // 8 B (VOP3P)
KERNEL(k_or_e32, "v_or_b32_e32 %0, %0, %1")            // 4 B
KERNEL(k_lshl_add, "v_lshl_add_u32 %0, %0, 3, %1")     // 8 B
KERNEL(k_add3, "v_add3_u32 %0, %0, %1, %1")            // 8 B, 2 adds

typedef void (*kfn)(unsigned*, unsigned, unsigned);

int main() {
  struct { const char* name; kfn f; int bytes; } ks[] = {
      {"v_add_u32_e32", k_add_e32, 4}, {"v_add_u32_e64", k_add_e64, 8}, {"v_add_u32_e32+literal", k_add_lit, 8},
      {"v_pk_add_u16", k_pk_add, 8},   {"v_or_b32_e32", k_or_e32, 4},   {"v_lshl_add_u32", k_lshl_add, 8},
      {"v_add3_u32", k_add3, 8}};
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const unsigned cus = prop.multiProcessorCount, threads = 256, iters = 2048;
  unsigned* out;
  hipMalloc(&out, cus * 16 * sizeof(unsigned));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  printf("{\"cus\": %u, \"rates\": [", cus);
  bool first = true;
  for (unsigned wps : {1u, 2u, 4u, 8u}) {  // waves per SIMD (4 waves per block, one block per SIMD-wave)
    for (unsigned i = 0; i < sizeof(ks) / sizeof(ks[0]); ++i) {
      const unsigned blocks = cus * wps;
      hipLaunchKernelGGL(ks[i].f, dim3(blocks), dim3(threads), 0, 0, out, 16u, 1u);
      hipEventRecord(e0);
      hipLaunchKernelGGL(ks[i].f, dim3(blocks), dim3(threads), 0, 0, out, iters, 1u);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double winstr = (double)blocks * (threads / 64) * iters * 32;  // wave-instructions
      const double per_cu_clk = winstr / cus / (ms * 1e-3 * prop.clockRate * 1e3);
      printf("%s{\"ins\": \"%s\", \"waves_per_simd\": %u, \"wave_instr_per_cu_clk\": %.3f, \"bytes_per_cu_clk\": %.2f, "
             "\"lanes_per_simd_clk\": %.2f}",
             first ? "" : ", ", ks[i].name, wps, per_cu_clk, per_cu_clk * ks[i].bytes, per_cu_clk * 64 / 4);
      first = false;
    }
  }
  printf("]}\n");
  return 0;
}
