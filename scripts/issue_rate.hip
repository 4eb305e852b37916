// VALU issue-rate probe for gfx950: chip-wide throughput of
// each instruction the sweep kernels are built from, 8 waves per SIMD, 8
// independent chains per lane.  Result (profiles/r02_issue_rate*.json): the
// encoding size does not matter (v_add_u32 e32 = e64 = with a literal), but
// packed (VOP3P), 3-source and multiply ops issue at ~58 % of the simple ops.
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
KERNEL(k_min_u32, "v_min_u32_e32 %0, %0, %1")
KERNEL(k_max_u32, "v_max_u32_e32 %0, %0, %1")
KERNEL(k_lshl, "v_lshlrev_b32_e32 %0, 3, %0")
KERNEL(k_lshr, "v_lshrrev_b32_e32 %0, %1, %0")
KERNEL(k_bfe, "v_bfe_u32 %0, %0, 16, 4")
KERNEL(k_and, "v_and_b32_e32 %0, %0, %1")
KERNEL(k_xor, "v_xor_b32_e32 %0, %0, %1")
KERNEL(k_perm, "v_perm_b32 %0, %0, %1, %1")
KERNEL(k_pk_min, "v_pk_min_u16 %0, %0, %1")
KERNEL(k_pk_lshr, "v_pk_lshrrev_b16 %0, 4, %0")
KERNEL(k_dot2, "v_dot2_u32_u16 %0, %1, %1, %0")
KERNEL(k_mul24, "v_mul_u32_u24_e32 %0, %0, %1")
KERNEL(k_mad24, "v_mad_u32_u24 %0, %0, %1, %1")
KERNEL(k_min3, "v_min3_u32 %0, %0, %1, %1")
KERNEL(k_and_or, "v_and_or_b32 %0, %0, %1, %1")
KERNEL(k_lshl_or, "v_lshl_or_b32 %0, %0, 3, %1")
KERNEL(k_alignbit, "v_alignbit_b32 %0, %0, %1, 7")
KERNEL(k_mul_lo, "v_mul_lo_u32 %0, %0, %1")
KERNEL(k_cvt_f32, "v_cvt_f32_u32_e32 %0, %0")
KERNEL(k_mul_f32, "v_mul_f32_e32 %0, %0, %1")
KERNEL(k_fma_f32, "v_fma_f32 %0, %0, %1, %1")
KERNEL(k_rcp_f32, "v_rcp_f32_e32 %0, %0")
KERNEL(k_cndmask, "v_cndmask_b32_e32 %0, %0, %1, vcc")
// round 5: candidates for the binned client loop's tag/address/value ops
KERNEL(k_add_sdwa_w1, "v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD")
KERNEL(k_add_sdwa_w0, "v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:DWORD")
KERNEL(k_mad_u16_hi, "v_mad_u32_u16 %0, %0, %1, %1 op_sel:[1,0,0,0]")
KERNEL(k_mad_u16, "v_mad_u32_u16 %0, %0, %1, %1")
KERNEL(k_and_const, "v_and_b32_e32 %0, 0xf000f, %0")
// v_cndmask_b32_e32 measured 0.175: which part is slow (the VCC read, any
// SGPR-pair mask, an SGPR operand)?
#define KERNEL_S(NAME, INS)                                                                              \
  __global__ void __launch_bounds__(256) NAME(unsigned* out, unsigned iters, unsigned seed) {           \
    unsigned a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, \
             a6 = a0 + 6, a7 = a0 + 7, k = seed * 3u + 1u;                                              \
    unsigned long long m = __ballot(threadIdx.x & 1);                                                   \
    unsigned sk = __builtin_amdgcn_readfirstlane(seed * 5u);                                            \
    for (unsigned i = 0; i < iters; ++i) {                                                               \
      C8S(INS) C8S(INS) C8S(INS) C8S(INS)                                                                \
    }                                                                                                    \
    unsigned s = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                                                 \
    if (s == 0x12345678u) out[blockIdx.x] = s;                                                           \
  }
#define C8S(INS)                                                                                         \
  asm volatile(INS : "+v"(a0) : "v"(k), "s"(m), "s"(sk)); asm volatile(INS : "+v"(a1) : "v"(k), "s"(m), "s"(sk)); \
  asm volatile(INS : "+v"(a2) : "v"(k), "s"(m), "s"(sk)); asm volatile(INS : "+v"(a3) : "v"(k), "s"(m), "s"(sk)); \
  asm volatile(INS : "+v"(a4) : "v"(k), "s"(m), "s"(sk)); asm volatile(INS : "+v"(a5) : "v"(k), "s"(m), "s"(sk)); \
  asm volatile(INS : "+v"(a6) : "v"(k), "s"(m), "s"(sk)); asm volatile(INS : "+v"(a7) : "v"(k), "s"(m), "s"(sk));
KERNEL_S(k_cnd_sgpr, "v_cndmask_b32_e64 %0, %0, %1, %2")
KERNEL_S(k_add_sgpr, "v_add_u32_e32 %0, %3, %0")
KERNEL_S(k_min_sgpr, "v_min_u32_e32 %0, %3, %0")
KERNEL_S(k_cnd_vcc_set, "s_mov_b64 vcc, %2\n v_cndmask_b32_e32 %0, %0, %1, vcc")
// mixes: 7 v_add + 1 mask select per 8 instructions
#define C8M(INS, SEL)                                                                                    \
  asm volatile(INS : "+v"(a0) : "v"(k), "s"(m), "s"(sk)); asm volatile(INS : "+v"(a1) : "v"(k), "s"(m), "s"(sk)); \
  asm volatile(INS : "+v"(a2) : "v"(k), "s"(m), "s"(sk)); asm volatile(INS : "+v"(a3) : "v"(k), "s"(m), "s"(sk)); \
  asm volatile(INS : "+v"(a4) : "v"(k), "s"(m), "s"(sk)); asm volatile(INS : "+v"(a5) : "v"(k), "s"(m), "s"(sk)); \
  asm volatile(INS : "+v"(a6) : "v"(k), "s"(m), "s"(sk)); asm volatile(SEL : "+v"(a7) : "v"(k), "s"(m), "s"(sk));
#define KERNEL_M(NAME, INS, SEL)                                                                         \
  __global__ void __launch_bounds__(256) NAME(unsigned* out, unsigned iters, unsigned seed) {           \
    unsigned a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, \
             a6 = a0 + 6, a7 = a0 + 7, k = seed * 3u + 1u;                                              \
    unsigned long long m = __ballot(threadIdx.x & 1);                                                   \
    unsigned sk = __builtin_amdgcn_readfirstlane(seed * 5u);                                            \
    for (unsigned i = 0; i < iters; ++i) {                                                               \
      C8M(INS, SEL) C8M(INS, SEL) C8M(INS, SEL) C8M(INS, SEL)                                            \
    }                                                                                                    \
    unsigned s = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                                                 \
    if (s == 0x12345678u) out[blockIdx.x] = s;                                                           \
  }
KERNEL_M(k_mix_add8, "v_add_u32_e32 %0, %0, %1", "v_add_u32_e32 %0, %0, %1")
KERNEL_M(k_mix_cndvcc, "v_add_u32_e32 %0, %0, %1", "v_cndmask_b32_e32 %0, %0, %1, vcc")
KERNEL_M(k_mix_cnds, "v_add_u32_e32 %0, %0, %1", "v_cndmask_b32_e64 %0, %0, %1, %2")
KERNEL_M(k_mix_addc, "v_add_u32_e32 %0, %0, %1", "v_addc_co_u32_e32 %0, vcc, %0, %1, vcc")
KERNEL_M(k_mix_sgpr, "v_add_u32_e32 %0, %0, %1", "v_add_u32_e32 %0, %3, %0")
KERNEL(k_add_co, "v_add_co_u32_e32 %0, vcc, %0, %1")
KERNEL(k_lshr_sdwa, "v_lshrrev_b32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1")

typedef void (*kfn)(unsigned*, unsigned, unsigned);

int main() {
  struct { const char* name; kfn f; int bytes; } ks[] = {
      {"v_add_u32_e32", k_add_e32, 4}, {"v_add_u32_e64", k_add_e64, 8}, {"v_add_u32_e32+literal", k_add_lit, 8},
      {"v_pk_add_u16", k_pk_add, 8},   {"v_or_b32_e32", k_or_e32, 4},   {"v_lshl_add_u32", k_lshl_add, 8},
      {"v_add3_u32", k_add3, 8},       {"v_min_u32", k_min_u32, 4},     {"v_max_u32", k_max_u32, 4},
      {"v_lshlrev_b32", k_lshl, 4},    {"v_lshrrev_b32", k_lshr, 4},    {"v_bfe_u32", k_bfe, 8},
      {"v_and_b32", k_and, 4},         {"v_xor_b32", k_xor, 4},         {"v_perm_b32", k_perm, 8},
      {"v_pk_min_u16", k_pk_min, 8},   {"v_pk_lshrrev_b16", k_pk_lshr, 8}, {"v_dot2_u32_u16", k_dot2, 8},
      {"v_mul_u32_u24", k_mul24, 4},   {"v_mad_u32_u24", k_mad24, 8},   {"v_min3_u32", k_min3, 8},
      {"v_and_or_b32", k_and_or, 8},   {"v_lshl_or_b32", k_lshl_or, 8}, {"v_alignbit_b32", k_alignbit, 8},
      {"v_mul_lo_u32", k_mul_lo, 8},   {"v_cvt_f32_u32", k_cvt_f32, 4}, {"v_mul_f32", k_mul_f32, 4},
      {"v_fma_f32", k_fma_f32, 8},     {"v_rcp_f32", k_rcp_f32, 4},
      {"v_cndmask_b32", k_cndmask, 4},
      {"v_add_u32_sdwa WORD_1", k_add_sdwa_w1, 8}, {"v_add_u32_sdwa WORD_0", k_add_sdwa_w0, 8},
      {"v_mad_u32_u16 op_sel hi", k_mad_u16_hi, 8}, {"v_mad_u32_u16", k_mad_u16, 8},
      {"v_and_b32 literal", k_and_const, 8},  {"v_lshrrev_b32_sdwa", k_lshr_sdwa, 8},
      {"v_cndmask_b32_e64 sgpr mask", k_cnd_sgpr, 8}, {"v_add_u32 sgpr operand", k_add_sgpr, 4},
      {"v_min_u32 sgpr operand", k_min_sgpr, 4}, {"s_mov vcc + v_cndmask (per op)", k_cnd_vcc_set, 8},
      {"mix 8 v_add", k_mix_add8, 4}, {"mix 7 v_add + 1 v_cndmask vcc", k_mix_cndvcc, 4},
      {"mix 7 v_add + 1 v_cndmask s-mask", k_mix_cnds, 4}, {"mix 7 v_add + 1 v_addc vcc", k_mix_addc, 4},
      {"mix 7 v_add + 1 v_add sgpr", k_mix_sgpr, 4}, {"v_add_co_u32 (writes vcc)", k_add_co, 4}};
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
  for (unsigned wps : {8u}) {  // waves per SIMD (4 waves per block, one block per SIMD-wave)
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
