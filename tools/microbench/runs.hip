// Does the gfx950 fast-class VALU rate (v_xor/v_add/v_bitop3 ~2.3 cycles) survive
// in longer runs between slow-class ops, or when fast and slow ops come from
// different waves of the same SIMD?  And which 16-bit packed ops are fast
// (candidates for a rotate-by-16 that does not leave the fast class).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
constexpr int IT = 1024;
#define X8(op) op " %0, %0, %8\n" op " %1, %1, %8\n" op " %2, %2, %8\n" op " %3, %3, %8\n" op " %4, %4, %8\n" op " %5, %5, %8\n" op " %6, %6, %8\n" op " %7, %7, %8\n"
#define AL8 "v_alignbit_b32 %0, %0, %0, 7\n" "v_alignbit_b32 %1, %1, %1, 7\n" "v_alignbit_b32 %2, %2, %2, 7\n" "v_alignbit_b32 %3, %3, %3, 7\n" "v_alignbit_b32 %4, %4, %4, 7\n" "v_alignbit_b32 %5, %5, %5, 7\n" "v_alignbit_b32 %6, %6, %6, 7\n" "v_alignbit_b32 %7, %7, %7, 7\n"
#define PK8(op, mods) op " %0, %0, 0 " mods "\n" op " %1, %1, 0 " mods "\n" op " %2, %2, 0 " mods "\n" op " %3, %3, 0 " mods "\n" op " %4, %4, 0 " mods "\n" op " %5, %5, 0 " mods "\n" op " %6, %6, 0 " mods "\n" op " %7, %7, 0 " mods "\n"
#define F32 X8("v_xor_b32") X8("v_add_u32") X8("v_xor_b32") X8("v_add_u32")
#define S32 AL8 AL8 AL8 AL8
#define OPS "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(m)
#define K(NAME, BODY)                                                             \
__global__ void __launch_bounds__(256) NAME(uint32_t *o, uint32_t s) {           \
  uint32_t a0=s+threadIdx.x,a1=a0*3,a2=a0*5,a3=a0*7,a4=a0*9,a5=a0*11,a6=a0*13,a7=a0*15; \
  uint32_t m = s | 1;                                                             \
  for (int i = 0; i < IT; ++i) { BODY }                                           \
  o[blockIdx.x*256+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;                        \
}
// 128 instructions per iteration in every kernel
K(k_fast, asm volatile(F32 F32 F32 F32 : OPS);)
K(k_slow, asm volatile(S32 S32 S32 S32 : OPS);)
K(k_run8, asm volatile(X8("v_xor_b32") AL8 X8("v_add_u32") AL8 X8("v_xor_b32") AL8 X8("v_add_u32") AL8
                       X8("v_xor_b32") AL8 X8("v_add_u32") AL8 X8("v_xor_b32") AL8 X8("v_add_u32") AL8 : OPS);)
K(k_run32, asm volatile(F32 S32 F32 S32 : OPS);)
K(k_run64, asm volatile(F32 F32 S32 S32 : OPS);)
K(k_2to1, asm volatile(X8("v_xor_b32") X8("v_add_u32") AL8 X8("v_xor_b32") X8("v_add_u32") AL8
                       X8("v_xor_b32") X8("v_add_u32") AL8 X8("v_xor_b32") X8("v_add_u32") AL8
                       X8("v_xor_b32") X8("v_add_u32") AL8 X8("v_xor_b32") X8("v_add_u32") X8("v_xor_b32") X8("v_add_u32") : OPS);)
// wave specialisation: even waves fast-only, odd waves slow-only (same SIMD mix)
K(k_spec, if ((threadIdx.x >> 6) & 1) { asm volatile(S32 S32 S32 S32 : OPS); } else { asm volatile(F32 F32 F32 F32 : OPS); })
// packed 16-bit candidates: v_pk_add_u16 with op_sel swapping the halves = rotl 16
K(k_pkswap, asm volatile(PK8("v_pk_add_u16", "op_sel:[1,0] op_sel_hi:[0,1]") PK8("v_pk_add_u16", "op_sel:[1,0] op_sel_hi:[0,1]")
                         PK8("v_pk_add_u16", "op_sel:[1,0] op_sel_hi:[0,1]") PK8("v_pk_add_u16", "op_sel:[1,0] op_sel_hi:[0,1]")
                         PK8("v_pk_add_u16", "op_sel:[1,0] op_sel_hi:[0,1]") PK8("v_pk_add_u16", "op_sel:[1,0] op_sel_hi:[0,1]")
                         PK8("v_pk_add_u16", "op_sel:[1,0] op_sel_hi:[0,1]") PK8("v_pk_add_u16", "op_sel:[1,0] op_sel_hi:[0,1]")
                         PK8("v_pk_add_u16", "op_sel:[1,0] op_sel_hi:[0,1]") PK8("v_pk_add_u16", "op_sel:[1,0] op_sel_hi:[0,1]")
                         PK8("v_pk_add_u16", "op_sel:[1,0] op_sel_hi:[0,1]") PK8("v_pk_add_u16", "op_sel:[1,0] op_sel_hi:[0,1]")
                         PK8("v_pk_add_u16", "op_sel:[1,0] op_sel_hi:[0,1]") PK8("v_pk_add_u16", "op_sel:[1,0] op_sel_hi:[0,1]")
                         PK8("v_pk_add_u16", "op_sel:[1,0] op_sel_hi:[0,1]") PK8("v_pk_add_u16", "op_sel:[1,0] op_sel_hi:[0,1]") : OPS);)
K(k_pkadd16, asm volatile(X8("v_pk_add_u16") X8("v_pk_add_u16") X8("v_pk_add_u16") X8("v_pk_add_u16")
                          X8("v_pk_add_u16") X8("v_pk_add_u16") X8("v_pk_add_u16") X8("v_pk_add_u16")
                          X8("v_pk_add_u16") X8("v_pk_add_u16") X8("v_pk_add_u16") X8("v_pk_add_u16")
                          X8("v_pk_add_u16") X8("v_pk_add_u16") X8("v_pk_add_u16") X8("v_pk_add_u16") : OPS);)
K(k_or, asm volatile(X8("v_or_b32") X8("v_or_b32") X8("v_or_b32") X8("v_or_b32") X8("v_or_b32") X8("v_or_b32") X8("v_or_b32") X8("v_or_b32")
                     X8("v_or_b32") X8("v_or_b32") X8("v_or_b32") X8("v_or_b32") X8("v_or_b32") X8("v_or_b32") X8("v_or_b32") X8("v_or_b32") : OPS);)
K(k_sub, asm volatile(X8("v_sub_u32") X8("v_sub_u32") X8("v_sub_u32") X8("v_sub_u32") X8("v_sub_u32") X8("v_sub_u32") X8("v_sub_u32") X8("v_sub_u32")
                      X8("v_sub_u32") X8("v_sub_u32") X8("v_sub_u32") X8("v_sub_u32") X8("v_sub_u32") X8("v_sub_u32") X8("v_sub_u32") X8("v_sub_u32") : OPS);)
K(k_cndmask_free, asm volatile(X8("v_max_u32") X8("v_max_u32") X8("v_max_u32") X8("v_max_u32") X8("v_max_u32") X8("v_max_u32") X8("v_max_u32") X8("v_max_u32")
                               X8("v_max_u32") X8("v_max_u32") X8("v_max_u32") X8("v_max_u32") X8("v_max_u32") X8("v_max_u32") X8("v_max_u32") X8("v_max_u32") : OPS);)

int main() {
  hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  uint32_t *d; hipMalloc(&d, p.multiProcessorCount * 8 * 256 * 4);
  auto run = [&](auto k, const char *n, int waves_per_simd) {
    int blocks = p.multiProcessorCount * waves_per_simd;  // 256 threads = 1 wave per SIMD
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 3u); hipDeviceSynchronize();
    hipEventRecord(e0); for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 3u);
    hipEventRecord(e1); hipEventSynchronize(e1); float ms; hipEventElapsedTime(&ms, e0, e1);
    double wi = 5.0 * blocks * 4.0 * IT * 128;
    double cyc = (ms * 1e-3) * 2.4e9 * p.multiProcessorCount * 4 / wi;
    printf("%-12s waves/SIMD %d  %7.3f ms  %5.2f SIMD-cycles/wave-instr(@2.4GHz)\n", n, waves_per_simd, ms, cyc);
  };
  for (int w : {2, 8}) {
    run(k_fast, "fast", w); run(k_slow, "slow", w); run(k_run8, "runs8", w); run(k_run32, "runs32", w);
    run(k_run64, "runs64", w); run(k_2to1, "2:1 runs8/16", w); run(k_spec, "wave-spec", w);
    run(k_pkswap, "pk_add_u16 sw", w); run(k_pkadd16, "pk_add_u16", w); run(k_or, "v_or_b32", w);
    run(k_sub, "v_sub_u32", w); run(k_cndmask_free, "v_max_u32", w);
  }
  return 0;
}
