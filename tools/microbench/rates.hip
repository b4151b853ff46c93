// Per-instruction VALU throughput on gfx950 (inline asm, 8 independent chains,
// 8 waves/SIMD) to price the AEAD kernels' instruction mix.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
constexpr int IT = 2048;
#define BODY8(S) S(0) S(1) S(2) S(3) S(4) S(5) S(6) S(7)
#define K(NAME, ASM)                                                              \
__global__ void __launch_bounds__(256) NAME(uint32_t *o, uint32_t s) {           \
  uint32_t a0=s+threadIdx.x,a1=a0*3,a2=a0*5,a3=a0*7,a4=a0*9,a5=a0*11,a6=a0*13,a7=a0*15; \
  uint32_t m = s | 1;                                                             \
  for (int i = 0; i < IT; ++i) {                                                 \
    asm volatile(ASM ASM ASM ASM : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(m)); \
  }                                                                               \
  o[blockIdx.x*256+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;                        \
}
#define X8(op) op " %0, %0, %8\n" op " %1, %1, %8\n" op " %2, %2, %8\n" op " %3, %3, %8\n" op " %4, %4, %8\n" op " %5, %5, %8\n" op " %6, %6, %8\n" op " %7, %7, %8\n"
#define X8_3(op) op " %0, %0, %8, %0\n" op " %1, %1, %8, %1\n" op " %2, %2, %8, %2\n" op " %3, %3, %8, %3\n" op " %4, %4, %8, %4\n" op " %5, %5, %8, %5\n" op " %6, %6, %8, %6\n" op " %7, %7, %8, %7\n"
#define AL8 "v_alignbit_b32 %0, %0, %0, 7\n" "v_alignbit_b32 %1, %1, %1, 7\n" "v_alignbit_b32 %2, %2, %2, 7\n" "v_alignbit_b32 %3, %3, %3, 7\n" "v_alignbit_b32 %4, %4, %4, 7\n" "v_alignbit_b32 %5, %5, %5, 7\n" "v_alignbit_b32 %6, %6, %6, 7\n" "v_alignbit_b32 %7, %7, %7, 7\n"
K(k_xor, X8("v_xor_b32"))
K(k_add, X8("v_add_u32"))
K(k_addf, X8("v_add_f32"))
K(k_align, AL8)
K(k_add3, X8_3("v_add3_u32"))
K(k_perm, X8_3("v_perm_b32"))
K(k_mullo, X8("v_mul_lo_u32"))
K(k_mul24, X8("v_mul_u32_u24"))
K(k_bitop3, "v_bitop3_b32 %0, %0, %8, %0 bitop3:0x96\n" "v_bitop3_b32 %1, %1, %8, %1 bitop3:0x96\n" "v_bitop3_b32 %2, %2, %8, %2 bitop3:0x96\n" "v_bitop3_b32 %3, %3, %8, %3 bitop3:0x96\n" "v_bitop3_b32 %4, %4, %8, %4 bitop3:0x96\n" "v_bitop3_b32 %5, %5, %8, %5 bitop3:0x96\n" "v_bitop3_b32 %6, %6, %8, %6 bitop3:0x96\n" "v_bitop3_b32 %7, %7, %8, %7 bitop3:0x96\n")

K(k_sdwa, "v_xor_b32_sdwa %0, %0, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n" "v_xor_b32_sdwa %1, %1, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n" "v_xor_b32_sdwa %2, %2, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n" "v_xor_b32_sdwa %3, %3, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n" "v_xor_b32_sdwa %4, %4, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n" "v_xor_b32_sdwa %5, %5, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n" "v_xor_b32_sdwa %6, %6, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n" "v_xor_b32_sdwa %7, %7, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n")
K(k_lshl, X8("v_lshlrev_b32"))
K(k_lshlor, X8_3("v_lshl_or_b32"))
K(k_lshladd, X8_3("v_lshl_add_u32"))
K(k_xad, X8_3("v_xad_u32"))
K(k_andor, X8_3("v_and_or_b32"))
K(k_or3, X8_3("v_or3_b32"))
K(k_bfe, X8_3("v_bfe_u32"))
K(k_alignbyte, X8_3("v_alignbyte_b32"))
K(k_and, X8("v_and_b32"))
K(k_xor_e64, X8("v_xor_b32_e64"))
K(k_mix_xa, "v_xor_b32 %0, %0, %8\n v_alignbit_b32 %1, %1, %1, 7\n v_xor_b32 %2, %2, %8\n v_alignbit_b32 %3, %3, %3, 7\n v_xor_b32 %4, %4, %8\n v_alignbit_b32 %5, %5, %5, 7\n v_xor_b32 %6, %6, %8\n v_alignbit_b32 %7, %7, %7, 7\n")
K(k_mix_xxa, "v_xor_b32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_alignbit_b32 %2, %2, %2, 7\n v_xor_b32 %3, %3, %8\n v_add_u32 %4, %4, %8\n v_alignbit_b32 %5, %5, %5, 7\n v_xor_b32 %6, %6, %8\n v_add_u32 %7, %7, %8\n")
// packed fp32 add on register pairs: a0:a1 ... 4 instr per body line
__global__ void __launch_bounds__(256) k_pkadd(uint32_t *o, uint32_t s) {
  float a[8]; for (int i=0;i<8;++i) a[i]=s+threadIdx.x*i;
  float m = s*0.5f;
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 x0={a[0],a[1]},x1={a[2],a[3]},x2={a[4],a[5]},x3={a[6],a[7]}; f2 mm={m,m};
  for (int i=0;i<IT;++i) {
    asm volatile("v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4\n"
                 "v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4\n"
                 "v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4\n"
                 "v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4\n"
                 "v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4\n"
                 "v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4\n"
                 "v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4\n"
                 "v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4\n"
                 : "+v"(x0),"+v"(x1),"+v"(x2),"+v"(x3) : "v"(mm));
  }
  o[blockIdx.x*256+threadIdx.x] = (uint32_t)(x0.x+x1.x+x2.x+x3.x+x0.y+x1.y+x2.y+x3.y);
}
// 64-bit ops
__global__ void __launch_bounds__(256) k_mad64(uint32_t *o, uint32_t s) {
  uint64_t a0=s+threadIdx.x,a1=a0*3,a2=a0*5,a3=a0*7; uint32_t m=s|1, b=threadIdx.x;
  for (int i=0;i<IT;++i) {
    asm volatile(
      "v_mad_u64_u32 %0, s[80:81], %4, %5, %0\n v_mad_u64_u32 %1, s[80:81], %4, %5, %1\n v_mad_u64_u32 %2, s[80:81], %4, %5, %2\n v_mad_u64_u32 %3, s[80:81], %4, %5, %3\n"
      "v_mad_u64_u32 %0, s[80:81], %4, %5, %0\n v_mad_u64_u32 %1, s[80:81], %4, %5, %1\n v_mad_u64_u32 %2, s[80:81], %4, %5, %2\n v_mad_u64_u32 %3, s[80:81], %4, %5, %3\n"
      "v_mad_u64_u32 %0, s[80:81], %4, %5, %0\n v_mad_u64_u32 %1, s[80:81], %4, %5, %1\n v_mad_u64_u32 %2, s[80:81], %4, %5, %2\n v_mad_u64_u32 %3, s[80:81], %4, %5, %3\n"
      "v_mad_u64_u32 %0, s[80:81], %4, %5, %0\n v_mad_u64_u32 %1, s[80:81], %4, %5, %1\n v_mad_u64_u32 %2, s[80:81], %4, %5, %2\n v_mad_u64_u32 %3, s[80:81], %4, %5, %3\n"
      "v_mad_u64_u32 %0, s[80:81], %4, %5, %0\n v_mad_u64_u32 %1, s[80:81], %4, %5, %1\n v_mad_u64_u32 %2, s[80:81], %4, %5, %2\n v_mad_u64_u32 %3, s[80:81], %4, %5, %3\n"
      "v_mad_u64_u32 %0, s[80:81], %4, %5, %0\n v_mad_u64_u32 %1, s[80:81], %4, %5, %1\n v_mad_u64_u32 %2, s[80:81], %4, %5, %2\n v_mad_u64_u32 %3, s[80:81], %4, %5, %3\n"
      "v_mad_u64_u32 %0, s[80:81], %4, %5, %0\n v_mad_u64_u32 %1, s[80:81], %4, %5, %1\n v_mad_u64_u32 %2, s[80:81], %4, %5, %2\n v_mad_u64_u32 %3, s[80:81], %4, %5, %3\n"
      "v_mad_u64_u32 %0, s[80:81], %4, %5, %0\n v_mad_u64_u32 %1, s[80:81], %4, %5, %1\n v_mad_u64_u32 %2, s[80:81], %4, %5, %2\n v_mad_u64_u32 %3, s[80:81], %4, %5, %3\n"
      : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3) : "v"(m), "v"(b) : "s80","s81");
  }
  o[blockIdx.x*256+threadIdx.x] = (uint32_t)(a0^a1^a2^a3);
}
__global__ void __launch_bounds__(256) k_shr64(uint32_t *o, uint32_t s) {
  uint64_t a0=s+threadIdx.x,a1=a0*3,a2=a0*5,a3=a0*7;
  for (int i=0;i<IT;++i) {
    asm volatile(
      "v_lshrrev_b64 %0, 1, %0\n v_lshrrev_b64 %1, 1, %1\n v_lshrrev_b64 %2, 1, %2\n v_lshrrev_b64 %3, 1, %3\n"
      "v_lshrrev_b64 %0, 1, %0\n v_lshrrev_b64 %1, 1, %1\n v_lshrrev_b64 %2, 1, %2\n v_lshrrev_b64 %3, 1, %3\n"
      "v_lshrrev_b64 %0, 1, %0\n v_lshrrev_b64 %1, 1, %1\n v_lshrrev_b64 %2, 1, %2\n v_lshrrev_b64 %3, 1, %3\n"
      "v_lshrrev_b64 %0, 1, %0\n v_lshrrev_b64 %1, 1, %1\n v_lshrrev_b64 %2, 1, %2\n v_lshrrev_b64 %3, 1, %3\n"
      "v_lshrrev_b64 %0, 1, %0\n v_lshrrev_b64 %1, 1, %1\n v_lshrrev_b64 %2, 1, %2\n v_lshrrev_b64 %3, 1, %3\n"
      "v_lshrrev_b64 %0, 1, %0\n v_lshrrev_b64 %1, 1, %1\n v_lshrrev_b64 %2, 1, %2\n v_lshrrev_b64 %3, 1, %3\n"
      "v_lshrrev_b64 %0, 1, %0\n v_lshrrev_b64 %1, 1, %1\n v_lshrrev_b64 %2, 1, %2\n v_lshrrev_b64 %3, 1, %3\n"
      "v_lshrrev_b64 %0, 1, %0\n v_lshrrev_b64 %1, 1, %1\n v_lshrrev_b64 %2, 1, %2\n v_lshrrev_b64 %3, 1, %3\n"
      : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3));
  }
  o[blockIdx.x*256+threadIdx.x] = (uint32_t)(a0^a1^a2^a3);
}
int main() {
  hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
  int blocks = p.multiProcessorCount * 8;   // 8 x 256 threads = 32 waves/CU = 8/SIMD
  uint32_t *d; hipMalloc(&d, blocks*256*4);
  hipEvent_t e0,e1; hipEventCreate(&e0); hipEventCreate(&e1);
  auto run=[&](auto k, const char *n, double instr_per_iter){
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 3u); hipDeviceSynchronize();
    hipEventRecord(e0); for(int r=0;r<5;++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 3u);
    hipEventRecord(e1); hipEventSynchronize(e1); float ms; hipEventElapsedTime(&ms,e0,e1);
    double wi = 5.0*blocks*4.0*IT*instr_per_iter;   // wave-instructions
    double cyc_per = (ms*1e-3)*2.4e9*p.multiProcessorCount*4/wi; // SIMD-cycles per wave-instr at 2.4 GHz
    printf("%-14s %8.3f ms  %6.2f T lane-instr/s  %5.2f SIMD-cycles/wave-instr(@2.4GHz)\n", n, ms, wi*64/(ms*1e-3)/1e12, cyc_per);
  };
  run(k_xor,"v_xor_b32",32); run(k_add,"v_add_u32",32); run(k_addf,"v_add_f32",32); run(k_align,"v_alignbit",32);
  run(k_add3,"v_add3_u32",32); run(k_perm,"v_perm_b32",32); run(k_bitop3,"v_bitop3_b32",32); run(k_mullo,"v_mul_lo_u32",32);
  run(k_mul24,"v_mul_u32_u24",32);
  run(k_sdwa,"v_xor_sdwa",32); run(k_lshl,"v_lshlrev_b32",32); run(k_lshlor,"v_lshl_or_b32",32); run(k_lshladd,"v_lshl_add_u32",32);
  run(k_xad,"v_xad_u32",32); run(k_andor,"v_and_or_b32",32); run(k_or3,"v_or3_b32",32); run(k_bfe,"v_bfe_u32",32);
  run(k_alignbyte,"v_alignbyte",32); run(k_and,"v_and_b32",32); run(k_xor_e64,"v_xor_b32_e64",32);
  run(k_mix_xa,"mix xor/align",32); run(k_mix_xxa,"mix xor/add/al",32); run(k_pkadd,"v_pk_add_f32",32); run(k_mad64,"v_mad_u64_u32",32); run(k_shr64,"v_lshrrev_b64",32);
  return 0;
}
