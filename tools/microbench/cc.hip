// ChaCha20 block throughput on gfx950: ILP (1 vs 2 blocks per lane), and
// per-instruction rates of rotate candidates.
#include "../../noise-c_amd/csrc/aead_device.h"
#include <cstdio>
using namespace na;
constexpr int BLOCKS = 24;  // blocks per lane

template <int ILP>
__global__ __launch_bounds__(256) void cc_bench(uint32_t *sink, uint32_t seed) {
  uint32_t key[8]; for (int i = 0; i < 8; ++i) key[i] = seed * (i + 3) ^ threadIdx.x;
  uint32_t acc = 0;
  const uint32_t gt = blockIdx.x * 256 + threadIdx.x;
  for (int b = 0; b < BLOCKS; b += ILP) {
    uint32_t x[ILP][16];
#pragma unroll
    for (int j = 0; j < ILP; ++j) chacha20_block(key, b + j, 0, gt, 0, x[j]);
#pragma unroll
    for (int j = 0; j < ILP; ++j) for (int i = 0; i < 16; ++i) acc ^= x[j][i];
  }
  if (acc == 0x9abcdef1u) sink[gt] = acc;
}

// 2-block ChaCha with interleaved quarter rounds written explicitly
#define QR2(a,b,c,d,A,B,C,D) \
  a += b; A += B; d ^= a; D ^= A; d = rotl(d,16); D = rotl(D,16); \
  c += d; C += D; b ^= c; B ^= C; b = rotl(b,12); B = rotl(B,12); \
  a += b; A += B; d ^= a; D ^= A; d = rotl(d,8); D = rotl(D,8); \
  c += d; C += D; b ^= c; B ^= C; b = rotl(b,7); B = rotl(B,7)

#define X8(op) op " %0, %0, %8\n" op " %1, %1, %8\n" op " %2, %2, %8\n" op " %3, %3, %8\n" op " %4, %4, %8\n" op " %5, %5, %8\n" op " %6, %6, %8\n" op " %7, %7, %8\n"
#define K(NAME, ASM) \
__global__ void __launch_bounds__(256) NAME(uint32_t *o, uint32_t s) { \
  uint32_t a0=s+threadIdx.x,a1=a0*3,a2=a0*5,a3=a0*7,a4=a0*9,a5=a0*11,a6=a0*13,a7=a0*15; uint32_t m = s | 1; \
  for (int i = 0; i < 2048; ++i) asm volatile(ASM ASM ASM ASM : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(m)); \
  o[blockIdx.x*256+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7; }
K(k_pkaddu16, "v_pk_add_u16 %0, %0, %8 op_sel:[1,0] op_sel_hi:[0,1]\n v_pk_add_u16 %1, %1, %8 op_sel:[1,0] op_sel_hi:[0,1]\n v_pk_add_u16 %2, %2, %8 op_sel:[1,0] op_sel_hi:[0,1]\n v_pk_add_u16 %3, %3, %8 op_sel:[1,0] op_sel_hi:[0,1]\n v_pk_add_u16 %4, %4, %8 op_sel:[1,0] op_sel_hi:[0,1]\n v_pk_add_u16 %5, %5, %8 op_sel:[1,0] op_sel_hi:[0,1]\n v_pk_add_u16 %6, %6, %8 op_sel:[1,0] op_sel_hi:[0,1]\n v_pk_add_u16 %7, %7, %8 op_sel:[1,0] op_sel_hi:[0,1]\n")
K(k_lshl, X8("v_lshlrev_b32"))
K(k_or, X8("v_or_b32"))
K(k_xor_sdwa, "v_xor_b32_sdwa %0, %0, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n v_xor_b32_sdwa %1, %1, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n v_xor_b32_sdwa %2, %2, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n v_xor_b32_sdwa %3, %3, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n v_xor_b32_sdwa %4, %4, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n v_xor_b32_sdwa %5, %5, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n v_xor_b32_sdwa %6, %6, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n v_xor_b32_sdwa %7, %7, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n")
K(k_xad, "v_xad_u32 %0, %0, %8, %0\n v_xad_u32 %1, %1, %8, %1\n v_xad_u32 %2, %2, %8, %2\n v_xad_u32 %3, %3, %8, %3\n v_xad_u32 %4, %4, %8, %4\n v_xad_u32 %5, %5, %8, %5\n v_xad_u32 %6, %6, %8, %6\n v_xad_u32 %7, %7, %8, %7\n")
K(k_alignbit, "v_alignbit_b32 %0, %0, %0, 7\n v_alignbit_b32 %1, %1, %1, 7\n v_alignbit_b32 %2, %2, %2, 7\n v_alignbit_b32 %3, %3, %3, 7\n v_alignbit_b32 %4, %4, %4, 7\n v_alignbit_b32 %5, %5, %5, 7\n v_alignbit_b32 %6, %6, %6, 7\n v_alignbit_b32 %7, %7, %7, 7\n")
// mixed: 2 xor + 1 alignbit pattern like ChaCha
K(k_mix, "v_xor_b32 %0, %0, %8\n v_xor_b32 %1, %1, %8\n v_alignbit_b32 %2, %2, %2, 7\n v_add_u32 %3, %3, %8\n v_xor_b32 %4, %4, %8\n v_alignbit_b32 %5, %5, %5, 9\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n")

int main() {
  hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
  uint32_t *d; hipMalloc(&d, 1 << 26);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const int lanes = 65536 * 4;  // C2 K=4 lane count
  auto run = [&](auto k, const char *n, int grid, double work) {
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, d, 7u); hipDeviceSynchronize();
    hipEventRecord(e0); for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, d, 7u);
    hipEventRecord(e1); hipEventSynchronize(e1); float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("%-26s %9.2f us  %s\n", n, ms * 100, work > 0 ? "" : "");
    (void)work;
  };
  for (int rep = 0; rep < 2; ++rep) {
    run(cc_bench<1>, "chacha ILP1 (24 blk/lane)", lanes / 256, 0);
    run(cc_bench<2>, "chacha ILP2 (24 blk/lane)", lanes / 256, 0);
    run(cc_bench<1>, "chacha ILP1 half lanes", lanes / 512, 0);
    run(cc_bench<2>, "chacha ILP2 half lanes", lanes / 512, 0);
  }
  int blocks = p.multiProcessorCount * 8;
  run(k_alignbit, "rate alignbit", blocks, 0); run(k_pkaddu16, "rate pk_add_u16 opsel", blocks, 0);
  run(k_lshl, "rate lshlrev", blocks, 0); run(k_or, "rate or", blocks, 0); run(k_xor_sdwa, "rate xor_sdwa", blocks, 0);
  run(k_xad, "rate xad_u32", blocks, 0); run(k_mix, "rate mix 5full+2align", blocks, 0);
  return 0;
}
