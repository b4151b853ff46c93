// ChaCha20 block throughput on gfx950 by rotate encoding, at 1..8 waves/SIMD.
// Each lane runs NB independent ChaCha20 blocks (register-resident, no memory
// in the loop); reports SIMD-cycles per wave-block at 2.4 GHz and the kernel's
// effective rate.  Variants:
//   0 alignbit  : every rotate is v_alignbit_b32 (what hipcc emits for rotl)
//   1 sdwa16    : d ^= a; d <<<= 16 as two v_xor_b32_sdwa word moves
//   2 perm      : <<<16 and <<<8 as v_perm_b32 (byte permutes)
//   3 sdwa16+perm8
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint32_t rotl_ab(uint32_t x, int n) {
  return __builtin_amdgcn_alignbit(x, x, 32 - n);
}
__device__ __forceinline__ uint32_t xor_rot16_sdwa(uint32_t d, uint32_t a) {
  uint32_t t;
  asm volatile("v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\n"
               "v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1"
               : "=&v"(t) : "v"(d), "v"(a));
  return t;
}
__device__ __forceinline__ uint32_t rot16_perm(uint32_t x) { return __builtin_amdgcn_perm(x, x, 0x01000302u); }
__device__ __forceinline__ uint32_t rot8_perm(uint32_t x) { return __builtin_amdgcn_perm(x, x, 0x02010003u); }

template <int V>
__device__ __forceinline__ void qr(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d) {
  a += b;
  if (V == 1 || V == 3) d = xor_rot16_sdwa(d, a);
  else if (V == 2) { d ^= a; d = rot16_perm(d); }
  else { d ^= a; d = rotl_ab(d, 16); }
  c += d; b ^= c; b = rotl_ab(b, 12);
  a += b; d ^= a;
  if (V >= 2) d = rot8_perm(d); else d = rotl_ab(d, 8);
  c += d; b ^= c; b = rotl_ab(b, 7);
}

template <int V>
__device__ __forceinline__ void block(uint32_t x[16]) {
  uint32_t s[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) s[i] = x[i];
#pragma unroll 1
  for (int r = 0; r < 10; ++r) {
    qr<V>(s[0], s[4], s[8], s[12]); qr<V>(s[1], s[5], s[9], s[13]);
    qr<V>(s[2], s[6], s[10], s[14]); qr<V>(s[3], s[7], s[11], s[15]);
    qr<V>(s[0], s[5], s[10], s[15]); qr<V>(s[1], s[6], s[11], s[12]);
    qr<V>(s[2], s[7], s[8], s[13]); qr<V>(s[3], s[4], s[9], s[14]);
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] += s[i];
}

constexpr int NB = 64;  // blocks per lane
template <int V>
__global__ void __launch_bounds__(256) kchacha(uint32_t *o, uint32_t seed) {
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = seed * (i + 1) + threadIdx.x + blockIdx.x * 977u;
  uint32_t acc = 0;
  for (int b = 0; b < NB; ++b) {
    block<V>(x);
    acc ^= x[0] ^ x[7];
    x[12] += 1;
  }
  o[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
  hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  uint32_t *d; hipMalloc(&d, (size_t)cus * 8 * 256 * 4);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  // reference check: all variants must produce the same words
  uint32_t h[4][256];
  auto run = [&](auto k, const char *name, int vi) {
    for (int w = 1; w <= 8; w *= 2) {
      int blocks = cus * w;   // 256 threads = 1 wave per SIMD per block
      hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 5u); hipDeviceSynchronize();
      hipEventRecord(e0);
      for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 5u);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      double wave_blocks = 3.0 * blocks * 4 * NB;
      double cyc = (ms * 1e-3) * 2.4e9 * cus * 4 / wave_blocks;
      double gbs = wave_blocks * 64 * 64 / (ms * 1e-3) / 1e9;
      printf("%-14s waves/SIMD %d  %7.1f SIMD-cyc/wave-block(@2.4GHz)  %7.0f GB/s keystream\n", name, w, cyc, gbs);
    }
    hipMemcpy(h[vi], d, 256 * 4, hipMemcpyDeviceToHost);
  };
  run(kchacha<0>, "alignbit", 0);
  run(kchacha<1>, "sdwa16", 1);
  run(kchacha<2>, "perm16+8", 2);
  run(kchacha<3>, "sdwa16+perm8", 3);
  int ok = 1;
  for (int v = 1; v < 4; ++v) for (int i = 0; i < 256; ++i) ok &= h[v][i] == h[0][i];
  printf("variants agree: %s\n", ok ? "yes" : "NO");
  return 0;
}
