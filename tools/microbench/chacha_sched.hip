// ChaCha20 double-round instruction ORDER on gfx950, at 1..8 waves/SIMD.
// gfx950 issues v_add_u32 / v_xor_b32 / v_and_b32 / v_bitop3_b32 in ~2.4
// SIMD-cycles per wave-instruction but v_alignbit_b32 (and every other
// shift/permute/3-operand integer op) in ~4.1, and an alternating fast/slow
// stream runs near 4 for every instruction (tools/microbench/rates.hip).
// This measures whole ChaCha20 blocks with the double round written in
// inline asm in different orders:
//   0 compiler : plain C++ quarter rounds, hipcc's schedule
//   1 grouped  : per half round, the 4 independent QRs advance in lock step:
//                4 add, 4 xor, 4 rotate, ... (runs of 8 fast then 4 slow)
//   2 serial   : one QR at a time, 12 dependent instructions
//   3 grouped2 : like 1 but two rotate groups merged: 8 fast, 4 slow, 4 fast ...
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define S_(x) #x
#define S(x) S_(x)
#define ADD(a, b) "v_add_u32 %" S(a) ", %" S(a) ", %" S(b) "\n"
#define XOR(d, a) "v_xor_b32 %" S(d) ", %" S(d) ", %" S(a) "\n"
#define ROT(d, n) "v_alignbit_b32 %" S(d) ", %" S(d) ", %" S(d) ", " S(n) "\n"
// rotl by r == alignbit by 32-r
#define STEP4(A0, B0, A1, B1, A2, B2, A3, B3, D0, D1, D2, D3, R)           \
  ADD(A0, B0) ADD(A1, B1) ADD(A2, B2) ADD(A3, B3)                           \
  XOR(D0, A0) XOR(D1, A1) XOR(D2, A2) XOR(D3, A3)                           \
  ROT(D0, R) ROT(D1, R) ROT(D2, R) ROT(D3, R)
#define HALF_G(a0, b0, c0, d0, a1, b1, c1, d1, a2, b2, c2, d2, a3, b3, c3, d3) \
  STEP4(a0, b0, a1, b1, a2, b2, a3, b3, d0, d1, d2, d3, 16)                    \
  STEP4(c0, d0, c1, d1, c2, d2, c3, d3, b0, b1, b2, b3, 20)                    \
  STEP4(a0, b0, a1, b1, a2, b2, a3, b3, d0, d1, d2, d3, 24)                    \
  STEP4(c0, d0, c1, d1, c2, d2, c3, d3, b0, b1, b2, b3, 25)
#define QR_S(a, b, c, d)                                                        \
  ADD(a, b) XOR(d, a) ROT(d, 16) ADD(c, d) XOR(b, c) ROT(b, 20)                 \
  ADD(a, b) XOR(d, a) ROT(d, 24) ADD(c, d) XOR(b, c) ROT(b, 25)
#define HALF_S(a0, b0, c0, d0, a1, b1, c1, d1, a2, b2, c2, d2, a3, b3, c3, d3) \
  QR_S(a0, b0, c0, d0) QR_S(a1, b1, c1, d1) QR_S(a2, b2, c2, d2) QR_S(a3, b3, c3, d3)
// variant 3: rotates of step k issued after the adds of step k+1 that do not
// depend on them (c += d needs the rotated d, so only the b-side overlaps):
// per step: 4 add | 4 xor | 4 rot ; this variant pairs each 4-rot group with
// the next step's independent 4 adds to give runs of 4 slow + 4 fast.
#define STEP4_NOROT(A0, B0, A1, B1, A2, B2, A3, B3, D0, D1, D2, D3)         \
  ADD(A0, B0) ADD(A1, B1) ADD(A2, B2) ADD(A3, B3)                           \
  XOR(D0, A0) XOR(D1, A1) XOR(D2, A2) XOR(D3, A3)
#define ROT4(D0, D1, D2, D3, R) ROT(D0, R) ROT(D1, R) ROT(D2, R) ROT(D3, R)

#define OPS16                                                                  \
  "+v"(s[0]), "+v"(s[1]), "+v"(s[2]), "+v"(s[3]), "+v"(s[4]), "+v"(s[5]),      \
      "+v"(s[6]), "+v"(s[7]), "+v"(s[8]), "+v"(s[9]), "+v"(s[10]), "+v"(s[11]), \
      "+v"(s[12]), "+v"(s[13]), "+v"(s[14]), "+v"(s[15])

__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }
#define QRC(a, b, c, d)                  \
  a += b; d ^= a; d = rotl(d, 16);       \
  c += d; b ^= c; b = rotl(b, 12);       \
  a += b; d ^= a; d = rotl(d, 8);        \
  c += d; b ^= c; b = rotl(b, 7)

template <int V>
__device__ __forceinline__ void dround(uint32_t s[16]) {
  if (V == 0) {
    QRC(s[0], s[4], s[8], s[12]); QRC(s[1], s[5], s[9], s[13]);
    QRC(s[2], s[6], s[10], s[14]); QRC(s[3], s[7], s[11], s[15]);
    QRC(s[0], s[5], s[10], s[15]); QRC(s[1], s[6], s[11], s[12]);
    QRC(s[2], s[7], s[8], s[13]); QRC(s[3], s[4], s[9], s[14]);
  } else if (V == 1) {
    asm volatile(HALF_G(0, 4, 8, 12, 1, 5, 9, 13, 2, 6, 10, 14, 3, 7, 11, 15)
                 HALF_G(0, 5, 10, 15, 1, 6, 11, 12, 2, 7, 8, 13, 3, 4, 9, 14) : OPS16);
  } else if (V == 2) {
    asm volatile(HALF_S(0, 4, 8, 12, 1, 5, 9, 13, 2, 6, 10, 14, 3, 7, 11, 15)
                 HALF_S(0, 5, 10, 15, 1, 6, 11, 12, 2, 7, 8, 13, 3, 4, 9, 14) : OPS16);
  } else {
    // two half-QR groups interleaved: rotates of QRs 0,1 between fast ops of QRs 2,3
    asm volatile(
#define HALF_I(a0, b0, c0, d0, a1, b1, c1, d1, a2, b2, c2, d2, a3, b3, c3, d3)                  \
  ADD(a0, b0) ADD(a1, b1) XOR(d0, a0) XOR(d1, a1) ADD(a2, b2) ADD(a3, b3) ROT(d0, 16) ROT(d1, 16) \
  XOR(d2, a2) XOR(d3, a3) ADD(c0, d0) ADD(c1, d1) ROT(d2, 16) ROT(d3, 16) XOR(b0, c0) XOR(b1, c1) \
  ADD(c2, d2) ADD(c3, d3) ROT(b0, 20) ROT(b1, 20) XOR(b2, c2) XOR(b3, c3) ADD(a0, b0) ADD(a1, b1) \
  ROT(b2, 20) ROT(b3, 20) XOR(d0, a0) XOR(d1, a1) ADD(a2, b2) ADD(a3, b3) ROT(d0, 24) ROT(d1, 24) \
  XOR(d2, a2) XOR(d3, a3) ADD(c0, d0) ADD(c1, d1) ROT(d2, 24) ROT(d3, 24) XOR(b0, c0) XOR(b1, c1) \
  ADD(c2, d2) ADD(c3, d3) ROT(b0, 25) ROT(b1, 25) XOR(b2, c2) XOR(b3, c3) ROT(b2, 25) ROT(b3, 25)
        HALF_I(0, 4, 8, 12, 1, 5, 9, 13, 2, 6, 10, 14, 3, 7, 11, 15)
        HALF_I(0, 5, 10, 15, 1, 6, 11, 12, 2, 7, 8, 13, 3, 4, 9, 14) : OPS16);
  }
}

constexpr int NB = 64;
template <int V, int SYNC = 0, int BS = 256>
__global__ void __launch_bounds__(BS) kchacha(uint32_t *o, uint32_t seed) {
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = seed * (i + 1) + threadIdx.x + blockIdx.x * 977u;
  uint32_t acc = 0;
  for (int b = 0; b < NB; ++b) {
    uint32_t s[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) s[i] = x[i];
#pragma unroll 2
    for (int r = 0; r < 10; ++r) {
      dround<V>(s);
      if (SYNC) __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) acc ^= s[i] + x[i];
    x[12] += 1;
  }
  o[blockIdx.x * BS + threadIdx.x] = acc;
}

int main() {
  hipDeviceProp_t p; (void)hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  uint32_t *d; (void)hipMalloc(&d, (size_t)cus * 8 * 256 * 4);
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  uint32_t h[4][256];
  const char *names[] = {"compiler", "grouped 8f/4s", "serial QR", "interleave 2f/2s"};
  auto run = [&](auto k, int vi) {
    for (int w = 1; w <= 8; w *= 2) {
      int blocks = cus * w;
      hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 5u); (void)hipDeviceSynchronize();
      (void)hipEventRecord(e0);
      for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 5u);
      (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
      float ms; (void)hipEventElapsedTime(&ms, e0, e1);
      double wave_blocks = 3.0 * blocks * 4 * NB;
      double cyc = (ms * 1e-3) * 2.4e9 * cus * 4 / wave_blocks;
      printf("%-18s waves/SIMD %d  %7.1f SIMD-cyc/wave-block(@2.4GHz)  %7.0f GB/s keystream\n",
             names[vi], w, cyc, wave_blocks * 64 * 64 / (ms * 1e-3) / 1e9);
    }
    (void)hipMemcpy(h[vi], d, 256 * 4, hipMemcpyDeviceToHost);
  };
  run(kchacha<0>, 0); run(kchacha<1>, 1); run(kchacha<2>, 2); run(kchacha<3>, 3);
  // lock-step waves: a workgroup of W waves per SIMD (BS = 256*W), barrier per double round
  auto run2 = [&](auto k, const char *name, int bs) {
    int wps = bs / 256;
    for (int rounds = 1; rounds <= 2; ++rounds) {
      int blocks = cus * rounds;   // rounds x wps waves per SIMD
      hipLaunchKernelGGL(k, dim3(blocks), dim3(bs), 0, 0, d, 5u); (void)hipDeviceSynchronize();
      (void)hipEventRecord(e0);
      for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(bs), 0, 0, d, 5u);
      (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
      float ms; (void)hipEventElapsedTime(&ms, e0, e1);
      double wave_blocks = 3.0 * blocks * (bs / 64) * NB;
      double cyc = (ms * 1e-3) * 2.4e9 * cus * 4 / wave_blocks;
      printf("%-26s waves/SIMD %d  %7.1f SIMD-cyc/wave-block(@2.4GHz)\n", name, wps * rounds, cyc);
    }
  };
  run2(kchacha<0, 0, 512>, "compiler bs512 nosync", 512);
  run2(kchacha<0, 1, 512>, "compiler bs512 sync/dr", 512);
  run2(kchacha<1, 1, 512>, "grouped bs512 sync/dr", 512);
  run2(kchacha<0, 0, 1024>, "compiler bs1024 nosync", 1024);
  run2(kchacha<0, 1, 1024>, "compiler bs1024 sync/dr", 1024);
  run2(kchacha<1, 1, 1024>, "grouped bs1024 sync/dr", 1024);
  int ok = 1;
  for (int v = 1; v < 4; ++v) for (int i = 0; i < 256; ++i) ok &= h[v][i] == h[0][i];
  printf("variants agree: %s\n", ok ? "yes" : "NO");
  return 0;
}
