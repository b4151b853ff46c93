// When does gfx950 issue a 32-bit integer VALU op in ~2.4 instead of ~4.1
// SIMD-cycles per wave-instruction?  Sweeps waves/SIMD (1..8) against the
// dependency distance of a v_xor_b32 stream and against runs of fast (xor)
// and slow (alignbit) instructions.  16 independent registers per lane.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
constexpr int IT = 1024;
#define X(i) "v_xor_b32 %" #i ", %" #i ", %16\n"
#define A(i) "v_alignbit_b32 %" #i ", %" #i ", %" #i ", 7\n"
#define XD(i, j) "v_xor_b32 %" #i ", %" #j ", %16\n"   /* i = j ^ m : depends on j */
#define OPS "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), \
            "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]), "+v"(r[12]), "+v"(r[13]), "+v"(r[14]), "+v"(r[15])
#define KERN(NAME, BODY)                                                       \
  __global__ void __launch_bounds__(256) NAME(uint32_t *o, uint32_t s) {       \
    uint32_t r[16];                                                            \
    for (int i = 0; i < 16; ++i) r[i] = s * (i + 3) + threadIdx.x;             \
    uint32_t m = s | 1;                                                        \
    for (int i = 0; i < IT; ++i) asm volatile(BODY : OPS : "v"(m));            \
    uint32_t a = 0;                                                            \
    for (int i = 0; i < 16; ++i) a ^= r[i];                                    \
    o[blockIdx.x * 256 + threadIdx.x] = a;                                     \
  }
// 32 instructions per body
#define X16 X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)
#define A16 A(0) A(1) A(2) A(3) A(4) A(5) A(6) A(7) A(8) A(9) A(10) A(11) A(12) A(13) A(14) A(15)
KERN(k_dist16, X16 X16)
// distance 1: one dependent chain
#define C8 X(0) X(0) X(0) X(0) X(0) X(0) X(0) X(0)
KERN(k_dist1, C8 C8 C8 C8)
// distance 2
#define C2 X(0) X(1) X(0) X(1) X(0) X(1) X(0) X(1)
KERN(k_dist2, C2 C2 C2 C2)
// distance 4
#define C4 X(0) X(1) X(2) X(3) X(0) X(1) X(2) X(3)
KERN(k_dist4, C4 C4 C4 C4)
// runs: 8 fast / 8 slow
KERN(k_run8, X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) A(8) A(9) A(10) A(11) A(12) A(13) A(14) A(15)
             X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) A(8) A(9) A(10) A(11) A(12) A(13) A(14) A(15))
// runs: 16 fast / 16 slow
KERN(k_run16, X16 A16)
// alternate 1/1
KERN(k_alt, X(0) A(8) X(1) A(9) X(2) A(10) X(3) A(11) X(4) A(12) X(5) A(13) X(6) A(14) X(7) A(15)
            X(0) A(8) X(1) A(9) X(2) A(10) X(3) A(11) X(4) A(12) X(5) A(13) X(6) A(14) X(7) A(15))
// 3 fast : 1 slow
KERN(k_3to1, X(0) X(1) X(2) A(8) X(3) X(4) X(5) A(9) X(6) X(7) X(0) A(10) X(1) X(2) X(3) A(11)
             X(4) X(5) X(6) A(12) X(7) X(0) X(1) A(13) X(2) X(3) X(4) A(14) X(5) X(6) X(7) A(15))
// pure slow
KERN(k_slow, A16 A16)
// xor chains with fresh-source (reads another reg written 8 earlier)
KERN(k_xdep8, XD(0, 8) XD(1, 9) XD(2, 10) XD(3, 11) XD(4, 12) XD(5, 13) XD(6, 14) XD(7, 15)
              XD(8, 0) XD(9, 1) XD(10, 2) XD(11, 3) XD(12, 4) XD(13, 5) XD(14, 6) XD(15, 7)
              XD(0, 8) XD(1, 9) XD(2, 10) XD(3, 11) XD(4, 12) XD(5, 13) XD(6, 14) XD(7, 15)
              XD(8, 0) XD(9, 1) XD(10, 2) XD(11, 3) XD(12, 4) XD(13, 5) XD(14, 6) XD(15, 7))

int main() {
  hipDeviceProp_t p; (void)hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  uint32_t *d; (void)hipMalloc(&d, (size_t)cus * 8 * 256 * 4);
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  auto run = [&](auto k, const char *name) {
    printf("%-22s", name);
    for (int w = 1; w <= 8; w *= 2) {
      int blocks = cus * w;
      hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 3u); (void)hipDeviceSynchronize();
      (void)hipEventRecord(e0);
      for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 3u);
      (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
      float ms; (void)hipEventElapsedTime(&ms, e0, e1);
      double wi = 3.0 * blocks * 4 * IT * 32.0;
      printf("  w%d %5.2f", w, (ms * 1e-3) * 2.4e9 * cus * 4 / wi);
    }
    printf("   SIMD-cyc/wave-instr @2.4GHz\n");
  };
  run(k_dist16, "xor dist16"); run(k_dist1, "xor dist1"); run(k_dist2, "xor dist2");
  run(k_dist4, "xor dist4"); run(k_xdep8, "xor fresh-src dist8"); run(k_slow, "alignbit");
  run(k_run16, "16 xor / 16 align"); run(k_run8, "8 xor / 8 align"); run(k_alt, "1 xor / 1 align");
  run(k_3to1, "3 xor / 1 align");
  return 0;
}
