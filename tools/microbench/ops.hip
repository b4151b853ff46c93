// Microbenchmark: VALU throughput of the integer ops the AEAD kernels lean on,
// and streaming bandwidth for the record access patterns (gfx950).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#define CHECK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("ERR %s line %d\n",hipGetErrorString(e),__LINE__); return 1;}}while(0)

constexpr int ITERS = 4096;

// 8 independent chains per lane to expose throughput, not latency.
template <int OP>
__global__ void __launch_bounds__(256) opk(uint32_t *out, uint32_t seed) {
  uint32_t a[8]; uint64_t b[8];
  for (int i = 0; i < 8; ++i) { a[i] = seed * (threadIdx.x + i) + i; b[i] = a[i] * 3ull; }
  uint32_t m = seed | 1;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (OP == 0) { a[i] = a[i] + m; }                                   // v_add_u32
      if constexpr (OP == 1) { a[i] = __builtin_amdgcn_alignbit(a[i], a[i], 7) ^ m; } // alignbit+xor (2 ops)
      if constexpr (OP == 2) { b[i] = (uint64_t)a[i] * m + b[i]; a[i] ^= (uint32_t)b[i]; } // mad_u64_u32 + xor
      if constexpr (OP == 3) { a[i] = a[i] * m + 1; }                               // mul_lo_u32 (+add)
      if constexpr (OP == 4) { a[i] = __umul24(a[i], m) ^ m; }                 // mul_u32_u24 + xor
      if constexpr (OP == 5) { a[i] = (uint32_t)(((uint64_t)(a[i] & 0xffffffu) * (m & 0xffffffu)) >> 32) ^ a[i]; }            // mul_hi_u32_u24 + xor
    }
  }
  uint32_t r = 0;
  for (int i = 0; i < 8; ++i) r ^= a[i] ^ (uint32_t)b[i] ^ (uint32_t)(b[i] >> 32);
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void __launch_bounds__(256) dopk(double *out, double seed) {
  double a[8];
  for (int i = 0; i < 8; ++i) a[i] = seed * (threadIdx.x + i);
  for (int it = 0; it < ITERS; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = __builtin_fma(a[i], seed, 1.0);
  double r = 0; for (int i = 0; i < 8; ++i) r += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

// Streaming: each lane owns one 64-B piece of a record; RPL lanes per record.
// pattern 0: lane loads its 64 B with 4 x 16-B loads (piece-per-lane)
// pattern 1: fully coalesced uint4 copy over the flat buffer
__global__ void __launch_bounds__(256) copy_flat(const uint4 *__restrict__ in, uint4 *__restrict__ out, size_t n16) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n16; i += stride) out[i] = in[i] ;
}
template <int K>
__global__ void __launch_bounds__(256) copy_records(const uint8_t *__restrict__ in, uint8_t *__restrict__ out,
                                                    uint32_t nrec, uint32_t len, uint32_t in_stride, uint32_t out_stride) {
  uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t rec = tid / K, k = tid % K;
  if (rec >= nrec) return;
  uint32_t units = (len + 63) / 64;
  const uint8_t *src = in + (size_t)rec * in_stride;
  uint8_t *dst = out + (size_t)rec * out_stride;
  for (uint32_t u = k; u < units; u += K) {
    const uint4 *s = (const uint4 *)(src + u * 64);
    uint4 *d = (uint4 *)(dst + u * 64);
    uint4 v0 = s[0], v1 = s[1], v2 = s[2], v3 = s[3];
    v0.x ^= u; d[0] = v0; d[1] = v1; d[2] = v2; d[3] = v3;
  }
}

int main() {
  hipDeviceProp_t prop; CHECK(hipGetDeviceProperties(&prop, 0));
  printf("device %s CUs %d clock %d kHz\n", prop.gcnArchName, prop.multiProcessorCount, prop.clockRate);
  int blocks = prop.multiProcessorCount * 16;  // 16 x 256 threads per CU = 16 waves/CU
  uint32_t *dout; CHECK(hipMalloc(&dout, blocks * 256 * 8));
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const char *names[] = {"add_u32", "alignbit+xor", "mad_u64_u32+xor", "mul_lo_u32+add", "mul_u24+xor", "mulhi_u24+xor"};
  auto run = [&](auto kern, const char *name, double ops_per_iter) {
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, dout, 12345u);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, dout, 12345u);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double lane_ops = 5.0 * blocks * 256.0 * ITERS * 8 * ops_per_iter;
    printf("%-18s %8.3f ms  %7.2f T lane-instr/s\n", name, ms, lane_ops / (ms * 1e-3) / 1e12);
  };
  run(opk<0>, names[0], 1); run(opk<1>, names[1], 2); run(opk<2>, names[2], 2);
  run(opk<3>, names[3], 2); run(opk<4>, names[4], 2); run(opk<5>, names[5], 2);
  {
    double *dd; CHECK(hipMalloc(&dd, blocks * 256 * 8));
    hipLaunchKernelGGL(dopk, dim3(blocks), dim3(256), 0, 0, dd, 1.0000001);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(dopk, dim3(blocks), dim3(256), 0, 0, dd, 1.0000001);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("%-18s %8.3f ms  %7.2f T lane-instr/s\n", "fma_f64", ms, 5.0 * blocks * 256.0 * ITERS * 8 / (ms * 1e-3) / 1e12);
  }
  // Bandwidth: rotate over 8 batches so the working set (> 1.4 GB) exceeds the 256 MB MALL.
  const uint32_t nrec = 65536, len = 1408;
  size_t bytes = (size_t)nrec * len;
  const int NB = 8;
  std::vector<uint8_t *> ins(NB), outs(NB);
  for (int b = 0; b < NB; ++b) { CHECK(hipMalloc(&ins[b], bytes)); CHECK(hipMalloc(&outs[b], bytes)); hipMemset(ins[b], b, bytes); }
  auto bw = [&](const char *name, auto launch) {
    for (int b = 0; b < NB; ++b) launch(b);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    const int R = 40;
    for (int r = 0; r < R; ++r) launch(r % NB);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("%-28s %8.2f us/batch  %7.2f TB/s (r+w)\n", name, ms * 1e3 / R, 2.0 * bytes * R / (ms * 1e-3) / 1e12);
  };
  bw("copy_flat grid=2048x256", [&](int b) { hipLaunchKernelGGL(copy_flat, dim3(2048), dim3(256), 0, 0, (const uint4 *)ins[b], (uint4 *)outs[b], bytes / 16); });
  bw("copy_flat grid=full", [&](int b) { hipLaunchKernelGGL(copy_flat, dim3((bytes / 16 + 255) / 256), dim3(256), 0, 0, (const uint4 *)ins[b], (uint4 *)outs[b], bytes / 16); });
  bw("copy_records K=1", [&](int b) { hipLaunchKernelGGL(copy_records<1>, dim3(nrec * 1 / 256), dim3(256), 0, 0, ins[b], outs[b], nrec, len, len, len); });
  bw("copy_records K=2", [&](int b) { hipLaunchKernelGGL(copy_records<2>, dim3(nrec * 2 / 256), dim3(256), 0, 0, ins[b], outs[b], nrec, len, len, len); });
  bw("copy_records K=4", [&](int b) { hipLaunchKernelGGL(copy_records<4>, dim3(nrec * 4 / 256), dim3(256), 0, 0, ins[b], outs[b], nrec, len, len, len); });
  bw("copy_records K=8", [&](int b) { hipLaunchKernelGGL(copy_records<8>, dim3(nrec * 8 / 256), dim3(256), 0, 0, ins[b], outs[b], nrec, len, len, len); });
  bw("copy_records K=16", [&](int b) { hipLaunchKernelGGL(copy_records<16>, dim3(nrec * 16 / 256), dim3(256), 0, 0, ins[b], outs[b], nrec, len, len, len); });
  bw("copy_records K=32", [&](int b) { hipLaunchKernelGGL(copy_records<32>, dim3(nrec * 32 / 256), dim3(256), 0, 0, ins[b], outs[b], nrec, len, len, len); });
  return 0;
}
