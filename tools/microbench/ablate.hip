// Ablation of the ChaChaPoly seal loop on the C2 shape (64Ki x 1400 B):
// which of load / ChaCha20 / Poly1305 / store bounds the kernel?
#include "../../noise-c_amd/csrc/aead_device.h"
#include <cstdio>
using namespace na;
constexpr int UNITS = 22;  // 1400 B -> 22 units (last one partial, treated full here)

template <int K, bool LD, bool CC, bool PL, bool ST>
__global__ __launch_bounds__(256) void ablate(const uint8_t *in, uint8_t *out, uint32_t n, uint32_t *sink,
                                              uint32_t stride_in, uint32_t stride_out) {
  uint32_t gtid = blockIdx.x * 256 + threadIdx.x, rec = gtid / K, k = gtid % K;
  if (rec >= n) return;
  const uint8_t *src = in + (size_t)rec * stride_in;
  uint8_t *dst = out + (size_t)rec * stride_out;
  uint32_t key[8]; for (int i = 0; i < 8; ++i) key[i] = 0x1234567u * (i + 1) ^ rec;
  R32 r = r32_from_key(key[0], key[1], key[2], key[3]);
  P32 acc = p32_zero();
  uint32_t wn[16];
  for (int i = 0; i < 16; ++i) wn[i] = rec + i;
  if (LD) { const uint4 *q = (const uint4 *)(src + 64 * k); uint4 a=q[0],b=q[1],c=q[2],d=q[3];
    wn[0]=a.x;wn[1]=a.y;wn[2]=a.z;wn[3]=a.w;wn[4]=b.x;wn[5]=b.y;wn[6]=b.z;wn[7]=b.w;wn[8]=c.x;wn[9]=c.y;wn[10]=c.z;wn[11]=c.w;wn[12]=d.x;wn[13]=d.y;wn[14]=d.z;wn[15]=d.w; }
  for (uint32_t u = k; u < UNITS; u += K) {
    uint32_t w[16];
    for (int i = 0; i < 16; ++i) w[i] = wn[i];
    uint32_t un = u + K < UNITS ? u + K : 0;
    if (LD) { const uint4 *q = (const uint4 *)(src + 64 * un); uint4 a=q[0],b=q[1],c=q[2],d=q[3];
      wn[0]=a.x;wn[1]=a.y;wn[2]=a.z;wn[3]=a.w;wn[4]=b.x;wn[5]=b.y;wn[6]=b.z;wn[7]=b.w;wn[8]=c.x;wn[9]=c.y;wn[10]=c.z;wn[11]=c.w;wn[12]=d.x;wn[13]=d.y;wn[14]=d.z;wn[15]=d.w; }
    else { for (int i = 0; i < 16; ++i) wn[i] = w[i] * 3 + u; }
    uint32_t x[16];
    if (CC) chacha20_block(key, u + 1, 0, rec, 0, x);
    else for (int i = 0; i < 16; ++i) x[i] = key[i & 7] + u;
    for (int i = 0; i < 16; ++i) w[i] ^= x[i];
    if (ST) { uint4 *q = (uint4 *)(dst + 64 * u);
      q[0]=make_uint4(w[0],w[1],w[2],w[3]); q[1]=make_uint4(w[4],w[5],w[6],w[7]); q[2]=make_uint4(w[8],w[9],w[10],w[11]); q[3]=make_uint4(w[12],w[13],w[14],w[15]); }
    if (PL) { for (int b = 0; b < 4; ++b) p32_block(acc, r, w[4*b], w[4*b+1], w[4*b+2], w[4*b+3]); }
    else { acc.h0 ^= w[0] ^ w[5] ^ w[10] ^ w[15]; }
  }
  uint32_t v = acc.h0 ^ acc.h1 ^ acc.h2 ^ acc.h3 ^ acc.h4;
  if (v == 0x12345678u) sink[gtid] = v;  // keeps everything live, (almost) never stores
}

int main() {
  const uint32_t N = 65536, SI = 1408, SO = 1424; const int NB = 4;
  uint8_t *in[NB], *out[NB]; uint32_t *sink;
  for (int b = 0; b < NB; ++b) { hipMalloc(&in[b], (size_t)N * SI + 4096); hipMalloc(&out[b], (size_t)N * SO + 4096); hipMemset(in[b], b + 1, (size_t)N * SI); }
  hipMalloc(&sink, N * 8 * 4);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  auto run = [&](auto kern, int K, const char *name) {
    dim3 g((N * K + 255) / 256);
    for (int b = 0; b < NB; ++b) hipLaunchKernelGGL(kern, g, dim3(256), 0, 0, in[b], out[b], N, sink, SI, SO);
    hipDeviceSynchronize();
    const int R = 40;
    hipEventRecord(e0);
    for (int r = 0; r < R; ++r) hipLaunchKernelGGL(kern, g, dim3(256), 0, 0, in[r % NB], out[r % NB], N, sink, SI, SO);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("K=%d %-22s %7.2f us/launch\n", K, name, ms * 1e3 / R);
  };
#define V(K, LD, CC, PL, ST, name) run(ablate<K, LD, CC, PL, ST>, K, name);
  for (int rep = 0; rep < 2; ++rep) {
  V(1, 1, 1, 1, 1, "all");  V(1, 0, 1, 1, 0, "compute(cc+poly)"); V(1, 0, 1, 0, 0, "chacha only");
  V(1, 0, 0, 1, 0, "poly only"); V(1, 1, 0, 0, 1, "load+store"); V(1, 1, 0, 0, 0, "load only"); V(1, 0, 0, 0, 1, "store only");
  V(4, 1, 1, 1, 1, "all");  V(4, 0, 1, 1, 0, "compute(cc+poly)"); V(4, 0, 1, 0, 0, "chacha only");
  V(4, 0, 0, 1, 0, "poly only"); V(4, 1, 0, 0, 1, "load+store"); V(4, 1, 0, 0, 0, "load only"); V(4, 0, 0, 0, 1, "store only");
  V(2, 1, 1, 1, 1, "all"); V(2, 0, 1, 1, 0, "compute(cc+poly)"); V(8, 1, 1, 1, 1, "all"); V(8, 0, 1, 1, 0, "compute(cc+poly)");
  }
  return 0;
}
