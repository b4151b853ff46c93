// Cross-wave VALU issue on gfx950, shaped like the ChaCha20 block (VERDICT r5
// item 6).  profiles/r01_runs_mix.log: waves of fast-class ops only (v_add,
// v_xor: ~2.1 SIMD-cycles per wave-instruction with >= 2 waves) sharing a
// SIMD with waves of slow-class ops only (v_alignbit: ~4.1) averaged 2.66,
// where ANY mix inside a wave's stream ran at ~4 (runs of 8..64 included).
// Can a real ChaCha20 stream use that?  A ChaCha quarter-round is
//   a += b; d ^= a; d <<<= 16; c += d; b ^= c; b <<<= 12; ...
// and with 4 blocks per lane in lock step (16 quarter-rounds) every sub-step
// is a run of 32 fast ops (16 v_add_u32, 16 v_xor_b32) followed by a run of
// 16 slow ops (16 v_alignbit_b32): 992-op block = 2/3 fast, 1/3 slow.
//
// Modes (every wave runs R double rounds on its lane's 4 blocks, the runs in
// fixed order through inline asm):
//   0 free       no synchronisation: the SIMD's 4 waves drift (baseline)
//   1 inphase    s_barrier at every run boundary (1024-thread workgroup = 4
//                waves per SIMD): all waves in their fast run, then all in
//                their slow run — the SIMD sees one class at a time
//   2 antiphase  as 1, but the odd waves of the workgroup run one interval
//                behind: at every interval half the SIMD's waves issue a fast
//                run and the other half a slow run (the wave-spec pattern)
//   3 prio       no barriers; s_setprio 2 before a slow run, 0 before a fast
//                run (slow runs first in the arbiter, fast runs fill)
//   4 compiler   the same 4-block ChaCha in plain C++ (hipcc's schedule)
// Output: SIMD-cycles per wave-instruction from the shader clock (s_memtime)
// of each workgroup's wave 0, the in-kernel clock (s_memtime over
// s_memrealtime), the waves' SIMD placement (HW_ID) and a check of every
// lane's final state against a host ChaCha20 double-round loop.
//
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 xwave.hip -o xwave
// run:   ./xwave [R]   (R double rounds per launch, default 2000)
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define DEV __device__ __forceinline__

// 8 v_add_u32 / v_xor_b32 (d_i op= s_i), one asm statement each: asm volatile
// statements keep their order, and nothing else sits between them
#define OP8(op)                                                                                              \
    asm volatile(op " %0, %0, %8\n\t" op " %1, %1, %9\n\t" op " %2, %2, %10\n\t" op " %3, %3, %11\n\t" op    \
                    " %4, %4, %12\n\t" op " %5, %5, %13\n\t" op " %6, %6, %14\n\t" op " %7, %7, %15"       \
                 : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7)           \
                 : "v"(s0), "v"(s1), "v"(s2), "v"(s3), "v"(s4), "v"(s5), "v"(s6), "v"(s7))

DEV void add8(uint32_t &d0, uint32_t &d1, uint32_t &d2, uint32_t &d3, uint32_t &d4, uint32_t &d5, uint32_t &d6,
              uint32_t &d7, uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3, uint32_t s4, uint32_t s5,
              uint32_t s6, uint32_t s7)
{
    OP8("v_add_u32");
}

DEV void xor8(uint32_t &d0, uint32_t &d1, uint32_t &d2, uint32_t &d3, uint32_t &d4, uint32_t &d5, uint32_t &d6,
              uint32_t &d7, uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3, uint32_t s4, uint32_t s5,
              uint32_t s6, uint32_t s7)
{
    OP8("v_xor_b32");
}

// rotl(x, n) = v_alignbit_b32(x, x, 32 - n)
template <int N>
DEV void rot8(uint32_t &d0, uint32_t &d1, uint32_t &d2, uint32_t &d3, uint32_t &d4, uint32_t &d5, uint32_t &d6,
              uint32_t &d7)
{
    asm volatile("v_alignbit_b32 %0, %0, %0, %8\n\tv_alignbit_b32 %1, %1, %1, %8\n\t"
                 "v_alignbit_b32 %2, %2, %2, %8\n\tv_alignbit_b32 %3, %3, %3, %8\n\t"
                 "v_alignbit_b32 %4, %4, %4, %8\n\tv_alignbit_b32 %5, %5, %5, %8\n\t"
                 "v_alignbit_b32 %6, %6, %6, %8\n\tv_alignbit_b32 %7, %7, %7, %8"
                 : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7)
                 : "i"(32 - N));
}

// quarter-round word indices: column round, then diagonal round
constexpr int HQR[2][4][4] = {{{0, 4, 8, 12}, {1, 5, 9, 13}, {2, 6, 10, 14}, {3, 7, 11, 15}},
                              {{0, 5, 10, 15}, {1, 6, 11, 12}, {2, 7, 8, 13}, {3, 4, 9, 14}}};

// sub-step s of round r over the 4 blocks x 4 QRs: dst += src (fast), x ^= dst
// (fast), x <<<= n (slow); sub-steps (a,b,d,16) (c,d,b,12) (a,b,d,8) (c,d,b,7)
template <int RND, int DST, int SRC, int X>
DEV void fast_run(uint32_t (&x)[4][16])
{
#define W(b, q, k) x[b][HQR[RND][q][k]]
    add8(W(0, 0, DST), W(0, 1, DST), W(0, 2, DST), W(0, 3, DST), W(1, 0, DST), W(1, 1, DST), W(1, 2, DST),
         W(1, 3, DST), W(0, 0, SRC), W(0, 1, SRC), W(0, 2, SRC), W(0, 3, SRC), W(1, 0, SRC), W(1, 1, SRC),
         W(1, 2, SRC), W(1, 3, SRC));
    add8(W(2, 0, DST), W(2, 1, DST), W(2, 2, DST), W(2, 3, DST), W(3, 0, DST), W(3, 1, DST), W(3, 2, DST),
         W(3, 3, DST), W(2, 0, SRC), W(2, 1, SRC), W(2, 2, SRC), W(2, 3, SRC), W(3, 0, SRC), W(3, 1, SRC),
         W(3, 2, SRC), W(3, 3, SRC));
    xor8(W(0, 0, X), W(0, 1, X), W(0, 2, X), W(0, 3, X), W(1, 0, X), W(1, 1, X), W(1, 2, X), W(1, 3, X),
         W(0, 0, DST), W(0, 1, DST), W(0, 2, DST), W(0, 3, DST), W(1, 0, DST), W(1, 1, DST), W(1, 2, DST),
         W(1, 3, DST));
    xor8(W(2, 0, X), W(2, 1, X), W(2, 2, X), W(2, 3, X), W(3, 0, X), W(3, 1, X), W(3, 2, X), W(3, 3, X),
         W(2, 0, DST), W(2, 1, DST), W(2, 2, DST), W(2, 3, DST), W(3, 0, DST), W(3, 1, DST), W(3, 2, DST),
         W(3, 3, DST));
}

template <int RND, int X, int N>
DEV void slow_run(uint32_t (&x)[4][16])
{
    rot8<N>(W(0, 0, X), W(0, 1, X), W(0, 2, X), W(0, 3, X), W(1, 0, X), W(1, 1, X), W(1, 2, X), W(1, 3, X));
    rot8<N>(W(2, 0, X), W(2, 1, X), W(2, 2, X), W(2, 3, X), W(3, 0, X), W(3, 1, X), W(3, 2, X), W(3, 3, X));
#undef W
}

DEV void sync_point(int mode)
{
    if (mode == 1 || mode == 2) __builtin_amdgcn_s_barrier();
}

// one round (column or diagonal) = 4 sub-steps = 8 runs; `lag` (mode 2, odd
// waves) runs the same code one interval later: the barrier count matches
template <int RND>
DEV void round_runs(uint32_t (&x)[4][16], int mode)
{
    if (mode == 3) __builtin_amdgcn_s_setprio(0);
    fast_run<RND, 0, 1, 3>(x);
    sync_point(mode);
    if (mode == 3) __builtin_amdgcn_s_setprio(2);
    slow_run<RND, 3, 16>(x);
    sync_point(mode);
    if (mode == 3) __builtin_amdgcn_s_setprio(0);
    fast_run<RND, 2, 3, 1>(x);
    sync_point(mode);
    if (mode == 3) __builtin_amdgcn_s_setprio(2);
    slow_run<RND, 1, 12>(x);
    sync_point(mode);
    if (mode == 3) __builtin_amdgcn_s_setprio(0);
    fast_run<RND, 0, 1, 3>(x);
    sync_point(mode);
    if (mode == 3) __builtin_amdgcn_s_setprio(2);
    slow_run<RND, 3, 8>(x);
    sync_point(mode);
    if (mode == 3) __builtin_amdgcn_s_setprio(0);
    fast_run<RND, 2, 3, 1>(x);
    sync_point(mode);
    if (mode == 3) __builtin_amdgcn_s_setprio(2);
    slow_run<RND, 1, 7>(x);
    sync_point(mode);
}

DEV uint32_t rotl(uint32_t v, int n) { return (v << n) | (v >> (32 - n)); }

// mode 4: the compiler's own schedule of the same 4 blocks
DEV void double_round_c(uint32_t (&x)[4][16])
{
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                uint32_t &a = x[b][HQR[r][q][0]], &bb = x[b][HQR[r][q][1]], &c = x[b][HQR[r][q][2]],
                         &d = x[b][HQR[r][q][3]];
                a += bb; d ^= a; d = rotl(d, 16);
                c += d; bb ^= c; bb = rotl(bb, 12);
                a += bb; d ^= a; d = rotl(d, 8);
                c += d; bb ^= c; bb = rotl(bb, 7);
            }
}

struct Out {
    unsigned long long c0, c1, t0, t1;
    uint32_t hw, lag;
};

template <int MODE>
__global__ __launch_bounds__(1024) void xwave(uint32_t *state, Out *out, int R)
{
    const uint32_t gt = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t x[4][16];
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i) x[b][i] = gt * 0x9E3779B9u + (uint32_t)(b * 16 + i) * 0x85EBCA6Bu;
    const int wave = threadIdx.x >> 6;
    /* mode 2: every other wave OF EACH SIMD lags (the SIMD of a wave from
       HW_ID: rank among the workgroup's waves on the same SIMD) */
    __shared__ uint32_t simd_of[16];
    const uint32_t hw = (uint32_t)__builtin_amdgcn_s_getreg(4 | (31 << 11));
    if ((threadIdx.x & 63) == 0) simd_of[wave] = (hw >> 4) & 3;
    __syncthreads();
    int rank = 0;
    for (int w = 0; w < wave; ++w) rank += simd_of[w] == ((hw >> 4) & 3);
    const bool lag = MODE == 2 && (rank & 1);
    __builtin_amdgcn_s_barrier();
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), t0 = __builtin_amdgcn_s_memrealtime();
    if (lag) __builtin_amdgcn_s_barrier(); /* one interval behind */
    for (int it = 0; it < R; ++it) {
        if constexpr (MODE == 4) {
            double_round_c(x);
        } else {
            round_runs<0>(x, MODE);
            round_runs<1>(x, MODE);
        }
    }
    if (MODE == 2 && !lag) __builtin_amdgcn_s_barrier(); /* the barrier counts match */
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), t1 = __builtin_amdgcn_s_memrealtime();
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i) state[((size_t)gt * 4 + b) * 16 + i] = x[b][i];
    if ((threadIdx.x & 63) == 0) {
        Out o;
        o.c0 = c0; o.c1 = c1; o.t0 = t0; o.t1 = t1;
        o.hw = hw;
        o.lag = lag;
        out[blockIdx.x * 16 + wave] = o;
    }
}


// ---- product shapes (round 6 follow-up): NB blocks per lane in lock step
// (runs of 8 NB fast / 4 NB slow ops), WPS waves per SIMD (workgroup of
// 256 WPS threads, one per CU), s_setprio PS before a slow run and PF before
// a fast run (PS < 0: no setprio; MODE 4 = the compiler's schedule).
template <int NB>
DEV void runs_nb(uint32_t (&x)[4][16], int rnd_unused);

template <int RND, int NB, int DST, int SRC, int X>
DEV void fast_nb(uint32_t (&x)[4][16])
{
#define W(b, q, k) x[b][HQR[RND][q][k]]
    if constexpr (NB == 1) {
        asm volatile("v_add_u32 %0, %0, %4\n\tv_add_u32 %1, %1, %5\n\tv_add_u32 %2, %2, %6\n\tv_add_u32 %3, %3, %7"
                     : "+v"(W(0, 0, DST)), "+v"(W(0, 1, DST)), "+v"(W(0, 2, DST)), "+v"(W(0, 3, DST))
                     : "v"(W(0, 0, SRC)), "v"(W(0, 1, SRC)), "v"(W(0, 2, SRC)), "v"(W(0, 3, SRC)));
        asm volatile("v_xor_b32 %0, %0, %4\n\tv_xor_b32 %1, %1, %5\n\tv_xor_b32 %2, %2, %6\n\tv_xor_b32 %3, %3, %7"
                     : "+v"(W(0, 0, X)), "+v"(W(0, 1, X)), "+v"(W(0, 2, X)), "+v"(W(0, 3, X))
                     : "v"(W(0, 0, DST)), "v"(W(0, 1, DST)), "v"(W(0, 2, DST)), "v"(W(0, 3, DST)));
    } else {
#pragma unroll
        for (int h = 0; h < NB; h += 2) {
            add8(W(h, 0, DST), W(h, 1, DST), W(h, 2, DST), W(h, 3, DST), W(h + 1, 0, DST), W(h + 1, 1, DST),
                 W(h + 1, 2, DST), W(h + 1, 3, DST), W(h, 0, SRC), W(h, 1, SRC), W(h, 2, SRC), W(h, 3, SRC),
                 W(h + 1, 0, SRC), W(h + 1, 1, SRC), W(h + 1, 2, SRC), W(h + 1, 3, SRC));
        }
#pragma unroll
        for (int h = 0; h < NB; h += 2) {
            xor8(W(h, 0, X), W(h, 1, X), W(h, 2, X), W(h, 3, X), W(h + 1, 0, X), W(h + 1, 1, X), W(h + 1, 2, X),
                 W(h + 1, 3, X), W(h, 0, DST), W(h, 1, DST), W(h, 2, DST), W(h, 3, DST), W(h + 1, 0, DST),
                 W(h + 1, 1, DST), W(h + 1, 2, DST), W(h + 1, 3, DST));
        }
    }
}

template <int RND, int NB, int X, int N>
DEV void slow_nb(uint32_t (&x)[4][16])
{
    if constexpr (NB == 1) {
        asm volatile("v_alignbit_b32 %0, %0, %0, %4\n\tv_alignbit_b32 %1, %1, %1, %4\n\t"
                     "v_alignbit_b32 %2, %2, %2, %4\n\tv_alignbit_b32 %3, %3, %3, %4"
                     : "+v"(W(0, 0, X)), "+v"(W(0, 1, X)), "+v"(W(0, 2, X)), "+v"(W(0, 3, X)) : "i"(32 - N));
    } else {
#pragma unroll
        for (int h = 0; h < NB; h += 2)
            rot8<N>(W(h, 0, X), W(h, 1, X), W(h, 2, X), W(h, 3, X), W(h + 1, 0, X), W(h + 1, 1, X),
                    W(h + 1, 2, X), W(h + 1, 3, X));
    }
#undef W
}

template <int PS>
DEV void prio_slow()
{
    if constexpr (PS >= 0) __builtin_amdgcn_s_setprio(PS);
}

template <int RND, int NB, int PS, int PF>
DEV void round_nb(uint32_t (&x)[4][16])
{
    prio_slow<PF>(); fast_nb<RND, NB, 0, 1, 3>(x); prio_slow<PS>(); slow_nb<RND, NB, 3, 16>(x);
    prio_slow<PF>(); fast_nb<RND, NB, 2, 3, 1>(x); prio_slow<PS>(); slow_nb<RND, NB, 1, 12>(x);
    prio_slow<PF>(); fast_nb<RND, NB, 0, 1, 3>(x); prio_slow<PS>(); slow_nb<RND, NB, 3, 8>(x);
    prio_slow<PF>(); fast_nb<RND, NB, 2, 3, 1>(x); prio_slow<PS>(); slow_nb<RND, NB, 1, 7>(x);
}

DEV void double_round_c_nb(uint32_t (&x)[4][16], int nb)
{
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int b = 0; b < 4; ++b)
            if (b < nb)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    uint32_t &a = x[b][HQR[r][q][0]], &bb = x[b][HQR[r][q][1]], &c = x[b][HQR[r][q][2]],
                             &d = x[b][HQR[r][q][3]];
                    a += bb; d ^= a; d = rotl(d, 16);
                    c += d; bb ^= c; bb = rotl(bb, 12);
                    a += bb; d ^= a; d = rotl(d, 8);
                    c += d; bb ^= c; bb = rotl(bb, 7);
                }
}

template <int NB, int WPS, int PS, int PF, bool COMPILER>
__global__ __launch_bounds__(256 * WPS) void xshape(uint32_t *state, Out *out, int R)
{
    const uint32_t gt = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t x[4][16];
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i) x[b][i] = gt * 0x9E3779B9u + (uint32_t)(b * 16 + i) * 0x85EBCA6Bu;
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), t0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < R; ++it) {
        if constexpr (COMPILER) {
            double_round_c_nb(x, NB);
        } else {
            round_nb<0, NB, PS, PF>(x);
            round_nb<1, NB, PS, PF>(x);
        }
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), t1 = __builtin_amdgcn_s_memrealtime();
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i) state[((size_t)gt * 4 + b) * 16 + i] = x[b][i];
    if ((threadIdx.x & 63) == 0) {
        Out o;
        o.c0 = c0; o.c1 = c1; o.t0 = t0; o.t1 = t1;
        o.hw = 0; o.lag = 0;
        out[blockIdx.x * 16 + (threadIdx.x >> 6)] = o;
    }
}

static uint32_t hrotl(uint32_t v, int n) { return (v << n) | (v >> (32 - n)); }

static void host_block(uint32_t gt, int b, int R, uint32_t o[16])
{
    uint32_t x[16];
    for (int i = 0; i < 16; ++i) x[i] = gt * 0x9E3779B9u + (uint32_t)(b * 16 + i) * 0x85EBCA6Bu;
    for (int it = 0; it < R; ++it)
        for (int r = 0; r < 2; ++r)
            for (int q = 0; q < 4; ++q) {
                uint32_t &a = x[HQR[r][q][0]], &bb = x[HQR[r][q][1]], &c = x[HQR[r][q][2]], &d = x[HQR[r][q][3]];
                a += bb; d ^= a; d = hrotl(d, 16);
                c += d; bb ^= c; bb = hrotl(bb, 12);
                a += bb; d ^= a; d = hrotl(d, 8);
                c += d; bb ^= c; bb = hrotl(bb, 7);
            }
    memcpy(o, x, sizeof(x));
}

int main(int argc, char **argv)
{
    const int R = argc > 1 ? atoi(argv[1]) : 2000;
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount, blocks = cus; /* one 1024-thread WG per CU: 4 waves per SIMD */
    const size_t threads = (size_t)blocks * 1024;
    uint32_t *d_state;
    Out *d_out;
    hipMalloc(&d_state, threads * 64 * 4);
    hipMalloc(&d_out, (size_t)blocks * 16 * sizeof(Out));
    std::vector<uint32_t> st(threads * 64);
    std::vector<Out> out((size_t)blocks * 16);
    const char *names[] = {"free", "inphase", "antiphase", "prio", "compiler"};
    void (*k[])(uint32_t *, Out *, int) = {xwave<0>, xwave<1>, xwave<2>, xwave<3>, xwave<4>};
    const double wave_instr = (double)R * 2 * 4 * 48; /* per wave: 2 rounds x 4 sub-steps x 48 VALU */
    for (int rep = 0; rep < 2; ++rep)
        for (int m = 0; m < 5; ++m) {
            /* settle: a few launches before the measured one (the clock) */
            for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k[m], dim3(blocks), dim3(1024), 0, 0, d_state, d_out, R);
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            hipEventRecord(e0);
            hipLaunchKernelGGL(k[m], dim3(blocks), dim3(1024), 0, 0, d_state, d_out, R);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            hipMemcpy(st.data(), d_state, st.size() * 4, hipMemcpyDeviceToHost);
            hipMemcpy(out.data(), d_out, out.size() * sizeof(Out), hipMemcpyDeviceToHost);
            /* correctness: sampled lanes vs the host */
            int bad = 0;
            for (size_t g = 0; g < threads; g += 4099)
                for (int b = 0; b < 4; ++b) {
                    uint32_t o[16];
                    host_block((uint32_t)g, b, R, o);
                    if (memcmp(o, &st[(g * 4 + b) * 16], 64)) ++bad;
                }
            /* per wave: shader cycles over its span; the clock */
            double cyc = 0, rt = 0;
            int simd_hist[4] = {0, 0, 0, 0}, odd_on[4] = {0, 0, 0, 0};
            for (int bidx = 0; bidx < blocks; ++bidx)
                for (int w = 0; w < 16; ++w) {
                    const Out &o = out[bidx * 16 + w];
                    cyc += (double)(o.c1 - o.c0);
                    rt += (double)(o.t1 - o.t0);
                    if (bidx == 0) {
                        const int simd = (o.hw >> 4) & 3;
                        simd_hist[simd]++;
                        if (o.lag) odd_on[simd]++;
                    }
                }
            cyc /= blocks * 16;
            rt /= blocks * 16;
            const double mhz = cyc / rt * 100.0; /* s_memrealtime: 100 MHz */
            /* a SIMD holds 4 of the workgroup's 16 waves: its cycles per wave-instruction */
            const double cpi = cyc / (4.0 * wave_instr);
            const double cpi_evt = (ms * 1e-3) * mhz * 1e6 / (4.0 * wave_instr);
            printf("%-9s R=%d  %8.3f ms  clock %6.0f MHz  SIMD-cycles/wave-instr %.3f (wave spans) %.3f (event)"
                   "  check %s  block0 waves/SIMD %d %d %d %d (lagging %d %d %d %d)\n",
                   names[m], R, ms, mhz, cpi, cpi_evt, bad ? "FAIL" : "ok", simd_hist[0], simd_hist[1],
                   simd_hist[2], simd_hist[3], odd_on[0], odd_on[1], odd_on[2], odd_on[3]);
            hipEventDestroy(e0);
            hipEventDestroy(e1);
        }
    /* product shapes: blocks per lane x waves per SIMD x prio */
    struct Shape { const char *name; void (*k)(uint32_t *, Out *, int); int nb, wps; };
    const Shape shapes[] = {
        {"nb1 w2 compiler", xshape<1, 2, -1, -1, true>, 1, 2}, {"nb1 w2 prio2/0", xshape<1, 2, 2, 0, false>, 1, 2},
        {"nb2 w2 compiler", xshape<2, 2, -1, -1, true>, 2, 2}, {"nb2 w2 free", xshape<2, 2, -1, -1, false>, 2, 2},
        {"nb2 w2 prio2/0", xshape<2, 2, 2, 0, false>, 2, 2},   {"nb2 w2 prio3/1", xshape<2, 2, 3, 1, false>, 2, 2},
        {"nb2 w2 prio0/2", xshape<2, 2, 0, 2, false>, 2, 2},
        {"nb4 w2 compiler", xshape<4, 2, -1, -1, true>, 4, 2}, {"nb4 w2 prio2/0", xshape<4, 2, 2, 0, false>, 4, 2},
        {"nb1 w4 compiler", xshape<1, 4, -1, -1, true>, 1, 4}, {"nb1 w4 prio2/0", xshape<1, 4, 2, 0, false>, 1, 4},
        {"nb2 w4 compiler", xshape<2, 4, -1, -1, true>, 2, 4}, {"nb2 w4 prio2/0", xshape<2, 4, 2, 0, false>, 2, 4},
        {"nb4 w4 compiler", xshape<4, 4, -1, -1, true>, 4, 4}, {"nb4 w4 prio2/0", xshape<4, 4, 2, 0, false>, 4, 4},
    };
    for (int rep = 0; rep < 2; ++rep)
        for (const Shape &sh : shapes) {
            const int threads_per = 256 * sh.wps;
            for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(sh.k, dim3(blocks), dim3(threads_per), 0, 0, d_state, d_out, R);
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            hipEventRecord(e0);
            hipLaunchKernelGGL(sh.k, dim3(blocks), dim3(threads_per), 0, 0, d_state, d_out, R);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            hipMemcpy(st.data(), d_state, st.size() * 4, hipMemcpyDeviceToHost);
            hipMemcpy(out.data(), d_out, out.size() * sizeof(Out), hipMemcpyDeviceToHost);
            int bad = 0;
            const size_t thr = (size_t)blocks * threads_per;
            for (size_t g = 0; g < thr; g += 4099)
                for (int b = 0; b < sh.nb; ++b) {
                    uint32_t o[16];
                    host_block((uint32_t)g, b, R, o);
                    if (memcmp(o, &st[(g * 4 + b) * 16], 64)) ++bad;
                }
            double cyc = 0, rt = 0;
            const int waves = threads_per / 64;
            for (int bidx = 0; bidx < blocks; ++bidx)
                for (int w = 0; w < waves; ++w) {
                    const Out &o = out[bidx * 16 + w];
                    cyc += (double)(o.c1 - o.c0);
                    rt += (double)(o.t1 - o.t0);
                }
            cyc /= blocks * waves;
            rt /= blocks * waves;
            const double mhz = cyc / rt * 100.0;
            const double wi = (double)R * 2 * 4 * 12 * sh.nb; /* per wave: 2 rounds x 4 sub-steps x 12 NB VALU */
            const double cpi_evt = (ms * 1e-3) * mhz * 1e6 / (sh.wps * wi);
            printf("%-16s R=%d %8.3f ms  clock %6.0f MHz  SIMD-cycles/wave-instr %.3f (event)  ns/block/SIMD %.3f  check %s\n",
                   sh.name, R, ms, mhz, cpi_evt, ms * 1e6 / ((double)sh.wps * sh.nb * 64 * R / 10.0 * 1.0) ,
                   bad ? "FAIL" : "ok");
            hipEventDestroy(e0);
            hipEventDestroy(e1);
        }
    hipFree(d_state);
    hipFree(d_out);
    return 0;
}
