// Hardware-queue probe: does a resident single-call worker hold up other
// streams' work?  Thread A makes single ChaChaPoly calls back to back (its
// worker stays resident); meanwhile the main thread creates streams one by
// one and times a small hipMemsetAsync on each (enqueue -> complete).  A
// stream that shares a hardware queue with the resident worker waits for the
// worker to leave.  prio "high": the application's streams are
// high-priority ones, the pool the workers' streams come from:
// the library leaves one queue of that pool to the application.  Prints one
// JSON line.  Build: tools/build_latency.sh.
//
//   queue_probe [streams] [worker threads] [normal|high]
#include <hip/hip_runtime.h>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>
#include "noise_aead_hip.h"

static double now_us()
{
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv)
{
    const int nstreams = argc > 1 ? atoi(argv[1]) : 8;
    const int workers = argc > 2 ? atoi(argv[2]) : 1;
    const bool high = argc > 3 && !strcmp(argv[3], "high");
    std::atomic<bool> stop{false};
    std::atomic<long> calls{0};
    std::vector<std::thread> th;
    for (int w = 0; w < workers; ++w)
        th.emplace_back([&, w] {
            NoiseCipherState *cs = nullptr;
            if (noise_cipherstate_new_by_id(&cs, NOISE_CIPHER_CHACHAPOLY) != 0) return;
            uint8_t key[32];
            for (int i = 0; i < 32; ++i) key[i] = (uint8_t)(i + w);
            noise_cipherstate_init_key(cs, key, 32);
            std::vector<uint8_t> buf(1400 + 16);
            while (!stop.load()) {
                NoiseBuffer b;
                noise_buffer_set_inout(b, buf.data(), 1400, buf.size());
                if (noise_cipherstate_encrypt(cs, &b) != 0) break;
                calls.fetch_add(1);
            }
            noise_cipherstate_free(cs);
        });
    std::this_thread::sleep_for(std::chrono::milliseconds(200)); /* workers resident */
    void *d = nullptr;
    if (hipMalloc(&d, 1 << 20) != hipSuccess) return 1;
    std::vector<double> us;
    std::vector<hipStream_t> ss;
    for (int i = 0; i < nstreams; ++i) {
        hipStream_t s;
        if (high) {
            int least = 0, greatest = 0;
            if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) return 1;
            if (hipStreamCreateWithPriority(&s, hipStreamNonBlocking, greatest) != hipSuccess) return 1;
        } else if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
            return 1;
        }
        ss.push_back(s);
        const double t0 = now_us();
        if (hipMemsetAsync(d, i, 1 << 20, s) != hipSuccess) return 1;
        if (hipStreamSynchronize(s) != hipSuccess) return 1;
        us.push_back(now_us() - t0);
    }
    stop.store(true);
    for (auto &t : th) t.join();
    printf("{\"streams\": %d, \"priority\": \"%s\", \"worker_threads\": %d, \"calls\": %ld, \"memset_us\": [",
           nstreams, high ? "high" : "normal", workers, calls.load());
    for (size_t i = 0; i < us.size(); ++i) printf("%s%.1f", i ? ", " : "", us[i]);
    printf("]}\n");
    for (auto s : ss) (void)hipStreamDestroy(s);
    (void)hipFree(d);
    return 0;
}
