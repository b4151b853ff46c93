"""Child process of test_gpu_worker.py (not collected by pytest): the time of
a C2-sized one-lane duplex batch (64 Ki x 1400 B sealed + 64 Ki opened, the
bench's kernel) launched right after a single CipherState call — the
resident worker then holds a CU's LDS — against the same batch with no
worker resident.  Rounds alternate the two cases on the warmed-up device.
NOISE_AEAD_WORKER_PARK (the parent's) decides whether batch launches ask the
workers to leave.  Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "noise-c_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import noise_aead as A  # noqa: E402


def main():
    A.lib()
    L, N, ins, outs = 1400, 65536, 1408, 1536
    sp = torch.cuda.current_stream().cuda_stream
    raw = torch.empty(32, dtype=torch.uint8, device="cuda")
    assert A.dev_fill_splitmix(raw.data_ptr(), 32, 0x6B6579, 0, sp) == 0
    ctx = torch.empty(A.dev_ctx_bytes(A.CHACHAPOLY), dtype=torch.uint8, device="cuda")
    assert A.dev_prepare(A.CHACHAPOLY, raw.data_ptr(), 1, ctx.data_ptr(), sp) == 0
    nb = torch.zeros(1, dtype=torch.int64, device="cuda")
    pt = torch.empty(N * ins, dtype=torch.uint8, device="cuda")
    assert A.dev_fill_splitmix(pt.data_ptr(), pt.numel(), 0x7074, 0, sp) == 0
    ct = torch.empty(N * outs, dtype=torch.uint8, device="cuda")
    back = torch.empty(N * ins, dtype=torch.uint8, device="cuda")
    st = torch.empty(N, dtype=torch.uint8, device="cuda")
    common = dict(ctx=ctx.data_ptr(), nonce_base=nb.data_ptr(), length=L, n_records=N,
                  recs_per_state=N)
    assert A.dev_uniform(False, A.CHACHAPOLY, inp=pt.data_ptr(), out=ct.data_ptr(), in_stride=ins,
                         out_stride=outs, stream=sp, **common) == 0
    ct2 = torch.empty_like(ct)
    sj = A.uniform_job(inp=pt.data_ptr(), out=ct2.data_ptr(), in_stride=ins, out_stride=outs, **common)
    oj = A.uniform_job(inp=ct.data_ptr(), out=back.data_ptr(), in_stride=outs, out_stride=ins,
                       status=st.data_ptr(), **common)

    def batch(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            assert A.dev_duplex(A.CHACHAPOLY, sj, oj, sp) == 0
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    import time
    t_end = time.time() + 0.5  # settle the clock (bench.py settle)
    while time.time() < t_end:
        batch(16)
    _, cs = A.CipherState.new_by_id(A.CHACHAPOLY)
    assert cs.init_key(bytes(range(32))) == 0
    lib = A.lib()
    lib.noise_aead_debug_workers_resident.restype = int
    cold, warm, resident_before = [], [], []
    for r in range(12):
        # cold: no worker (the last one has idled out: 2 ms without requests)
        t0 = time.time()
        while lib.noise_aead_debug_workers_resident() and time.time() - t0 < 1.0:
            time.sleep(0.005)
        cold.append(batch(1))
        # warm: a single call leaves the worker resident, then the batch
        cs.seal(bytes(1400))
        resident_before.append(lib.noise_aead_debug_workers_resident())
        warm.append(batch(1))
    assert int(st.max().item()) == 0
    cold.sort()
    warm.sort()
    print(json.dumps({"park": os.environ.get("NOISE_AEAD_WORKER_PARK", "1"),
                      "cold_ms_median": cold[len(cold) // 2], "warm_ms_median": warm[len(warm) // 2],
                      "cold_ms": cold, "warm_ms": warm, "resident_before_warm": resident_before,
                      "ratio": warm[len(warm) // 2] / cold[len(cold) // 2]}))
    cs.free()
    return 0


if __name__ == "__main__":
    sys.exit(main())
