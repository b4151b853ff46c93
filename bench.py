#!/usr/bin/env python3
"""bench.py — device-resident Noise transport AEAD throughput on MI355X.

Metric (BASELINE.json): GiB/s device-resident AEAD encrypt+decrypt of
64 Ki x 1400 B records per GPU.  One "step" = one seal pass (encrypt +
Poly1305/GHASH tag) over the batch followed by one open pass (verify + decrypt)
of the sealed batch, both through the C ABI of noise-c_amd
(noise_aead_dev_{seal,open}_uniform).  Payload processed per step per GPU =
2 x records x len (every byte goes through one AEAD op in each direction).
Inputs are resident in HBM before timing; the batch sets rotate so that the
working set (> 1 GiB) cannot be served from the 256 MiB Infinity Cache.

Multi-GPU: one process per GPU (torchrun), records sharded by range with no
data-path collective — each rank seals/opens its own 64 Ki records of the
global stream (nonce base = rank x records): weak scaling.  Only the timing
barrier and a max-over-ranks all_reduce use the process group.

The CPU baseline is the reference noise-c itself (oracle/_ref/ref_bench: the
reference's CipherState API compiled from its own sources), timed on this
host's cores on a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "noise-c_amd"))

CHACHA, AES = 0x4301, 0x4302
GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, MI355X_MICROARCH.md chip table

CONFIGS = {
    # name: cipher, records per GPU, record length, key states per GPU
    "c2": dict(cipher=CHACHA, records=65536, len=1400, states=1,
               workload="ChaCha20-Poly1305 64Ki x 1400B records, one CipherState key"),
    "c3": dict(cipher=AES, records=65536, len=1400, states=1,
               workload="AES-256-GCM 64Ki x 1400B records, one CipherState key"),
    # C4: 1 Mi records / 4096 states IN TOTAL, sharded by state
    # block over the ranks (strong scaling)
    "c4": dict(cipher=CHACHA, records=1048576, len=1400, states=4096, strong=True,
               workload="ChaCha20-Poly1305 1Mi x 1400B records, 4096 CipherStates x 256"),
    # noise-c's own tests/performance perf_cipher shape (test-performance.c
    # :140-179): 1024-B records with 32 B of associated data each
    "perf": dict(cipher=CHACHA, records=65536, len=1024, states=1, ad=32,
                 workload="ChaCha20-Poly1305 64Ki x 1024B records + 32B AD (tests/performance shape)"),
    # C5 per GPU = 1/8 of the 8-GPU job (1 Mi records, 4096 states in total):
    # lengths 64 + splitmix64(seed_len + i) mod 16321, cipher by state parity.
    "c5": dict(cipher=None, records=131072, len=None, states=512,
               workload="Mixed ChaChaPoly (even states) + AESGCM (odd states), 64 B-16 KiB "
                        "records (SURVEY.md 8d C5), 128 Ki records / 512 CipherStates per GPU, "
                        "ragged descriptors"),
}
SEED_LEN, SEED_PT, SEED_KEY = 0x6C656E, 0x7074, 0x6B6579
# NOISE_BENCH_REHEARSE=1: rehearse the N>1 code path on a one-GPU box — every
# rank on cuda:0, gloo process group, collectives on CPU copies.  Only the
# transport differs from the real run (RCCL refuses two ranks on one GPU).
REHEARSE = os.environ.get("NOISE_BENCH_REHEARSE") == "1"


def cpu_if_rehearsal(t):
    return t.cpu() if REHEARSE else t
# Device record slots: strides roundup(len, SLOT_ALIGN) / roundup(len + 16,
# SLOT_ALIGN).  Whole 128-B lines per slot keep a record's first and last
# lines its own: with 16-B slots (1408 / 1424 B at 1400 B) the open re-read
# the line shared with the neighbouring record and the tag's line (duplex HBM
# bytes 1.13x vs 1.10x algorithmic); +0.6-0.8 % at C2/C3/C4 in three
# interleaved rounds (profiles/r02/align_all_ab.jsonl).  DESIGN.md §3.
IN_ALIGN = 16
SLOT_ALIGN = 128


def shard(records_per_gpu: int, states: int, rank: int, world: int):
    """Records of rank `rank` in the global stream (weak scaling): the rank's
    records are [rank*R, (rank+1)*R); with S states per GPU, global state
    rank*S + s owns records rank*R + s*(R/S) ... and its nonces start at 0.
    With a single state per GPU the ranks share one logical CipherState whose
    nonce runs across the ranks' ranges (nonce base = rank*R)."""
    first = rank * records_per_gpu
    rps = records_per_gpu // states
    if states == 1:
        nonce_base = [first]
    else:
        nonce_base = [0] * states
    key_ids = [rank * states + s for s in range(states)] if states > 1 else [0]
    return dict(first=first, count=records_per_gpu, rps=rps, nonce_base=nonce_base,
                key_ids=key_ids)


def splitmix64_np(x):
    """SplitMix64 of uint64 array x (oracle_splitmix64)."""
    import numpy as np
    with np.errstate(over="ignore"):
        z = x.astype(np.uint64) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def mixed_layout(records_per_gpu: int, states: int, rank: int):
    """C5 shard of rank: global record i = rank*R + j, length
    64 + splitmix64(SEED_LEN + i) % 16321, state rank*S + j // (R/S),
    ChaChaPoly for even global states, AESGCM for odd; record slots are
    roundup64(len + 16) bytes (FAST: 16-B aligned, readable past the tag)."""
    import numpy as np
    R, S = records_per_gpu, states
    gi = np.arange(rank * R, (rank + 1) * R, dtype=np.uint64)
    lens = (np.uint64(64) + splitmix64_np(np.uint64(SEED_LEN) + gi) % np.uint64(16321)).astype(np.int64)
    slot = (lens + 16 + 63) // 64 * 64
    off = np.zeros(R, dtype=np.int64)
    off[1:] = np.cumsum(slot)[:-1]
    rps = R // S
    st_local = np.arange(R) // rps
    st_global = rank * S + st_local
    nonce = (np.arange(R) % rps).astype(np.uint64)
    return dict(lens=lens, off=off, total=int(off[-1] + slot[-1]), st_local=st_local,
                st_global=st_global, nonce=nonce, rps=rps)


def stride(n: int, align: int = IN_ALIGN) -> int:
    return (n + align - 1) // align * align


def physical_cores(cpus):
    """Distinct physical cores (package, core id) among the logical CPUs."""
    seen = set()
    for c in cpus:
        base = f"/sys/devices/system/cpu/cpu{c}/topology/"
        try:
            with open(base + "physical_package_id") as f:
                pkg = f.read().strip()
            with open(base + "core_id") as f:
                core = f.read().strip()
        except OSError:
            return None
        seen.add((pkg, core))
    return len(seen) or None


def host_cpu():
    """CPU model, logical CPUs, the affinity set, its physical cores and the
    CPU share this job is given (SURVEY.md 8d asks for the core count)."""
    model = None
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = sorted(os.sched_getaffinity(0))
    except AttributeError:
        aff = list(range(os.cpu_count() or 1))
    share = os.environ.get("OMP_NUM_THREADS")
    return {"cpu_model": model, "nproc": os.cpu_count(), "usable_cpus": len(aff),
            "physical_cores": physical_cores(aff),
            "cpu_share": int(share) if share and share.isdigit() else None}


def cpu_baseline(cfg, budget_cpu_s: float = 12.0):
    """Reference noise-c on this host's cores, bounded sample."""
    r = _cpu_baseline(cfg, budget_cpu_s)
    return None if r is None else {**r, **host_cpu()}


def ref_perf_cipher(path, timeout_s=120.0):
    """Run the reference's tests/performance program (oracle/_ref/
    test-performance, built from its own sources) and read its ChaChaPoly and
    AESGCM perf_cipher lines (MiB/s; test-performance.c:140-179, 420-422).
    It goes on to time DH and signatures, which this baseline does not need:
    once both cipher lines are out the child is stopped (by its own PID)."""
    p = subprocess.Popen([path], stdout=subprocess.PIPE, text=True)
    out, t0 = {}, time.time()
    try:
        for line in p.stdout:
            f = line.split()
            if len(f) >= 3 and f[0] in ("ChaChaPoly", "AESGCM"):
                out[f[0]] = float(f[1])
            if len(out) == 2 or time.time() - t0 > timeout_s:
                break
    finally:
        p.kill()
        p.wait()
    return out


def _cpu_baseline(cfg, budget_cpu_s):
    ref = os.path.join(ROOT, "oracle", "_ref", "ref_bench")
    kind = "reference"
    if not os.path.exists(ref):
        ref = os.path.join(ROOT, "oracle", "_build", "port_bench")
        kind = "port"
    if not os.path.exists(ref):
        return None
    cname = "aesgcm" if cfg["cipher"] == AES else "chachapoly"
    if cfg.get("ad"):
        # the reference's own tests/performance program, unchanged: 1 thread,
        # 200 MiB of 1024-B records with 32 B AD, encrypt only, CPU-time clock
        tp = os.path.join(ROOT, "oracle", "_ref", "test-performance")
        if os.path.exists(tp):
            r = ref_perf_cipher(tp)
            name = "AESGCM" if cfg["cipher"] == AES else "ChaChaPoly"
            return {"value": round(r[name] / 1024.0, 4), "unit": "GiB/s", "cores": 1,
                    "kind": "reference",
                    "sample": f"noise-c tests/performance/test-performance (built from the reference's "
                              f"sources, run unchanged): perf_cipher {name}, 200 MiB of 1024 B + 32 B AD "
                              f"encrypts, one thread, CPU-time clock (encrypt only); its AESGCM/ChaChaPoly "
                              f"lines: {r}"}
        out = subprocess.run([ref, "perf", cname, str(cfg["len"]), "200000", "1"],
                             capture_output=True, text=True, timeout=300, check=True)
        r = json.loads(out.stdout)
        return {"value": round(r["mib_per_s"] / 1024.0, 4), "unit": "GiB/s", "cores": 1,
                "kind": kind, "sample": f"{'reference library' if kind == 'reference' else 'oracle port'} "
                f"in a restatement of perf_cipher's loop (oracle/ref_bench.c perf; the reference's "
                f"test-performance binary was not built): 200000 x 1024 B + 32 B AD encrypts, one "
                f"thread, CPU-time clock (encrypt only)"}
    hc = host_cpu()
    usable, phys = hc["usable_cpus"], hc["physical_cores"] or hc["usable_cpus"]
    # one thread per physical core of the affinity set, within the CPU share
    # this job is given on the box (OMP_NUM_THREADS: 16 of the host's cores
    # per GPU on the pool; other jobs share the host)
    threads = max(1, min(phys, usable, hc["cpu_share"] or phys))
    # calibrate on one thread (~0.3 s), then size the sample to the budget
    probe_n = 200 if cfg["cipher"] == AES else 2000
    out = subprocess.run([ref, "roundtrip", cname, str(cfg["len"]), str(probe_n), "1"],
                         capture_output=True, text=True, timeout=120, check=True)
    p = json.loads(out.stdout)
    rec_per_s = probe_n / max(p["seconds"], 1e-6)
    per_thread = max(probe_n, int(rec_per_s * budget_cpu_s / threads))
    out = subprocess.run([ref, "roundtrip", cname, str(cfg["len"]), str(per_thread),
                          str(threads)], capture_output=True, text=True, timeout=600, check=True)
    r = json.loads(out.stdout)
    one = subprocess.run([ref, "roundtrip", cname, str(cfg["len"]), str(max(probe_n, int(rec_per_s * 2))), "1"],
                         capture_output=True, text=True, timeout=120, check=True)
    r1 = json.loads(one.stdout)
    res = {"value": round(r["gib_per_s"], 4), "unit": "GiB/s", "cores": threads, "kind": kind,
           "single_thread": round(r1["gib_per_s"], 4),
           "sample": (f"{'noise-c ref backend CipherState API' if kind == 'reference' else 'oracle restatement'}"
                      f" {cname}: {threads} threads (one per physical core, within this job's CPU share) x "
                      f"{per_thread} records x {cfg['len']} B, each encrypted then decrypted+verified "
                      f"(send/recv CipherState pair per thread), wall clock; 1 thread: "
                      f"{r1['gib_per_s']:.3f} GiB/s"),
           "ok": r["ok"]}
    if phys > threads:
        # not run (the box gives this job `threads` cores): per-thread rate x
        # the affinity set's physical cores, an upper bound for linear scaling
        res["all_physical_cores_linear_estimate"] = round(r["gib_per_s"] / threads * phys, 3)
    return res


def kernel_name(cipher, n, rps, lanes, in_stride, out_stride, length, duplex=False, ct=False):
    """The kernel the library dispatches for this uniform job's seal
    (aead_api.hip run_uniform) or, duplex, for the whole step (run_duplex), as
    rocprofv3 names it."""
    fast = in_stride % 16 == 0 and out_stride % 16 == 0 and in_stride >= (max(length, 1) + 63) // 64 * 64
    if duplex and cipher == CHACHA and fast and lanes in (4, 8):
        return f"chachapoly_duplex_staged<{lanes}, {'true' if rps % (64 // lanes) == 0 else 'false'}>"
    if cipher == AES:
        c = "true" if ct else "false"
        if fast and rps % 256 == 0:
            return f"gcm_duplex_staged<{c}>" if duplex else f"gcm_staged<false, {c}>"
        return f"gcm_uniform<false, {c}>"
    if fast and lanes >= 4:
        return f"chachapoly_seal_staged<{lanes}, {'true' if rps % (64 // lanes) == 0 else 'false'}>"
    return f"chachapoly_seal_uniform<{lanes}, {'true' if fast else 'false'}>"


def load_pmc(config_name: str, kernel: str, scale: float = 1.0):
    """Per-launch PMC counters of `kernel` from profiles/traffic_<cfg>.json
    (tools/gpu/pmc.sh + tools/pmc_report.py, collected at N = 1), or {}.
    `scale`: this launch's share of the profiled one (1/N for a strong-scaling
    shard; the counters are per-launch totals proportional to the records)."""
    path = os.path.join(ROOT, "profiles", f"traffic_{config_name}.json")
    if not os.path.exists(path):
        return {}
    with open(path) as f:
        t = json.load(f)
    k = t.get("kernels", {}).get(kernel) or {}
    return {n: v * scale for n, v in k.items()} if scale != 1.0 else k


# VALU issue ceiling: a SIMD issues one wave64 integer VALU
# instruction per ~4 cycles for the shift/rotate/multiply class and whenever
# fast (add/xor) and slow ops interleave (profiles/r01_rates_dep.log), so the
# chip-wide ceiling is 1024 SIMDs x 2.4 GHz / 4 wave-instructions per second.
VALU_ISSUE_PEAK = 1024 * 2.4e9 / 4


def issue_bound(pmc, avg_launch_ms):
    n = pmc.get("SQ_INSTS_VALU")
    if not n or not avg_launch_ms:
        return None
    rate = n / (avg_launch_ms * 1e-3)
    return {"resource": "VALU issue (wave-instructions/s)", "valu_insts_per_launch": int(n),
            "achieved": round(rate / 1e9, 1), "peak": round(VALU_ISSUE_PEAK / 1e9, 1),
            "unit": "G wave-instr/s", "frac": round(rate / VALU_ISSUE_PEAK, 4),
            "source": "SQ_INSTS_VALU from the committed PMC profile / live launch time"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--lanes", type=int, default=0, help="lanes per record (0 = library default)")
    ap.add_argument("--sets", type=int, default=4, help="rotating batch sets (> MALL)")
    ap.add_argument("--align", type=int, default=SLOT_ALIGN, choices=(16, 64, 128, 256),
                    help="record slot alignment of the device batch (strides roundup(len, align), "
                         "roundup(len + 16, align))")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verify", action="store_true", help="check every open status after timing")
    ap.add_argument("--no-xfer", action="store_true",
                    help="skip the N>1 scatter/seal/gather leg (RCCL, SURVEY.md 8e)")
    ap.add_argument("--xfer-reps", type=int, default=5)
    ap.add_argument("--n1-value", type=float, default=None,
                    help="value of the same config at N = 1: adds per_gpu_efficiency for N > 1")
    ap.add_argument("--mode", default="duplex", choices=("duplex", "separate"),
                    help="duplex: each step seals one set and opens another in ONE launch "
                         "(noise_aead_dev_duplex_uniform); separate: a seal launch then an open launch")
    ap.add_argument("--events", default="ends", choices=("ends", "step"),
                    help="ends: HIP events only around the timed region (per-launch time = "
                         "its interval / launches); step: events at every launch boundary")
    ap.add_argument("--streams", type=int, default=1, choices=(1, 2),
                    help="C2-C4/perf: 2 = consecutive steps alternate between two streams")
    ap.add_argument("--ct-ghash", action="store_true",
                    help="AES-GCM: NOISE_AEAD_FLAG_CT_GHASH (table-free GHASH)")
    ap.add_argument("--c5-streams", type=int, default=2, choices=(1, 2),
                    help="C5: 2 = the AES-GCM and ChaChaPoly halves on two streams, concurrently")
    args = ap.parse_args()

    import torch
    import noise_aead as A

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if REHEARSE:
        local = 0
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if REHEARSE:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    cfg = CONFIGS[args.config]
    if args.config == "c5":
        return run_mixed(args, cfg, A, torch, dev, rank, world, dist)
    cipher, N, L, S = cfg["cipher"], cfg["records"], cfg["len"], cfg["states"]
    if cfg.get("strong"):
        if N % world or S % world:
            raise SystemExit(f"{args.config}: {N} records / {S} states do not split over {world} ranks")
        N, S = N // world, S // world
    sh = shard(N, S, rank, world)
    in_stride, out_stride = stride(L, args.align), stride(L + 16, args.align)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream

    # keys: SplitMix64 words of seed 0x6B6579 at 4*(global key id)
    key_ids = torch.tensor(sh["key_ids"], dtype=torch.int64)
    raw = torch.empty(len(sh["key_ids"]) * 32, dtype=torch.uint8, device=dev)
    for i, kid in enumerate(sh["key_ids"]):
        assert A.dev_fill_splitmix(raw[32 * i:].data_ptr(), 32, 0x6B6579, 4 * kid, sp) == 0
    ctx = torch.empty(len(sh["key_ids"]) * A.dev_ctx_bytes(cipher), dtype=torch.uint8, device=dev)
    assert A.dev_prepare(cipher, raw.data_ptr(), len(sh["key_ids"]), ctx.data_ptr(), sp) == 0
    nonce = torch.tensor(sh["nonce_base"], dtype=torch.int64, device=dev)
    del key_ids
    AD = cfg.get("ad", 0)
    ad_buf = None
    if AD:
        ad_buf = torch.empty(N * AD, dtype=torch.uint8, device=dev)
        assert A.dev_fill_splitmix(ad_buf.data_ptr(), ad_buf.numel(), 0x6164, sh["first"] * AD // 8, sp) == 0
    ad_kw = dict(ad=ad_buf.data_ptr() if AD else 0, ad_stride=AD, ad_len=AD)

    sets = []
    for b in range(args.sets):
        pt = torch.empty(N * in_stride, dtype=torch.uint8, device=dev)
        # plaintext word w of the global stream = splitmix64(seed_pt + w)
        word0 = (sh["first"] * in_stride + b * (1 << 40)) // 8
        assert A.dev_fill_splitmix(pt.data_ptr(), pt.numel(), 0x7074, word0, sp) == 0
        ct = torch.empty(N * out_stride, dtype=torch.uint8, device=dev)
        back = torch.empty(N * in_stride, dtype=torch.uint8, device=dev)
        st = torch.empty(N, dtype=torch.uint8, device=dev)
        sets.append((pt, ct, back, st))
    torch.cuda.synchronize(dev)

    lanes = args.lanes or A.dev_default_lanes(cipher, N)
    jflags = A.FLAG_CT_GHASH if args.ct_ghash else 0

    def seal(b, pt=None, ct=None, stream=sp):
        if pt is None:
            pt, ct, _, _ = sets[b]
        return A.dev_uniform(False, cipher, ctx=ctx.data_ptr(), nonce_base=nonce.data_ptr(),
                             inp=pt.data_ptr(), out=ct.data_ptr(), in_stride=in_stride,
                             out_stride=out_stride, length=L, n_records=N,
                             recs_per_state=sh["rps"], lanes=lanes, flags=jflags, stream=stream,
                             **ad_kw)

    def open_(b, stream=sp):
        _, ct, back, st = sets[b]
        return A.dev_uniform(True, cipher, ctx=ctx.data_ptr(), nonce_base=nonce.data_ptr(),
                             inp=ct.data_ptr(), out=back.data_ptr(), in_stride=out_stride,
                             out_stride=in_stride, length=L, n_records=N,
                             recs_per_state=sh["rps"], status=st.data_ptr(), lanes=lanes,
                             flags=jflags, stream=stream, **ad_kw)

    # Each step seals set b = s % sets and opens set (s - LAG) % sets, sealed LAG
    # steps earlier: the ciphertext an open reads was written two full steps
    # (> 700 MB of traffic) before, so it comes from HBM, not from the 256 MiB
    # Infinity Cache.  Every set is sealed once before timing, so every open
    # has ciphertext; a set's ciphertext is the same at every seal.
    lag = 2 if args.sets >= 3 else 0
    duplex = args.mode == "duplex"

    def jobs(b, bo, stream):
        pt, ct, _, _ = sets[b]
        _, cto, back, st = sets[bo]
        common = dict(ctx=ctx.data_ptr(), nonce_base=nonce.data_ptr(), length=L, n_records=N,
                      recs_per_state=sh["rps"], lanes=lanes, flags=jflags, **ad_kw)
        sj = A.uniform_job(inp=pt.data_ptr(), out=ct.data_ptr(), in_stride=in_stride,
                           out_stride=out_stride, **common)
        oj = A.uniform_job(inp=cto.data_ptr(), out=back.data_ptr(), in_stride=out_stride,
                           out_stride=in_stride, status=st.data_ptr(), **common)
        return sj, oj

    def step_duplex(b, bo, stream=sp):
        sj, oj = jobs(b, bo, stream)
        return A.dev_duplex(cipher, sj, oj, stream)

    # --streams 2 (separate mode): consecutive steps (independent batch sets)
    # alternate between two streams, so step s+1's seal can start on CUs that
    # step s's open is leaving.  Set b is reused only every `sets` steps.
    streams = [stream] + ([torch.cuda.Stream(dev)] if args.streams == 2 and not duplex else [])

    for b in range(args.sets):
        assert seal(b) == 0
    for w in range(args.warmup):
        b, bo = w % args.sets, (w - lag) % args.sets
        if duplex:
            assert step_duplex(b, bo) == 0
        else:
            assert seal(b) == 0
            assert open_(bo) == 0
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    per_step = args.events == "step"
    if duplex or not per_step:  # launch boundaries (duplex) or just the region's ends
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    else:
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
               torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if duplex or not per_step:
        ev[0].record(stream)
    for s in range(args.steps):
        b, bo = s % args.sets, (s - lag) % args.sets
        if duplex or not per_step:
            if duplex:
                rc = step_duplex(b, bo)
            else:
                st_ = streams[s % len(streams)].cuda_stream
                rc = seal(b, stream=st_) or open_(bo, stream=st_)
            if per_step or s == args.steps - 1:
                ev[s + 1].record(stream)
            if rc:
                raise RuntimeError(f"launch failed {rc:#x}")
            continue
        st_ = streams[s % len(streams)]
        ev[s][0].record(st_)
        rc1 = seal(b, stream=st_.cuda_stream)
        ev[s][1].record(st_)
        rc2 = open_(bo, stream=st_.cuda_stream)
        ev[s][2].record(st_)
        if rc1 or rc2:
            raise RuntimeError(f"launch failed {rc1:#x} {rc2:#x}")
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if dist:
        t = cpu_if_rehearsal(torch.tensor([elapsed], dtype=torch.float64, device=dev))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.barrier()

    if duplex or not per_step:
        # average launch interval over the timed region, gaps included
        launch_ms = ev[0].elapsed_time(ev[args.steps]) / args.steps / (1 if duplex else 2)
    else:
        seal_ms = sum(e[0].elapsed_time(e[1]) for e in ev) / args.steps
        open_ms = sum(e[1].elapsed_time(e[2]) for e in ev) / args.steps
    if duplex or not per_step or len(streams) > 1:
        # per-direction launch times (separate kernels) from a serial, untimed pass
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        reps = 5
        e[0].record(stream)
        for r in range(reps):
            seal(r % args.sets)
        e[1].record(stream)
        for r in range(reps):
            open_((r - lag) % args.sets)
        e[2].record(stream)
        torch.cuda.synchronize(dev)
        seal_ms = e[0].elapsed_time(e[1]) / reps
        open_ms = e[1].elapsed_time(e[2]) / reps

    ok = True
    if args.verify:
        for b in range(args.sets):
            pt, _, back, st = sets[b]
            ok &= bool((st == 0).all().item())
            v = pt.view(N, in_stride)[:, :L]
            ok &= bool(torch.equal(back.view(N, in_stride)[:, :L], v))

    payload_step = 2.0 * N * L * world                         # both directions, all ranks
    value = payload_step * args.steps / elapsed / GIB
    alg_seal = N * (2 * L + 16 + AD) + len(sh["key_ids"]) * 40  # SURVEY §8d algorithmic bytes (+AD read)
    kname = kernel_name(cipher, N, sh["rps"], lanes, in_stride, out_stride, L, duplex, args.ct_ghash)
    if "_duplex_" in kname:
        # the one launch of a step: one seal + one open of N records each
        alg_launch, launch_ms_ = 2 * alg_seal, launch_ms
    elif not duplex and not per_step:
        # seal and open alternate: the mean interval per launch, gaps included
        alg_launch, launch_ms_ = alg_seal, launch_ms
    else:
        alg_launch, launch_ms_ = alg_seal, seal_ms
    achieved = alg_launch / (launch_ms_ * 1e-3) / 1e9
    pmc = load_pmc(args.config, kname, 1.0 / world if cfg.get("strong") else 1.0)
    traffic = pmc.get("hbm_bytes_per_launch")
    result = {
        "metric": (f"GiB/s device-resident AEAD encrypt+decrypt, {N * world // 1024}Ki x {L}B "
                   f"records in total over {S * world} CipherStates, sharded by state"
                   if cfg.get("strong") else
                   f"GiB/s device-resident AEAD encrypt+decrypt, {N // 1024}Ki x {L}B records"
                   + (f" + {AD}B AD" if AD else "") + " per GPU"),
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "strong" if cfg.get("strong") else "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (SplitMix64 plaintext and keys, SURVEY.md 8d), resident in HBM",
        "config": {"workload": cfg["workload"], "config": args.config, "records_per_gpu": N,
                   "record_len": L, "states_per_gpu": S, "lanes_per_record": lanes,
                   "in_stride": in_stride, "out_stride": out_stride,
                   "payload_bytes_per_step": int(payload_step), "parallelism": f"records x{world}",
                   "streams": len(streams), "mode": args.mode, "events": args.events,
                   "open_reads_set_sealed_steps_before": lag,
                   **({"ct_ghash": True} if args.ct_ghash else {})},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "kernel": kname,
                     "algorithmic_bytes_per_launch": alg_launch,
                     "avg_launch_ms": round(launch_ms_, 5),
                     "issue_bound": issue_bound(pmc, launch_ms_)},
        "seal_gibs": round(N * L * world / (seal_ms * 1e-3) / GIB, 2),
        "open_gibs": round(N * L * world / (open_ms * 1e-3) / GIB, 2),
        "open_roofline_frac": round(alg_seal / (open_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
    }
    if args.verify:
        result["verified"] = ok
    if world > 1 and not args.no_xfer:
        try:  # reported beside the value; a failure here never voids the bench line
            result["scatter_gather"] = xfer_leg(args, torch, dist, dev, A, rank, world, N, L,
                                                in_stride, out_stride, sh, sets, seal)
        except Exception as e:
            result["scatter_gather"] = {"error": repr(e)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            result["cpu_baseline"] = cpu_baseline(cfg)
        except Exception as e:  # reported, never fatal to the GPU number
            result["cpu_baseline"] = {"error": str(e)}
    finish(args, result, rank, world, dist)


def finish(args, result, rank, world, dist):
    """Per-GPU efficiency when an N = 1 value is given, the
    rehearsal label, then rank 0 prints the one JSON line."""
    if args.n1_value and world > 1:
        # (aggregate GiB/s at N) / (N x GiB/s at N = 1), for weak and strong
        # scaling alike (strong: total work fixed, so this is speedup / N)
        result["per_gpu_efficiency"] = round(result["value"] / (world * args.n1_value), 4)
        result["n1_value"] = args.n1_value
    if REHEARSE and world > 1:
        # every rank on one GPU, collectives on gloo: exercises the N > 1 code
        # path only; per-kernel rates of ranks sharing a GPU mean nothing
        result.pop("roofline", None)
        result["rehearsal"] = (f"{world} ranks on ONE GPU, gloo process group (collectives via host "
                               "memory): a code-path rehearsal, not a multi-GPU measurement")
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


def xfer_leg(args, torch, dist, dev, A, rank, world, N, L, in_stride, out_stride, sh, sets, seal):
    """the batch starts and ends on rank 0's GPU.  Rank 0 holds
    the whole job's plaintext (world shards, each equal to that rank's set-0
    input), RCCL scatters the shards, every rank seals its own, RCCL gathers
    the sealed shards back to rank 0.  Timed per phase (max over ranks);
    reported beside, never instead of, the device-resident value."""
    from distribute import scatter_records, gather_records
    sp = torch.cuda.current_stream(dev).cuda_stream
    shard_in, shard_out = N * in_stride, N * out_stride
    full_in = full_out = None
    if rank == 0:
        full_in = torch.empty(world * shard_in, dtype=torch.uint8, device=dev)
        full_out = torch.empty(world * shard_out, dtype=torch.uint8, device=dev)
        for g in range(world):  # shard g = rank g's set-0 plaintext (same SplitMix64 words)
            assert A.dev_fill_splitmix(full_in[g * shard_in:].data_ptr(), shard_in, 0x7074,
                                       (g * N * in_stride) // 8, sp) == 0
    local_in = torch.empty(shard_in, dtype=torch.uint8, device=dev)
    local_out = torch.empty(shard_out, dtype=torch.uint8, device=dev)
    phases = []
    for rep in range(args.xfer_reps + 1):
        torch.cuda.synchronize(dev)
        dist.barrier()
        t0 = time.perf_counter()
        if REHEARSE:  # gloo scatters CPU tensors
            tmp = torch.empty(shard_in, dtype=torch.uint8)
            scatter_records(tmp, full_in.cpu() if rank == 0 else None, src=0)
            local_in.copy_(tmp)
        else:
            scatter_records(local_in, full_in, src=0)
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        if seal(0, local_in, local_out):
            raise RuntimeError("seal launch failed")
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        if REHEARSE:
            tmp = torch.empty(world * shard_out, dtype=torch.uint8) if rank == 0 else None
            gather_records(local_out.cpu(), tmp, dst=0)
            if rank == 0:
                full_out.copy_(tmp)
        else:
            gather_records(local_out, full_out, dst=0)
        torch.cuda.synchronize(dev)
        t3 = time.perf_counter()
        if rep:  # rep 0 warms RCCL's channels
            phases.append((t1 - t0, t2 - t1, t3 - t2, t3 - t0))
    ph = cpu_if_rehearsal(torch.tensor(phases, dtype=torch.float64, device=dev).mean(0))
    dist.all_reduce(ph, op=dist.ReduceOp.MAX)
    # checks: scattered shard == this rank's own input; gathered shard g ==
    # rank g's sealed output (int64 checksums, all_gathered)
    ok = cpu_if_rehearsal(torch.tensor([1 if torch.equal(local_in, sets[0][0]) else 0], device=dev))
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    mine = cpu_if_rehearsal(local_out.view(torch.int64).sum().reshape(1))
    sums = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(sums, mine)
    good = bool(ok.item())
    if rank == 0:
        for g in range(world):
            got = full_out[g * shard_out:(g + 1) * shard_out].view(torch.int64).sum()
            good &= bool(got.item() == sums[g].item())
    sc, se, ga, tot = (float(x) * 1e3 for x in ph.tolist())
    return {"collective": ("torch.distributed scatter/gather on gloo via host memory (one-GPU rehearsal)"
                           if REHEARSE else
                           "torch.distributed scatter/gather on nccl (RCCL grouped send/recv over xGMI)"),
            "src_dst_rank": 0, "shard_in_bytes": shard_in, "shard_out_bytes": shard_out,
            "scatter_ms": round(sc, 4), "seal_ms": round(se, 4), "gather_ms": round(ga, 4),
            "total_ms": round(tot, 4),
            "seal_gibs_incl_xfer": round(N * L * world / (tot * 1e-3) / GIB, 2),
            "scatter_gbs": round((world - 1) * shard_in / (sc * 1e-3) / 1e9, 1),
            "gather_gbs": round((world - 1) * shard_out / (ga * 1e-3) / 1e9, 1),
            "verified": good, "reps": args.xfer_reps}


def run_mixed(args, cfg, A, torch, dev, rank, world, dist):
    """C5: mixed-cipher ragged batch, seal then open (tags verified)."""
    import numpy as np
    R, S = cfg["records"], cfg["states"]
    lay = mixed_layout(R, S, rank)
    sp = torch.cuda.current_stream(dev).cuda_stream
    rec_dt = np.dtype([("in_off", "<u8"), ("out_off", "<u8"), ("nonce", "<u8"), ("ctx_off", "<u8"),
                       ("ad_off", "<u8"), ("len", "<u4"), ("ad_len", "<u4")])
    assert rec_dt.itemsize == 48
    pt = torch.empty(lay["total"], dtype=torch.uint8, device=dev)
    assert A.dev_fill_splitmix(pt.data_ptr(), pt.numel(), SEED_PT, rank << 40, sp) == 0
    ct = torch.empty_like(pt)
    back = torch.empty_like(pt)
    groups = []
    for cipher, parity in ((CHACHA, 0), (AES, 1)):
        states = [s for s in range(S) if (rank * S + s) % 2 == parity]
        if not states:
            continue
        cb = A.dev_ctx_bytes(cipher)
        raw = torch.empty(len(states) * 32, dtype=torch.uint8, device=dev)
        for i, s in enumerate(states):
            assert A.dev_fill_splitmix(raw[32 * i:].data_ptr(), 32, SEED_KEY, 4 * (rank * S + s), sp) == 0
        ctx = torch.empty(len(states) * cb, dtype=torch.uint8, device=dev)
        assert A.dev_prepare(cipher, raw.data_ptr(), len(states), ctx.data_ptr(), sp) == 0
        slot_of = {s: i for i, s in enumerate(states)}
        idx = np.nonzero((lay["st_global"] % 2) == parity)[0]
        recs = np.zeros(len(idx), dtype=rec_dt)
        recs["in_off"] = lay["off"][idx]
        recs["out_off"] = lay["off"][idx]
        recs["nonce"] = lay["nonce"][idx]
        recs["ctx_off"] = np.array([slot_of[s] for s in lay["st_local"][idx]], dtype=np.uint64) * cb
        recs["len"] = lay["lens"][idx]
        d_recs = torch.from_numpy(recs.view(np.uint8)).to(dev)
        st = torch.empty(len(idx), dtype=torch.uint8, device=dev)
        groups.append(dict(cipher=cipher, ctx=ctx, recs=d_recs, n=len(idx), st=st,
                           bytes=int(lay["lens"][idx].sum()), states=len(states)))
    torch.cuda.synchronize(dev)

    def launch(g, open_, stream=sp, inp=None, out=None):
        inp = inp if inp is not None else (ct if open_ else pt)
        out = out if out is not None else (back if open_ else ct)
        return A.dev_ragged(open_, g["cipher"], ctx_base=g["ctx"].data_ptr(),
                            recs=g["recs"].data_ptr(), inp=inp.data_ptr(),
                            out=out.data_ptr(), n_records=g["n"],
                            status=g["st"].data_ptr() if open_ else 0, lanes=args.lanes,
                            flags=A.FLAG_FAST, stream=stream)

    # Two streams: the LDS-bound AES-GCM kernel and the VALU-bound ChaChaPoly
    # kernel share the CUs instead of running back to back; the open phase
    # waits for both seals (fork/join by events, no host sync).
    main_s = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev) if args.c5_streams == 2 and len(groups) == 2 else None
    fork = [torch.cuda.Event() for _ in range(2)]
    join = [torch.cuda.Event() for _ in range(2)]

    def step():
        for open_ in (False, True):
            if side is None:
                for g in groups:
                    rc = launch(g, open_)
                    if rc:
                        raise RuntimeError(f"launch failed {rc:#x}")
                continue
            fork[open_].record(main_s)
            side.wait_event(fork[open_])
            rc = launch(groups[1], open_, side.cuda_stream) or launch(groups[0], open_)
            if rc:
                raise RuntimeError(f"launch failed {rc:#x}")
            join[open_].record(side)
            main_s.wait_event(join[open_])

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if dist:
        t = cpu_if_rehearsal(torch.tensor([elapsed], dtype=torch.float64, device=dev))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.barrier()
    # per-kernel times (separate, untimed pass) for the roofline line
    per = []
    for open_ in (False, True):
        for g in groups:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                launch(g, open_)
            e1.record()
            torch.cuda.synchronize(dev)
            per.append((e0.elapsed_time(e1) / 5, g, open_))
    ok = all(bool((g["st"] == 0).all().item()) for g in groups)
    if args.verify:  # round trip on a sample of records (statuses: all of them, above)
        rng = np.random.default_rng(rank)
        for j in rng.choice(R, size=min(512, R), replace=False):
            o, n = int(lay["off"][j]), int(lay["lens"][j])
            ok &= bool(torch.equal(back[o:o + n], pt[o:o + n]))
    payload = sum(g["bytes"] for g in groups)
    value = 2.0 * payload * world * args.steps / elapsed / GIB
    ms, g, open_ = max(per, key=lambda x: x[0])
    alg = 2 * g["bytes"] + 16 * g["n"] + 40 * g["states"]
    achieved = alg / (ms * 1e-3) / 1e9
    # the kernel the library dispatches (aead_api.hip run_ragged), as rocprofv3 names it
    if g["cipher"] == CHACHA:  # run_ragged: 8 lanes below 128 Ki records, else 4
        k = args.lanes or (8 if g["n"] < 131072 else 4)
        kname = f"chachapoly_{'open' if open_ else 'seal'}_ragged<{k}, true>"
    else:  # gcm_ragged_shape: (threads, records per group, lanes per record) by batch size
        n_aes = g["n"]
        wg, r, kl = (1024, 2, 4) if n_aes >= 131072 else ((1024, 2, 8) if n_aes >= 65536 else (256, 1, 4))
        kname = f"gcm_ragged_staged<{'true' if open_ else 'false'}, true, {wg}, false, {r}, {kl}>"
    pmc = load_pmc("c5", kname)
    result = {
        "metric": "GiB/s device-resident AEAD encrypt+decrypt, mixed 64B-16KiB records per GPU",
        "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic (SplitMix64 lengths, plaintext and keys, SURVEY.md 8d C5), resident in HBM",
        "config": {"workload": cfg["workload"], "config": "c5", "records_per_gpu": R,
                   "states_per_gpu": S, "payload_bytes_per_step": int(2 * payload * world),
                   "streams": 2 if side is not None else 1,
                   "parallelism": f"states x{world}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": pmc.get("hbm_bytes_per_launch"),
                     "kernel": kname, "algorithmic_bytes_per_launch": alg,
                     "avg_launch_ms": round(ms, 5), "issue_bound": issue_bound(pmc, ms)},
        "kernels_ms": {(("chacha" if gg["cipher"] == CHACHA else "aes") + ("_open" if o else "_seal")): round(m, 4)
                       for m, gg, o in per},
        "all_tags_verified": ok,
    }
    if world > 1 and not args.no_xfer:
        try:  # reported beside the value; a failure here never voids the bench line
            result["scatter_gather"] = xfer_leg_mixed(args, torch, dist, dev, A, rank, world, R, S,
                                                      lay, pt, groups, launch)
        except Exception as e:
            result["scatter_gather"] = {"error": repr(e)}
    finish(args, result, rank, world, dist)


def xfer_leg_mixed(args, torch, dist, dev, A, rank, world, R, S, lay, pt, groups, launch):
    """The C5 form of xfer_leg: rank 0 holds every rank's
    ragged plaintext shard, RCCL scatters them (shards differ in size, so each
    travels in a slot of the largest shard's size), every rank seals its own
    records of both ciphers, RCCL gathers the sealed shards back.  The record
    descriptors are not sent: each rank derives its own from the shared layout
    rule (mixed_layout).  Timed per phase, max over ranks; verified."""
    from distribute import scatter_records, gather_records
    sp = torch.cuda.current_stream(dev).cuda_stream
    totals = [mixed_layout(R, S, g)["total"] for g in range(world)]
    slot = (max(totals) + 63) // 64 * 64
    full_in = full_out = None
    if rank == 0:
        full_in = torch.zeros(world * slot, dtype=torch.uint8, device=dev)
        full_out = torch.zeros(world * slot, dtype=torch.uint8, device=dev)
        for g in range(world):  # slot g = rank g's plaintext (its SplitMix64 words)
            assert A.dev_fill_splitmix(full_in[g * slot:].data_ptr(), totals[g], SEED_PT, g << 40, sp) == 0
    local_in = torch.zeros(slot, dtype=torch.uint8, device=dev)
    local_out = torch.zeros(slot, dtype=torch.uint8, device=dev)
    phases = []
    for rep in range(args.xfer_reps + 1):
        torch.cuda.synchronize(dev)
        dist.barrier()
        t0 = time.perf_counter()
        if REHEARSE:
            tmp = torch.empty(slot, dtype=torch.uint8)
            scatter_records(tmp, full_in.cpu() if rank == 0 else None, src=0)
            local_in.copy_(tmp)
        else:
            scatter_records(local_in, full_in, src=0)
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        for g in groups:
            if launch(g, False, inp=local_in, out=local_out):
                raise RuntimeError("seal launch failed")
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        if REHEARSE:
            tmp = torch.empty(world * slot, dtype=torch.uint8) if rank == 0 else None
            gather_records(local_out.cpu(), tmp, dst=0)
            if rank == 0:
                full_out.copy_(tmp)
        else:
            gather_records(local_out, full_out, dst=0)
        torch.cuda.synchronize(dev)
        t3 = time.perf_counter()
        if rep:
            phases.append((t1 - t0, t2 - t1, t3 - t2, t3 - t0))
    ph = cpu_if_rehearsal(torch.tensor(phases, dtype=torch.float64, device=dev).mean(0))
    dist.all_reduce(ph, op=dist.ReduceOp.MAX)
    total = lay["total"]
    ok = cpu_if_rehearsal(torch.tensor([1 if torch.equal(local_in[:total], pt[:total]) else 0],
                                       device=dev))
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    mine = cpu_if_rehearsal(local_out.view(torch.int64).sum().reshape(1))
    sums = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(sums, mine)
    good = bool(ok.item())
    if rank == 0:
        for g in range(world):
            got = full_out[g * slot:(g + 1) * slot].view(torch.int64).sum()
            good &= bool(got.item() == sums[g].item())
    sc, se, ga, tot = (float(x) * 1e3 for x in ph.tolist())
    payload = sum(int(mixed_layout(R, S, g)["lens"].sum()) for g in range(world))
    return {"collective": ("torch.distributed scatter/gather on gloo via host memory (one-GPU rehearsal)"
                           if REHEARSE else
                           "torch.distributed scatter/gather on nccl (RCCL grouped send/recv over xGMI)"),
            "src_dst_rank": 0, "slot_bytes": slot, "shard_bytes": totals,
            "scatter_ms": round(sc, 4), "seal_ms": round(se, 4), "gather_ms": round(ga, 4),
            "total_ms": round(tot, 4),
            "seal_gibs_incl_xfer": round(payload / (tot * 1e-3) / GIB, 2),
            "verified": good, "reps": args.xfer_reps}


if __name__ == "__main__":
    main()
