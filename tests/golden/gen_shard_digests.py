"""Per-rank golden digests of the bench workloads.

Test infrastructure.  bench.py verifies, after its timed region, that the
records its timed kernels sealed hash to these digests — for every rank of
an N-GPU run, so each rank checks its own shard:

  c2, c3, perf (weak scaling): rank r seals global records [r*N, (r+1)*N) of
      the one-key stream, nonces r*N + i, plaintext = the SplitMix64 words of
      the global byte offsets (bench.py: word0 = r*N*in_stride/8), set 0.
      perf also has 32 B of AD per record (seed 0x6164).  Ranks 0..7.
  c4 (strong scaling): 1 Mi records over 4096 states x 256 in total; rank r
      of W holds states [r*4096/W, (r+1)*4096/W).  The digest of every such
      slice for W = 1, 2, 4, 8.
  c5 (weak): rank r's mixed ChaChaPoly/AES-GCM ragged batch (bench.py
      mixed_layout), ranks 0..7, sealed through the reference build (its AES
      is ~30x faster than the bit-serial oracle); every 128th record
      re-sealed by the oracle as a cross-check.
  c5s: the same layout rule at 16 Ki records / 64 states per rank (the GPU
      tests' multi-rank rehearsal), ranks 0..7 (`--c5s` adds it alone).

Each digest is SHA-256 over the sealed records (ct || tag) in record order,
stride padding excluded.  Rank 0 / W = 1 entries equal config_digests.json's.

    python tests/golden/gen_shard_digests.py  ->  tests/golden/shard_digests.json
"""
import hashlib
import json
import os
import sys
import time
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)
from oracle import Oracle, RefLib  # noqa: E402

CHACHA, AES = 0x4301, 0x4302
SEED_PT, SEED_KEY, SEED_AD = 0x7074, 0x6B6579, 0x6164
RANKS = 8
N = 65536


def weak_shard(args):
    """Rank r's set-0 sealed digest of a one-key uniform config."""
    name, cipher, L, ad, ins, outs, r = args
    o = Oracle()
    first = r * N
    key = np.frombuffer(o.fill(SEED_KEY, 32, 0), dtype=np.uint8).copy()
    pt = np.frombuffer(o.fill(SEED_PT, N * ins, first * ins // 8), dtype=np.uint8).copy()
    h = hashlib.sha256()
    if not ad:
        ct = np.zeros(N * outs, dtype=np.uint8)
        o.seal_uniform(cipher, key, np.array([first], dtype=np.uint64), N, pt, ins, ct, outs, L, N)
        h.update(ct.reshape(N, outs)[:, :L + 16].tobytes())
    else:
        adb = o.fill(SEED_AD, N * ad, first * ad // 8)
        kb = key.tobytes()
        for i in range(N):
            h.update(o.encrypt(cipher, kb, first + i, pt[i * ins:i * ins + L].tobytes(),
                               adb[i * ad:(i + 1) * ad]))
    return name, r, h.hexdigest()


def c4_slices():
    """The 1 Mi-record C4 stream sealed state by state; digests of every
    rank's slice for W = 1, 2, 4, 8."""
    o = Oracle()
    S, rps, L, ins, outs = 4096, 256, 1400, 1408, 1424
    hs = {W: [hashlib.sha256() for _ in range(W)] for W in (1, 2, 4, 8)}
    chunk = 64  # states per oracle call
    for s0 in range(0, S, chunk):
        keys = np.frombuffer(b"".join(o.fill(SEED_KEY, 32, 4 * s) for s in range(s0, s0 + chunk)),
                             dtype=np.uint8).copy()
        n = chunk * rps
        pt = np.frombuffer(o.fill(SEED_PT, n * ins, s0 * rps * ins // 8), dtype=np.uint8).copy()
        ct = np.zeros(n * outs, dtype=np.uint8)
        o.seal_uniform(CHACHA, keys, np.zeros(chunk, dtype=np.uint64), rps, pt, ins, ct, outs, L, n)
        packed = ct.reshape(n, outs)[:, :L + 16]
        for W in hs:
            per = S // W  # states per rank
            for s in range(s0, s0 + chunk, per if per < chunk else chunk):
                r = s // per
                cnt = min(per, s0 + chunk - s)
                a = (s - s0) * rps
                hs[W][r].update(packed[a:a + cnt * rps].tobytes())
    return {str(W): [h.hexdigest() for h in v] for W, v in hs.items()}


def c5_rank(r, name="c5"):
    from bench import CONFIGS as BC, mixed_layout
    o = Oracle()
    ref = RefLib()
    R, S = BC[name]["records"], BC[name]["states"]
    lay = mixed_layout(R, S, r)
    pt = o.fill(SEED_PT, lay["total"], r << 40)
    keys = {}
    h = hashlib.sha256()
    for j in range(R):
        s = int(lay["st_global"][j])
        if s not in keys:
            keys[s] = o.fill(SEED_KEY, 32, 4 * s)
        off, L, n = int(lay["off"][j]), int(lay["lens"][j]), int(lay["nonce"][j])
        cipher = CHACHA if s % 2 == 0 else AES
        p = pt[off:off + L]
        c = ref.encrypt(cipher, keys[s], n, p)
        if j % 128 == 0:
            assert c == o.encrypt(cipher, keys[s], n, p), (r, j)
        h.update(c)
    return r, h.hexdigest()


def c5s_rank(r):
    return c5_rank(r, "c5s")


def add_c5s():
    """`--c5s`: add the reduced C5 rehearsal layout's rank digests (bench.py
    CONFIGS["c5s"]: 16 Ki records / 64 states per rank) to the existing file."""
    path = os.path.join(ROOT, "tests", "golden", "shard_digests.json")
    with open(path) as f:
        out = json.load(f)
    with Pool(8) as p:
        res = p.map(c5s_rank, range(RANKS))
    out["configs"]["c5s"] = {"rank_sealed_sha256": [d for _, d in sorted(res)]}
    with open(path, "w") as f:
        json.dump(out, f, indent=1)


def main():
    if sys.argv[1:2] == ["--c5s"]:
        return add_c5s()
    t = time.time()
    jobs = []
    for name, cipher, L, ad, ins, outs in (("c2", CHACHA, 1400, 0, 1408, 1536),
                                           ("c3", AES, 1400, 0, 1408, 1536),
                                           ("perf", CHACHA, 1024, 32, 1024, 1152)):
        jobs += [(name, cipher, L, ad, ins, outs, r) for r in range(RANKS)]
    out = {"generator": "tests/golden/gen_shard_digests.py (CPU oracle; c5 via the reference build)",
           "configs": {"c2": {}, "c3": {}, "perf": {}}}
    with Pool(8) as p:
        res = p.map(weak_shard, jobs)
        c5 = p.map(c5_rank, range(RANKS))
    for name, r, d in res:
        out["configs"][name].setdefault("rank_sealed_sha256", [None] * RANKS)[r] = d
    out["configs"]["c5"] = {"rank_sealed_sha256": [d for _, d in sorted(c5)]}
    with Pool(8) as p:
        out["configs"]["c5s"] = {"rank_sealed_sha256": [d for _, d in sorted(p.map(c5s_rank, range(RANKS)))]}
    print("weak + c5", f"{time.time() - t:.0f}s")
    t = time.time()
    out["configs"]["c4"] = {"world_rank_sealed_sha256": c4_slices()}
    print("c4", f"{time.time() - t:.0f}s")
    with open(os.path.join(ROOT, "tests", "golden", "config_digests.json")) as f:
        base = json.load(f)["configs"]
    for name in ("c2", "c3"):
        assert out["configs"][name]["rank_sealed_sha256"][0] == base[name]["sealed_sha256"], name
    assert out["configs"]["c4"]["world_rank_sealed_sha256"]["1"][0] == base["c4"]["sealed_sha256"]
    assert out["configs"]["c5"]["rank_sealed_sha256"][0] == base["c5"]["sealed_sha256"]
    with open(os.path.join(ROOT, "tests", "golden", "shard_digests.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
