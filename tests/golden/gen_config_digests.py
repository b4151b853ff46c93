"""Full-size golden digests of the bench workloads.

Test infrastructure: runs the CPU oracle (oracle/_build/liboracle.so, pinned
against the reference's own vectors in tests/test_oracle.py) over the exact
synthetic inputs bench.py generates at N = 1 (SplitMix64
plaintext of seed 0x7074 over the strided input slots, keys of seed 0x6B6579
at word 4*key_id, nonce base 0) and records, per config, the SHA-256 of the
packed plaintexts (pins the generator) and of the packed sealed records
(ct || tag, record after record, stride padding excluded).

    python tests/golden/gen_config_digests.py   ->  tests/golden/config_digests.json
    python tests/golden/gen_config_digests.py --ref-check c3 c4
        (re-derives the committed digests through the reference build,
         oracle/_ref, and marks them reference_checked)
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from oracle import REF_SO, Oracle, RefLib  # noqa: E402

CHACHA, AES = 0x4301, 0x4302
SEED_PT, SEED_KEY = 0x7074, 0x6B6579
ALIGN = 16
# bench.py CONFIGS at N = 1 (C5 is ragged and covered by its own tests)
CONFIGS = {
    "c2": dict(cipher=CHACHA, records=65536, len=1400, states=1),
    "c3": dict(cipher=AES, records=65536, len=1400, states=1),
    "c4": dict(cipher=CHACHA, records=1048576, len=1400, states=4096),
    # noise-c's tests/performance shape (bench.py "perf"): 1024-B records with
    # 32 B of AD each, the AD the SplitMix64 stream of seed 0x6164
    "perf": dict(cipher=CHACHA, records=65536, len=1024, states=1, ad=32),
}
SEED_AD = 0x6164


def stride(n):
    return (n + ALIGN - 1) // ALIGN * ALIGN


def digests(o, name, cfg):
    N, L, S = cfg["records"], cfg["len"], cfg["states"]
    ins, outs = stride(L), stride(L + 16)
    keys = np.frombuffer(b"".join(o.fill(SEED_KEY, 32, 4 * k) for k in range(S)), dtype=np.uint8).copy()
    nb = np.zeros(S, dtype=np.uint64)
    pt = np.frombuffer(o.fill(SEED_PT, N * ins, 0), dtype=np.uint8).copy()
    ct = np.zeros(N * outs, dtype=np.uint8)
    AD = cfg.get("ad", 0)
    if AD:
        ad = np.frombuffer(o.fill(SEED_AD, N * AD, 0), dtype=np.uint8).copy()
        o.seal_uniform_ad(cfg["cipher"], keys, nb, N // S, pt, ins, ct, outs, L, N, ad, AD, AD)
    else:
        o.seal_uniform(cfg["cipher"], keys, nb, N // S, pt, ins, ct, outs, L, N)
    return dict(cipher=cfg["cipher"], records=N, len=L, states=S, recs_per_state=N // S,
                in_stride=ins, out_stride=outs, ad=AD,
                pt_sha256=hashlib.sha256(pt.reshape(N, ins)[:, :L].tobytes()).hexdigest(),
                sealed_sha256=hashlib.sha256(ct.reshape(N, outs)[:, :L + 16].tobytes()).hexdigest())


def ref_digest(o, cfg):
    """A config's sealed digest through the reference's own CipherState API
    (oracle/_ref, built from /root/reference), one call per record: record i
    belongs to state i // rps (key = SplitMix64 words at 4 * state) and is
    sealed at nonce i % rps — C2 / C3 / perf (one state) and C4 (4096 states
    x 256 records)."""
    ref = RefLib()
    N, L, AD, S = cfg["records"], cfg["len"], cfg.get("ad", 0), cfg["states"]
    rps = N // S
    ins = stride(L)
    keys = [o.fill(SEED_KEY, 32, 4 * s) for s in range(S)]
    pt = o.fill(SEED_PT, N * ins, 0)
    ad = o.fill(SEED_AD, N * AD, 0) if AD else b""
    h = hashlib.sha256()
    for i in range(N):
        h.update(ref.encrypt(cfg["cipher"], keys[i // rps], i % rps, pt[i * ins:i * ins + L],
                             ad[i * AD:(i + 1) * AD]))
    return h.hexdigest()


def c5_digest(o):
    """C5 at N = 1 (bench.py run_mixed, rank 0): 128 Ki records of 64 B-16 KiB
    over 512 states, ChaChaPoly for even states and AES-GCM for odd, record j
    at slot offset off[j] with nonce j % rps.  Sealed through the reference
    build (its AES is ~30x faster than the bit-serial oracle here); every
    64th record is re-sealed by the oracle as a cross-check."""
    sys.path.insert(0, ROOT)
    from bench import CONFIGS as BC, mixed_layout
    R, S = BC["c5"]["records"], BC["c5"]["states"]
    lay = mixed_layout(R, S, 0)
    pt = o.fill(SEED_PT, lay["total"], 0)
    ref = RefLib()
    keys = [o.fill(SEED_KEY, 32, 4 * s) for s in range(S)]
    hp, hs = hashlib.sha256(), hashlib.sha256()
    for j in range(R):
        s, off, L, n = int(lay["st_global"][j]), int(lay["off"][j]), int(lay["lens"][j]), int(lay["nonce"][j])
        cipher = CHACHA if s % 2 == 0 else AES
        p = pt[off:off + L]
        c = ref.encrypt(cipher, keys[s], n, p)
        if j % 64 == 0:
            assert c == o.encrypt(cipher, keys[s], n, p), j
        hp.update(p)
        hs.update(c)
    return dict(records=R, states=S, lens_sum=int(lay["lens"].sum()), total=lay["total"],
                pt_sha256=hp.hexdigest(), sealed_sha256=hs.hexdigest(), reference_checked=True)


def main():
    o = Oracle()
    out = {"generator": "tests/golden/gen_config_digests.py (CPU oracle)", "configs": {}}
    if sys.argv[1:2] == ["--ref-check"]:
        # reference-check the committed digests of the named configs (no
        # oracle re-run): `--ref-check c3 c4`
        path = os.path.join(ROOT, "tests", "golden", "config_digests.json")
        with open(path) as f:
            out = json.load(f)
        for name in sys.argv[2:]:
            t = time.time()
            d = ref_digest(o, CONFIGS[name])
            assert d == out["configs"][name]["sealed_sha256"], f"oracle != reference on {name}"
            out["configs"][name]["reference_checked"] = True
            print(name, f"reference build agrees ({time.time() - t:.1f}s)")
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
        return
    only = sys.argv[1:]  # e.g. `perf`: add that config to the existing file, keep the others
    path = os.path.join(ROOT, "tests", "golden", "config_digests.json")
    if only:
        with open(path) as f:
            out = json.load(f)
        for name in only:
            t = time.time()
            out["configs"][name] = digests(o, name, CONFIGS[name])
            print(name, f"{time.time() - t:.1f}s", out["configs"][name]["sealed_sha256"][:16])
            if os.path.exists(REF_SO):
                assert ref_digest(o, CONFIGS[name]) == out["configs"][name]["sealed_sha256"], name
                out["configs"][name]["reference_checked"] = True
                print(name, "reference build agrees")
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
        return
    for name, cfg in CONFIGS.items():
        t = time.time()
        out["configs"][name] = digests(o, name, cfg)
        print(name, f"{time.time() - t:.1f}s", out["configs"][name]["sealed_sha256"][:16])
    if os.path.exists(REF_SO):
        for name in CONFIGS:
            t = time.time()
            d = ref_digest(o, CONFIGS[name])
            assert d == out["configs"][name]["sealed_sha256"], f"oracle != reference on {name}"
            out["configs"][name]["reference_checked"] = True
            print(name, f"reference build agrees ({time.time() - t:.1f}s)")
        t = time.time()
        out["configs"]["c5"] = c5_digest(o)
        print("c5", f"{time.time() - t:.1f}s", out["configs"]["c5"]["sealed_sha256"][:16])
    with open(os.path.join(ROOT, "tests", "golden", "config_digests.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
