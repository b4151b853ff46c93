"""Cycle accounting of the persistent ragged ChaChaPoly kernel (debug
variant built with -DNA_SEG_TL: make -C noise-c_amd variant NAME=tl
DEFS=-DNA_SEG_TL) on C5's ChaChaPoly half, standalone: per-wave sums of
set-up, DMA waits, passes, combine + tag and the end-of-job drain, as
fractions of the waves' lives.  Prints one JSON line per direction.

    NOISE_AEAD_LIB=noise-c_amd/ab/libnoise_aead_hip_tl.so python tools/seg_tl.py
"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "noise-c_amd"))


def main():
    import numpy as np
    import torch
    import bench
    import noise_aead as A
    lib = A.lib()
    lib.noise_aead_debug_seg_tl.restype = C.c_int
    dev = torch.device("cuda", 0)
    R, S = bench.CONFIGS["c5"]["records"], bench.CONFIGS["c5"]["states"]
    lay = bench.mixed_layout(R, S, 0)
    sp = torch.cuda.current_stream(dev).cuda_stream
    pt = torch.empty(lay["total"], dtype=torch.uint8, device=dev)
    assert A.dev_fill_splitmix(pt.data_ptr(), pt.numel(), bench.SEED_PT, 0, sp) == 0
    ct = torch.empty_like(pt)
    back = torch.empty_like(pt)
    states = [s for s in range(S) if s % 2 == 0]
    cb = A.dev_ctx_bytes(bench.CHACHA)
    raw = torch.empty(len(states) * 32, dtype=torch.uint8, device=dev)
    for i, s in enumerate(states):
        assert A.dev_fill_splitmix(raw[32 * i:].data_ptr(), 32, bench.SEED_KEY, 4 * s, sp) == 0
    ctx = torch.empty(len(states) * cb, dtype=torch.uint8, device=dev)
    assert A.dev_prepare(bench.CHACHA, raw.data_ptr(), len(states), ctx.data_ptr(), sp) == 0
    slot_of = {s: i for i, s in enumerate(states)}
    idx = np.nonzero((lay["st_global"] % 2) == 0)[0]
    rec_dt = np.dtype([("in_off", "<u8"), ("out_off", "<u8"), ("nonce", "<u8"), ("ctx_off", "<u8"),
                       ("ad_off", "<u8"), ("len", "<u4"), ("ad_len", "<u4")])
    recs = np.zeros(len(idx), dtype=rec_dt)
    recs["in_off"] = recs["out_off"] = lay["off"][idx]
    recs["nonce"] = lay["nonce"][idx]
    recs["ctx_off"] = np.array([slot_of[s] for s in lay["st_local"][idx]], dtype=np.uint64) * cb
    recs["len"] = lay["lens"][idx]
    d_recs = torch.from_numpy(recs.view(np.uint8)).to(dev)
    st = torch.empty(len(idx), dtype=torch.uint8, device=dev)

    def launch(open_):
        return A.dev_ragged(open_, bench.CHACHA, ctx_base=ctx.data_ptr(), recs=d_recs.data_ptr(),
                            inp=(ct if open_ else pt).data_ptr(), out=(back if open_ else ct).data_ptr(),
                            n_records=len(idx), status=st.data_ptr() if open_ else 0,
                            flags=A.FLAG_FAST, stream=sp)
    out = (C.c_uint64 * 8)()
    for open_ in (False, True):
        for _ in range(30):
            assert launch(open_) == 0
        torch.cuda.synchronize()
        lib.noise_aead_debug_seg_tl(out, 1)
        assert launch(open_) == 0
        torch.cuda.synchronize()
        waves = lib.noise_aead_debug_seg_tl(out, 1)
        c = list(out)
        life = c[0] or 1
        names = ["life", "setup", "wait_first", "wait_steps", "passes", "combine_tag", "drain", "jobs"]
        print(json.dumps({"open": open_, "waves": waves, "jobs": c[7],
                          "cycles_per_wave": round(life / max(waves, 1)),
                          "frac_of_life": {n: round(v / life, 4) for n, v in zip(names[1:7], c[1:7])},
                          "pass_compute_frac": round((c[4] - c[2] - c[3]) / life, 4)}))


if __name__ == "__main__":
    main()
