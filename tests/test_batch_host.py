"""noise_cipherstate_decrypt_batch host logic on the CPU.

These run only against the sanitized host build (noise-c_amd/asan: the real
cipherstate.c over CPU stubs of the device calls, which compute with the
oracle — test infrastructure), started by tests/test_sanitizers.py with
NOISE_AEAD_LIB pointing at it.  The same cases run on the MI355X against the
product library in tests/test_gpu_hardening.py.

- a run of k forged records costs O(log k) GPU rounds (forge windows of 1, 2,
  4, ... records tried at the same nonce), not one round per forgery;
- random forgery patterns over several interleaved states equal the
  sequential calls (cipherstate.c:373-410) record for record.
"""
import math
import os

import numpy as np
import pytest

from batch_cases import check_against_model, make_records, run_batch

CHACHA, AES = 0x4301, 0x4302

pytestmark = pytest.mark.skipif(
    not os.environ.get("NOISE_AEAD_LIB", "").endswith("libnoise_aead_asan.so"),
    reason="host-logic test: runs under tests/test_sanitizers.py (sanitized CPU stub)")


@pytest.mark.parametrize("cipher", [CHACHA, AES])
@pytest.mark.parametrize("before,forged,after", [(3, 60, 80), (0, 1000, 5), (50, 7, 0), (1, 1, 1)])
def test_forged_run_costs_log_rounds(aead, oracle, cipher, before, forged, after):
    rng = np.random.default_rng(before * 7 + forged + after + (cipher & 3))
    key = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
    pattern = [False] * before + [True] * forged + [False] * after
    records = make_records(oracle, cipher, key, pattern, rng, max_len=120)
    st = aead.CipherState.new_by_id(cipher)[1]
    st.init_key(key)
    rc, res, mems, bufs, rounds, disp = run_batch(aead, [st] * len(records), records)
    assert rc == 0
    check_against_model(oracle, cipher, key, 0, records, res, mems, bufs, st)
    total = len(records)
    # one optimistic round, log2(k) forge rounds, log2 of the tail's windows
    assert rounds <= 2 * math.log2(total + 1) + 3, (rounds, disp)
    assert disp <= 3 * total + 64, (rounds, disp)
    st.free()


@pytest.mark.parametrize("seed", range(6))
def test_random_forgeries_equal_sequential(aead, oracle, seed):
    """Interleaved states, forgeries at random (isolated and in runs), one
    state close to nonce exhaustion."""
    rng = np.random.default_rng(900 + seed)
    nstates = 4
    keys = [bytes(rng.integers(0, 256, 32, dtype=np.uint8)) for _ in range(nstates)]
    ciphers = [CHACHA if s % 2 == 0 else AES for s in range(nstates)]
    n0 = [0, 5, 2**64 - 4, 1 << 40]
    per = [int(rng.integers(5, 60)) for _ in range(nstates)]
    pat = []
    for s in range(nstates):
        p = rng.random(per[s]) < [0.05, 0.3, 0.2, 0.6][s]
        if seed % 2:  # add a run
            a = int(rng.integers(0, per[s]))
            p[a:a + 9] = True
        pat.append(list(p))
    recs = [make_records(oracle, ciphers[s], keys[s], pat[s], rng, n0=n0[s], max_len=80)
            for s in range(nstates)]
    states = []
    for s in range(nstates):
        st = aead.CipherState.new_by_id(ciphers[s])[1]
        st.init_key(keys[s])
        assert st.set_nonce(n0[s]) == 0
        states.append(st)
    labels = np.repeat(np.arange(nstates), per)
    rng.shuffle(labels)  # interleave the states, each state's records in order
    seqs = [iter(range(per[s])) for s in range(nstates)]
    idx = [(int(s), next(seqs[s])) for s in labels]
    rc, res, mems, bufs, rounds, disp = run_batch(aead, [states[s] for s, _ in idx],
                                                  [recs[s][i] for s, i in idx])
    assert rc == 0
    for s in range(nstates):
        pos = [k for k, (ss, _) in enumerate(idx) if ss == s]
        check_against_model(oracle, ciphers[s], keys[s], n0[s], [recs[s][i] for _, i in
                            (idx[k] for k in pos)], [res[k] for k in pos], [mems[k] for k in pos],
                            [bufs[k] for k in pos], states[s])
    for st in states:
        st.free()
