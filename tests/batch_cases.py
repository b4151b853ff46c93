"""Shared cases for noise_cipherstate_decrypt_batch (host logic).

The batch must leave results, buffers, sizes and nonces exactly as the
sequential calls would (src/protocol/cipherstate.c:373-410: a MAC failure
leaves the record and n untouched, so the next record of the state is tried
at the same n).  Used by tests/test_gpu_hardening.py (real library, MI355X)
and tests/test_batch_host.py (the sanitized CPU stub of the device calls).
"""
import ctypes as C

import numpy as np

NONCE_LIMIT = 2**64 - 1


def sequential_model(oracle, cipher, key, n0, records):
    """What per-record noise_cipherstate_decrypt calls return, in order."""
    n, out = n0, []
    for r in records:
        if n == NONCE_LIMIT:
            out.append((0x450D, None))  # NOISE_ERROR_INVALID_NONCE
            continue
        rc, pt = oracle.decrypt(cipher, key, n, r)
        if rc == 0:
            out.append((0, pt))
            n += 1
        else:
            out.append((0x4504, None))  # NOISE_ERROR_MAC_FAILURE
    return out, n


def make_records(oracle, cipher, key, pattern, rng, n0=0, max_len=300):
    """pattern[i] True = a forged record.  Good records are sealed at the
    nonce the sequential calls will have reached for them."""
    records, n = [], n0
    for forged in pattern:
        L = int(rng.integers(0, max_len))
        if forged or n >= NONCE_LIMIT:  # past exhaustion nothing can be sealed
            records.append(bytes(rng.integers(0, 256, L + 16, dtype=np.uint8)))
        else:
            records.append(oracle.encrypt(cipher, key, n, bytes(rng.integers(0, 256, L, dtype=np.uint8))))
            n += 1
    return records


def run_batch(aead, states, records):
    mems = [(C.c_uint8 * max(1, len(r))).from_buffer_copy(r or b"\0") for r in records]
    bufs = [aead.NoiseBuffer.input(m, len(r)) for m, r in zip(mems, records)]
    rc, res = aead.decrypt_batch(states, bufs)
    rounds, disp = C.c_uint64(), C.c_uint64()
    aead.lib().noise_aead_debug_batch_stats(C.byref(rounds), C.byref(disp))
    return rc, res, mems, bufs, rounds.value, disp.value


def check_against_model(oracle, cipher, key, n0, records, res, mems, bufs, state):
    exp, n_end = sequential_model(oracle, cipher, key, n0, records)
    for i, ((erc, ept), r) in enumerate(zip(exp, records)):
        assert res[i] == erc, (i, res[i], erc)
        if erc == 0:
            assert bufs[i].size == len(ept) and bytes(mems[i])[:len(ept)] == ept, i
        else:  # untouched (verify-then-decrypt, cipherstate.c:400-405)
            assert bufs[i].size == len(r) and bytes(mems[i])[:len(r)] == r, i
    assert state.nonce == n_end
