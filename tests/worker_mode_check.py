"""Child process of test_gpu_worker.py's placement test (not collected by
pytest): single-record seal/open through the resident worker, checked
against the oracle, under whatever NOISE_AEAD_WORKER_VRAM the parent set.
The worker picks its request placement once per process, hence the child.
Prints "placement N" (noise_aead_debug_worker_placement) and exits non-zero
on the first mismatch."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "noise-c_amd")):
    sys.path.insert(0, p)

import noise_aead as aead  # noqa: E402
import oracle as O  # noqa: E402


def main():
    if not os.path.exists(O.ORACLE_SO):
        O.build(ref=False)
    orc = O.Oracle()
    aead.lib()
    for cipher in (0x4301, 0x4302):
        rnd = random.Random(cipher ^ 0x77)
        key = bytes(rnd.randrange(256) for _ in range(32))
        _, tx = aead.CipherState.new_by_id(cipher)
        _, rx = aead.CipherState.new_by_id(cipher)
        assert tx.init_key(key) == 0 and rx.init_key(key) == 0
        n = 0
        for L in (0, 1, 17, 1024, 1400, 2100, 3100, 4033, 8000, 16384):
            if cipher == 0x4302 and L > 4096:
                continue
            for A in (0, 32):
                pt = bytes(rnd.randrange(256) for _ in range(L))
                ad = bytes(rnd.randrange(256) for _ in range(A))
                ct = tx.seal(pt, ad)
                if ct != orc.encrypt(cipher, key, n, pt, ad):
                    print("seal mismatch", hex(cipher), L, A)
                    return 1
                bad = bytearray(ct)
                bad[rnd.randrange(len(bad))] ^= 1
                rc, back = rx.open(bytes(bad), ad)
                if rc != aead.ERROR_MAC_FAILURE or back != bytes(bad) or rx.nonce != n:
                    print("tamper not rejected", hex(cipher), L, A)
                    return 1
                rc, back = rx.open(ct, ad)
                if rc != 0 or back != pt:
                    print("open mismatch", hex(cipher), L, A)
                    return 1
                n += 1
        tx.free()
        rx.free()
    print("placement", aead.lib().noise_aead_debug_worker_placement())
    return 0


def free_check():
    """--free-check (run with NOISE_AEAD_DEBUG_WORKER_IDLE_MS=10000, so no
    worker leaves by idling): an AES-GCM single call leaves the worker
    resident with the state's context cached in LDS; freeing the state must
    make it leave (it zeroes that cache on the way out) within 200 ms.
    Prints "left_ms X"."""
    import time
    lib = aead.lib()
    lib.noise_aead_debug_workers_resident.restype = int
    _, st = aead.CipherState.new_by_id(0x4302)
    assert st.init_key(bytes(range(32))) == 0
    st.seal(bytes(100))
    time.sleep(0.05)
    if lib.noise_aead_debug_workers_resident() < 1:
        print("no resident worker after the call")
        return 1
    t0 = time.time()
    st.free()
    while lib.noise_aead_debug_workers_resident() and time.time() - t0 < 0.2:
        time.sleep(0.001)
    left = lib.noise_aead_debug_workers_resident() == 0
    print("left_ms", round((time.time() - t0) * 1e3, 3) if left else -1)
    return 0 if left else 1


def free_concurrent():
    """--free-concurrent (run with NOISE_AEAD_WORKER_QUEUES=2,
    NOISE_AEAD_WORKER_SLOTS=1 and NOISE_AEAD_DEBUG_WORKER_IDLE_MS=10000:
    two groups of one slot each): thread A keeps making ChaChaPoly
    single calls (its worker stays resident, its request headers keep being
    written); the main thread's AES-GCM state S, used once from the main
    thread (the other worker caches its context), is freed.  The worker that
    was sent S's context must leave — its stop word is no longer part of the
    header A's calls rewrite — and A's worker, which never saw
    S's context, must stay (no relaunch of it).  Prints "parked_ok 1"."""
    import threading
    import time
    lib = aead.lib()
    lib.noise_aead_debug_workers_resident.restype = int
    lib.noise_aead_debug_worker_launches.restype = int
    stop = [False]
    errs = []
    started = threading.Event()

    def caller():
        _, cs = aead.CipherState.new_by_id(0x4301)
        cs.init_key(bytes(range(32)))
        n = 0
        while not stop[0]:
            if len(cs.seal(bytes(1400))) != 1416:
                errs.append("seal")
            n += 1
            if n == 50:
                started.set()
        cs.free()

    T0 = time.time()
    marks = []
    th = threading.Thread(target=caller)
    th.start()
    started.wait(30)
    marks.append(time.time())
    _, st = aead.CipherState.new_by_id(0x4302)
    assert st.init_key(bytes(range(1, 33))) == 0
    st.seal(bytes(100))
    marks.append(time.time())
    time.sleep(0.05)
    import ctypes as C

    def per_group():
        a = (C.c_uint * 12)()
        lib.noise_aead_debug_worker_group_launches(a, 12)
        return list(a)
    g0 = per_group()
    res0, l0 = lib.noise_aead_debug_workers_resident(), lib.noise_aead_debug_worker_launches()
    st.free()
    t0 = time.time()
    while lib.noise_aead_debug_workers_resident() >= res0 and time.time() - t0 < 0.5:
        time.sleep(0.001)
    res1 = lib.noise_aead_debug_workers_resident()
    marks.append(time.time())
    time.sleep(0.1)
    l1 = lib.noise_aead_debug_worker_launches()
    stop[0] = True
    th.join()
    ok = res0 == 2 and res1 == 1 and l1 == l0 and not errs
    print("resident", res0, res1, "launches", l0, l1, "errs", errs[:3])
    print("per group + ensure causes", g0, per_group())
    lib.noise_aead_debug_worker_leave_reason.restype = C.c_uint
    print("leave reasons g0 g1", lib.noise_aead_debug_worker_leave_reason(0, 0),
          lib.noise_aead_debug_worker_leave_reason(1, 0))
    for gi in (0, 1):
        a = (C.c_uint * 4)()
        lib.noise_aead_debug_worker_leave_info(gi, 0, a)
        print("leave info", gi, list(a), "age_s", ((a[1] - a[0]) & 0xffffffff) / 1e8)
    print("timeline", [round(x - T0, 3) for x in marks])
    print("parked_ok", 1 if ok else 0)
    return 0 if ok else 1


def relaunch_free():
    """--relaunch-free (run with NOISE_AEAD_DEBUG_WORKER_LEAVE=1 and
    NOISE_AEAD_DEBUG_WORKER_IDLE_MS=10000): every single call's group leaves
    after the call checked it was up and before the request is posted, so the
    call's wait loop relaunches the group and the new workgroup serves the
    request and caches the AES-GCM context.  Freeing the state must still park
    that group within 200 ms (the relaunch used to wipe the slot's
    context history).  The call's result is checked against the oracle.
    Prints "relaunch_free_ok 1"."""
    import time
    lib = aead.lib()
    lib.noise_aead_debug_workers_resident.restype = int
    orc = O.Oracle()
    key = bytes(range(7, 39))
    _, st = aead.CipherState.new_by_id(0x4302)
    assert st.init_key(key) == 0
    pt = bytes(range(200))
    ct = st.seal(pt)
    if ct != orc.encrypt(0x4302, key, 0, pt):
        print("seal mismatch")
        return 1
    time.sleep(0.05)
    res0 = lib.noise_aead_debug_workers_resident()
    t0 = time.time()
    st.free()
    while lib.noise_aead_debug_workers_resident() and time.time() - t0 < 0.2:
        time.sleep(0.001)
    res1 = lib.noise_aead_debug_workers_resident()
    ok = res0 >= 1 and res1 == 0
    print("resident", res0, res1)
    print("relaunch_free_ok", 1 if ok else 0)
    return 0 if ok else 1


def group_idle():
    """--group-idle (run with NOISE_AEAD_WORKER_QUEUES=1,
    NOISE_AEAD_WORKER_SLOTS=2, NOISE_AEAD_DEBUG_WORKER_IDLE_MS=20): one
    group of two slots.  The main thread makes one call (its slot then stays
    idle) while thread A keeps calling for 300 ms: the group must not leave
    for the idle slot's sake (a workgroup leaves for idleness only when every
    slot of its group is idle), so no relaunch happens; once both are quiet
    the group leaves by itself.  Prints "group_idle_ok 1"."""
    import threading
    import time
    lib = aead.lib()
    lib.noise_aead_debug_workers_resident.restype = int
    lib.noise_aead_debug_worker_launches.restype = int
    _, mine = aead.CipherState.new_by_id(0x4301)
    mine.init_key(bytes(range(32)))
    started = threading.Event()
    stop = [False]
    errs = []

    def caller():
        _, cs = aead.CipherState.new_by_id(0x4301)
        cs.init_key(bytes(range(3, 35)))
        started.set()
        while not stop[0]:
            if len(cs.seal(bytes(1400))) != 1416:
                errs.append("seal")
        cs.free()

    assert len(mine.seal(bytes(100))) == 116  # slot 0: launches the group
    th = threading.Thread(target=caller)
    th.start()
    started.wait(30)
    time.sleep(0.05)
    l0 = lib.noise_aead_debug_worker_launches()
    time.sleep(0.3)  # 15 idle timeouts of the main thread's slot
    l1 = lib.noise_aead_debug_worker_launches()
    stop[0] = True
    th.join()
    t0 = time.time()
    while lib.noise_aead_debug_workers_resident() and time.time() - t0 < 2.0:
        time.sleep(0.005)
    left = lib.noise_aead_debug_workers_resident() == 0
    mine.free()
    ok = l0 == l1 and left and not errs
    print("launches", l0, l1, "left", left, "errs", errs[:3])
    print("group_idle_ok", 1 if ok else 0)
    return 0 if ok else 1


if __name__ == "__main__":
    if "--group-idle" in sys.argv:
        sys.exit(group_idle())
    if "--free-check" in sys.argv:
        sys.exit(free_check())
    if "--free-concurrent" in sys.argv:
        sys.exit(free_concurrent())
    if "--relaunch-free" in sys.argv:
        sys.exit(relaunch_free())
    sys.exit(main())
