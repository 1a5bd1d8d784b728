"""The thread-safe service (include/blsverify.h blsv_service_*) and the per-context chunk cap.

The reference verifies every arrival in its own goroutine: one per partial packet
(core/drand_public.go:39 -> chain/beacon/node.go:112,125), one per gossip message
(lp2p/client/validator.go:64), one per client.Get (client/verify.go:185-207). Here 64 host threads
(ctypes releases the GIL inside each call) each call VerifyPartial / VerifyRecovered for ONE item at
the same moment; the service coalesces them into one launch. Checked: every verdict and reject class
equals the C oracle's (oracle/c/bls_oracle.c, pinned to the reference KAT), the 64 concurrent calls
are coalesced (at most two launches per burst; the wall time against a lone call is reported, with
one loose sanity bound), a bad key fails only its own call, a batch spanning several pipeline passes
keeps every item's own key, a burst overflowing the key arena runs as sub-batches, and a context
capped at a 256 Ki chunk verifies a 2^20 + 4,099-round history with the verdicts of the uncapped
context.
"""
import hashlib
import sys
import threading
import time

import pytest

pytestmark = pytest.mark.gpu

NONE = (1 << 64) - 1


@pytest.fixture(scope="module")
def C():
    from oracle import c_oracle

    c_oracle.load()
    return c_oracle


@pytest.fixture(scope="module")
def svc():
    from drand_amd.engine import Service

    s = Service(0)
    yield s
    s.close()


def _burst(fns):
    """Run every fn on its own thread, released together by a barrier; (results, wall seconds)."""
    n = len(fns)
    bar = threading.Barrier(n + 1)
    out = [None] * n
    err = []

    def worker(i):
        bar.wait()
        try:
            out[i] = fns[i]()
        except Exception as e:  # noqa: BLE001 - reported below
            err.append(e)

    ths = [threading.Thread(target=worker, args=(i,)) for i in range(n)]
    for t in ths:
        t.start()
    bar.wait()
    t0 = time.perf_counter()
    for t in ths:
        t.join()
    dt = time.perf_counter() - t0
    assert not err, err
    return out, dt


def _mixed_partials(golden):
    """The 64 golden shares of one round with corruptions of several kinds (indices intact)."""
    th = golden["threshold"]
    parts = [bytes.fromhex(p) for p in th["partials"]]
    bad = dict(enumerate(parts))
    bad[3] = parts[3][:50] + bytes([parts[3][50] ^ 4]) + parts[3][51:]          # bit flip
    bad[20] = parts[20][:2] + bytes.fromhex(golden["mixed"]["sigs"][24])       # on curve, not in G2
    bad[41] = ((int.from_bytes(parts[41][:2], "big") + 1) % th["n"]).to_bytes(2, "big") + parts[41][2:]
    bad[63] = bytes.fromhex(th["partials_v2"][0])                              # signs MessageV2
    return [bad[i] for i in range(len(parts))]


BURSTS = 8
# The wall-time bound of a 64-call burst against one lone call. Coalescing itself is asserted
# exactly (launch counts); the time is a report plus one loose sanity bound on the MEDIAN burst:
# the r05 runs measured 1.1-2.3x through Python threads (r05b 5.96 ms against a 2.55 ms lone call,
# thread start-up jitter; the plain-C pthread burst of tools/cabi_smoke.c measures <= 1.5x), while
# an uncoalesced service would take ~64x. 4x separates the two with margin on either side.
BURST_BOUND = 4.0


def _partial_world(golden):
    th = golden["threshold"]
    commits = [bytes.fromhex(c) for c in th["commits"]]
    return th, commits, bytes.fromhex(th["msg"])


def test_service_64_concurrent_partials(svc, golden, C):
    """64 concurrent VerifyPartial calls, each verdict and reject class equal to the C oracle's, in
    at most two launches per burst."""
    th, commits, msg = _partial_world(golden)
    parts = _mixed_partials(golden)
    grp = C.Group(commits)
    want = [grp.verify_partial(msg, p) for p in parts]
    assert sum(1 for c in want if c) == 4
    # the flip at byte 50 lands in x.c0 of the signature: x^3 + 4(u + 1) has no root (NOT_ON_CURVE);
    # the wrong index and the V2-message share reach the pairing and fail it
    assert want[3] == 5 and want[20] == 6 and want[41] == 7 and want[63] == 7

    # arguments marshalled in advance: each thread holds the GIL only for its ctypes call
    calls = [svc.prepare_partial(commits, th["n"], msg, p) for p in parts]
    # warm: the group's PK_i table is built on its first sight, the kernels are loaded
    assert calls[0]() == (True, 0)
    lone = []
    for _ in range(7):
        t0 = time.perf_counter()
        assert calls[1]() == (True, 0)
        lone.append(time.perf_counter() - t0)
    lone_s = sorted(lone)[len(lone) // 2]
    l0, i0, _ = svc.stats()
    times = []
    # a short GIL switch interval so that the 64 Python threads reach their ctypes calls together (the
    # default 5 ms interval can hold the late ones back past the service's coalescing window -- a
    # Python artefact: the plain-C burst in tools/cabi_smoke.c measures the same contract with pthreads)
    old_iv = sys.getswitchinterval()
    sys.setswitchinterval(1e-5)
    try:
        for _ in range(BURSTS):
            res, dt = _burst(calls)
            assert [c for _, c in res] == want
            assert [ok for ok, _ in res] == [c == 0 for c in want]
            times.append(dt)
    finally:
        sys.setswitchinterval(old_iv)
    l1, i1, mb = svc.stats()
    med = sorted(times)[len(times) // 2]
    print(f"lone {lone_s * 1e3:.2f} ms, 64 concurrent median {med * 1e3:.2f} ms (best {min(times) * 1e3:.2f}), "
          f"{l1 - l0} launches for {i1 - i0} items, largest batch {mb}")
    assert i1 - i0 == BURSTS * 64
    assert l1 - l0 <= 2 * BURSTS  # coalesced: at most two launches per burst
    assert med <= BURST_BOUND * lone_s, (med, lone_s)


def _mixed_items(golden, C, reps=3, beyond=0, seed=7):
    """Partials of the golden round (with corruptions) and chained beacons under the chain key
    (right and wrong messages), repeated and shuffled: (callables, expected classes). `beyond` extra
    partials carry share indices >= n (kyber still evaluates the polynomial there; they fail the
    pairing)."""
    import random

    th, commits, msg = _partial_world(golden)
    parts = _mixed_partials(golden)
    grp = C.Group(commits)
    ch = golden["chained"]
    pk = bytes.fromhex(ch["pk"])
    items = []
    for p in parts:
        items.append((lambda p=p: svc_holder[0].verify_partial(commits, th["n"], msg, p), grp.verify_partial(msg, p)))
    for j in range(beyond):
        p = (th["n"] + 1 + j).to_bytes(2, "big") + parts[j][2:]
        items.append((lambda p=p: svc_holder[0].verify_partial(commits, th["n"], msg, p), grp.verify_partial(msg, p)))
    for b in ch["beacons"][:8]:
        m = hashlib.sha256(bytes.fromhex(b["prev"]) + b["round"].to_bytes(8, "big")).digest()
        sig = bytes.fromhex(b["sig"])
        for wrong in (False, True):
            mm = hashlib.sha256(m).digest() if wrong else m
            items.append((lambda mm=mm, sig=sig: svc_holder[0].verify_recovered(pk, mm, sig), C.verify(pk, mm, sig)))
    items = items * reps
    random.Random(seed).shuffle(items)
    return [f for f, _ in items], [w for _, w in items]


svc_holder = [None]


def test_service_multipass_per_item_keys(golden, C):
    """A service batch spanning several pipeline passes keeps every item's own key: with the
    dispatcher's pass shrunk to 64 items and the latency path off, a ~250-item burst of partials of
    64 members and beacons under another key runs in >= 2 passes of the batch pipeline, and every
    verdict equals the C oracle's (pass 2+ used to read pass 1's key entries)."""
    from drand_amd.engine import Service

    with Service(0) as s:
        svc_holder[0] = s
        s.test_limits(chunk=64, lat_max=0)
        fns, want = _mixed_items(golden, C, reps=3)
        assert len(fns) > 2 * 64
        old_iv = sys.getswitchinterval()
        sys.setswitchinterval(1e-5)
        try:
            res, _ = _burst(fns)
        finally:
            sys.setswitchinterval(old_iv)
        _, items, mb = s.stats()
        print(f"{len(fns)} items, largest batch {mb} (passes of 64)")
        assert items == len(fns)
        assert mb > 64, mb  # at least one batch really spanned two passes
        assert [c for _, c in res] == want
        assert [ok for ok, _ in res] == [c == 0 for c in want]


def test_service_arena_overflow_sub_batches(golden, C):
    """A burst whose keys overflow the key arena (one group table of 64 entries, a chain key and 40
    out-of-table share indices, each needing a tail entry, against an arena capped at 72) runs as
    consecutive sub-batches: no honest call fails, every verdict equals the C oracle's (ADVICE r05:
    the whole batch used to fail with BLSV_EINVAL)."""
    from drand_amd.engine import Service

    with Service(0) as s:
        svc_holder[0] = s
        s.test_limits(chunk=1 << 14, lat_max=(1 << 64) - 1, arena_entries=72)
        fns, want = _mixed_items(golden, C, reps=1, beyond=40, seed=11)
        sub0 = s.test_limits()
        old_iv = sys.getswitchinterval()
        sys.setswitchinterval(1e-5)
        try:
            res, _ = _burst(fns)
        finally:
            sys.setswitchinterval(old_iv)
        sub1 = s.test_limits()
        launches, items, mb = s.stats()
        print(f"{len(fns)} items in {launches} coalesced batches, {sub1 - sub0} device sub-batches, largest {mb}")
        assert items == len(fns)
        assert [c for _, c in res] == want
        assert sum(1 for w in want if w == 7) >= 40  # the out-of-table shares fail the pairing
        assert sub1 - sub0 > launches  # an overflowing batch was split, not failed


def test_service_mixed_kinds_and_bad_key(svc, golden, C):
    """Partials, beacons under the chain key and a call with an undecodable key, all at once: each
    call gets its own verdict, the bad key fails only its own call (BLSV_EINVAL)."""
    from drand_amd.engine import EngineError

    th = golden["threshold"]
    commits = [bytes.fromhex(c) for c in th["commits"]]
    msg = bytes.fromhex(th["msg"])
    parts = _mixed_partials(golden)[:24]
    ch = golden["chained"]
    pk = bytes.fromhex(ch["pk"])
    beacons = ch["beacons"]
    fns, want = [], []
    grp = C.Group(commits)
    for p in parts:
        fns.append(lambda p=p: svc.verify_partial(commits, th["n"], msg, p))
        want.append(grp.verify_partial(msg, p))
    for b in beacons:
        m = hashlib.sha256(bytes.fromhex(b["prev"]) + b["round"].to_bytes(8, "big")).digest()
        s = bytes.fromhex(b["sig"])
        for wrong in (False, True):
            mm = hashlib.sha256(m).digest() if wrong else m
            fns.append(lambda mm=mm, s=s: svc.verify_recovered(pk, mm, s))
            want.append(C.verify(pk, mm, s))
    bad_pk = bytes([pk[0] & 0x7F]) + pk[1:]  # compression flag cleared: G1.FromCompressed fails

    def bad_call():
        try:
            svc.verify_recovered(bad_pk, msg, bytes.fromhex(beacons[0]["sig"]))
        except EngineError as e:
            return ("error", e.code)
        return ("no error", None)

    fns.append(bad_call)
    res, _ = _burst(fns)
    assert res[-1] == ("error", -1)
    got = [c for _, c in res[:-1]]
    assert got == want
    assert [ok for ok, _ in res[:-1]] == [c == 0 for c in want]


def test_service_host_side_share_rejects(svc, golden):
    """tbls IndexOf / SigShare rejects never reach the GPU: a share shorter than its index prefix and
    a share of the wrong length."""
    th = golden["threshold"]
    commits = [bytes.fromhex(c) for c in th["commits"]]
    msg = bytes.fromhex(th["msg"])
    p = bytes.fromhex(th["partials"][0])
    assert svc.verify_partial(commits, th["n"], msg, p[:1]) == (False, 8)
    assert svc.verify_partial(commits, th["n"], msg, p[:97]) == (False, 1)
    assert svc.verify_partial(commits, th["n"], msg, p) == (True, 0)


def test_chunk_cap_same_verdicts(engine, golden, C):
    """A context capped at a 256 Ki chunk (blsv_set_chunk) verifies a 2^20 + 4,099-round device
    history in five passes with the bitmap, first bad round and classes of the uncapped context, and
    holds at most the capped staging."""
    import torch

    from drand_amd.engine import Engine

    n, seg = (1 << 20) + 4099, 64
    ch = golden["chained"]
    sk32 = int(ch["sk"], 16).to_bytes(32, "big")
    dev = torch.device("cuda", 0)
    nseg = (n + seg - 1) // seg
    sb = b"".join(hashlib.sha256(b"cap-%d" % i).digest() * 3 for i in range(nseg))
    seeds = torch.frombuffer(bytearray(sb), dtype=torch.uint8).to(dev)
    sigs = torch.empty(n * 96, dtype=torch.uint8, device=dev)
    engine.set_public_key(bytes.fromhex(ch["pk"]))
    engine.generate_chained_dev(sk32, 1, seg, seeds.data_ptr(), 96, sigs.data_ptr(), n)
    torch.cuda.synchronize()
    # corruptions at both sides of the 256 Ki pass edges and of the 2^20 edge, and mid-segment
    hit = (0, (1 << 18) - 1, 1 << 18, (3 << 18) + 5, (1 << 20) - 1, 1 << 20, n - 1)
    for i in hit:
        sigs[i * 96 + 50] ^= 1
    words = (n + 63) // 64

    def run(eng):
        bm = torch.zeros(words, dtype=torch.int64, device=dev)
        fb = torch.zeros(1, dtype=torch.int64, device=dev)
        cls = torch.zeros(n, dtype=torch.uint8, device=dev)
        eng.verify_chained_dev(1, seg, seeds.data_ptr(), 96, sigs.data_ptr(), n, bm.data_ptr(), fb.data_ptr(),
                               cls.data_ptr())
        eng.synchronize()
        return bm.cpu(), int(fb.cpu()[0]) & NONE, cls.cpu()

    bm0, fb0, cls0 = run(engine)
    with Engine(0) as capped:
        capped.set_public_key(bytes.fromhex(ch["pk"]))
        assert capped.set_chunk(1 << 18) == 1 << 20
        bm1, fb1, cls1 = run(capped)
        ws = capped.workspace_bytes()
    assert torch.equal(bm0, bm1) and fb0 == fb1 and torch.equal(cls0, cls1)
    assert fb0 == 1
    bad = (cls0 != 0).nonzero().flatten().tolist()
    # a corrupted sig_i fails round i and round i + 1 unless i + 1 starts a segment (its prev is a seed)
    want = sorted({i for i in hit} | {i + 1 for i in hit if i + 1 < n and (i + 1) % seg})
    assert bad == want
    assert 0 < ws <= (1 << 18) * 42500, ws  # ~42.4 KB of staging per item (engine_ctx.h)
