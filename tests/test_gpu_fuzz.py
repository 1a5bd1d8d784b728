"""Seeded random parity beyond the fixtures: the GPU against the C oracle (oracle/c/bls_oracle.c,
pinned to the reference KAT) on inputs no golden file holds.

* Sign (key.Scheme's ThresholdScheme.Sign / blsv_sign) of random messages whose lengths cross
  expand_message_xmd's block edges (0 .. 300 bytes): every 96-byte signature equals the oracle's, so
  hash-to-G2 of arbitrary messages, the G2 scalar multiplication and the compression are bit-exact.
* Verify (kyber bls.Verify: VerifyRecovered's and VerifyBeaconV2's check, blsv_verify_messages) of
  signatures under the golden chain key with half of them corrupted at random -- a flipped bit at
  a random position (flags, x, the sign bit), the sign bit alone, another message's signature, a
  random 96-byte string with the compression flag set, the infinity encoding with and without stray
  bits: every reject class equals the oracle's, on the latency path and on the batch pipeline.

DRAND_AMD_FUZZ_SCALE=k (default 1) runs k times as many random cases, each block with its own seeds
(profiles/r06w_pytest_gpu_fuzz_x10.log is one such run).
"""
import os
import random

import pytest

pytestmark = pytest.mark.gpu

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
LENGTHS = (0, 1, 31, 32, 33, 63, 64, 65, 100, 135, 136, 137, 200, 255, 256, 300)
SCALE = max(1, int(os.environ.get("DRAND_AMD_FUZZ_SCALE", "1")))


@pytest.fixture(scope="module")
def C():
    from oracle import c_oracle

    c_oracle.load()
    return c_oracle


def _msgs(rng, n):
    return [bytes(rng.getrandbits(8) for _ in range(rng.choice(LENGTHS))) for _ in range(n)]


def test_sign_random_messages_equal_oracle(engine, C):
    for blk in range(SCALE):
        rng = random.Random(0x5157 + 1000 * blk)
        sk = rng.randrange(1, R)
        msgs = _msgs(rng, 160)
        got = engine.sign(sk.to_bytes(32, "big"), msgs)
        bad = [i for i, (m, s) in enumerate(zip(msgs, got)) if s != C.sign(sk, m)]
        assert not bad, (blk, bad[:8])


def _corrupt(rng, sigs, i):
    s = bytearray(sigs[i])
    kind = rng.randrange(7)
    if kind == 0:  # one bit anywhere
        s[rng.randrange(96)] ^= 1 << rng.randrange(8)
    elif kind == 1:  # the sign bit alone: -sigma decodes, the pairing rejects
        s[0] ^= 0x20
    elif kind == 2:  # another message's signature
        s = bytearray(sigs[(i + 1 + rng.randrange(len(sigs) - 1)) % len(sigs)])
    elif kind == 3:  # random bytes with the compression flag (x >= p, off the curve, or outside G2)
        s = bytearray(rng.getrandbits(8) for _ in range(96))
        s[0] = (s[0] & 0x3F) | 0x80 | (rng.getrandbits(1) << 5)
    elif kind == 4:  # the infinity encoding
        s = bytearray(96)
        s[0] = 0xC0
    elif kind == 5:  # infinity flag with stray bits
        s[0] |= 0xC0
    else:  # compression flag cleared
        s[0] &= 0x7F
    return bytes(s)


@pytest.mark.parametrize("route", ["lat", "batch"])
def test_verify_random_corruptions_equal_oracle(engine, golden, C, route):
    for blk in range(SCALE):
        _verify_block(engine, golden, C, route, random.Random(0xF022 + (route == "batch") + 1000 * blk))


def _verify_block(engine, golden, C, route, rng):
    ch = golden["chained"]
    sk, pk = int(ch["sk"], 16), bytes.fromhex(ch["pk"])
    msgs = _msgs(rng, 240)
    sigs = engine.sign(sk.to_bytes(32, "big"), msgs)
    sigs = [_corrupt(rng, sigs, i) if rng.random() < 0.5 else sigs[i] for i in range(len(sigs))]
    want = [C.verify(pk, m, s) for m, s in zip(msgs, sigs)]
    assert len(set(want)) >= 5, sorted(set(want))  # the corruptions reach several reject classes
    prev = engine.set_lat_max(0 if route == "batch" else 1536)
    try:
        res = engine.verify_messages(msgs, sigs, pk48=pk)
    finally:
        engine.set_lat_max(prev)
    assert res.reject_class == want
    assert res.ok == [c == 0 for c in want]
    fb = next((i for i, c in enumerate(want) if c), None)
    assert res.first_bad == fb


def _mangle_shares(rng, parts, n):
    """Random corruptions of a round's shares: a flipped signature bit, a wrong share index, a
    duplicate of another share (the dedup rule), a truncated-to-garbage signature."""
    parts = list(parts)
    for j in rng.sample(range(len(parts)), min(len(parts), rng.choice([0, 0, 1, 2, 5, 12, 30]))):
        p = bytearray(parts[j])
        kind = rng.randrange(4)
        if kind == 0:
            p[2 + rng.randrange(96)] ^= 1 << rng.randrange(8)
        elif kind == 1:
            idx = ((p[0] << 8 | p[1]) + 1 + rng.randrange(n - 1)) % n
            p[0], p[1] = idx >> 8, idx & 0xFF
        elif kind == 2:
            p = bytearray(parts[rng.randrange(len(parts))])
        else:
            p[2:] = bytes(96)
            p[2] = 0x80
        parts[j] = bytes(p)
    return parts


def test_aggregate_random_rounds_equal_oracle(engine, golden, C):
    """blsv_aggregate (VerifyPartial x k, Recover from the first t valid shares, VerifyRecovered) on
    random share sets of the golden n=64 / t=33 round -- shuffled, between t - 2 and 64 shares, some
    corrupted -- against the oracle's verdicts and Recover: the classes, the group signature bytes,
    the group verdict, "not enough shares" as an error; both the speculative recovery's hits and its
    misses are reached (spec_stats)."""
    from drand_amd.engine import EngineError

    th = golden["threshold"]
    t, n = th["t"], th["n"]
    commits = [bytes.fromhex(c) for c in th["commits"]]
    msg = bytes.fromhex(th["msg"])
    engine.set_group(commits, n)
    grp = C.Group(commits)
    rng = random.Random(0xA66)
    h0, m0 = engine.spec_stats()
    rounds = fails = 0
    for _ in range(14 * SCALE):
        parts = [bytes.fromhex(p) for p in th["partials"]]
        rng.shuffle(parts)
        parts = _mangle_shares(rng, parts[:rng.randrange(t - 2, n + 1)], n)
        want_cls = [grp.verify_partial(msg, p) for p in parts]
        want_sig = grp.recover(msg, parts, t, n)
        if want_sig is None:
            with pytest.raises(EngineError):
                engine.aggregate(msg, parts, t, n)
            fails += 1
            continue
        ok, cls, sig, gok = engine.aggregate(msg, parts, t, n)
        assert cls == want_cls
        assert ok == [c == 0 for c in want_cls]
        assert sig == want_sig
        assert gok == (C.verify(commits[0], msg, sig) == 0)
        rounds += 1
    h1, m1 = engine.spec_stats()
    print(f"{rounds} rounds recovered, {fails} short; speculation hits {h1 - h0}, misses {m1 - m0}")
    assert rounds >= 5 and fails >= 2 and h1 > h0 and m1 > m0


def test_aggregate_round_v1_v2_random_equal_oracle(engine, golden, C):
    """blsv_aggregate_round (chain/beacon/chain.go:131-166: V1 and V2 partials verified in one pass,
    both Recovers, both group verifications) on random V1 / V2 share sets: the status follows the
    oracle (V1 recover failure, V2 recover failure blocking the beacon, OK, OK_V2 with v2_valid), and
    the verdicts and both signatures equal the oracle's."""
    from drand_amd import _lib

    th = golden["threshold"]
    t, n = th["t"], th["n"]
    commits = [bytes.fromhex(c) for c in th["commits"]]
    msg1, msg2 = bytes.fromhex(th["msg"]), bytes.fromhex(th["msg_v2"])
    engine.set_group(commits, n)
    grp = C.Group(commits)
    rng = random.Random(0xB22)
    seen = set()
    for _ in range(12 * SCALE):
        p1 = [bytes.fromhex(p) for p in th["partials"]]
        p2 = [bytes.fromhex(p) for p in th["partials_v2"]]
        rng.shuffle(p1)
        rng.shuffle(p2)
        p1 = _mangle_shares(rng, p1[:rng.randrange(t - 1, n + 1)], n)
        p2 = _mangle_shares(rng, p2[:rng.choice([0, t - 1, t, rng.randrange(t, n + 1)])], n)
        st, ok1, ok2, sig1, sig2, v2 = engine.aggregate_round(msg1, p1, msg2, p2, t, n)
        assert ok1 == [grp.verify_partial(msg1, p) == 0 for p in p1]
        assert ok2 == [grp.verify_partial(msg2, p) == 0 for p in p2]
        w1 = grp.recover(msg1, p1, t, n)
        if w1 is None:
            assert st == _lib.AGG_V1_RECOVER_FAIL
        elif C.verify(commits[0], msg1, w1) != 0:
            assert st == _lib.AGG_V1_INVALID and sig1 == w1
        elif len(p2) >= t:
            w2 = grp.recover(msg2, p2, t, n)
            if w2 is None:
                assert st == _lib.AGG_V2_RECOVER_FAIL and sig1 == w1
            else:
                assert st == _lib.AGG_OK_V2 and sig1 == w1 and sig2 == w2
                assert v2 == (C.verify(commits[0], msg2, w2) == 0)
        else:
            assert st == _lib.AGG_OK and sig1 == w1 and sig2 is None
        seen.add(st)
    print("statuses:", sorted(seen))
    assert len(seen) >= 3


def test_chained_random_kinds_single_lane_f_pass(engine, golden, C):
    """A 70,003-round device-generated chained history (above the 3-lane f pass's 64 Ki limit, so the
    single-lane Miller f pass and the batch pipeline verify it) with 48 rounds corrupted by random
    kinds (_corrupt): exactly the corrupted rounds and their successors in the same 64-round segment
    reject, first_bad is the smallest, and the class of every rejected round equals the C oracle's
    on its own message (chain.Message of its round and the stored previous signature)."""
    import hashlib

    import torch

    from test_gpu_scale import _history, _verify, NONE

    n, seg = 70003, 64
    seeds, sigs, s0 = _history(engine, golden, n, seg, seed=23)
    host = bytearray(sigs.cpu().numpy().tobytes())
    orig = bytes(host)
    rng = random.Random(0xC4A1)
    bad = sorted(rng.sample(range(n), 48))
    view = [orig[i * 96:(i + 1) * 96] for i in range(n)]
    for i in bad:
        host[i * 96:(i + 1) * 96] = _corrupt(rng, view, i)
    sigs.copy_(torch.frombuffer(bytearray(host), dtype=torch.uint8).to("cuda:0"))
    prev = engine.set_lat_max(0)
    try:
        ok, fb, cls = _verify(engine, 1, seg, seeds, s0, sigs, n)
    finally:
        engine.set_lat_max(prev)
    sd = seeds.cpu().numpy().tobytes()
    pk = bytes.fromhex(golden["chained"]["pk"])

    def prev_of(i):
        if i % seg == 0:
            s = i // seg
            return sd[s * 96: s * 96 + (s0 if s == 0 else 96)]
        return bytes(host[(i - 1) * 96: i * 96])

    cand = sorted(set(bad) | {i + 1 for i in bad if i + 1 < n and (i + 1) % seg})
    want = {}
    for i in cand:
        msg = hashlib.sha256(prev_of(i) + (i + 1).to_bytes(8, "big")).digest()
        want[i] = C.verify(pk, msg, bytes(host[i * 96:(i + 1) * 96]))
    rejected = {i for i, v in enumerate(ok) if not v}
    assert rejected == {i for i, c in want.items() if c}
    assert all(cls[i] == want[i] for i in cand)
    assert fb == (1 + min(rejected) if rejected else NONE)
