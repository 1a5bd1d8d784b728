"""GPU parity of the latency path (drand_amd/csrc/k_lat.hip: one wave per item, limbs across lanes)
against the golden fixtures and, on the same inputs, against the batch pipeline (one lane per item):
every verdict, reject class, first_bad and recovered signature byte must agree.
"""
import hashlib

import pytest

from oracle import bls12381 as O

pytestmark = pytest.mark.gpu

BIG = 1 << 40


@pytest.fixture
def both(engine):
    """run(fn) -> (latency-path result, batch-path result) of the same call"""
    def run(fn):
        old = engine.set_lat_max(BIG)
        try:
            lat = fn()
            engine.set_lat_max(0)
            batch = fn()
        finally:
            engine.set_lat_max(old)
        return lat, batch
    return run


def test_lat_kat_and_chain(engine, golden, both):
    kat = golden["kat"]
    ch = golden["chained"]
    sigs = [bytes.fromhex(b["sig"]) for b in ch["beacons"]]
    seed = bytes.fromhex(ch["genesis_seed"])

    def go():
        engine.set_public_key(bytes.fromhex(ch["pk"]))
        r = engine.verify_chained(1, seed, sigs)
        m = engine.verify_messages([bytes.fromhex(kat["msg"]), b"\x00" + bytes.fromhex(kat["msg"])],
                                   [bytes.fromhex(kat["sig"])] * 2, pk48=bytes.fromhex(kat["pk"]))
        return r.ok, r.first_bad, r.reject_class, m.ok, m.reject_class

    lat, batch = both(go)
    assert lat == batch
    assert all(lat[0]) and lat[1] is None and lat[3] == [True, False] and lat[4] == [0, 7]


def test_lat_mixed_golden_classes(engine, golden, both):
    m = golden["mixed"]
    sigs = [bytes.fromhex(s) for s in m["sigs"]]

    def go():
        engine.set_public_key(bytes.fromhex(m["pk"]))
        r = engine.verify_chained(1, bytes.fromhex(m["genesis_seed"]), sigs)
        return r.reject_class, r.first_bad

    lat, batch = both(go)
    assert lat == batch
    assert lat[0] == m["expect_class"]


def test_lat_unchained_and_wrong_round(engine, golden, both):
    ch = golden["chained"]
    sigs2 = [bytes.fromhex(b["sig_v2"]) for b in ch["beacons"]]
    r0 = ch["beacons"][0]["round"]

    def go():
        engine.set_public_key(bytes.fromhex(ch["pk"]))
        a = engine.verify_unchained(sigs2, first_round=r0)
        b = engine.verify_unchained(sigs2, first_round=r0 + 1)
        return a.ok, a.first_bad, b.ok, b.first_bad

    lat, batch = both(go)
    assert lat == batch
    assert all(lat[0]) and lat[1] is None and not any(lat[2]) and lat[3] == r0 + 1


def test_lat_threshold_round_bit_exact(engine, golden, both):
    th = golden["threshold"]
    commits = [bytes.fromhex(c) for c in th["commits"]]
    msg = bytes.fromhex(th["msg"])
    partials = [bytes.fromhex(p) for p in th["partials"]]
    bad = bytes.fromhex(th["bad_partial"])

    def go():
        engine.set_group(commits, th["n"])
        ok, cls = engine.verify_partials(msg, partials + [bad])
        sig = engine.recover(msg, [bytes.fromhex(p) for p in th["recover_subset"]], th["t"], th["n"])
        agg = engine.aggregate(msg, partials, th["t"], th["n"])
        return ok, cls, sig, agg

    lat, batch = both(go)
    assert lat == batch
    ok, cls, sig, agg = lat
    assert all(ok[:-1]) and not ok[-1]
    assert sig.hex() == th["group_sig"] and agg[2].hex() == th["group_sig"] and agg[3]


def test_lat_random_corruptions_match_batch(engine, golden, both):
    """Device-signed beacons with corruptions of every class; both paths give identical classes."""
    ch = golden["chained"]
    sk32 = int(ch["sk"], 16).to_bytes(32, "big")
    n = 40
    msgs = [hashlib.sha256(b"lat %d" % i).digest() for i in range(n)]
    sigs = [bytearray(s) for s in engine.sign(sk32, msgs)]
    sigs[1][60] ^= 0x10                  # bit flip in x
    sigs[2][0] &= 0x7F                   # compression flag cleared
    sigs[3] = bytearray(b"\xc0" + bytes(95))  # infinity
    sigs[4][48:96] = O.P.to_bytes(48, "big")   # x.c0 = p
    sigs[5] = bytearray(sigs[6])         # a valid signature of another message
    sigs[7][0] ^= 0x20                   # sign bit flipped: the other root
    pk = bytes.fromhex(ch["pk"])

    def go():
        r = engine.verify_messages(msgs, [bytes(s) for s in sigs], pk48=pk)
        return r.ok, r.reject_class, r.first_bad

    lat, batch = both(go)
    assert lat == batch
    assert lat[1][1:8] != [0] * 7 and lat[1][8:] == [0] * (n - 8)
