"""Batched callers (drand_amd/callers.py) and wire ingest (drand_amd/ingest.py).

The same scenarios run twice: on CPU against ``OracleEngine`` (a test double that answers the
engine's verify calls with the C oracle, so the host logic is checked without a GPU), and with the
``gpu`` mark against the real HIP engine through the C ABI. Inputs are the 24-round chained golden
history (tests/golden/golden.json, pinned to the reference KAT) and the round-367 JSON example of
the reference README (README.md:200-207; randomness == sha256(signature), the only pin it gives).
"""
from __future__ import annotations

import hashlib
import json

import pytest

from drand_amd.callers import (Beacon, ChainInfo, FetchError, RandomData, VerifyError, VerifyingClient,
                               randomness_from_signature, sync_chain, verify_beacons)
from drand_amd import ingest
from tests.support.oracle_engine import OracleEngine

README_367 = {
    "round": 367,
    "signature": "b62dd642e939191af1f9e15bef0f0b0e9562a5f570a12a231864afe468377e2a6424a92ccfc34ef1471cbd58c37c6b020cf75"
                 "ce9446d2aa1252a090250b2b1441f8a2a0d22208dcc09332eaa0143c4a508be13de63978dbed273e3b9813130d5",
    "previous_signature": "afc545efb57f591dbdf833c339b3369f569566a93e49578db46b6586299422483b7a2d595814046e2847494b401"
                          "650a0050981e716e531b6f4b620909c2bf1476fd82cf788a110becbc77e55746a7cccd47fb171e8ae2eea2a22fc"
                          "c6a512486d",
    "randomness": "d7aed3686bf2be657e6d38c20999831308ee6244b68c8825676db580e7e3bec6",
}


@pytest.fixture(scope="module")
def chain(golden):
    ch = golden["chained"]
    seed = bytes.fromhex(ch["genesis_seed"])
    beacons = [Beacon(bytes.fromhex(b["prev"]), b["round"], bytes.fromhex(b["sig"]), bytes.fromhex(b["sig_v2"]))
               for b in ch["beacons"]]
    return bytes.fromhex(ch["pk"]), seed, beacons


def _getter(beacons, tamper=None, fail_at=None, log=None):
    by_round = {b.round: b for b in beacons}

    def get(r):
        if log is not None:
            log.append(r)
        if fail_at is not None and r == fail_at:
            raise IOError("connection reset")
        b = by_round[r]
        sig = tamper.get(r, b.signature) if tamper else b.signature
        return RandomData(round=r, signature=sig, previous_signature=b.previous_sig, signature_v2=b.signature_v2)
    return get


# ------------------------------------------------------------------ scenarios (engine-agnostic)
def _trusted(bs):
    """``WithVerifiedResult(&results[0])`` as the reference's client tests use (verify_test.go:19,36)."""
    return RandomData(round=1, signature=bs[0].signature, previous_signature=bs[0].previous_sig)


def scenario_walk(eng, chain):
    pk, seed, bs = chain
    log = []
    vc = VerifyingClient(eng, ChainInfo(pk, seed), _getter(bs, log=log), chunk=5, point_of_trust=_trusted(bs))
    r = RandomData(round=24, signature=bs[23].signature)          # no previous_signature -> walk
    vc.verify(r)
    assert r.randomness == randomness_from_signature(bs[23].signature)
    assert log == list(range(2, 24))
    assert vc.point_of_trust.round == 23
    # from the point of trust only the new rounds are fetched
    log.clear()
    vc.verify(RandomData(round=24, signature=bs[23].signature))
    assert log == []
    # round 2 right after the point of trust: no fetch, prev = round 1's signature
    vc2 = VerifyingClient(eng, ChainInfo(pk, seed), _getter(bs), point_of_trust=_trusted(bs))
    vc2.verify(RandomData(round=2, signature=bs[1].signature))
    # round 1 always takes GroupHash as its previous signature (verify.go:122-124)
    vc2.verify(RandomData(round=1, signature=bs[0].signature))
    # a round below the point of trust restarts at round 1 with GroupHash as the trusted signature
    # (verify.go:131-137): the reference then checks round 2 against Message(2, GroupHash) and fails
    with pytest.raises(VerifyError) as ei:
        vc.verify(RandomData(round=20, signature=bs[19].signature))
    assert ei.value.round == 2 and vc.point_of_trust.round == 23
    # wrong signature for the requested round
    with pytest.raises(VerifyError):
        vc.verify(RandomData(round=24, signature=bs[22].signature, previous_signature=bs[22].signature))


def scenario_walk_errors(eng, chain):
    pk, seed, bs = chain
    # a corrupted round 10 stops the walk there; the point of trust stays at round 1
    vc = VerifyingClient(eng, ChainInfo(pk, seed), _getter(bs, tamper={10: bs[8].signature}), chunk=6, point_of_trust=_trusted(bs))
    with pytest.raises(VerifyError) as ei:
        vc.verify(RandomData(round=20, signature=bs[19].signature))
    assert ei.value.round == 10 and vc.point_of_trust.round == 1
    # fetch failure at 12 with an earlier bad round in the same chunk: the verify error wins
    vc = VerifyingClient(eng, ChainInfo(pk, seed), _getter(bs, tamper={10: bs[8].signature}, fail_at=12), chunk=16, point_of_trust=_trusted(bs))
    with pytest.raises(VerifyError) as ei:
        vc.verify(RandomData(round=20, signature=bs[19].signature))
    assert ei.value.round == 10
    # fetch failure with a clean prefix
    vc = VerifyingClient(eng, ChainInfo(pk, seed), _getter(bs, fail_at=12), chunk=16, point_of_trust=_trusted(bs))
    with pytest.raises(FetchError) as ei:
        vc.verify(RandomData(round=20, signature=bs[19].signature))
    assert ei.value.round == 12
    # a wrong-length signature mid-walk (grpcserver.go:66-69 serves 3 bytes) rejects that round
    vc = VerifyingClient(eng, ChainInfo(pk, seed), _getter(bs, tamper={7: b"\x01\x02\x03"}), chunk=16, point_of_trust=_trusted(bs))
    with pytest.raises(VerifyError) as ei:
        vc.verify(RandomData(round=20, signature=bs[19].signature))
    assert ei.value.round == 7


def scenario_v2(eng, chain):
    pk, seed, bs = chain
    vc = VerifyingClient(eng, ChainInfo(pk, seed), _getter(bs), v2from=10)
    r = RandomData(round=15, signature_v2=bs[14].signature_v2, version=2)
    vc.verify(r)                                                     # V2: no walk, msg = sha256(BE64(round))
    assert r.randomness == hashlib.sha256(bs[14].signature_v2).digest()
    with pytest.raises(VerifyError):
        vc.verify(RandomData(round=16, signature_v2=bs[14].signature_v2, version=2))
    # below v2from with a previous signature given and strict=False: no walk
    r = RandomData(round=5, signature=bs[4].signature, previous_signature=bs[3].signature)
    vc.verify(r)
    assert vc.point_of_trust is None


def scenario_sync(eng, chain):
    pk, seed, bs = chain
    genesis = Beacon(b"", 0, seed)                                   # chain/store.go:234-238
    put = []
    out = sync_chain(eng, pk, genesis, iter(bs), 24, put.append, chunk=7)
    assert out.finished and out.stored == 24 and out.last.round == 24 and [b.round for b in put] == list(range(1, 25))
    # stop at up_to mid-chunk
    put = []
    out = sync_chain(eng, pk, genesis, iter(bs), 10, put.append, chunk=7)
    assert out.finished and out.stored == 10 and out.last.round == 10
    # resume from a stored beacon
    out = sync_chain(eng, pk, bs[9], iter(bs[10:]), 24, lambda b: None, chunk=64)
    assert out.finished and out.stored == 14
    # bad signature at round 9: rounds 1..8 stored, reason invalid_beacon
    bad = list(bs)
    bad[8] = Beacon(bs[8].previous_sig, 9, bs[7].signature)
    out = sync_chain(eng, pk, genesis, iter(bad), 24, lambda b: None, chunk=5)
    assert not out.finished and out.stored == 8 and out.reason == "invalid_beacon" and out.bad_round == 9
    # a repeated (valid) beacon breaks linkage: appendStore.Put's round check
    dup = bs[:11] + [bs[10]] + bs[11:]
    out = sync_chain(eng, pk, genesis, iter(dup), 24, lambda b: None, chunk=64)
    assert not out.finished and out.stored == 11 and out.reason == "invalid round inserted"
    # the stream ends before up_to
    out = sync_chain(eng, pk, genesis, iter(bs[:5]), 24, lambda b: None)
    assert not out.finished and out.stored == 5 and out.reason == "stream ended"
    # store error
    def failing_put(b):
        if b.round == 4:
            raise IOError("disk full")
    out = sync_chain(eng, pk, genesis, iter(bs), 24, failing_put)
    assert not out.finished and out.stored == 3 and out.reason == "store" and out.bad_round == 4


def scenario_verify_beacons(eng, chain):
    pk, seed, bs = chain
    mixed = [bs[20], bs[3], bs[4], bs[5], bs[0], bs[1], Beacon(bs[7].previous_sig, 8, b"\x00" * 3), bs[8], bs[12]]
    ok = verify_beacons(eng, pk, mixed)
    assert ok == [True, True, True, True, True, True, False, True, True]
    wrong_round = [Beacon(bs[4].previous_sig, 6, bs[4].signature)]
    assert verify_beacons(eng, pk, wrong_round) == [False]
    assert verify_beacons(eng, pk, []) == []


SCENARIOS = [scenario_walk, scenario_walk_errors, scenario_v2, scenario_sync, scenario_verify_beacons]


@pytest.mark.parametrize("scenario", SCENARIOS, ids=lambda f: f.__name__)
def test_callers_cpu(scenario, chain):
    scenario(OracleEngine(), chain)


@pytest.mark.gpu
@pytest.mark.parametrize("scenario", SCENARIOS, ids=lambda f: f.__name__)
def test_callers_gpu(scenario, chain, engine):
    scenario(engine, chain)


@pytest.mark.gpu
def test_sync_batches_calls(chain, engine):
    """The sync loop reaches the GPU once per chunk, not once per beacon."""
    pk, seed, bs = chain
    calls = []
    real = engine.verify_chained

    def counting(*a, **k):
        calls.append(len(a[2]))
        return real(*a, **k)
    engine.verify_chained = counting
    try:
        out = sync_chain(engine, pk, Beacon(b"", 0, seed), iter(bs), 24, lambda b: None, chunk=8)
    finally:
        del engine.verify_chained
    assert out.finished and calls == [8, 8, 8]


# ------------------------------------------------------------------ ingest (host logic only)
def test_readme_json_round_367():
    r = ingest.random_from_json(json.dumps(README_367))
    assert r.round == 367 and r.version == 1 and len(r.signature) == 96 and len(r.previous_signature) == 96
    assert randomness_from_signature(r.signature) == r.randomness


def test_hexjson_beacon_roundtrip(chain):
    _, _, bs = chain
    for b in (bs[0], bs[5], Beacon(bs[1].previous_sig, 2, bs[1].signature)):
        j = ingest.beacon_to_json(b)
        assert json.loads(j)["Round"] == b.round
        assert ingest.beacon_from_json(j) == b
    assert b"SignatureV2" not in ingest.beacon_to_json(Beacon(b"\x01", 1, b"\x02"))


def test_protobuf_packets(chain):
    _, _, bs = chain
    for b in bs[:4]:
        pkt = ingest.beacon_to_packet(b)
        back = ingest.beacon_from_packet(pkt)
        assert (back.previous_sig, back.round, back.signature, back.signature_v2) == \
               (b.previous_sig, b.round, b.signature, b"")  # convert.go drops SignatureV2
    # hand-built PublicRandResponse with an unknown field and a big round
    sig = bs[0].signature
    buf = bytes([0x08]) + bytes([0xff, 0xff, 0xff, 0xff, 0x0f]) + bytes([0x12, 96]) + sig + \
        bytes([0x32, 2, 0xaa, 0xbb]) + bytes([0x22, 32]) + hashlib.sha256(sig).digest()
    r = ingest.random_from_response(buf)
    assert r.round == 0xffffffff and r.signature == sig and r.previous_signature is None
    assert r.randomness == randomness_from_signature(sig)
    with pytest.raises(ingest.WireError):
        ingest.beacon_from_packet(bytes([0x0a, 96]) + sig[:10])


def test_segments(chain):
    _, seed, bs = chain
    segs = ingest.segments(bs)
    assert len(segs) == 1 and segs[0].first_round == 1 and segs[0].prev0 == seed and segs[0].n == 24
    gap = bs[:5] + bs[6:10] + [Beacon(bs[10].previous_sig, 11, b"\x00")] + bs[11:]
    segs = ingest.segments(gap)
    assert [(s.first_round, s.n, s.start) for s in segs] == [(1, 5, 0), (7, 4, 5), (11, 1, 9), (12, 13, 10)]
    assert ingest.segments([]) == []


def scenario_wire_to_sync(eng, chain):
    """protobuf BeaconPackets off the sync stream (protocol.proto:88-92) straight into sync_chain."""
    pk, seed, bs = chain
    stream = [ingest.beacon_to_packet(b) for b in bs]
    put = []
    out = sync_chain(eng, pk, Beacon(b"", 0, seed), (ingest.beacon_from_packet(x) for x in stream), 24, put.append,
                     chunk=10)
    assert out.finished and [b.round for b in put] == list(range(1, 25))
    # an odd-length PreviousSig is still a message (sha256(prev || round)): it rejects, via the message form
    odd = [Beacon(bs[4].previous_sig[:10], 5, bs[4].signature), bs[5]]
    assert verify_beacons(eng, pk, odd) == [False, True]




@pytest.mark.parametrize("scenario", [scenario_wire_to_sync], ids=lambda f: f.__name__)
def test_wire_cpu(scenario, chain):
    scenario(OracleEngine(), chain)


@pytest.mark.gpu
@pytest.mark.parametrize("scenario", [scenario_wire_to_sync], ids=lambda f: f.__name__)
def test_wire_gpu(scenario, chain, engine):
    scenario(engine, chain)
