"""CPU tests of the oracle (oracle/bls12381.py) against the reference's own known answers, and of
the committed golden fixtures against the oracle. No GPU.

Pins:
  * key/curve_test.go:10-30 TestBLS12381Compatv112: sk, msg "pass the signature", 96-byte sig.
  * chain/store_test.go:9-14 TestRoundToBytes: big-endian round encoding.
  * README.md:203-206: round-367 randomness == sha256(signature).
"""
import hashlib
import struct

import pytest

from oracle import bls12381 as O


def test_kat_sign_verify(golden):
    kat = golden["kat"]
    sk = int(kat["sk"], 16)
    msg = bytes.fromhex(kat["msg"])
    assert msg == b"pass the signature"
    sig = O.sign(sk, msg)
    assert sig.hex() == kat["sig"]  # key/curve_test.go:26-29
    pk = O.sk_to_pk(sk)
    assert O.g1_compress(pk).hex() == kat["pk"]
    O.verify(pk, msg, sig)
    with pytest.raises(O.VerifyError):
        O.verify(pk, msg + b"x", sig)


def test_round_to_bytes():
    # chain/store_test.go:9-14
    assert O.round_to_bytes(1) == struct.pack(">Q", 1)
    assert O.round_to_bytes(0x0102030405060708) == bytes(range(1, 9))


def test_readme_randomness_pin():
    # README.md:203-206 (round 367 of the League of Entropy chain)
    sig = bytes.fromhex(
        "b62dd642e939191af1f9e15bef0f0b0e9562a5f570a12a231864afe468377e2a6424a92ccfc34ef1471cbd58c37c6b020cf75ce9446d2aa1252a090250b2b1441f8a2a0d22208dcc09332eaa0143c4a508be13de63978dbed273e3b9813130d5")
    assert O.randomness(sig).hex() == "d7aed3686bf2be657e6d38c20999831308ee6244b68c8825676db580e7e3bec6"


def test_golden_chained_sample(golden):
    ch = golden["chained"]
    pk = O.g1_decompress(bytes.fromhex(ch["pk"]))
    assert O.g1_compress(O.sk_to_pk(int(ch["sk"], 16))).hex() == ch["pk"]
    bs = ch["beacons"]
    assert bs[0]["prev"] == ch["genesis_seed"] and len(bytes.fromhex(bs[0]["prev"])) == 32
    for a, b in zip(bs, bs[1:]):
        assert b["prev"] == a["sig"] and b["round"] == a["round"] + 1
    for b in (bs[0], bs[-1]):
        O.verify_beacon(pk, b["round"], bytes.fromhex(b["prev"]), bytes.fromhex(b["sig"]))
        O.verify_beacon_v2(pk, b["round"], bytes.fromhex(b["sig_v2"]))
    with pytest.raises(O.VerifyError):  # wrong round (test/mock/grpcserver.go:145-147)
        O.verify_beacon(pk, bs[1]["round"] + 1, bytes.fromhex(bs[1]["prev"]), bytes.fromhex(bs[1]["sig"]))


def test_golden_mixed_classes_sample(golden):
    mx = golden["mixed"]
    pk = O.g1_decompress(bytes.fromhex(mx["pk"]))
    sigs = [bytes.fromhex(s) for s in mx["sigs"]]
    seed = bytes.fromhex(mx["genesis_seed"])
    # decode-class rejects are cheap to recheck: every non-pairing class
    for i, c in enumerate(mx["expect_class"]):
        if c in (O.REJ_FLAG, O.REJ_INF_NONZERO, O.REJ_X_GE_P, O.REJ_NOT_ON_CURVE, O.REJ_NOT_IN_SUBGROUP):
            prev = seed if i == 0 else sigs[i - 1]
            assert O.verify_class(pk, O.message(i + 1, prev), sigs[i]) == c, i


def test_decode_edge_cases():
    # infinity must be exactly 0xc0 || 0...; compression flag required; x >= p rejected
    inf = bytes([0xC0]) + bytes(95)
    assert O.g2_decompress(inf) is None
    with pytest.raises(O.DecodeError) as e:
        O.g2_decompress(bytes([0xC0]) + bytes(94) + b"\x01")
    assert e.value.cls == O.REJ_INF_NONZERO
    with pytest.raises(O.DecodeError) as e:
        O.g2_decompress(bytes(96))
    assert e.value.cls == O.REJ_FLAG
    pbytes = O.P.to_bytes(48, "big")
    with pytest.raises(O.DecodeError) as e:
        O.g2_decompress(bytes([0x80 | pbytes[0]]) + pbytes[1:] + bytes(48))
    assert e.value.cls == O.REJ_X_GE_P


def test_threshold_fixture_consistency(golden):
    th = golden["threshold"]
    assert th["t"] == 33 and th["n"] == 64  # MinimumT(64), key/group.go:312-314
    assert len(th["partials"]) == 64 and len(th["recover_subset"]) == 33
    idx = [O.tbls_index_of(bytes.fromhex(p)) for p in th["partials"]]
    assert sorted(idx) == list(range(64))
