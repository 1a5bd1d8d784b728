"""CPU tests of the C oracle (oracle/c/bls_oracle.c, the cpu_baseline restatement) against the
reference KAT (key/curve_test.go:10-30), the committed golden vectors (made by the pinned Python
oracle) and the Python oracle itself. No GPU."""
import os
import subprocess

import pytest

from oracle import bls12381 as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def C():
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    from oracle import c_oracle

    c_oracle.load()
    return c_oracle


def test_kat(C, golden):
    kat = golden["kat"]
    msg = bytes.fromhex(kat["msg"])
    assert C.sign(int(kat["sk"], 16), msg).hex() == kat["sig"]  # key/curve_test.go:26-29
    assert C.verify(bytes.fromhex(kat["pk"]), msg, bytes.fromhex(kat["sig"])) == O.REJ_OK
    assert C.verify(bytes.fromhex(kat["pk"]), msg + b"x", bytes.fromhex(kat["sig"])) == O.REJ_PAIRING


def test_hash_to_g2_golden(C, golden):
    for v in golden["hash_to_g2"]:
        x = (int(v["x"][0], 16), int(v["x"][1], 16))
        y = (int(v["y"][0], 16), int(v["y"][1], 16))
        assert C.hash_to_g2(bytes.fromhex(v["msg"])) == O.g2_compress((x, y))


def test_chained_golden(C, golden):
    ch = golden["chained"]
    sigs = b"".join(bytes.fromhex(b["sig"]) for b in ch["beacons"])
    cls = C.verify_chained(bytes.fromhex(ch["pk"]), ch["beacons"][0]["round"], bytes.fromhex(ch["genesis_seed"]), sigs)
    assert cls == [O.REJ_OK] * len(ch["beacons"])
    # wrong round rejects (test/mock/grpcserver.go:145-147)
    assert C.verify_chained(bytes.fromhex(ch["pk"]), 2, bytes.fromhex(ch["genesis_seed"]), sigs[:96]) == [O.REJ_PAIRING]


def test_mixed_golden_classes(C, golden):
    mx = golden["mixed"]
    sigs = b"".join(bytes.fromhex(s) for s in mx["sigs"])
    assert C.verify_chained(bytes.fromhex(mx["pk"]), 1, bytes.fromhex(mx["genesis_seed"]), sigs) == mx["expect_class"]


def test_decode_edge_cases(C):
    assert C.g2_decode_class(bytes([0xC0]) + bytes(95)) == O.REJ_OK  # canonical infinity decodes
    assert C.g2_decode_class(bytes([0xC0]) + bytes(94) + b"\x01") == O.REJ_INF_NONZERO
    assert C.g2_decode_class(bytes(96)) == O.REJ_FLAG
    assert C.g2_decode_class(bytes(95)) == O.REJ_LENGTH
    pb = O.P.to_bytes(48, "big")
    assert C.g2_decode_class(bytes([0x80 | pb[0]]) + pb[1:] + bytes(48)) == O.REJ_X_GE_P


def test_cross_check_python_oracle(C):
    sk = 0x1234567890ABCDEF1234567890ABCDEF1234567890ABCDEF % O.R
    pk48 = O.g1_compress(O.sk_to_pk(sk))
    msg = O.message(42, bytes(range(96)))
    sig = C.sign(sk, msg)
    assert sig == O.sign(sk, msg)
    assert C.verify(pk48, msg, sig) == O.verify_class(O.g1_decompress(pk48), msg, sig) == O.REJ_OK


def test_threshold_golden(C, golden):
    """tbls VerifyPartial / Recover of the C oracle (the configs[2] CPU baseline) against the golden
    n = 64 / t = 33 round made by the Python oracle: every V1 and V2 partial accepts, the bad partial
    rejects, and Recover reproduces both group signatures byte for byte."""
    th = golden["threshold"]
    g = C.Group([bytes.fromhex(c) for c in th["commits"]])
    try:
        for key, sig_key, bad_key in (("msg", "partials", "bad_partial"), ("msg_v2", "partials_v2", "bad_partial_v2")):
            msg = bytes.fromhex(th[key])
            parts = [bytes.fromhex(p) for p in th[sig_key]]
            assert all(g.verify_partial(msg, p) == O.REJ_OK for p in parts[:8])
            assert g.verify_partial(msg, bytes.fromhex(th[bad_key])) != O.REJ_OK
            assert g.verify_partial(msg, b"\x00") == O.REJ_LENGTH
        msg = bytes.fromhex(th["msg"])
        sub = [bytes.fromhex(p) for p in th["recover_subset"]]
        assert g.recover(msg, sub, th["t"], th["n"]).hex() == th["group_sig"]
        parts2 = [bytes.fromhex(p) for p in th["partials_v2"]]
        assert g.recover(bytes.fromhex(th["msg_v2"]), [bytes.fromhex(th["bad_partial_v2"])] + parts2,
                         th["t"], th["n"]).hex() == th["group_sig_v2"]
        assert g.recover(msg, sub[:-1], th["t"], th["n"]) is None            # t - 1 good shares
        assert g.recover(msg, sub[:-1] + [sub[0]], th["t"], th["n"]) is None  # a duplicate counts, collapses
    finally:
        g.close()


def test_chain2049_fixture_is_the_golden_chain(golden):
    """tests/golden/chain2049.bin (make_chain_fixture.py) continues the golden chained history: its
    first rounds are the golden beacons byte for byte, and the C oracle accepts samples further on."""
    from oracle import c_oracle

    c_oracle.load()
    with open(os.path.join(os.path.dirname(__file__), "golden", "chain2049.bin"), "rb") as f:
        raw = f.read()
    assert len(raw) == 2049 * 96
    ch = golden["chained"]
    assert [raw[i * 96:(i + 1) * 96].hex() for i in range(len(ch["beacons"]))] == [b["sig"] for b in ch["beacons"]]
    pk = bytes.fromhex(ch["pk"])
    for lo in (1999, 2047):
        assert c_oracle.verify_chained(pk, lo + 1, raw[(lo - 1) * 96:lo * 96], raw[lo * 96:(lo + 2) * 96]) == [0, 0]
