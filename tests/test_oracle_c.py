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
