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
"""
import random

import pytest

pytestmark = pytest.mark.gpu

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
LENGTHS = (0, 1, 31, 32, 33, 63, 64, 65, 100, 135, 136, 137, 200, 255, 256, 300)


@pytest.fixture(scope="module")
def C():
    from oracle import c_oracle

    c_oracle.load()
    return c_oracle


def _msgs(rng, n):
    return [bytes(rng.getrandbits(8) for _ in range(rng.choice(LENGTHS))) for _ in range(n)]


def test_sign_random_messages_equal_oracle(engine, C):
    rng = random.Random(0x5157)
    sk = rng.randrange(1, R)
    msgs = _msgs(rng, 160)
    got = engine.sign(sk.to_bytes(32, "big"), msgs)
    bad = [i for i, (m, s) in enumerate(zip(msgs, got)) if s != C.sign(sk, m)]
    assert not bad, bad[:8]


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
    rng = random.Random(0xF022 + (route == "batch"))
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
