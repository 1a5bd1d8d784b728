"""Generate the committed golden fixtures under tests/golden/ from the CPU oracle.

The oracle (oracle/bls12381.py) is first pinned against the reference's only fixed known answer,
key/curve_test.go:10-30 (TestBLS12381Compatv112); this script refuses to run if that KAT fails.
Recipes follow the reference's own generators:
  * chained/unchained history: client/test/result/mock/result.go:98-132 (single key, random 32-byte
    genesis seed as round-1 PreviousSig, sig_i signs Message(i, sig_{i-1}), SigV2 signs MessageV2(i))
  * threshold round: chain/beacon/node_test.go:52-102 (summed PriPoly shares at x = i+1, Sign every
    share, Recover, VerifyRecovered), sized n = 64, t = MinimumT(64) = 33 (key/group.go:312-314)
  * malformed signatures: SURVEY.md §8d config 5 classes; test/mock/grpcserver.go:66-69 (3-byte
    bad signature) and :145-147 (signature of the wrong round).
Deterministic: all randomness from random.Random(seed).

Usage: python tests/golden/make_golden.py [--threshold-n 64 --threshold-t 33]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import bls12381 as O  # noqa: E402

KAT_SK = 0x643D6C704505385387A20D98ABA19664E3EE81C600D21A0DA910CC87F5DC4AB3
KAT_MSG = bytes.fromhex("7061737320746865207369676e6174757265")
KAT_SIG = bytes.fromhex("9940ca447bab3bab393c3a07866349343630437167eaeab063ef1e47acedc51e85c513121cf319a8832c3d13"
                        "6d7f36490fa7241194b403a3bbbba9e7d5e73c9a86f67a9585c6fe077cd6576b2f76560efbab3550d9d5124242"
                        "c728e3a7ef6989")


def hx(b):
    return bytes(b).hex()


def seeded_sk(label):
    return int.from_bytes(hashlib.sha256(label.encode()).digest(), "big") % O.R


def chained(label, n, v2=True):
    rng = random.Random(label)
    sk = seeded_sk(label)
    pk = O.g1_compress(O.sk_to_pk(sk))
    prev = bytes(rng.getrandbits(8) for _ in range(32))
    seed = prev
    out = []
    for i in range(1, n + 1):
        sig = O.sign(sk, O.message(i, prev))
        rec = {"round": i, "prev": hx(prev), "sig": hx(sig)}
        if v2:
            rec["sig_v2"] = hx(O.sign(sk, O.message_v2(i)))
        out.append(rec)
        prev = sig
    return {"label": label, "sk": hex(sk), "pk": hx(pk), "genesis_seed": hx(seed), "beacons": out}


def non_g2_point(rng):
    """On-curve E2' point outside G2 (no cofactor clearing), compressed."""
    while True:
        x = (rng.randrange(O.P), rng.randrange(O.P))
        y = O.f2_sqrt(O.f2_add(O.f2_mul(O.f2_sqr(x), x), O.B2))
        if y is not None and not O.g2_in_subgroup((x, y)):
            return O.g2_compress((x, y))


def malformed(base_sigs, rng, sk):
    """List of (name, sig_bytes) per class; base_sigs valid for their rounds."""
    cases = []
    s = bytearray(base_sigs[0])
    s[rng.randrange(1, 96)] ^= 1 << rng.randrange(8)
    cases.append(("bitflip_x", bytes(s)))
    s = bytearray(base_sigs[1])
    s[0] &= 0x7F
    cases.append(("flag_cleared", bytes(s)))
    cases.append(("infinity", bytes([0xC0]) + bytes(95)))
    cases.append(("infinity_stray_bits", bytes([0xC0]) + bytes(94) + b"\x01"))
    cases.append(("infinity_sign_bit", bytes([0xE0]) + bytes(95)))
    # x.c1 >= p (keep flags)
    s = bytearray(O.P.to_bytes(48, "big") + base_sigs[2][48:])
    s[0] |= 0x80
    cases.append(("x_c1_ge_p", bytes(s)))
    s = bytearray(base_sigs[3][:48] + (O.P + 5).to_bytes(48, "big"))
    cases.append(("x_c0_ge_p", bytes(s)))
    # x with no square root for x^3 + b
    while True:
        x1, x0 = rng.randrange(O.P), rng.randrange(O.P)
        if O.f2_sqrt(O.f2_add(O.f2_mul(O.f2_sqr((x0, x1)), (x0, x1)), O.B2)) is None:
            b = bytearray(x1.to_bytes(48, "big") + x0.to_bytes(48, "big"))
            b[0] |= 0x80
            cases.append(("not_on_curve", bytes(b)))
            break
    cases.append(("not_in_subgroup", non_g2_point(rng)))
    cases.append(("wrong_round", base_sigs[5]))  # a valid signature of another round
    cases.append(("sign_bit_flipped", bytes([base_sigs[6][0] ^ 0x20]) + base_sigs[6][1:]))
    return cases


# Decode edge classes whose verdict follows the ZCash encoding rules as kilic/bls12-381 is documented
# to apply them, with no reference fixture or test behind them: parity unpinned.
UNPINNED_DECODE_CLASSES = ("infinity", "infinity_stray_bits", "infinity_sign_bit", "x_c1_ge_p", "x_c0_ge_p")


def mixed_batch(label, n, rng):
    """Config 5 recipe in small: chained history with injected corruptions."""
    ch = chained(label, n, v2=False)
    sk = int(ch["sk"], 16)
    sigs = [bytes.fromhex(b["sig"]) for b in ch["beacons"]]
    cases = malformed(sigs, rng, sk)
    positions = sorted(rng.sample(range(2, n), len(cases)))
    corrupted = list(sigs)
    injected = []
    for pos, (name, bad) in zip(positions, cases):
        if name == "wrong_round":
            bad = sigs[pos - 1]  # the previous round's (valid) signature
        corrupted[pos] = bad
        injected.append({"index": pos, "class": name,
                         "parity": "unpinned" if name in UNPINNED_DECODE_CLASSES else "spec"})
    pk = O.g1_decompress(bytes.fromhex(ch["pk"]))
    prev0 = bytes.fromhex(ch["genesis_seed"])
    expect = []
    for i, s in enumerate(corrupted):
        prev = prev0 if i == 0 else corrupted[i - 1]
        expect.append(O.verify_class(pk, O.message(i + 1, prev), s))
    return {"label": label, "pk": ch["pk"], "genesis_seed": ch["genesis_seed"],
            "sigs": [hx(s) for s in corrupted], "injected": injected, "expect_class": expect,
            "parity_note": "classes marked parity=unpinned follow the published ZCash/kilic decoding rules; "
                           "no reference fixture pins them"}


def threshold(label, n, t, rng):
    coeffs = [rng.randrange(1, O.R) for _ in range(t)]
    commits = [O.g1_mul(O.G1, c) for c in coeffs]
    prev = bytes(rng.getrandbits(8) for _ in range(96))
    rnd = 1234
    msg = O.message(rnd, prev)
    partials = []
    for i in range(n):
        share = O.pripoly_eval(coeffs, i)
        partials.append(O.tbls_sign(i, share, msg))
    group_sig = O.sign(coeffs[0], msg)
    subset = sorted(rng.sample(range(n), t))
    shuffled = [partials[i] for i in subset]
    rng.shuffle(shuffled)
    rec = O.tbls_recover(commits, msg, shuffled, t, n)
    assert rec == group_sig, "recover != a0*H(m)"
    # a corrupted partial (valid point, wrong share) for the negative path
    bad = O.tbls_sign(3, (O.pripoly_eval(coeffs, 3) + 1) % O.R, msg)
    # the same round's V2 partials (node.go:298-299: SignPartial over MessageV2(round)); no rng draws
    msg2 = O.message_v2(rnd)
    partials_v2 = [O.tbls_sign(i, O.pripoly_eval(coeffs, i), msg2) for i in range(n)]
    group_sig_v2 = O.sign(coeffs[0], msg2)
    bad_v2 = O.tbls_sign(5, (O.pripoly_eval(coeffs, 5) + 1) % O.R, msg2)
    return {"label": label, "n": n, "t": t, "round": rnd, "prev": hx(prev), "msg": hx(msg),
            "commits": [hx(O.g1_compress(c)) for c in commits], "partials": [hx(p) for p in partials],
            "recover_subset": [hx(p) for p in shuffled], "group_sig": hx(group_sig), "bad_partial": hx(bad),
            "msg_v2": hx(msg2), "partials_v2": [hx(p) for p in partials_v2], "group_sig_v2": hx(group_sig_v2),
            "bad_partial_v2": hx(bad_v2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threshold-n", type=int, default=64)
    ap.add_argument("--threshold-t", type=int, default=33)
    ap.add_argument("--chain-len", type=int, default=24)
    args = ap.parse_args()
    # pin the oracle first
    assert O.sign(KAT_SK, KAT_MSG) == KAT_SIG, "oracle fails key/curve_test.go KAT"
    O.verify(O.sk_to_pk(KAT_SK), KAT_MSG, KAT_SIG)
    rng = random.Random(20250114)
    out = {}
    out["kat"] = {"sk": hex(KAT_SK), "msg": hx(KAT_MSG), "sig": hx(KAT_SIG),
                  "pk": hx(O.g1_compress(O.sk_to_pk(KAT_SK))), "source": "key/curve_test.go:10-30"}
    print("chained...", flush=True)
    out["chained"] = chained("drand-gpu-cfg1", args.chain_len)
    print("mixed...", flush=True)
    out["mixed"] = mixed_batch("drand-gpu-cfg5", 32, rng)
    print("threshold...", flush=True)
    out["threshold"] = threshold("drand-gpu-cfg3", args.threshold_n, args.threshold_t, rng)
    # hash-to-curve vectors (arbitrary lengths, incl. empty and > 1 block)
    print("h2c...", flush=True)
    h2c = []
    for m in [b"", b"abc", KAT_MSG, bytes(range(32)), bytes(range(64)) + bytes(range(64)), b"q" * 200]:
        h = O.hash_to_g2(m)
        h2c.append({"msg": hx(m), "x": [hex(h[0][0]), hex(h[0][1])], "y": [hex(h[1][0]), hex(h[1][1])]})
    out["hash_to_g2"] = h2c
    # pairing vectors e(aG1, bG2)
    pv = []
    for _ in range(2):
        a, b = rng.randrange(1, O.R), rng.randrange(1, O.R)
        p, q = O.g1_mul(O.G1, a), O.g2_mul(O.G2, b)
        e = O.pairing(p, q)
        pv.append({"p": [hex(p[0]), hex(p[1])], "q": [hex(q[0][0]), hex(q[0][1]), hex(q[1][0]), hex(q[1][1])],
                   "e": [[hex(c[0]), hex(c[1])] for c in e]})
    out["pairing"] = pv
    path = os.path.join(HERE, "golden.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
