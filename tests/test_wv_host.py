"""The latency engine (drand_amd/csrc/w*.h: one item per wave, one 25-bit limb per lane) compiled
for the host with wv.h's lane emulation (tools/wvtest) and checked on the CPU against Python
integers, the reference KAT (key/curve_test.go:10-30) and the golden fixtures. The host build also
checks every arithmetic contract (operand bounds, subtrahends below their constant) as it runs."""
import json
import os
import random
import subprocess

import pytest

from oracle import bls12381 as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# WVTEST_TARGET=wvtest-asan runs the module on the ASan+UBSan build (tests/test_sanitize.py)
TARGET = os.environ.get("WVTEST_TARGET", "wvtest")
BIN = os.path.join(ROOT, "tools", TARGET)
P = O.P


@pytest.fixture(scope="module")
def wvtest():
    subprocess.run(["make", "-C", os.path.join(ROOT, "tools"), TARGET], check=True, capture_output=True)
    return BIN


def run(binary, cmd, lines):
    r = subprocess.run([binary, cmd], input="\n".join(lines) + "\n", capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return r.stdout.strip().split("\n")


def _m2(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def test_field_ops_match_integers(wvtest):
    rng = random.Random(11)
    cases = [tuple(rng.randrange(P) for _ in range(4)) for _ in range(40)]
    cases += [(0, 0, 1, 0), (1, 0, 1, 0), (P - 1, P - 1, P - 1, P - 1), (0, 1, 0, 1), (2 ** 380, 3, 7, 2 ** 200)]
    out = run(wvtest, "field", [" ".join("%x" % v for v in c) for c in cases])
    half = (P + 1) // 2
    for c, line in zip(cases, out):
        a, b = (c[0], c[1]), (c[2], c[3])
        f = [int(x, 16) for x in line.split()[:22]]
        got = [tuple(f[i:i + 2]) for i in range(0, 22, 2)]
        n = (a[0] ** 2 + a[1] ** 2) % P
        inv = (a[0] * pow(n, P - 2, P) % P, -a[1] * pow(n, P - 2, P) % P) if n else (0, 0)
        want = [_m2(a, b), _m2(a, a), (a[0] * b[0] % P, a[1] * b[1] % P), ((a[0] + b[0]) % P, (a[1] + b[1]) % P),
                ((a[0] - b[0]) % P, (a[1] - b[1]) % P), ((a[0] - a[1]) % P, (a[0] + a[1]) % P), (a[0], -a[1] % P),
                (a[0] * half % P, a[1] * half % P), inv, (n, n),
                tuple((x + y + z) % P for x, y, z in zip(_m2(a, b), _m2(b, a), _m2(a, a)))]
        assert got == want, c
        eq, z = map(int, line.split()[22:])
        assert eq == (a == b) and z == (a == (0, 0))


def test_lane_gcd_inverse(wvtest):
    """wfield.h inv_gcd_lanes (the lane-parallel binary GCD behind every latency-path inversion):
    random values and the structured inputs of tools/opcount invfuzz (powers of two, p minus powers
    of two, p / 2^k, values next to p, small values), each inverse against Python's, and every input
    must converge (no exponentiation fallback)."""
    rng = random.Random(25)
    vals = [0, 1, 2, 3, P - 1, P - 2, (P + 1) // 2, (P - 1) // 2]
    vals += [1 << k for k in range(0, 381, 7)] + [P - (1 << k) for k in range(0, 380, 9)]
    vals += [P >> k for k in range(1, 380, 11)] + [rng.randrange(1, 1 << 32) for _ in range(10)]
    vals += [rng.randrange(P) for _ in range(400)]
    vals = [v % P for v in vals]
    out = run(wvtest, "inv", ["%x" % v for v in vals])
    assert len(out) == len(vals)
    for v, line in zip(vals, out):
        assert line != "nc", hex(v)
        want = pow(v, P - 2, P)
        assert [int(x, 16) for x in line.split()] == [want, want], hex(v)


def test_team_g2_addition_cases(wvtest, golden):
    """wvteam.h team_g2_add (the hash team's five-round G2 addition, three host threads) against the
    one-wave wcurve.h g2_add on the cases a hash never reaches: P + P (doubling), P + (-P) (infinity),
    O + Q, Q + O, besides a generic sum; and the team [|x|] chain (team_mul_x_abs) against
    g2_mul_x_abs -- on golden signature points in scaled Jacobian coordinates."""
    sigs = [golden["kat"]["sig"]] + [b["sig"] for b in golden["chained"]["beacons"][:2]]
    lines = ["%s %s" % (s, c) for s in sigs for c in ("sum", "dbl", "neg", "ainf", "binf", "chain")]
    assert run(wvtest, "teamadd", lines) == ["ok"] * len(lines)


def test_hash_to_g2_golden(wvtest, golden):
    cases = golden["hash_to_g2"]
    out = run(wvtest, "hash", [h["msg"] or "-" for h in cases])
    for h, line in zip(cases, out):
        assert line == "0 %x %x %x %x" % tuple(int(v, 16) for v in h["x"] + h["y"]), h["msg"]


def test_decompress_matches_oracle(wvtest, golden):
    m = golden["mixed"]
    sigs = [golden["kat"]["sig"]] + [b["sig"] for b in golden["chained"]["beacons"][:4]] + m["sigs"]
    out = run(wvtest, "decompress", sigs)
    for s, line in zip(sigs, out):
        try:
            pt = O.g2_decompress(bytes.fromhex(s))
            want = "0 1 0 0 0 0" if pt is None else "0 0 %x %x %x %x" % (pt[0][0], pt[0][1], pt[1][0], pt[1][1])
        except O.DecodeError as e:
            want = "%d 0 0 0 0 0" % e.cls
        assert line == want, s


@pytest.mark.parametrize("cmd", ["verify", "tverify", "tverify_pre"])
def test_verify_kat_and_chain(wvtest, golden, cmd):
    """verify = one wave (wverify.h); tverify = the eight-wave team of the device kernels (wvteam.h),
    one host thread per wave; tverify_pre = the fused round's two launches (H hashed on its own, the
    signature handed over as an affine point: wvteam.h team_hash_key / verify_team_pre)"""
    kat = golden["kat"]
    ch = golden["chained"]
    seed = bytes.fromhex(ch["genesis_seed"])
    lines = ["%s %s %s" % (kat["pk"], kat["msg"], kat["sig"])]
    beacons = ch["beacons"][:3]
    for i, b in enumerate(beacons):
        prev = seed if i == 0 else bytes.fromhex(beacons[i - 1]["sig"])
        lines.append("%s %s %s" % (ch["pk"], O.message(b["round"], prev).hex(), b["sig"]))
    # negative controls: the KAT signature on another message, a beacon under the wrong round
    lines.append("%s %s %s" % (kat["pk"], "00" + kat["msg"], kat["sig"]))
    lines.append("%s %s %s" % (ch["pk"], O.message(beacons[0]["round"] + 1, seed).hex(), beacons[0]["sig"]))
    assert run(wvtest, cmd, lines) == ["0"] * 4 + ["7", "7"]


@pytest.mark.slow
@pytest.mark.parametrize("cmd", ["verify", "tverify"])
def test_verify_mixed_golden_classes(wvtest, golden, cmd):
    """Every reject class of the mixed golden batch (configs[4] classes, chained messages)."""
    m = golden["mixed"]
    seed = bytes.fromhex(m["genesis_seed"])
    sigs = [bytes.fromhex(s) for s in m["sigs"]]
    lines = []
    for i, s in enumerate(sigs):
        prev = seed if i == 0 else sigs[i - 1]
        lines.append("%s %s %s" % (m["pk"], O.message(i + 1, prev).hex(), s.hex()))
    assert [int(x) for x in run(wvtest, cmd, lines)] == m["expect_class"]


def test_verify_pre_infinity_signature(wvtest, golden):
    """The split VerifyRecovered with the signature at infinity (the interpolated sum of a degenerate
    share set): only the key pair runs, e(pk, H) != 1 rejects it -- the class verify_team gives the
    compressed infinity, whose decoding is the point at infinity. And with the key at infinity: the
    signature pair alone (rejected), or no pair at all (the empty product accepts, as kilic's Check)"""
    kat = golden["kat"]
    inf = "c0" + "00" * 95
    line = "%s %s %s" % (kat["pk"], kat["msg"], inf)
    assert run(wvtest, "tverify_pre", [line]) == run(wvtest, "tverify", [line]) == ["7"]
    # the key at infinity (the key pair inactive): the signature pair alone, and both inactive
    pk_inf = "c0" + "00" * 47
    lines = ["%s %s %s" % (pk_inf, kat["msg"], kat["sig"]), "%s %s %s" % (pk_inf, kat["msg"], inf)]
    assert run(wvtest, "tverify_pre", lines) == run(wvtest, "tverify", lines) == ["7", "0"]


def test_recover_four_wave_lambda_product(wvtest, golden):
    """wrecover.h's four-wave form of [lambda] S (k_lat_recover_mul: wave j computes [d_j] P_j with
    the exception-free mixed addition) against the joint-table g2_mul_lambda, for the golden partials'
    signatures and scalars below r: small ones, one-digit ones, and random full-width ones."""
    import random
    rng = random.Random(7)
    r = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
    x = 0xD201000000010000
    sigs = [p[4:] for p in golden["threshold"]["partials"][:6]]
    ks = [1, 2, 3, x - 1, x, x + 1, x * x + 5, r - 1] + [rng.randrange(1, r) for _ in range(10)]
    lines = ["%s %x" % (sigs[i % len(sigs)], k) for i, k in enumerate(ks)]
    assert run(wvtest, "smul4", lines) == ["ok"] * len(lines)
