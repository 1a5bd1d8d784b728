"""CPU ORACLE (test infrastructure only) -- pure-Python restatement of drand's BLS12-381 path.

ONLY tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and
only as the checker. The product path (drand_amd/) never imports it.

What it restates (the reference's arithmetic lives in un-vendored Go modules):
  * github.com/kilic/bls12-381 @ v0.0.0-20200820230200-6b2c19996391 (go.sum:344): Fp..Fp12,
    G1/G2, ZCash compressed encoding, hash-to-curve, Engine.AddPair/AddPairInv/Check.
  * github.com/drand/kyber-bls12381 v0.2.1 (go.mod:10): Suite.ValidatePairing, KyberG2.Hash with
    DST "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_".
  * github.com/drand/kyber @ d59c3367dcde (go.mod:9): sign/bls Verify, sign/tbls (2-byte index
    prefix), share.PubPoly.Eval / RecoverCommit (x = i+1, Lagrange at 0).
Published algorithms followed: RFC 9380 (hash_to_curve suite BLS12381G2_XMD:SHA-256_SSWU_RO_),
the ZCash BLS12-381 serialization, and the optimal-ate pairing for BLS12.

The oracle is deliberately *naive* where kilic is naive (cofactor clearing by the 636-bit h_eff
scalar multiplication, subgroup check by [r]P == O) and uses textbook affine Miller-loop
arithmetic over E(Fp12), so that it shares no algorithm with the GPU engine (which uses
psi-based cofactor clearing / subgroup checks and projective sparse-line Miller loops).

Pinned by the reference's only fixed known-answer test, key/curve_test.go:10-30
(TestBLS12381Compatv112), see tests/test_oracle.py.
"""
from __future__ import annotations

import hashlib
import struct

# ----------------------------------------------------------------------------------------------
# Parameters
# ----------------------------------------------------------------------------------------------
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
X_ABS = 0xD201000000010000          # BLS parameter x = -X_ABS
X = -X_ABS
H_EFF_G2 = 0xBC69F08F2EE75B3584C6A0EA91B352888E2A8E9145AD7689986FF031508FFE1329C2F178731DB956D82BF015D1212B02EC0EC69D7477C1AE954CBC06689F6A359894C0ADEBBF6B4E8020005AAA95551

DST_G2 = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_"

G1_X = 0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB
G1_Y = 0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1
G2_X = (0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
        0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E)
G2_Y = (0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
        0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE)


class VerifyError(Exception):
    """Reject of a signature / encoding (kyber returns a non-nil error)."""


# ----------------------------------------------------------------------------------------------
# Fp and Fp2 = Fp[i]/(i^2+1)
# ----------------------------------------------------------------------------------------------
def fp_inv(a):
    return pow(a % P, P - 2, P)


def fp_sqrt(a):
    """Square root in Fp (p = 3 mod 4) or None."""
    a %= P
    s = pow(a, (P + 1) // 4, P)
    return s if s * s % P == a else None


F2_ZERO = (0, 0)
F2_ONE = (1, 0)
XI = (1, 1)  # non-residue 1 + i used for the sextic twist


def f2_add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2_sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2_neg(a):
    return ((-a[0]) % P, (-a[1]) % P)


def f2_mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def f2_sqr(a):
    return f2_mul(a, a)


def f2_muls(a, k):
    return (a[0] * k % P, a[1] * k % P)


def f2_conj(a):
    return (a[0], (-a[1]) % P)


def f2_inv(a):
    n = (a[0] * a[0] + a[1] * a[1]) % P
    ni = fp_inv(n)
    return (a[0] * ni % P, (-a[1]) * ni % P)


def f2_pow(a, e):
    r = F2_ONE
    b = a
    while e:
        if e & 1:
            r = f2_mul(r, b)
        b = f2_sqr(b)
        e >>= 1
    return r


def f2_is_zero(a):
    return a[0] % P == 0 and a[1] % P == 0


def f2_eq(a, b):
    return (a[0] - b[0]) % P == 0 and (a[1] - b[1]) % P == 0


def f2_is_square(a):
    """Euler criterion in Fp2 through the norm map (a is a square in Fp2 iff N(a) is in Fp)."""
    n = (a[0] * a[0] + a[1] * a[1]) % P
    return n == 0 or pow(n, (P - 1) // 2, P) == 1


def f2_sqrt(a):
    """A square root in Fp2 (p = 3 mod 4 'complex method'), or None."""
    if f2_is_zero(a):
        return F2_ZERO
    a1 = f2_pow(a, (P - 3) // 4)
    alpha = f2_mul(f2_sqr(a1), a)
    x0 = f2_mul(a1, a)
    if f2_eq(alpha, (P - 1, 0)):
        cand = f2_mul((0, 1), x0)
    else:
        b = f2_pow(f2_add(F2_ONE, alpha), (P - 1) // 2)
        cand = f2_mul(b, x0)
    return cand if f2_eq(f2_sqr(cand), a) else None


def f2_sgn0(a):
    """RFC 9380 sgn0 for Fp2."""
    sign_0 = a[0] % 2
    zero_0 = a[0] == 0
    sign_1 = a[1] % 2
    return sign_0 | (zero_0 & sign_1)


# ----------------------------------------------------------------------------------------------
# Fp12 as Fp2[w]/(w^6 - xi): element = sum c_k w^k, k = 0..5 (list of 6 Fp2).
# (The GPU engine uses the Fp2 -> Fp6 -> Fp12 tower; the coefficient map is
#  c0 + c1 w with c0 = a0 + a1 v + a2 v^2, c1 = b0 + b1 v + b2 v^2, v = w^2
#  <=> [a0, b0, a1, b1, a2, b2] here; see to_tower()/from_tower().)
# ----------------------------------------------------------------------------------------------
F12_ONE = [F2_ONE] + [F2_ZERO] * 5


def f12_mul(a, b):
    t = [F2_ZERO] * 11
    for i in range(6):
        if f2_is_zero(a[i]):
            continue
        for j in range(6):
            if f2_is_zero(b[j]):
                continue
            t[i + j] = f2_add(t[i + j], f2_mul(a[i], b[j]))
    out = t[:6]
    for k in range(6, 11):
        out[k - 6] = f2_add(out[k - 6], f2_mul(t[k], XI))
    return out


def f12_sqr(a):
    return f12_mul(a, a)


def f12_eq(a, b):
    return all(f2_eq(x, y) for x, y in zip(a, b))


def f12_pow(a, e):
    r = F12_ONE
    b = a
    while e:
        if e & 1:
            r = f12_mul(r, b)
        b = f12_sqr(b)
        e >>= 1
    return r


# Frobenius x -> x^(p^2): coefficients are in Fp2 (fixed by p^2) and w^(p^2) = w * xi^((p^2-1)/6)
_GAMMA2 = f2_pow(XI, (P * P - 1) // 6)
_GAMMA2_POW = [F2_ONE]
for _k in range(1, 6):
    _GAMMA2_POW.append(f2_mul(_GAMMA2_POW[-1], _GAMMA2))


def f12_frob2(a):
    return [f2_mul(a[k], _GAMMA2_POW[k]) for k in range(6)]


def f12_inv(a):
    """a^-1 = (prod_{k=1..5} a^(p^(2k))) / N(a), N(a) = prod_{k=0..5} a^(p^(2k)) in Fp2."""
    conjs = F12_ONE
    c = a
    for _ in range(5):
        c = f12_frob2(c)
        conjs = f12_mul(conjs, c)
    n = f12_mul(a, conjs)
    assert all(f2_is_zero(n[k]) for k in range(1, 6))
    ni = f2_inv(n[0])
    return [f2_mul(x, ni) for x in conjs]


def f12_from_fp(a):
    return [(a % P, 0)] + [F2_ZERO] * 5


def f12_from_f2(a, k=0):
    out = [F2_ZERO] * 6
    out[k] = a
    return out


def to_tower(a):
    """poly rep [c0..c5] -> tower ((a0,a1,a2),(b0,b1,b2)) with a_j = c_{2j}, b_j = c_{2j+1}."""
    return ((a[0], a[2], a[4]), (a[1], a[3], a[5]))


def from_tower(t):
    (a0, a1, a2), (b0, b1, b2) = t
    return [a0, b0, a1, b1, a2, b2]


# ----------------------------------------------------------------------------------------------
# Generic short-Weierstrass affine arithmetic (y^2 = x^3 + b) over a field given by ops.
# Points are tuples (x, y) or None for the point at infinity O.
# ----------------------------------------------------------------------------------------------
class _Field:
    def __init__(self, add, sub, mul, inv, neg, eq, zero, one, muls):
        self.add, self.sub, self.mul, self.inv, self.neg, self.eq = add, sub, mul, inv, neg, eq
        self.zero, self.one, self.muls = zero, one, muls


FP = _Field(lambda a, b: (a + b) % P, lambda a, b: (a - b) % P, lambda a, b: a * b % P,
            fp_inv, lambda a: (-a) % P, lambda a, b: (a - b) % P == 0, 0, 1,
            lambda a, k: a * k % P)
FP2 = _Field(f2_add, f2_sub, f2_mul, f2_inv, f2_neg, f2_eq, F2_ZERO, F2_ONE, f2_muls)

B1 = 4
B2 = (4, 4)  # 4 * (1 + i)


def ec_on_curve(F, b, pt):
    if pt is None:
        return True
    x, y = pt
    return F.eq(F.mul(y, y), F.add(F.mul(F.mul(x, x), x), b))


def ec_neg(F, pt):
    if pt is None:
        return None
    return (pt[0], F.neg(pt[1]))


def ec_add(F, p1, p2):
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    x1, y1 = p1
    x2, y2 = p2
    if F.eq(x1, x2):
        if F.eq(y1, F.neg(y2)):
            return None
        lam = F.mul(F.muls(F.mul(x1, x1), 3), F.inv(F.muls(y1, 2)))
    else:
        lam = F.mul(F.sub(y2, y1), F.inv(F.sub(x2, x1)))
    x3 = F.sub(F.sub(F.mul(lam, lam), x1), x2)
    y3 = F.sub(F.mul(lam, F.sub(x1, x3)), y1)
    return (x3, y3)


def ec_mul(F, pt, k):
    if k < 0:
        return ec_mul(F, ec_neg(F, pt), -k)
    acc = None
    add = pt
    while k:
        if k & 1:
            acc = ec_add(F, acc, add)
        add = ec_add(F, add, add)
        k >>= 1
    return acc


G1 = (G1_X, G1_Y)
G2 = (G2_X, G2_Y)


def g1_mul(pt, k):
    return ec_mul(FP, pt, k)


def g2_mul(pt, k):
    return ec_mul(FP2, pt, k)


def g1_add(a, b):
    return ec_add(FP, a, b)


def g2_add(a, b):
    return ec_add(FP2, a, b)


def g1_in_subgroup(pt):
    return ec_mul(FP, pt, R) is None


def g2_in_subgroup(pt):
    """kilic G2.InCorrectSubgroup: naive [r]P == O."""
    return ec_mul(FP2, pt, R) is None


# ----------------------------------------------------------------------------------------------
# ZCash compressed serialization (kilic G1/G2 ToCompressed / FromCompressed)
# ----------------------------------------------------------------------------------------------
def _fp_to_bytes(a):
    return (a % P).to_bytes(48, "big")


def _fp_largest(a):
    return a % P > (P - 1) // 2


def g1_compress(pt):
    if pt is None:
        return bytes([0xC0]) + bytes(47)
    x, y = pt
    out = bytearray(_fp_to_bytes(x))
    out[0] |= 0x80
    if _fp_largest(y):
        out[0] |= 0x20
    return bytes(out)


def g2_compress(pt):
    if pt is None:
        return bytes([0xC0]) + bytes(95)
    (x0, x1), y = pt
    out = bytearray(_fp_to_bytes(x1) + _fp_to_bytes(x0))
    out[0] |= 0x80
    y0, y1 = y
    largest = _fp_largest(y1) if y1 % P != 0 else _fp_largest(y0)
    if largest:
        out[0] |= 0x20
    return bytes(out)


# reject classes (shared vocabulary with include/blsverify.h BLSV_REJ_*)
REJ_OK = 0
REJ_LENGTH = 1
REJ_FLAG = 2
REJ_INF_NONZERO = 3
REJ_X_GE_P = 4
REJ_NOT_ON_CURVE = 5
REJ_NOT_IN_SUBGROUP = 6
REJ_PAIRING = 7


class DecodeError(VerifyError):
    def __init__(self, cls, msg):
        super().__init__(msg)
        self.cls = cls


def g1_decompress(buf):
    """kilic G1.FromCompressed: length, 0x80 flag, infinity exactly 0xc0||0, x<p, sqrt, sign, [r]P."""
    if len(buf) != 48:
        raise DecodeError(REJ_LENGTH, "bad length")
    b = bytearray(buf)
    if not b[0] & 0x80:
        raise DecodeError(REJ_FLAG, "bad compression flag")
    if b[0] & 0x40:
        if b[0] != 0xC0 or any(b[1:]):
            raise DecodeError(REJ_INF_NONZERO, "infinity with non-zero bits")
        return None
    sign = bool(b[0] & 0x20)
    b[0] &= 0x1F
    x = int.from_bytes(b, "big")
    if x >= P:
        raise DecodeError(REJ_X_GE_P, "x >= p")
    y = fp_sqrt(x * x * x + B1)
    if y is None:
        raise DecodeError(REJ_NOT_ON_CURVE, "not on curve")
    if _fp_largest(y) != sign:
        y = (-y) % P
    pt = (x, y)
    if not g1_in_subgroup(pt):
        raise DecodeError(REJ_NOT_IN_SUBGROUP, "not in subgroup")
    return pt


def g2_decompress(buf, check_subgroup=True):
    """kilic G2.FromCompressed (see SURVEY.md §8a row a8 for the check order)."""
    if len(buf) != 96:
        raise DecodeError(REJ_LENGTH, "bad length")
    b = bytearray(buf)
    if not b[0] & 0x80:
        raise DecodeError(REJ_FLAG, "bad compression flag")
    if b[0] & 0x40:
        if b[0] != 0xC0 or any(b[1:]):
            raise DecodeError(REJ_INF_NONZERO, "infinity with non-zero bits")
        return None
    sign = bool(b[0] & 0x20)
    b[0] &= 0x1F
    x1 = int.from_bytes(b[:48], "big")
    x0 = int.from_bytes(b[48:], "big")
    if x1 >= P or x0 >= P:
        raise DecodeError(REJ_X_GE_P, "x >= p")
    x = (x0, x1)
    y = f2_sqrt(f2_add(f2_mul(f2_sqr(x), x), B2))
    if y is None:
        raise DecodeError(REJ_NOT_ON_CURVE, "not on curve")
    largest = _fp_largest(y[1]) if y[1] != 0 else _fp_largest(y[0])
    if largest != sign:
        y = f2_neg(y)
    pt = (x, y)
    if check_subgroup and not g2_in_subgroup(pt):
        raise DecodeError(REJ_NOT_IN_SUBGROUP, "not in subgroup")
    return pt


# ----------------------------------------------------------------------------------------------
# RFC 9380 hash_to_curve for G2 (BLS12381G2_XMD:SHA-256_SSWU_RO_)
# ----------------------------------------------------------------------------------------------
def expand_message_xmd(msg, dst, len_in_bytes):
    b_in_bytes, r_in_bytes = 32, 64
    ell = (len_in_bytes + b_in_bytes - 1) // b_in_bytes
    assert ell <= 255 and len(dst) <= 255
    dst_prime = dst + bytes([len(dst)])
    z_pad = bytes(r_in_bytes)
    l_i_b = len_in_bytes.to_bytes(2, "big")
    b0 = hashlib.sha256(z_pad + msg + l_i_b + b"\x00" + dst_prime).digest()
    b = [hashlib.sha256(b0 + b"\x01" + dst_prime).digest()]
    for i in range(2, ell + 1):
        prev = bytes(x ^ y for x, y in zip(b0, b[-1]))
        b.append(hashlib.sha256(prev + bytes([i]) + dst_prime).digest())
    return b"".join(b)[:len_in_bytes]


def hash_to_field_fp2(msg, count=2, dst=DST_G2):
    L = 64
    ub = expand_message_xmd(msg, dst, count * 2 * L)
    out = []
    for i in range(count):
        e = []
        for j in range(2):
            off = L * (j + i * 2)
            e.append(int.from_bytes(ub[off:off + L], "big") % P)
        out.append((e[0], e[1]))
    return out


SSWU_A = (0, 240)
SSWU_B = (1012, 1012)
SSWU_Z = ((-2) % P, (-1) % P)


def map_to_curve_sswu_g2(u):
    """RFC 9380 §6.6.2 straight-line simplified SWU onto E2': y^2 = x^3 + A'x + B'."""
    A, B, Z = SSWU_A, SSWU_B, SSWU_Z
    u2 = f2_sqr(u)
    zu2 = f2_mul(Z, u2)
    den = f2_add(f2_sqr(zu2), zu2)
    tv1 = F2_ZERO if f2_is_zero(den) else f2_inv(den)
    if f2_is_zero(tv1):
        x1 = f2_mul(B, f2_inv(f2_mul(Z, A)))
    else:
        x1 = f2_mul(f2_mul(f2_neg(B), f2_inv(A)), f2_add(F2_ONE, tv1))
    gx1 = f2_add(f2_add(f2_mul(f2_sqr(x1), x1), f2_mul(A, x1)), B)
    x2 = f2_mul(zu2, x1)
    gx2 = f2_add(f2_add(f2_mul(f2_sqr(x2), x2), f2_mul(A, x2)), B)
    if f2_is_square(gx1):
        x, y = x1, f2_sqrt(gx1)
    else:
        x, y = x2, f2_sqrt(gx2)
    assert y is not None
    if f2_sgn0(u) != f2_sgn0(y):
        y = f2_neg(y)
    return (x, y)


def _h(v):
    return v % P


# RFC 9380 Appendix E.3: 3-isogeny E2' -> E2
ISO_XNUM = [
    (_h(0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97D6),
     _h(0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97D6)),
    (0, _h(0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71A)),
    (_h(0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71E),
     _h(0x8AB05F8BDD54CDE190937E76BC3E447CC27C3D6FBD7063FCD104635A790520C0A395554E5C6AAAA9354FFFFFFFFE38D)),
    (_h(0x171D6541FA38CCFAED6DEA691F5FB614CB14B4E7F4E810AA22D6108F142B85757098E38D0F671C7188E2AAAAAAAA5ED1), 0),
]
ISO_XDEN = [
    (0, _h(0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA63)),
    (0xC, _h(0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA9F)),
    (1, 0),
]
ISO_YNUM = [
    (_h(0x1530477C7AB4113B59A4C18B076D11930F7DA5D4A07F649BF54439D87D27E500FC8C25EBF8C92F6812CFC71C71C6D706),
     _h(0x1530477C7AB4113B59A4C18B076D11930F7DA5D4A07F649BF54439D87D27E500FC8C25EBF8C92F6812CFC71C71C6D706)),
    (0, _h(0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97BE)),
    (_h(0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71C),
     _h(0x8AB05F8BDD54CDE190937E76BC3E447CC27C3D6FBD7063FCD104635A790520C0A395554E5C6AAAA9354FFFFFFFFE38F)),
    (_h(0x124C9AD43B6CF79BFBF7043DE3811AD0761B0F37A1E26286B0E977C69AA274524E79097A56DC4BD9E1B371C71C718B10), 0),
]
ISO_YDEN = [
    (_h(0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA8FB),
     _h(0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA8FB)),
    (0, _h(0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA9D3)),
    (0x12, _h(0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA99)),
    (1, 0),
]


def _poly(coeffs, x):
    acc = F2_ZERO
    for c in reversed(coeffs):
        acc = f2_add(f2_mul(acc, x), c)
    return acc


def iso_map_g2(pt):
    x, y = pt
    xn, xd = _poly(ISO_XNUM, x), _poly(ISO_XDEN, x)
    yn, yd = _poly(ISO_YNUM, x), _poly(ISO_YDEN, x)
    if f2_is_zero(xd) or f2_is_zero(yd):
        return None
    return (f2_mul(xn, f2_inv(xd)), f2_mul(y, f2_mul(yn, f2_inv(yd))))


def clear_cofactor_g2(pt):
    """kilic ClearCofactor: naive multiplication by h_eff (RFC 9380 §8.8.2)."""
    return g2_mul(pt, H_EFF_G2)


def hash_to_g2(msg, dst=DST_G2):
    u0, u1 = hash_to_field_fp2(msg, 2, dst)
    q0 = iso_map_g2(map_to_curve_sswu_g2(u0))
    q1 = iso_map_g2(map_to_curve_sswu_g2(u1))
    return clear_cofactor_g2(g2_add(q0, q1))


# ----------------------------------------------------------------------------------------------
# Optimal-ate pairing, textbook affine Miller loop over E(Fp12)
# ----------------------------------------------------------------------------------------------
def _f12_ops():
    def add(a, b):
        return [f2_add(x, y) for x, y in zip(a, b)]

    def sub(a, b):
        return [f2_sub(x, y) for x, y in zip(a, b)]

    def neg(a):
        return [f2_neg(x) for x in a]

    def muls(a, k):
        return [f2_muls(x, k) for x in a]

    return _Field(add, sub, f12_mul, f12_inv, neg, f12_eq, [F2_ZERO] * 6, F12_ONE, muls)


FP12 = _f12_ops()
_XI_INV = f2_inv(XI)


def untwist(q):
    """E2'(Fp2) -> E(Fp12): (x, y) -> (x w^-2, y w^-3), w^-2 = w^4/xi, w^-3 = w^3/xi."""
    x, y = q
    return (f12_from_f2(f2_mul(x, _XI_INV), 4), f12_from_f2(f2_mul(y, _XI_INV), 3))


def _line(t, q, p):
    """Value at P of the line through T and Q (tangent if T == Q), all in E(Fp12) affine."""
    F = FP12
    (xt, yt), (xq, yq) = t, q
    xp, yp = p
    if F.eq(xt, xq):
        if F.eq(yt, yq):
            lam = F.mul(F.muls(F.mul(xt, xt), 3), F.inv(F.muls(yt, 2)))
        else:  # vertical line
            return F.sub(xp, xt)
    else:
        lam = F.mul(F.sub(yq, yt), F.inv(F.sub(xq, xt)))
    return F.sub(F.sub(yp, yt), F.mul(lam, F.sub(xp, xt)))


def miller_loop(p, q):
    """f_{|x|,Q}(P), conjugated for x < 0 (optimal ate for BLS12). O inputs give 1."""
    if p is None or q is None:
        return F12_ONE
    pe = (f12_from_fp(p[0]), f12_from_fp(p[1]))
    qe = untwist(q)
    f = F12_ONE
    t = qe
    for i in range(X_ABS.bit_length() - 2, -1, -1):
        f = f12_mul(f12_sqr(f), _line(t, t, pe))
        t = ec_add(FP12, t, t)
        if (X_ABS >> i) & 1:
            f = f12_mul(f, _line(t, qe, pe))
            t = ec_add(FP12, t, qe)
    # x < 0: f_{x} = 1 / f_{|x|} up to factors killed by the final exponentiation
    return f12_conj6(f)


def f12_conj6(a):
    """a^(p^6): w^(p^6) = -w (xi^((p^6-1)/6) = -1), Fp2 coefficients fixed."""
    return [a[k] if k % 2 == 0 else f2_neg(a[k]) for k in range(6)]


FINAL_EXP_HARD = (P ** 4 - P ** 2 + 1) // R
assert (P ** 4 - P ** 2 + 1) % R == 0


def final_exponentiation(f):
    """f^((p^12-1)/r) = ((f^(p^6-1))^(p^2+1))^((p^4-p^2+1)/r)."""
    f = f12_mul(f12_conj6(f), f12_inv(f))
    f = f12_mul(f12_frob2(f), f)
    return f12_pow(f, FINAL_EXP_HARD)


def pairing(p, q):
    return final_exponentiation(miller_loop(p, q))


def pairing_check(pairs):
    """kilic Engine: multi-Miller loop over non-O pairs, one final exp, == 1."""
    f = F12_ONE
    for p, q in pairs:
        if p is None or q is None:
            continue
        f = f12_mul(f, miller_loop(p, q))
    return f12_eq(final_exponentiation(f), F12_ONE)


# ----------------------------------------------------------------------------------------------
# BLS (kyber sign/bls on G2, tbls) and drand messages
# ----------------------------------------------------------------------------------------------
def sk_to_pk(sk):
    return g1_mul(G1, sk % R)


def sign(sk, msg):
    """kyber bls.Sign on G2: compress(sk * H(msg))."""
    return g2_compress(g2_mul(hash_to_g2(msg), sk % R))


def verify(pk, msg, sig):
    """kyber bls.Verify: H(msg), unmarshal sig (decompress + subgroup),
    ValidatePairing(pk, H, g1, sig) <=> e(pk, H) * e(-g1, sig) == 1. Raises VerifyError."""
    hm = hash_to_g2(msg)
    s = g2_decompress(sig)
    if not pairing_check([(pk, hm), (ec_neg(FP, G1), s)]):
        raise DecodeError(REJ_PAIRING, "bls: invalid signature")


def verify_class(pk, msg, sig):
    """Reject class code (REJ_*) for one signature; REJ_OK on accept."""
    try:
        verify(pk, msg, sig)
    except DecodeError as e:
        return e.cls
    return REJ_OK


def round_to_bytes(r):
    """chain/store.go:39-44 RoundToBytes (8-byte big endian)."""
    return struct.pack(">Q", r)


def message(round_, prev_sig):
    """chain/beacon.go:103-108 Message = sha256(prevSig || RoundToBytes(round))."""
    return hashlib.sha256(bytes(prev_sig) + round_to_bytes(round_)).digest()


def message_v2(round_):
    """chain/beacon.go:110-114 MessageV2 = sha256(RoundToBytes(round))."""
    return hashlib.sha256(round_to_bytes(round_)).digest()


def randomness(sig):
    """chain/beacon.go:66-69 RandomnessFromSignature = sha256(sig)."""
    return hashlib.sha256(bytes(sig)).digest()


def verify_beacon(pk, round_, prev_sig, sig):
    """chain/beacon.go:87-92 VerifyBeacon -> Scheme.VerifyRecovered(pk, Message(round, prev), sig)."""
    verify(pk, message(round_, prev_sig), sig)


def verify_beacon_v2(pk, round_, sig_v2):
    """chain/beacon.go:94-98 VerifyBeaconV2."""
    verify(pk, message_v2(round_), sig_v2)


# tbls: 2-byte big-endian index prefix (kyber sign/tbls SigShare)
def tbls_sign(index, sk_share, msg):
    return struct.pack(">H", index) + sign(sk_share, msg)


def tbls_index_of(sig):
    if len(sig) < 2:
        raise VerifyError("tbls: invalid signature share")
    return struct.unpack(">H", bytes(sig[:2]))[0]


def pubpoly_eval(commits, i):
    """share.PubPoly.Eval(i): sum_j C_j * (i+1)^j (Horner)."""
    xi = (i + 1) % R
    v = None
    for c in reversed(commits):
        v = g1_add(g1_mul(v, xi) if v is not None else None, c)
    return v


def pripoly_eval(coeffs, i):
    xi = (i + 1) % R
    v = 0
    for c in reversed(coeffs):
        v = (v * xi + c) % R
    return v


def tbls_verify_partial(commits, msg, partial):
    i = tbls_index_of(partial)
    verify(pubpoly_eval(commits, i), msg, bytes(partial[2:]))


def tbls_recover(commits, msg, partials, t, n):
    """tbls.Recover -> share.RecoverCommit ([ext] drand/kyber@d59c3367dcde, restated from the
    published source; parity unpinned by any reference test): walk the shares in input order, skip
    invalid ones, append valid ones until t are held (a duplicate index COUNTS toward t); xyCommit
    then keys them by index (duplicates collapse) and drops indices >= n; fewer than t distinct ->
    "not enough good public shares". Lagrange-interpolate at 0 over x = i+1, compress."""
    taken = []
    for ps in partials:
        if len(taken) >= t:
            break
        try:
            i = tbls_index_of(ps)
            tbls_verify_partial(commits, msg, ps)
            taken.append((i, g2_decompress(bytes(ps[2:]))))
        except VerifyError:
            continue
    shares = {}
    for i, pt in taken:
        if 0 <= i < n:
            shares[i] = pt
    if len(shares) < t:
        raise VerifyError("share: not enough good public shares to reconstruct secret commitment")
    xs = {i: (i + 1) % R for i in shares}
    acc = None
    for i, pt in shares.items():
        num, den = 1, 1
        for j in shares:
            if j == i:
                continue
            num = num * xs[j] % R
            den = den * (xs[j] - xs[i]) % R
        lam = num * pow(den, R - 2, R) % R
        acc = g2_add(acc, g2_mul(pt, lam))
    return g2_compress(acc)
