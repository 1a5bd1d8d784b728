"""Generate wv_constants.h: constants of the wave-cooperative latency engine (wfield.h).

Representation: an Fp value is 16 limbs of 25 bits held one per lane in the even DPP row of a
half-wave (lanes 32h + 0..15), Montgomery form with R = 2^400. A constant is stored as 64 words in
that lane layout ("value form": odd rows zero), so a lane loads its own word of it:
  FP2 constants  half 0 = c0, half 1 = c1          (an Fp2 value)
  DUP constants  both halves = the same Fp value    (an Fp scalar multiplying an Fp2, or a pair)
Everything is computed from first principles with Python integers (gen_constants.py supplies the
curve constants). Run:  python drand_amd/csrc/gen_wv_constants.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_constants as G  # noqa: E402

P = G.P
W = 25
NL = 16
MASK = (1 << W) - 1
R = 1 << (W * NL)  # 2^400


def mont(v):
    return (v % P) * R % P


def limbs25(v):
    assert 0 <= v < R
    return [(v >> (W * k)) & MASK for k in range(NL)]


def lanes_fp2(c0, c1):
    a, b = limbs25(c0), limbs25(c1)
    return a + [0] * 16 + b + [0] * 16


def lanes_dup(c):
    return lanes_fp2(c, c)


def dominating(m, lower_min):
    """m*p as 16 redundant digits with digits 0..14 >= lower_min (borrowing c = 2 from each next
    digit): lets x + D - y be formed limb-wise with no borrows for any y whose limbs are < lower_min
    and whose value is < the top-digit bound this returns."""
    v = m * P
    d = limbs25(v)
    c = 2
    D = [d[0] + c * (1 << W)] + [d[k] + c * (1 << W) - c for k in range(1, 15)] + [d[15] - c]
    assert sum(x << (W * k) for k, x in enumerate(D)) == v
    assert all(x >= lower_min for x in D[:15]) and D[15] > 0
    # a subtrahend y < B p with non-negative digits has y_15 <= B p / 2^375: largest B covered
    b_max = (D[15] << 375) // P
    return D, b_max


def main():
    names, rows = [], []

    def add(name, lanes):
        assert len(lanes) == 64
        names.append(name)
        rows.append(lanes)

    def add_fp2(name, c, montgomery=True):
        f = mont if montgomery else (lambda v: v % P)
        add(name, lanes_fp2(f(c[0]), f(c[1])))

    def add_dup(name, c, montgomery=True):
        add(name, lanes_dup(mont(c) if montgomery else c))  # RAW values are taken as they are (P_DUP = p)

    m2, inv2, pow2 = G.m2, G.inv2, G.pow2
    add_fp2("ONE2", (1, 0))
    for c in (1, 2, 3, 4, 6, 8):  # small Montgomery multipliers folded into dot products as one more term
        add_fp2(f"NEG{c}", ((-c) % P, 0))
        add_fp2(f"POS{c}", (c, 0))
    add_dup("ONE_DUP", 1)
    add_dup("RAW_ONE_DUP", 1, montgomery=False)
    add_dup("R2_DUP", R * R % P, montgomery=False)
    add_dup("H256_R2_DUP", (1 << 256) * R * R % P, montgomery=False)
    add_dup("C408_DUP", pow(2, 408, P), montgomery=False)  # 392-form (batch engine) -> 400-form
    add_dup("C392_DUP", pow(2, 392, P), montgomery=False)  # 400-form -> 392-form
    add_dup("C416_DUP", pow(2, 416, P), montgomery=False)  # fp.h inverse of a 400-form value -> 400-form
    add_dup("P_DUP", P, montgomery=False)
    add_dup("PM1H_DUP", (P - 1) // 2, montgomery=False)
    add_dup("PP1H_DUP", (P + 1) // 2, montgomery=False)  # x > (p-1)/2  <=>  x >= (p+1)/2
    add_fp2("B2", (4, 4))
    add_fp2("B2X3", (12, 12))  # 3 b' (Miller doubling line)
    A, B, Z = (0, 240), (1012, 1012), ((-2) % P, (-1) % P)
    add_fp2("SSWU_A", A)
    add_fp2("SSWU_B", B)
    add_fp2("SSWU_Z", Z)
    add_fp2("SSWU_NBA", m2(((-B[0]) % P, (-B[1]) % P), inv2(A)))
    add_fp2("SSWU_BZA", m2(B, inv2(m2(Z, A))))
    nz = (Z[0] * Z[0] + Z[1] * Z[1]) % P
    c = (-nz * nz * nz) % P
    cr = pow(c, (P + 1) // 4, P)
    assert cr * cr % P == c
    add_dup("SSWU_SQRT_MNZ3", cr)
    iso = G.ISO if hasattr(G, "ISO") else None
    h = lambda v: v % P  # noqa: E731
    iso = {
        "ISO_XNUM": [(h(0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97D6),
                      h(0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97D6)),
                     (0, h(0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71A)),
                     (h(0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71E),
                      h(0x8AB05F8BDD54CDE190937E76BC3E447CC27C3D6FBD7063FCD104635A790520C0A395554E5C6AAAA9354FFFFFFFFE38D)),
                     (h(0x171D6541FA38CCFAED6DEA691F5FB614CB14B4E7F4E810AA22D6108F142B85757098E38D0F671C7188E2AAAAAAAA5ED1), 0)],
        "ISO_XDEN": [(0, (-72) % P), (12, (-12) % P)],
        "ISO_YNUM": [(h(0x1530477C7AB4113B59A4C18B076D11930F7DA5D4A07F649BF54439D87D27E500FC8C25EBF8C92F6812CFC71C71C6D706),
                      h(0x1530477C7AB4113B59A4C18B076D11930F7DA5D4A07F649BF54439D87D27E500FC8C25EBF8C92F6812CFC71C71C6D706)),
                     (0, h(0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97BE)),
                     (h(0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71C),
                      h(0x8AB05F8BDD54CDE190937E76BC3E447CC27C3D6FBD7063FCD104635A790520C0A395554E5C6AAAA9354FFFFFFFFE38F)),
                     (h(0x124C9AD43B6CF79BFBF7043DE3811AD0761B0F37A1E26286B0E977C69AA274524E79097A56DC4BD9E1B371C71C718B10), 0)],
        "ISO_YDEN": [((-432) % P, (-432) % P), (0, (-216) % P), (18, (-18) % P)],
    }
    for name, coeffs in iso.items():
        for i, cc in enumerate(coeffs):
            add_fp2(f"{name}{i}", cc)
    xi = G.XI
    kx = inv2(pow2(xi, (P - 1) // 3))
    ky = inv2(pow2(xi, (P - 1) // 2))
    add_fp2("PSI_KX", kx)
    add_fp2("PSI_KY", ky)
    kx2 = m2((kx[0], (-kx[1]) % P), kx)
    ky2 = m2((ky[0], (-ky[1]) % P), ky)
    assert kx2[1] == 0 and ky2[1] == 0
    add_dup("PSI2_KX", kx2[0])
    add_dup("PSI2_KY", ky2[0])
    g1 = pow2(xi, (P - 1) // 6)
    g2 = pow2(xi, (P * P - 1) // 6)
    f1, f2 = [(1, 0)], [(1, 0)]
    for _ in range(5):
        f1.append(m2(f1[-1], g1))
        f2.append(m2(f2[-1], g2))
    for k in range(6):
        add_fp2(f"FROB1_{k}", f1[k])
        assert f2[k][1] == 0
        add_dup(f"FROB2_{k}", f2[k][0])
    add_dup("NEG_G1_X", G.G1_X)
    add_dup("NEG_G1_Y", (-G.G1_Y) % P)
    # subtraction / negation constants (RAW digits, not reduced): x + D - y limb-wise
    levels = (4, 32, 128)
    dl = []
    for m in levels:
        D, bmax = dominating(m, (1 << 26) - 2)
        dl.append(bmax)
        add(f"DSUB{len(dl) - 1}", D + [0] * 16 + D + [0] * 16)
    DM, bmul = dominating(129, (1 << 26) - 2)
    add("DMUL", DM + [0] * 16 + DM + [0] * 16)
    # per-lane p table of the m * p product: PC_i[lane] = p_{k - i} for k = lane % 32 in [i, i + 15]
    pl = limbs25(P)
    for i in range(16):
        add(f"PC{i}", [pl[(l % 32) - i] if i <= (l % 32) <= i + 15 else 0 for l in range(64)])
    add_dup("C1200_DUP", pow(2, 1200, P), montgomery=False)  # wave GCD's y^-1 (y = a 2^400) -> 400-form
    np25 = limbs25((-pow(P, -1, R)) % R)
    p_over_r = P / R

    out = []
    w = out.append
    w("// GENERATED by drand_amd/csrc/gen_wv_constants.py -- do not edit.")
    w("// Latency-engine constants (wfield.h): 16 x 25-bit limbs, one per lane, Montgomery R = 2^400,")
    w("// each constant 64 words in the value-form lane layout (see the generator's docstring).")
    w("#pragma once")
    w("#include <stdint.h>")
    w("namespace wv {")
    w("enum WC : int {")
    for i, n in enumerate(names):
        w(f"  WC_{n} = {i},")
    w(f"  WC_COUNT = {len(names)}")
    w("};")
    w("#ifdef WV_HOST")
    w("static const uint32_t WV_CONST_TABLE[WC_COUNT * 64] = {")
    w("#else")
    w("__device__ const uint32_t WV_CONST_TABLE[WC_COUNT * 64] = {")
    w("#endif")
    for n, r in zip(names, rows):
        w(f"  // {n}")
        w("  " + ", ".join(hex(x) + "u" for x in r) + ",")
    w("};")
    w("static constexpr uint32_t NP25[16] = {" + ", ".join(hex(x) + "u" for x in np25) + "};  // -p^-1 mod 2^400")
    w("static constexpr uint32_t P25[16] = {" + ", ".join(hex(x) + "u" for x in pl) + "};")
    w("// value bounds (units of p) the host build checks: a subtrahend of sub<L> must stay below")
    w("// DSUB_BMAX[L]; an Fp2 product operand below DMUL_BMAX; P_OVER_R = p / 2^400")
    w("static constexpr double DSUB_M[3] = {" + ", ".join(str(float(m)) for m in levels) + "};")
    w("static constexpr double DSUB_BMAX[3] = {" + ", ".join(str(float(b)) for b in dl) + "};")
    w(f"static constexpr double DMUL_M = 129.0;")
    w(f"static constexpr double DMUL_BMAX = {float(bmul)};")
    w(f"static constexpr double P_OVER_R = {p_over_r!r};")
    w("}  // namespace wv")
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "wv_constants.h")
    with open(path, "w") as f:
        f.write("\n".join(out) + "\n")
    print("wrote", path, len(names), "constants; DSUB_BMAX", dl, "DMUL_BMAX", bmul)


if __name__ == "__main__":
    main()
