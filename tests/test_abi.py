"""CPU tests of the drop-in boundary: the C-ABI library loads and exports every symbol declared in
include/*.h, the Python binding declares exactly those symbols, and the host build of the engine's
own device algorithms (tools/opcount, -DBLS_HOST) verifies golden beacons and reproduces the frozen
op counts in profiles/opcount.json. No GPU calls."""
import ctypes
import json
import os
import re
import subprocess

import pytest

from drand_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    syms = set()
    for h in ("blsverify.h", "blsverify_testing.h"):
        txt = open(os.path.join(ROOT, "include", h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        syms |= set(re.findall(r"\b(blsv_\w+)\s*\(", txt))
    return syms


def test_binding_matches_headers():
    assert header_symbols() == set(_lib.SIGNATURES), header_symbols() ^ set(_lib.SIGNATURES)


def test_library_exports_every_symbol():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libblsverify.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for s in header_symbols():
        assert hasattr(lib, s), s
    lib.blsv_version.restype = ctypes.c_char_p
    assert b"gfx950" in lib.blsv_version()


def test_host_lagrange_matches_integers():
    """blsv_test_lagrange (the host Lagrange basis blsv_recover / blsv_aggregate* interpolate with,
    blsverify.cpp host_lagrange) against Python integers: lambda_i = prod x_j / (x_j - x_i) mod r,
    x = index + 1, for the golden round's first 33 shares, a scattered set and t = 1; repeated indices
    are refused. No GPU: the function is host arithmetic."""
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libblsverify.so not built (run __graft_entry__.build())")
    lib = _lib.load()
    R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
    for idx in (list(range(33)), [65535, 0, 7, 40000, 12, 3, 999], [5]):
        t = len(idx)
        arr = (ctypes.c_uint32 * t)(*idx)
        out = (ctypes.c_uint32 * (8 * t))()
        assert lib.blsv_test_lagrange(arr, t, out) == 0
        for i in range(t):
            num = den = 1
            for j in range(t):
                if j != i:
                    num = num * (idx[j] + 1) % R
                    den = den * (idx[j] - idx[i]) % R
            want = num * pow(den, R - 2, R) % R
            got = sum(out[8 * i + w] << (32 * w) for w in range(8))
            assert got == want, (idx, i)
    arr = (ctypes.c_uint32 * 2)(4, 4)
    assert lib.blsv_test_lagrange(arr, 2, (ctypes.c_uint32 * 16)()) == -1


def test_boltload_exports_every_symbol():
    """include/boltload.h (drand.db bulk loader) against libboltload.so."""
    from drand_amd import boltdb
    if not os.path.exists(boltdb.LIB_PATH):
        pytest.skip("libboltload.so not built (run __graft_entry__.build())")
    txt = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "boltload.h")).read(), flags=re.S)
    syms = set(re.findall(r"\b(dl_\w+)\s*\(", txt))
    assert syms == {"dl_open", "dl_count", "dl_load", "dl_last_error", "dl_close"}
    lib = ctypes.CDLL(boltdb.LIB_PATH)
    for s in syms:
        assert hasattr(lib, s), s


def test_engine_refuses_without_library(monkeypatch, tmp_path):
    """No CPU fallback: a missing library is a loud error."""
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(_lib.EngineUnavailable):
        _lib.load()


@pytest.fixture(scope="module")
def opcount_bin():
    subprocess.run(["make", "-C", os.path.join(ROOT, "tools"), "opcount"], check=True, capture_output=True)
    return os.path.join(ROOT, "tools", "opcount")


def run_opcount(binp, pk, rnd, prev, sig):
    r = subprocess.run([binp, pk, str(rnd), prev, sig], capture_output=True, text=True)
    return r.returncode, json.loads(r.stdout)


def test_host_build_verifies_golden(opcount_bin, golden):
    ch = golden["chained"]
    for b in ch["beacons"]:
        rc, out = run_opcount(opcount_bin, ch["pk"], b["round"], b["prev"], b["sig"])
        assert rc == 0 and out["verified"], out
        rc2, out2 = run_opcount(opcount_bin, ch["pk"], b["round"], "-", b["sig_v2"])
        assert rc2 == 0 and out2["verified"], out2
    frozen = json.load(open(os.path.join(ROOT, "profiles", "opcount.json")))
    assert out["fp_mul"] == frozen["fp_mul"], "profiles/opcount.json is stale: regenerate it"
    b = ch["beacons"][2]  # wrong round -> pairing reject
    rc, out = run_opcount(opcount_bin, ch["pk"], b["round"] + 1, b["prev"], b["sig"])
    assert rc == 1 and not out["verified"]


def test_host_build_hash_to_g2_golden(opcount_bin, golden):
    for v in golden["hash_to_g2"]:
        r = subprocess.run([opcount_bin, "hash", v["msg"]], capture_output=True, text=True, check=True)
        got = json.loads(r.stdout)
        assert [int(x, 16) for x in got["x"]] == [int(x, 16) for x in v["x"]]
        assert [int(x, 16) for x in got["y"]] == [int(x, 16) for x in v["y"]]


def test_host_build_decode_classes(opcount_bin, golden):
    mx = golden["mixed"]
    for i, c in enumerate(mx["expect_class"]):
        if c in (2, 3, 4, 5, 6):
            prev = mx["genesis_seed"] if i == 0 else mx["sigs"][i - 1]
            rc, out = run_opcount(opcount_bin, mx["pk"], i + 1, prev, mx["sigs"][i])
            assert out.get("class") == c, (i, out)


def test_host_build_inversion_matches_exponentiation(opcount_bin):
    """fp_inv (Pornin binary GCD, fp.h) == a^(p-2) on 20,000 seeded inputs in [0, 2p), the edge
    values 0, 1, p, p-1, 2p-1, p+1, and ~2,100 structured inputs (2^k, 2^k - 1, p - 2^k, (p +- 1)/2^k,
    p +- d, 2p - d) -- the same device source compiled for the host. The GCD is checked WITHOUT the
    exponentiation fallback of fp_inv_bingcd: every input must also converge (b == 1)."""
    r = subprocess.run([opcount_bin, "invfuzz", "20000"], capture_output=True, text=True)
    out = json.loads(r.stdout)
    assert r.returncode == 0 and out["bad"] == 0 and out["unconverged"] == 0 and out["structured"] > 2000, out



def test_host_sqrt_window_and_fp2_sqr_fuzz(opcount_bin):
    """The 4-bit sliding-window square-root exponentiation (radix-2^28 running value) equals the fixed
    2-bit-window one, and the Fp2 square with radix-2^28 sums equals (a0 + a1)(a0 - a1), 2 a0 a1 from
    Fp products, for reduced operands and lazy sums (< 4p), on the host build of fp.h."""
    r = subprocess.run([opcount_bin, "powfuzz", "3000"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    out = json.loads(r.stdout)
    assert out["pow_mismatch"] == 0 and out["fp2_sqr_mismatch"] == 0, out


def test_host_cofactor_addition_flags_exceptions(opcount_bin):
    """The cofactor chains' branch-free addition (curve.h g2_add_inl_exc) and the subgroup check's mixed
    addition (g2_madd_inl_exc) equal jac_add on distinct
    points given in different Jacobian representations, and raises its exceptional flag for P + P,
    P + (-P) and a point at infinity on either side (k_hash.hip then recomputes such lanes with the
    generic formulas) -- the device source compiled for the host."""
    r = subprocess.run([opcount_bin, "addfuzz", "2000"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert json.loads(r.stdout)["add_mismatch"] == 0


def test_fused_cyclotomic_combination_host(opcount_bin):
    """tower.h fp2_3u_pm_2x, the 3-lane cyclotomic square's 3u +- 2x with one reduction by an estimated
    multiple of p, equals fp2_addsub + fp2_dbl + fp2_add mod p and stays in [0, 2p) on random
    operands, the range edges and operands aimed at every boundary of its quotient correction."""
    r = subprocess.run([opcount_bin, "linfuzz", "3000"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    out = json.loads(r.stdout)
    assert out["lin_mismatch"] == 0 and out["boundary_cases"] > 10000


def test_one_reduction_fp6_product_host(opcount_bin):
    """tower.h fp6_mul_lin / fp12_sqr_lin (the Karatsuba Fp6 outputs as linear forms reduced once, the
    Miller f pass's products) equal fp6_mul / fp12_sqr mod p and stay in [0, 2p): random operands,
    operands at 2p - 1 and the lazily added (< 4p) operands of the squaring's second product."""
    r = subprocess.run([opcount_bin, "f6fuzz", "2000"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert json.loads(r.stdout)["f6_mismatch"] == 0


def _split_top(args):
    out, depth, cur = [], 0, ""
    for ch in args:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def header_prototypes():
    """name -> list of parameter types of every blsv_* function in include/*.h"""
    protos = {}
    for h in ("blsverify.h", "blsverify_testing.h"):
        txt = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", h)).read(), flags=re.S)
        for m in re.finditer(r"\b(blsv_\w+)\s*\(([^;{]*?)\)\s*;", txt):
            params = _split_top(m.group(2))
            protos[m.group(1)] = [] if params == ["void"] else [re.sub(r"\s*\b\w+$", "", p) if "*" not in p.split()[-1]
                                                                else p for p in params]
    return protos


def _arg_kind(expr):
    m = re.match(r"C\.(size_t|uint64_t|int32_t|uint32_t|int|uint8_t)\(", expr)
    if m:
        return m.group(1)
    if re.match(r"(ptr\(|&|e\.ctx$|ctx$|nil$|unsafe\.Pointer\(|\(\*C\.)", expr):
        return "ptr"
    return None


def _param_kind(ptype):
    if "*" in ptype:
        return "ptr"
    for k in ("size_t", "uint64_t", "int32_t", "uint32_t", "uint8_t", "int"):
        if re.search(r"\b%s\b" % k, ptype):
            return k
    return None


def test_integration_cgo_calls_match_header():
    """Compile-shape check of the Go adapter in INTEGRATION.md against include/*.h: every C.blsv_*
    call names a declared function with the declared number of arguments, each scalar argument is
    converted to the declared C type (C.size_t(...) for size_t, ...) and each pointer parameter gets
    a pointer expression; every C.BLSV_* constant is defined by the header."""
    protos = header_prototypes()
    md = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    go = "\n".join(re.findall(r"```go\n(.*?)```", md, flags=re.S))
    calls = 0
    for m in re.finditer(r"\bC\.(blsv_\w+)\(", go):
        name = m.group(1)
        assert name in protos, "INTEGRATION.md calls undeclared %s" % name
        depth, i = 1, m.end()
        while depth:
            depth += {"(": 1, ")": -1}.get(go[i], 0)
            i += 1
        args = _split_top(go[m.end():i - 1])
        params = protos[name]
        assert len(args) == len(params), "%s: %d args, header declares %d" % (name, len(args), len(params))
        for a, p in zip(args, params):
            ak, pk = _arg_kind(a), _param_kind(p)
            if ak is not None and pk is not None:
                assert ak == pk, "%s: argument %r for parameter %r" % (name, a, p)
        calls += 1
    assert calls >= 10
    hdr = open(os.path.join(ROOT, "include", "blsverify.h")).read()
    for c in set(re.findall(r"\bC\.(BLSV_\w*[A-Z0-9])\b", go)):
        assert re.search(r"\b%s\b\s*=|#define\s+%s\b" % (c, c), hdr), c
