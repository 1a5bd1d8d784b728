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
