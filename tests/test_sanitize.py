"""Host-side code under the sanitizers (CPU only; tools/Makefile sanitizer targets).

* the service's request coalescer (drand_amd/csrc/coalesce.h) under ASan+UBSan and under TSan:
  many submitting threads, the dispatcher thread, shutdown while requests are queued;
* the drand.db bulk loader (drand_amd/csrc/boltload.cpp) under ASan+UBSan on bbolt files from
  tests/support/boltwriter.py and 200 truncated / bit-flipped mutants of each (must fail cleanly,
  never fault);
* the engine's device algorithms compiled for the host (tools/opcount.cpp, -DBLS_HOST) under
  ASan+UBSan: field fuzzers and one golden beacon verified end to end.

The GPU-side library cannot run here; its host logic beyond these parts (blsverify.cpp, service.cpp)
is exercised by the GPU suite. DESIGN.md records the one-off run of the whole CPU suite with the
ASan runtime preloaded and the ASan build of libboltload.so.
"""
from __future__ import annotations

import json
import sys
import os
import struct
import subprocess

import pytest

from drand_amd import ingest
from drand_amd.callers import Beacon
from tests.support.boltwriter import write_db

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOLS = os.path.join(ROOT, "tools")
SAN_ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", TSAN_OPTIONS="halt_on_error=1")


def _build(target):
    r = subprocess.run(["make", "-C", TOOLS, target], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return os.path.join(TOOLS, target)


def _run(args, timeout=300):
    r = subprocess.run(args, capture_output=True, text=True, env=SAN_ENV, timeout=timeout)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "runtime error" not in r.stderr and "Sanitizer" not in r.stderr, r.stderr[-4000:]
    return r.stdout


@pytest.mark.parametrize("target", ["hosttest-asan", "hosttest-tsan"])
def test_coalescer_sanitized(target):
    out = json.loads(_run([_build(target), "coalesce"]).strip().splitlines()[-1])
    assert out["coalesce"]["items"] > 0


def test_boltload_fuzz_asan(tmp_path, golden):
    ch = golden["chained"]
    bs = [Beacon(bytes.fromhex(b["prev"]), b["round"], bytes.fromhex(b["sig"]), bytes.fromhex(b["sig_v2"]))
          for b in ch["beacons"]]
    items = [(struct.pack(">Q", b.round), ingest.beacon_to_json(b)) for b in bs]
    files = []
    for k, layout in enumerate([dict(per_leaf=5), dict(inline=True), dict(page_size=1024, per_leaf=1)]):
        p = tmp_path / f"f{k}.db"
        write_db(p, items, **layout)
        files.append(str(p))
    out = json.loads(_run([_build("hosttest-asan"), "boltload", *files]).strip().splitlines()[-1])
    assert out["boltload"] == {"files": 3, "mutants": 600}


def test_device_algorithms_on_host_asan(golden):
    exe = _build("opcount-asan")
    assert json.loads(_run([exe, "powfuzz", "200"]))["fp4_sqr_mismatch"] == 0
    assert json.loads(_run([exe, "addfuzz", "100"]))["add_mismatch"] == 0
    out = json.loads(_run([exe, "invfuzz", "500"]))
    assert out["bad"] == 0 and out["unconverged"] == 0
    ch = golden["chained"]
    b = ch["beacons"][1]
    assert json.loads(_run([exe, ch["pk"], str(b["round"]), b["prev"], b["sig"]]))["verified"]
    assert json.loads(_run([exe, ch["pk"], str(b["round"]), "-", b["sig_v2"]]))["verified"]


def test_latency_engine_on_host_asan():
    """tests/test_wv_host.py (the latency engine's lane code compiled for the host, against Python
    integers and the golden fixtures) on the ASan+UBSan build of tools/wvtest."""
    _build("wvtest-asan")
    env = dict(SAN_ENV, WVTEST_TARGET="wvtest-asan")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider", os.path.join(ROOT, "tests",
                        "test_wv_host.py")], capture_output=True, text=True, env=env, cwd=ROOT, timeout=900)
    assert r.returncode == 0, r.stdout[-4000:]
