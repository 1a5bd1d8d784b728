"""Generate tests/golden/chain2049.bin: one CONTINUOUS 2,049-round chained history (raw 96-byte
compressed signatures, rounds 1..2049) for the latency-path parity tests at the sizes that path
serves (tests/test_gpu_lat_scale.py: 1,000 = configs[0], 1,536 = the default cutover, 1,537 = one
past it, 2,048 = above it; the tests force each route through set_lat_max, so the cutover a fixture
was made at does not matter). A continuous chain is sequential to sign (sig_i signs Message(i, sig_{i-1})), which is why
it is committed instead of generated on the test box.

Recipe: client/test/result/mock/result.go:98-132 with the golden chained key and genesis seed
(tests/golden/golden.json "chained": sk, pk, genesis_seed): round 1 signs sha256(seed || BE64(1))
(chain/beacon.go:103-108, the 32-byte genesis seed as PreviousSig), round i signs
sha256(sig_{i-1} || BE64(i)). Signed by the C oracle (oracle/c/bls_oracle.c, pinned to the
reference KAT key/curve_test.go:10-30 in tests/test_oracle_c.py); the script re-verifies samples.

Usage: python tests/golden/make_chain_fixture.py   (~20 s)
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import c_oracle  # noqa: E402

N = 2049
OUT = os.path.join(HERE, "chain2049.bin")


def main():
    c_oracle.load()
    with open(os.path.join(HERE, "golden.json")) as f:
        ch = json.load(f)["chained"]
    sk, pk, seed = int(ch["sk"], 16), bytes.fromhex(ch["pk"]), bytes.fromhex(ch["genesis_seed"])
    sigs, prev = [], seed
    for r in range(1, N + 1):
        s = c_oracle.sign(sk, hashlib.sha256(prev + r.to_bytes(8, "big")).digest())
        sigs.append(s)
        prev = s
    # the golden fixture's first rounds are the same chain
    assert [s.hex() for s in sigs[:len(ch["beacons"])]] == [b["sig"] for b in ch["beacons"]]
    assert c_oracle.verify_chained(pk, 1, seed, b"".join(sigs[:4])) == [0] * 4
    for lo in (1000, 2040):
        assert c_oracle.verify_chained(pk, lo + 1, sigs[lo - 1], b"".join(sigs[lo:lo + 9])) == [0] * 9
    with open(OUT, "wb") as f:
        f.write(b"".join(sigs))
    print("wrote", OUT, N, "signatures")


if __name__ == "__main__":
    main()
