"""CPU test double of drand_amd.engine.Engine answered by the C oracle: TEST INFRASTRUCTURE ONLY."""
from __future__ import annotations

import hashlib

from drand_amd.engine import BatchResult


class OracleEngine:
    """CPU test double with the Engine's verify surface, answered by the C oracle (tests only)."""

    def __init__(self):
        from oracle import c_oracle
        self.o = c_oracle
        self.pk = None
        self.calls = []

    def set_public_key(self, pk48):
        self.pk = bytes(pk48)

    def _res(self, cls, base):
        ok = [c == 0 for c in cls]
        bad = next((i for i, v in enumerate(ok) if not v), None)
        return BatchResult(ok, None if bad is None else base + bad, list(cls))

    def verify_chained(self, first_round, prev0, sigs):
        assert len(prev0) in (32, 96) and all(len(s) == 96 for s in sigs)
        self.calls.append(("chained", first_round, len(sigs)))
        return self._res(self.o.verify_chained(self.pk, first_round, bytes(prev0), b"".join(sigs)), first_round)

    def verify_chained_packed(self, first_round, prev0, sigs96, n):
        b = bytes(memoryview(sigs96).cast("B"))
        return self.verify_chained(first_round, prev0, [b[96 * i:96 * (i + 1)] for i in range(n)])

    def verify_prevs(self, first_round, prev0_len, prevs96, sigs96, n):
        p, q = bytes(memoryview(prevs96).cast("B")), bytes(memoryview(sigs96).cast("B"))
        self.calls.append(("prevs", first_round, n))
        cls = []
        for i in range(n):
            prev = p[96 * i:96 * i + (prev0_len if i == 0 else 96)]
            msg = hashlib.sha256(prev + (first_round + i).to_bytes(8, "big")).digest()
            cls.append(self.o.verify(self.pk, msg, q[96 * i:96 * (i + 1)]))
        return self._res(cls, first_round)

    def verify_unchained(self, sigs, first_round=None, rounds=None):
        rounds = rounds if rounds is not None else [first_round + i for i in range(len(sigs))]
        self.calls.append(("unchained", rounds[0], len(sigs)))
        cls = [self.o.verify(self.pk, hashlib.sha256(r.to_bytes(8, "big")).digest(), s) for r, s in zip(rounds, sigs)]
        return self._res(cls, 0)

    def verify_messages(self, msgs, sigs, pk48=None):
        self.calls.append(("messages", 0, len(sigs)))
        return self._res([self.o.verify(pk48 or self.pk, m, s) for m, s in zip(msgs, sigs)], 0)

    # ---- threshold surface (test double of blsv_set_group / blsv_aggregate_round)
    def set_group(self, commits, n=None):
        self.commits = [bytes(c) for c in commits]
        self.n = n if n is not None else len(self.commits)
        self.pk = self.commits[0]
        self.calls.append(("set_group", len(self.commits), self.n))

    def _partial_ok(self, msg, p):
        from oracle import bls12381 as O
        if len(p) != 98:
            return False
        pts = [O.g1_decompress(c) for c in self.commits]
        pk = O.g1_compress(O.pubpoly_eval(pts, int.from_bytes(p[:2], "big")))
        return self.o.verify(pk, msg, bytes(p[2:])) == 0

    def _recover(self, parts, oks, t, n):
        """kyber rule (blsv_recover): first t valid in order, duplicates count, keyed by index < n."""
        from oracle import bls12381 as O
        taken = [(int.from_bytes(p[:2], "big"), p) for p, ok in zip(parts, oks) if ok][:t]
        shares = {i: O.g2_decompress(bytes(p[2:])) for i, p in taken if i < n}
        if len(shares) < t:
            return None
        acc = None
        for i, pt in shares.items():
            num, den = 1, 1
            for j in shares:
                if j != i:
                    num = num * (j + 1) % O.R
                    den = den * (j - i) % O.R
            acc = O.g2_add(acc, O.g2_mul(pt, num * pow(den, O.R - 2, O.R) % O.R))
        return O.g2_compress(acc)

    def aggregate_round(self, msg1, partials1, msg2, partials2, t, n):
        from drand_amd import callers as C
        self.calls.append(("aggregate_round", len(partials1), len(partials2)))
        ok1 = [self._partial_ok(msg1, p) for p in partials1]
        ok2 = [self._partial_ok(msg2, p) for p in partials2]
        sig1 = self._recover(partials1, ok1, t, n)
        if sig1 is None:
            return C.AGG_V1_RECOVER_FAIL, ok1, ok2, None, None, False
        if self.o.verify(self.commits[0], msg1, sig1) != 0:
            return C.AGG_V1_INVALID, ok1, ok2, sig1, None, False
        if len(partials2) < t:
            return C.AGG_OK, ok1, ok2, sig1, None, False
        sig2 = self._recover(partials2, ok2, t, n)
        if sig2 is None:
            return C.AGG_V2_RECOVER_FAIL, ok1, ok2, sig1, None, False
        return C.AGG_OK_V2, ok1, ok2, sig1, sig2, self.o.verify(self.commits[0], msg2, sig2) == 0
