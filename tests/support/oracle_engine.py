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
