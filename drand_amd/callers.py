"""Batched rewrites of drand's two serial verification loops.

The reference walks a chain one round at a time, with one full BLS verify per round:

* ``verifyingClient.getTrustedPreviousSignature`` (client/verify.go:115-174) fetches rounds
  ``trust+1 .. round-1`` and calls ``chain.VerifyBeacon`` on each (verify.go:146-163).
* ``verifyingClient.verify`` (client/verify.go:176-208) then checks the requested round, V1 or V2
  depending on ``v2from``, and sets ``Random = sha256(sig)`` (chain/beacon.go:66-75).
* ``syncer.tryNode`` (chain/beacon/sync.go:83-131) streams ``BeaconPacket``s, verifies each
  (sync.go:105) and appends it through ``appendStore.Put`` (chain/beacon/store.go:40-54), which
  checks ``Round == last.Round+1`` and ``PreviousSig == last.Signature``.

Here both loops keep their observable behaviour (same accepted prefix, same first failing round,
same point-of-trust update, same error kinds) but hand whole ranges to the GPU engine in one
``Engine.verify_chained`` call per chunk. Fetching and storing stay with the caller (network and
storage are out of scope); the callables passed in stand for ``indirectClient.Get`` and
``chain.Store.Put``.

Every verdict comes from the HIP kernels through the C ABI; there is no CPU verify here.
"""
from __future__ import annotations

import hashlib
import threading
from dataclasses import dataclass
from typing import Callable, Iterable, Optional

UINT64_MAX = 2 ** 64 - 1
SIG_LEN = 96


class VerifyError(Exception):
    """A beacon failed verification (kyber's "bls: invalid signature" or a decode error)."""

    def __init__(self, round_, msg):
        super().__init__(msg)
        self.round = round_


class FetchError(Exception):
    """``indirectClient.Get`` failed for a round (client/verify.go:149-152)."""

    def __init__(self, round_, cause):
        super().__init__(f"could not get round {round_}: {cause}")
        self.round = round_
        self.__cause__ = cause


@dataclass
class ChainInfo:
    """The two fields of ``chain.Info`` the walk uses (chain/info.go): G1 public key (48 B
    compressed) and ``GroupHash``, which is the previous signature of round 1
    (client/verify.go:122-124)."""
    public_key: bytes
    group_hash: bytes


@dataclass
class RandomData:
    """``client.RandomData`` (client/random.go:5-12). ``version`` is 2 once ``round >= v2from``."""
    round: int
    signature: bytes = b""
    previous_signature: Optional[bytes] = None
    signature_v2: bytes = b""
    randomness: bytes = b""
    version: int = 1

    def sig(self):
        return self.signature_v2 if self.version == 2 else self.signature


@dataclass
class Beacon:
    """``chain.Beacon`` (chain/beacon.go:16-25)."""
    previous_sig: bytes
    round: int
    signature: bytes
    signature_v2: bytes = b""


def randomness_from_signature(sig: bytes) -> bytes:
    """``chain.RandomnessFromSignature`` (chain/beacon.go:66-69): sha256 of the signature bytes.
    Host-side, like the reference: it runs only after the GPU verdict accepted the beacon."""
    return hashlib.sha256(sig).digest()


def _verify_run(engine, first_round, prev0, sigs):
    """Verify ``sigs`` as consecutive rounds starting at ``first_round`` whose first previous
    signature is ``prev0``. Returns the index of the first rejected beacon, or None.

    A wrong-length signature is a reject in the reference (kyber's unmarshal fails); the engine
    refuses such input host-side, so the run is cut there and that index is reported."""
    n = len(sigs)
    cut = next((i for i, s in enumerate(sigs) if len(s) != SIG_LEN), n)
    if cut and len(prev0) not in (32, 96):
        # Only the first round's prev may be another length; the C ABI takes 32 or 96 bytes.
        # A kyber verify of such a message is still well defined, so route it through the
        # message-form entry point.
        first = engine.verify_messages([hashlib.sha256(bytes(prev0) + first_round.to_bytes(8, "big")).digest()],
                                       [sigs[0]])
        if not first.ok[0]:
            return 0
        rest = _verify_run(engine, first_round + 1, sigs[0], sigs[1:cut])
        return None if rest is None else rest + 1
    if cut:
        res = engine.verify_chained(first_round, bytes(prev0), [bytes(s) for s in sigs[:cut]])
        if res.first_bad is not None:
            return res.first_bad - first_round
    return None if cut == n else cut


class VerifyingClient:
    """Batched ``verifyingClient`` (client/verify.go:22-214) over one GPU engine.

    ``get(round) -> RandomData`` stands for ``indirectClient.Get``. ``chunk`` bounds how many rounds
    are fetched before one batched verify; the reference's order of errors is kept (a verify
    failure at round k is reported before a fetch failure at a later round).

    ``point_of_trust`` is ``WithVerifiedResult`` (client/client.go options; verify_test.go:19 seeds it
    with round 1). Reference quirk kept as is: without one, or for a round below it, the walk
    restarts at round 1 with ``GroupHash`` as the trusted signature (verify.go:131-137), so round 2
    is checked against ``Message(2, GroupHash)`` and rejects on a real chain."""

    def __init__(self, engine, info: ChainInfo, get: Callable[[int], RandomData], strict=False,
                 v2from=UINT64_MAX, chunk=1 << 16, point_of_trust: Optional[RandomData] = None):
        self.engine = engine
        self.info = info
        self.get = get
        self.strict = strict
        self.v2from = v2from
        self.chunk = int(chunk)
        self.point_of_trust: Optional[RandomData] = point_of_trust
        self._pot_lk = threading.Lock()
        engine.set_public_key(info.public_key)

    def get_trusted_previous_signature(self, round_: int) -> bytes:
        """client/verify.go:115-174."""
        if round_ == 1:
            return self.info.group_hash
        with self._pot_lk:
            pot = self.point_of_trust
        if pot is None or pot.round > round_:
            trust_round, trust_prev = 1, self.get_trusted_previous_signature(1)
        else:
            trust_round, trust_prev = pot.round, pot.sig()
        initial = trust_round
        last_result = None
        while trust_round < round_ - 1:
            lo = trust_round + 1
            hi = min(round_ - 1, trust_round + self.chunk)
            results, fetch_err = [], None
            for r in range(lo, hi + 1):
                try:
                    results.append(self.get(r))
                except Exception as e:  # noqa: BLE001 - the reference wraps any client error
                    fetch_err = FetchError(r, e)
                    break
            sigs = [res.sig() for res in results]
            bad = _verify_run(self.engine, lo, trust_prev, sigs)
            if bad is not None:
                raise VerifyError(lo + bad, f"verifying beacon: round {lo + bad}: bls: invalid signature")
            if fetch_err is not None:
                raise fetch_err
            trust_round = hi
            trust_prev = sigs[-1]
            last_result = results[-1]
        if trust_round == round_ - 1 and trust_round > initial:
            with self._pot_lk:
                self.point_of_trust = last_result
        if trust_round != round_ - 1:
            raise VerifyError(round_, f"unexpected trust round {trust_round}")
        return trust_prev

    def verify(self, r: RandomData) -> None:
        """client/verify.go:176-208: verify one result (V1 or V2) and set its randomness."""
        ps = r.previous_signature
        if r.round < self.v2from and (self.strict or r.previous_signature is None):
            ps = self.get_trusted_previous_signature(r.round)
        if r.round >= self.v2from:
            res = self.engine.verify_unchained([r.signature_v2], rounds=[r.round]) if len(r.signature_v2) == SIG_LEN \
                else None
            if res is None or not res.ok[0]:
                raise VerifyError(r.round, f"verification v2 of round {r.round} failed: bls: invalid signature")
            r.randomness = randomness_from_signature(r.signature_v2)
        else:
            bad = _verify_run(self.engine, r.round, ps, [r.signature])
            if bad is not None:
                raise VerifyError(r.round, f"verification v1 of round {r.round} failed: bls: invalid signature")
            r.randomness = randomness_from_signature(r.signature)


@dataclass
class SyncOutcome:
    """What ``syncer.tryNode`` (chain/beacon/sync.go:83-131) returns, plus why it stopped."""
    finished: bool            # the bool tryNode returns: last.Round == upTo was reached
    last: Beacon              # the store's last beacon afterwards
    stored: int               # beacons appended in this call
    reason: str = ""          # "", "invalid_beacon", "invalid round inserted", "invalid previous signature",
                              # "store", "stream ended"
    bad_round: Optional[int] = None


def sync_chain(engine, public_key: bytes, last: Beacon, packets: Iterable[Beacon], up_to: int,
               put: Callable[[Beacon], None], chunk=1 << 16) -> SyncOutcome:
    """Batched ``syncer.tryNode`` + ``appendStore.Put`` over one GPU engine.

    Per chunk of the stream: the longest prefix that links (``Round == last.Round+1`` and
    ``PreviousSig == last.Signature``, store.go:43-48) is one chained range, verified in one call.
    Beacons are stored in order up to the first failure, exactly where the serial loop would stop
    (verify before Put, sync.go:105-113). The first unlinked beacon is verified on its own so the
    stop reason matches the reference's (a bad signature is reported before a linkage error).
    Unlike the serial loop, up to ``chunk`` packets are read from the stream ahead of the verify."""
    engine.set_public_key(public_key)
    stored = 0
    it = iter(packets)
    while True:
        batch = []
        for b in it:
            batch.append(b)
            if len(batch) >= chunk or b.round == up_to:
                break
        if not batch:
            return SyncOutcome(False, last, stored, "stream ended")
        # linked prefix
        linked, prev_r, prev_s = 0, last.round, last.signature
        for b in batch:
            if b.round != prev_r + 1 or bytes(b.previous_sig) != bytes(prev_s):
                break
            linked += 1
            prev_r, prev_s = b.round, b.signature
        bad = None
        if linked:
            bad = _verify_run(engine, batch[0].round, batch[0].previous_sig, [b.signature for b in batch[:linked]])
        ok_upto = linked if bad is None else bad
        for b in batch[:ok_upto]:
            try:
                put(b)
            except Exception:  # noqa: BLE001 - sync.go:110-113 logs and gives up on any store error
                return SyncOutcome(False, last, stored, "store", b.round)
            last = b
            stored += 1
            if last.round == up_to:
                return SyncOutcome(True, last, stored)
        if bad is not None:
            return SyncOutcome(False, last, stored, "invalid_beacon", batch[bad].round)
        if linked < len(batch):
            b = batch[linked]
            if _verify_run(engine, b.round, b.previous_sig, [b.signature]) is not None:
                return SyncOutcome(False, last, stored, "invalid_beacon", b.round)
            reason = "invalid round inserted" if b.round != last.round + 1 else "invalid previous signature"
            return SyncOutcome(False, last, stored, reason, b.round)


def verify_beacons(engine, public_key: bytes, beacons) -> list:
    """``chain.VerifyBeacon`` (chain/beacon.go:87-92) over an arbitrary list of beacons, e.g. a
    range loaded from a store or a relay: one ``verify_chained`` call per maximal linked run
    (``ingest.segments``). Returns one bool per beacon, in input order."""
    from .ingest import segments
    engine.set_public_key(public_key)
    ok = [False] * len(beacons)
    for seg in segments(beacons):
        if len(seg.sigs[0]) != SIG_LEN or len(seg.prev0) not in (32, 96):
            # a lone malformed beacon (wrong signature length) or an odd-length prev: one at a time
            for k, s in enumerate(seg.sigs):
                prev = seg.prev0 if k == 0 else seg.sigs[k - 1]
                ok[seg.start + k] = _verify_run(engine, seg.first_round + k, prev, [s]) is None
            continue
        res = engine.verify_chained(seg.first_round, seg.prev0, seg.sigs)
        ok[seg.start:seg.start + seg.n] = res.ok
    return ok


# --------------------------------------------------------------------------------------------------
# Threshold aggregation: chainStore.runAggregator (chain/beacon/chain.go:91-190)
# and its partialCache / roundCache (chain/beacon/cache.go:18-182), restated. The cache, the gate and
# the flush rules are host bookkeeping, as in the reference; the aggregation step itself (verify every
# cached V1 and V2 partial, Recover both, VerifyRecovered both) is ONE engine call,
# ``Engine.aggregate_round`` -> blsv_aggregate_round: two device passes for the whole round.

MAX_PARTIALS_PER_NODE = 100     # chain/beacon/constants.go:14
PARTIAL_CACHE_STORE_LIMIT = 3   # chain/beacon/chain.go:87

AGG_OK, AGG_OK_V2, AGG_V1_RECOVER_FAIL, AGG_V1_INVALID, AGG_V2_RECOVER_FAIL = range(5)  # include/blsverify.h


@dataclass
class PartialBeaconPacket:
    """``drand.PartialBeaconPacket`` (protobuf/drand/protocol.proto:62-72)."""
    round: int
    previous_sig: bytes
    partial_sig: bytes
    partial_sig_v2: bytes = b""


def index_of(partial: bytes) -> int:
    """``key.Scheme.IndexOf`` ([ext] tbls): the 2-byte big-endian share index; -1 on a short share
    (the callers ignore the error, cache.go:42,91,133)."""
    return int.from_bytes(bytes(partial[:2]), "big") if len(partial) >= 2 else -1


def message(round_: int, prev: bytes) -> bytes:
    """``chain.Message`` (chain/beacon.go:103-108)."""
    return hashlib.sha256(bytes(prev) + round_.to_bytes(8, "big")).digest()


def message_v2(round_: int) -> bytes:
    """``chain.MessageV2`` (chain/beacon.go:110-114)."""
    return hashlib.sha256(round_.to_bytes(8, "big")).digest()


class RoundCache:
    """``roundCache`` (cache.go:112-182): the partials of one (round, prev) keyed by share index."""

    def __init__(self, id_: bytes, p: PartialBeaconPacket):
        self.round = p.round
        self.prev = bytes(p.previous_sig)
        self.id = id_
        self.sigs: dict = {}
        self.sigs_v2: dict = {}

    def append(self, p: PartialBeaconPacket) -> bool:
        idx = index_of(p.partial_sig)
        if idx in self.sigs:
            return False
        self.sigs[idx] = bytes(p.partial_sig)
        if len(p.partial_sig_v2) > 0:  # a V2 partial missing the first time is never added later
            self.sigs_v2[idx] = bytes(p.partial_sig_v2)
        return True

    def __len__(self):
        return len(self.sigs)

    def len_v2(self):
        return len(self.sigs_v2)

    def msg(self):
        return message(self.round, self.prev)

    def partials(self):
        return list(self.sigs.values())

    def partials_v2(self):
        return list(self.sigs_v2.values())

    def flush_index(self, idx):
        self.sigs.pop(idx, None)


def round_id(round_: int, prev: bytes) -> bytes:
    """cache.go:33-38: BE64(round) || previous."""
    return round_.to_bytes(8, "big") + bytes(prev)


class PartialCache:
    """``partialCache`` (cache.go:18-110): per-round caches plus the per-signer round list that
    bounds a signer to MAX_PARTIALS_PER_NODE cached rounds (the oldest is evicted)."""

    def __init__(self, log=None):
        self.rounds: dict = {}
        self.rcvd: dict = {}
        self.log = log or (lambda *a: None)

    def append(self, p: PartialBeaconPacket):
        id_ = round_id(p.round, p.previous_sig)
        idx = index_of(p.partial_sig)
        rc = self._get_cache(id_, p)
        if rc is None:
            return
        if rc.append(p):
            self.rcvd.setdefault(idx, []).append(id_)

    def flush_rounds(self, round_: int):
        for id_, rc in list(self.rounds.items()):
            if rc.round > round_:
                continue
            del self.rounds[id_]
            for idx in list(rc.sigs):
                keep = [x for x in self.rcvd.get(idx, []) if x != id_]
                if keep:
                    self.rcvd[idx] = keep
                else:
                    self.rcvd.pop(idx, None)

    def get_round_cache(self, round_: int, prev: bytes):
        return self.rounds.get(round_id(round_, prev))

    def _get_cache(self, id_, p):
        if id_ in self.rounds:
            return self.rounds[id_]
        idx = index_of(p.partial_sig)
        if len(self.rcvd.get(idx, [])) >= MAX_PARTIALS_PER_NODE:
            to_evict = self.rcvd[idx][0]
            rc = self.rounds.get(to_evict)
            if rc is None:
                self.log("cache miss", idx, p.round)
                return None
            rc.flush_index(idx)
            self.rcvd[idx] = self.rcvd[idx][1:] + [id_]
            if len(rc) == 0:
                del self.rounds[to_evict]
        rc = RoundCache(id_, p)
        self.rounds[id_] = rc
        return rc


@dataclass
class AggregateEvent:
    """What one partial did to the aggregator (the reference only logs these)."""
    kind: str                       # "ignored", "stored", "invalid_recovery", "invalid_sig",
                                    # "invalid_recovery_v2", "aggregated"
    round: int
    beacon: Optional[Beacon] = None
    appended: bool = False          # tryAppend succeeded (chain.go:192-208)
    v2_valid: Optional[bool] = None  # VerifyRecovered V2 (a failure only logs, chain.go:162-164)


class Aggregator:
    """``chainStore.runAggregator`` (chain/beacon/chain.go:91-190) over one GPU engine.

    ``on_partial`` is the ``newPartials`` case (partials already passed ``ProcessPartialBeacon``'s
    VerifyPartial, node.go:112); ``on_beacon_stored`` the ``beaconStoredAgg`` case. ``put`` stands for
    ``CallbackStore.Put`` (raises on a rejected beacon). ``commits``/``t``/``n`` are the current
    group's (``c.crypto.GetPub()``, ``GetGroup().Threshold``/``Len()``); ``set_group`` follows a
    reshare transition (node.go:190)."""

    def __init__(self, engine, commits, t: int, n: int, last: Beacon, put: Callable[[Beacon], None]):
        self.engine = engine
        self.put = put
        self.last = last
        self.cache = PartialCache()
        self.set_group(commits, t, n)

    def set_group(self, commits, t, n):
        self.commits, self.t, self.n = [bytes(c) for c in commits], int(t), int(n)

    def on_beacon_stored(self, b: Beacon):
        self.last = b
        self.cache.flush_rounds(b.round)

    def on_partial(self, p: PartialBeaconPacket) -> AggregateEvent:
        r = p.round
        if not (self.last.round < r <= self.last.round + PARTIAL_CACHE_STORE_LIMIT + 1):
            return AggregateEvent("ignored", r)
        self.cache.append(p)
        rc = self.cache.get_round_cache(r, p.previous_sig)
        if rc is None or len(rc) < self.t:
            return AggregateEvent("stored", r)
        self.engine.set_group(self.commits, self.n)
        status, _, _, sig1, sig2, v2_valid = self.engine.aggregate_round(
            rc.msg(), rc.partials(), message_v2(r), rc.partials_v2(), self.t, self.n)
        if status == AGG_V1_RECOVER_FAIL:
            return AggregateEvent("invalid_recovery", r)
        if status == AGG_V1_INVALID:
            return AggregateEvent("invalid_sig", r)
        if status == AGG_V2_RECOVER_FAIL:
            return AggregateEvent("invalid_recovery_v2", r)
        b = Beacon(rc.prev, rc.round, sig1, sig2 if status == AGG_OK_V2 else b"")
        self.cache.flush_rounds(r)
        ev = AggregateEvent("aggregated", r, b, v2_valid=v2_valid if status == AGG_OK_V2 else None)
        if self.last.round + 1 == b.round:  # tryAppend (chain.go:192-208)
            try:
                self.put(b)
                ev.appended = True
                self.last = b
            except Exception:  # noqa: BLE001 - chain.go:197-200 logs and returns false
                pass
        return ev
