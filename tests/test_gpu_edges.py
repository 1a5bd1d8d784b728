"""GPU edge cases through the C ABI, each checked against the Python oracle or the goldens:
empty and ragged batches, wrong-length inputs (rejected host-side, grpcserver.go:66-69), the
point-at-infinity rules of kilic's pairing engine (O pairs are skipped, empty product = 1), and
tbls Recover's share selection (first t VALID shares in input order, duplicates keep the first,
fewer than t valid -> error; the group signature a0*H(m) is the same for every valid t-subset)."""
import random

import pytest

from drand_amd import _lib
from drand_amd.engine import EngineError
from oracle import bls12381 as O

pytestmark = pytest.mark.gpu

INF_G1 = bytes([0xC0]) + bytes(47)
INF_G2 = bytes([0xC0]) + bytes(95)


def test_empty_batches(engine, golden):
    ch = golden["chained"]
    engine.set_public_key(bytes.fromhex(ch["pk"]))
    res = engine.verify_chained(1, bytes.fromhex(ch["genesis_seed"]), [])
    assert res.ok == [] and res.first_bad is None
    res = engine.verify_unchained([], first_round=1)
    assert res.ok == [] and res.first_bad is None
    assert engine.verify_messages([], []).ok == []


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65])
def test_ragged_chained_prefixes(engine, golden, n):
    ch = golden["chained"]
    engine.set_public_key(bytes.fromhex(ch["pk"]))
    sigs = [bytes.fromhex(b["sig"]) for b in ch["beacons"]]
    seed = bytes.fromhex(ch["genesis_seed"])
    reps = (n + len(sigs) - 1) // len(sigs)
    # beyond the golden chain: rounds past the end reject (their messages differ) -- prefix only
    m = min(n, len(sigs))
    res = engine.verify_chained(1, seed, sigs[:m])
    assert all(res.ok) and len(res.ok) == m
    if n > len(sigs):  # a ragged batch of n: the golden chain twice; the second copy rejects
        batch = (sigs * reps)[:n]
        res = engine.verify_chained(1, seed, batch)
        assert all(res.ok[:len(sigs)]) and not any(res.ok[len(sigs):])
        assert res.first_bad == len(sigs) + 1


def test_wrong_length_rejected_host_side(engine, golden):
    ch = golden["chained"]
    engine.set_public_key(bytes.fromhex(ch["pk"]))
    with pytest.raises(ValueError):
        engine.verify_chained(1, bytes.fromhex(ch["genesis_seed"]), [bytes(3)])  # grpcserver.go:66-69
    with pytest.raises(ValueError):
        engine.verify_unchained([b""], first_round=1)


def test_infinity_rules_parity_unpinned(engine, golden):
    """PARITY UNPINNED: kilic's treatment of points at infinity in the pairing product (a pair with an
    infinity point is skipped), restated from its published source; no reference fixture."""
    kat = golden["kat"]
    msg = bytes.fromhex(kat["msg"])
    sig = bytes.fromhex(kat["sig"])
    cases = [(bytes.fromhex(kat["pk"]), INF_G2),  # valid pk, sigma = O: e(pk, H) != 1 -> reject
             (INF_G1, INF_G2),                    # both pairs skipped: empty product -> kilic accepts
             (INF_G1, sig)]                       # only e(-g1, sigma) left -> reject
    for pk48, s in cases:
        pk = O.g1_decompress(pk48)
        want = O.verify_class(pk, msg, s)
        res = engine.verify_messages([msg], [s], pk48=pk48)
        assert res.reject_class == [want], (pk48[:1].hex(), s[:1].hex())


def test_recover_selection_rules_dedup_parity_unpinned(engine, golden):
    """Any t valid shares give the group signature (pinned by the threshold fixture); the duplicate-
    index rule at the end is PARITY UNPINNED (kyber's published Recover/xyCommit, no reference test)."""
    th = golden["threshold"]
    engine.set_group([bytes.fromhex(c) for c in th["commits"]], th["n"])
    msg = bytes.fromhex(th["msg"])
    partials = [bytes.fromhex(p) for p in th["partials"]]
    t = th["t"]
    rng = random.Random(9)
    for _ in range(2):  # any t valid shares give the same group signature
        sub = rng.sample(partials, t)
        assert engine.recover(msg, sub, t, th["n"]).hex() == th["group_sig"]
    bad = bytes.fromhex(th["bad_partial"])
    dup = partials[0]
    # invalid shares are skipped, the next valid ones complete the set
    sub = [bad, dup] + partials[1:t]
    assert engine.recover(msg, sub, t, th["n"]).hex() == th["group_sig"]
    # fewer than t valid shares -> BLSV_ENOTENOUGH
    with pytest.raises(EngineError) as e:
        engine.recover(msg, [bad] + partials[: t - 1], t, th["n"])
    assert e.value.code == _lib.BLSV_ENOTENOUGH
    # PARITY UNPINNED ([ext] kyber tbls.Recover / share.xyCommit, restated from the published
    # source): a duplicate index among the first t valid shares counts toward t and then
    # collapses -> not enough distinct shares, even though a later share would have completed the set
    with pytest.raises(EngineError) as e:
        engine.recover(msg, [bad, dup, dup] + partials[1:t], t, th["n"])
    assert e.value.code == _lib.BLSV_ENOTENOUGH


def test_recover_index_beyond_n_parity_unpinned(engine, golden):
    """PARITY UNPINNED (xyCommit drops s.I >= n): a single-key group (t = 1, Eval(i) = C0 for every
    i) accepts a share at index 5 as VALID, but Recover with n = 1 drops it -> ENOTENOUGH; index 0
    recovers the signature itself (lambda = 1)."""
    import hashlib
    ch = golden["chained"]
    b = ch["beacons"][0]
    msg = hashlib.sha256(bytes.fromhex(b["prev"]) + b["round"].to_bytes(8, "big")).digest()
    sig = bytes.fromhex(b["sig"])
    engine.set_group([bytes.fromhex(ch["pk"])], 1)
    assert engine.verify_partials(msg, [b"\0\5" + sig])[0] == [True]
    with pytest.raises(EngineError) as e:
        engine.recover(msg, [b"\0\5" + sig], 1, 1)
    assert e.value.code == _lib.BLSV_ENOTENOUGH
    assert engine.recover(msg, [b"\0\0" + sig], 1, 1) == sig
    assert engine.recover(msg, [b"\0\5" + sig], 1, 6) == sig


@pytest.mark.gpu
def test_aggregate_round(engine, golden):
    """blsv_aggregate = VerifyPartial x k + Recover(first t valid) + VerifyRecovered (chain.go:119-166)."""
    from drand_amd.engine import EngineError
    th = golden["threshold"]
    engine.set_group([bytes.fromhex(c) for c in th["commits"]], th["n"])
    msg = bytes.fromhex(th["msg"])
    partials = [bytes.fromhex(p) for p in th["partials"]]
    # the recovery is speculated beside the partials' verification (blsverify.cpp spec_recover_*):
    # kept when every selected share verifies, recomputed from the valid shares otherwise
    h0, m0 = engine.spec_stats()
    ok, cls, sig, gok = engine.aggregate(msg, partials, th["t"], th["n"])
    assert all(ok) and gok and sig.hex() == th["group_sig"]
    assert engine.spec_stats() == (h0 + 1, m0)
    bad = bytes.fromhex(th["bad_partial"])
    # the golden bad share repeats index 3: assumed valid it would leave only 32 distinct indices
    # among the first 33 shares, so nothing is speculated and the sequential recovery runs
    ok, cls, sig, gok = engine.aggregate(msg, [bad] + partials[:th["t"]], th["t"], th["n"])
    assert ok[0] is False and all(ok[1:]) and gok and sig.hex() == th["group_sig"]
    assert engine.spec_stats() == (h0 + 1, m0)
    # share 0 with a flipped signature bit: speculated, fails verification, recomputed from 1..33
    flip = partials[0][:40] + bytes([partials[0][40] ^ 1]) + partials[0][41:]
    ok, cls, sig, gok = engine.aggregate(msg, [flip] + partials[1:th["t"] + 1], th["t"], th["n"])
    assert ok[0] is False and all(ok[1:]) and gok and sig.hex() == th["group_sig"]
    assert engine.spec_stats() == (h0 + 1, m0 + 1)
    # a bad share after the first t: the speculated selection stands
    ok, cls, sig, gok = engine.aggregate(msg, partials[:th["t"]] + [flip], th["t"], th["n"])
    assert all(ok[:-1]) and ok[-1] is False and gok and sig.hex() == th["group_sig"]
    assert engine.spec_stats() == (h0 + 2, m0 + 1)
    with pytest.raises(EngineError):
        engine.aggregate(msg, [bad] + partials[:th["t"] - 1], th["t"], th["n"])


@pytest.mark.gpu
def test_verify_partials_multi_rounds(engine, golden):
    """Partials of 24 different rounds in one pass. Group = the single golden key (t = 1, share index
    0, as mock/result.go:88-95 signs with PriShare{I: 0}); partial_i = BE16(0) || sig_i over
    Message(round_i, prev_i)."""
    import hashlib
    ch = golden["chained"]
    engine.set_group([bytes.fromhex(ch["pk"])], 1)
    msgs = [hashlib.sha256(bytes.fromhex(b["prev"]) + b["round"].to_bytes(8, "big")).digest() for b in ch["beacons"]]
    parts = [b"\0\0" + bytes.fromhex(b["sig"]) for b in ch["beacons"]]
    ok, cls = engine.verify_partials_multi(msgs, parts)
    assert all(ok) and set(cls) == {0}
    swapped = msgs[:]
    swapped[3], swapped[17] = swapped[17], swapped[3]
    ok, cls = engine.verify_partials_multi(swapped, parts)
    assert [i for i, v in enumerate(ok) if not v] == [3, 17] and cls[3] == O.REJ_PAIRING
    # agrees with the single-message entry point round by round
    for i in (0, 9, 23):
        assert engine.verify_partials(msgs[i], [parts[i]])[0] == [True]


@pytest.mark.gpu
def test_verify_messages_null_message_buffer(engine, golden):
    """A message length without a message buffer is refused (BLSV_EINVAL), not dereferenced; zero-length
    messages need no buffer."""
    import ctypes

    from drand_amd import _lib

    kat = golden["kat"]
    sig = bytes.fromhex(kat["sig"])
    lens = (ctypes.c_uint32 * 1)(5)
    bm, cls = _lib.out_buf(1), _lib.out_buf(1)
    fb = ctypes.c_uint64()
    rc = engine.lib.blsv_verify_messages(engine._h, _lib.buf(bytes.fromhex(kat["pk"])), None, lens, 1, _lib.buf(sig),
                                         bm, ctypes.byref(fb), cls)
    assert rc == -1
    lens[0] = 0
    rc = engine.lib.blsv_verify_messages(engine._h, _lib.buf(bytes.fromhex(kat["pk"])), None, lens, 1, _lib.buf(sig),
                                         bm, ctypes.byref(fb), cls)
    assert rc == 0 and cls[0] == 7  # the KAT signature over the empty message fails the pairing
