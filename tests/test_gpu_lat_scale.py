"""Parity of the latency path at the sizes it serves.

Every host call of 1..lat_max items (default 1,536) runs on the latency engine (k_lat.hip: one
workgroup per item, limbs across lanes), a second implementation of the arithmetic beside the batch
pipeline (one lane per item). This file puts full-size batches through the DEFAULT routing and checks
them three ways: against the same call forced onto the batch pipeline (set_lat_max(0)), forced onto
the latency path, and against the C oracle's reject classes (oracle/c/bls_oracle.c, pinned to the
reference KAT) at every injected position and its successor:

  * a continuous 2,049-round chained history (tests/golden/chain2049.bin, make_chain_fixture.py)
    through host verify_chained at n = 1,000 (configs[0]), 1,536 (= lat_max), 1,537 (= lat_max + 1,
    the batch side of the cut-over) and 2,048, with every class of the mixed golden injected at the first, a
    middle, the last item and a 64-item edge (client/verify.go:146-163, chain/beacon.go:87-108);
  * the same through blsv_verify_prevs (stored PreviousSig per row: the drand.db loader's call);
  * a device-generated SEGMENTED history through blsv_verify_chained_dev's latency branch with a
    user stream, first_round > 1, seg_phase != 0 and a device class buffer, first_bad as a ROUND;
  * verify_partials over k = 256 partials of one round (indices in every order, corruptions, an
    index >= n) (chain/beacon/node.go:112);
  * verify_messages at 2,048 (client/verify.go:185-207 per item, key/keys.go:60-63).
"""
import hashlib
import os

import pytest


pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NONE = (1 << 64) - 1
BIG = 1 << 20
LAT_MAX = 1536  # blsverify.cpp kLatMaxDefault (test_default_cutover)

# classes of the mixed golden (tests/golden/golden.json "mixed"): name -> source index there; the
# decode classes are copied as bytes, the others are made from the local signature
MIXED = {"flag_cleared": 3, "infinity": 5, "infinity_stray_bits": 6, "infinity_sign_bit": 11, "x_c1_ge_p": 15,
         "x_c0_ge_p": 18, "not_on_curve": 22, "not_in_subgroup": 24}
LOCAL = ("bitflip_x", "wrong_round", "sign_bit_flipped")


@pytest.fixture(scope="module")
def C():
    from oracle import c_oracle

    c_oracle.load()
    return c_oracle


@pytest.fixture(scope="module")
def chain():
    with open(os.path.join(ROOT, "tests", "golden", "chain2049.bin"), "rb") as f:
        raw = f.read()
    assert len(raw) == 2049 * 96
    return [raw[i * 96:(i + 1) * 96] for i in range(2049)]


def _corrupt(kind, sigs, i, golden):
    s = bytearray(sigs[i])
    if kind in MIXED:
        return bytes.fromhex(golden["mixed"]["sigs"][MIXED[kind]])
    if kind == "bitflip_x":
        s[50] ^= 0x04
    elif kind == "sign_bit_flipped":
        s[0] ^= 0x20
    elif kind == "wrong_round":  # a valid signature of another round (test/mock/grpcserver.go:145-147)
        return bytes(sigs[i - 1 if i else i + 1])
    return bytes(s)


def _positions(n):
    return sorted({0, n // 2, n - 1, 64})


def _routes(engine, call, n):
    """(default routing, forced batch, forced latency) results of the same call"""
    old = engine.set_lat_max(LAT_MAX)
    try:
        default = call()
        engine.set_lat_max(0)
        batch = call()
        engine.set_lat_max(n)
        lat = call()
    finally:
        engine.set_lat_max(old)
    return default, batch, lat


def _expected_chained(C, pk, seed, sigs, touched):
    """C-oracle classes at the corrupted items and their successors; 0 elsewhere (the uncorrupted
    history verifies, checked once in test_chain_fixture_accepts)."""
    want = [0] * len(sigs)
    for i in sorted({j for t in touched for j in (t, t + 1) if j < len(sigs)}):
        prev = seed if i == 0 else sigs[i - 1]
        want[i] = C.verify_chained(pk, i + 1, prev, sigs[i])[0]
    return want


def test_default_cutover(engine):
    prev = engine.set_lat_max(0)
    engine.set_lat_max(prev)
    assert prev == LAT_MAX


def test_chain_fixture_accepts(engine, golden, chain, C):
    ch = golden["chained"]
    pk, seed = bytes.fromhex(ch["pk"]), bytes.fromhex(ch["genesis_seed"])
    engine.set_public_key(pk)
    for n in (1000, LAT_MAX, LAT_MAX + 1, 2048):
        d, b, l = _routes(engine, lambda: engine.verify_chained(1, seed, chain[:n]), n)
        for r in (d, b, l):
            assert all(r.ok) and r.first_bad is None and not any(r.reject_class)


@pytest.mark.parametrize("n", [1000, LAT_MAX, LAT_MAX + 1, 2048])
@pytest.mark.parametrize("kind", list(MIXED) + list(LOCAL))
def test_chained_every_class_at_size(engine, golden, chain, C, n, kind):
    ch = golden["chained"]
    pk, seed = bytes.fromhex(ch["pk"]), bytes.fromhex(ch["genesis_seed"])
    engine.set_public_key(pk)
    sigs = list(chain[:n])
    pos = _positions(n)
    for i in pos:
        sigs[i] = _corrupt(kind, chain, i, golden)
    want = _expected_chained(C, pk, seed, sigs, pos)
    assert all(want[i] != 0 for i in pos)
    d, b, l = _routes(engine, lambda: engine.verify_chained(1, seed, sigs), n)
    assert d.reject_class == b.reject_class == l.reject_class == want
    assert d.ok == b.ok == l.ok == [c == 0 for c in want]
    assert d.first_bad == b.first_bad == l.first_bad == 1 + min(i for i, c in enumerate(want) if c)


@pytest.mark.parametrize("n", [LAT_MAX, LAT_MAX + 1])
def test_verify_prevs_at_size(engine, golden, chain, C, n):
    """blsv_verify_prevs: every row carries its own stored PreviousSig (chain/boltdb/store.go
    values); a corrupted stored prev rejects only its own round, a corrupted signature only its own
    round too (the next row's prev is the stored, uncorrupted one)."""
    ch = golden["chained"]
    pk, seed = bytes.fromhex(ch["pk"]), bytes.fromhex(ch["genesis_seed"])
    engine.set_public_key(pk)
    sigs = list(chain[:n])
    prevs = [seed.ljust(96, b"\0")] + sigs[:-1]
    bad_sig, bad_prev = [5, n // 2, n - 1], [64, n - 2]
    for i in bad_sig:
        sigs[i] = _corrupt("bitflip_x", chain, i, golden)
    for i in bad_prev:
        p = bytearray(prevs[i])
        p[10] ^= 1
        prevs[i] = bytes(p)
    want = [0] * n
    for i in bad_sig + bad_prev:
        want[i] = C.verify_chained(pk, i + 1, prevs[i] if i else seed, sigs[i])[0]
    P, S = b"".join(prevs), b"".join(sigs)
    d, b, l = _routes(engine, lambda: engine.verify_prevs(1, 32, P, S, n), n)
    for r in (d, b, l):
        assert list(r.reject_class) == want
        assert r.first_bad == 1 + min(bad_sig + bad_prev)


@pytest.mark.parametrize("n,seg,phase,first_round", [(1500, 64, 17, 10_001), (LAT_MAX, 64, 63, 100), (700, 32, 1, 2)])
def test_chained_dev_latency_branch(engine, golden, C, n, seg, phase, first_round):
    """blsv_verify_chained_dev on the latency path (a small per-rank shard of bench.py
    --total-rounds): user stream, label = first_round, seg_phase != 0, device reject classes; a
    corrupted signature inside a segment rejects it and its successor, one at a segment's last round
    only itself; first_bad is a ROUND. Same verdicts as the batch pipeline."""
    import torch

    from drand_amd import shard

    ch = golden["chained"]
    pk = bytes.fromhex(ch["pk"])
    engine.set_public_key(pk)
    sk32 = int(ch["sk"], 16).to_bytes(32, "big")
    gen_n = n + phase
    n_seg = (gen_n + seg - 1) // seg
    g = torch.Generator(device="cuda:0")
    g.manual_seed(n + phase)
    seg_seeds = torch.randint(0, 256, (n_seg, 96), dtype=torch.uint8, device="cuda:0", generator=g)
    gen_first = first_round - phase
    s0 = 32 if gen_first == 1 else 96
    gen = torch.empty((gen_n, 96), dtype=torch.uint8, device="cuda:0")
    engine.generate_chained_dev(sk32, gen_first, seg, seg_seeds.data_ptr(), s0, gen.data_ptr(), gen_n)
    torch.cuda.synchronize()
    sl = shard.SegmentedSlice(shard.Shard(0, phase, n), 0, 0, phase, n_seg)
    loc = shard.local_seeds(sl, seg_seeds, gen)
    mine = gen[phase:].clone()
    last_in_seg = next(i for i in range(n) if (i + 1 + phase) % seg == 0)
    bad = [3, last_in_seg, n - 1]
    for i in bad:
        mine[i, 50] ^= 0x04
    stream = torch.cuda.Stream()
    s0_local = 32 if first_round == 1 else 96

    def call():
        bm = torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda:0")
        fb = torch.empty(1, dtype=torch.int64, device="cuda:0")
        cls = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda:0")
        torch.cuda.synchronize()
        engine.verify_chained_dev(first_round, seg, loc.data_ptr(), s0_local, mine.data_ptr(), n, bm.data_ptr(),
                                  fb.data_ptr(), cls.data_ptr(), stream.cuda_stream, seg_phase=phase)
        stream.synchronize()
        words = [w & NONE for w in bm.cpu().tolist()]
        return ([(words[i // 64] >> (i % 64)) & 1 == 1 for i in range(n)], int(fb.item()) & NONE,
                cls.cpu().tolist())

    d, b, l = _routes(engine, call, n)
    assert d == b == l
    ok, fb, cls = d
    rows = [bytes(loc[k].cpu().tolist()) for k in range(loc.shape[0])]
    host = [bytes(mine[i].cpu().tolist()) for i in range(n)]
    want_bad = set(bad) | {i + 1 for i in bad if i + 1 < n and (i + 1 + phase) % seg != 0}
    assert {i for i, v in enumerate(ok) if not v} == want_bad
    assert fb == first_round + min(want_bad)
    for i in sorted(want_bad):
        prev = shard.chained_prev(i, phase, seg, rows, host, s0_local)
        assert cls[i] == C.verify_chained(pk, first_round + i, prev, host[i])[0] != 0
    assert sum(1 for c in cls if c) == len(want_bad)


def test_verify_partials_256_mixed(engine, golden, C):
    """k = 256 partials of one round: the 64 golden shares four times in shuffled orders, with
    corruptions (bit flip, a decode class, a share presented under another index, an index >= n,
    the V2 share of the same signer, which signs MessageV2) -- every class equal on all three
    routes and to the C oracle's tbls VerifyPartial."""
    import random

    th = golden["threshold"]
    commits = [bytes.fromhex(c) for c in th["commits"]]
    msg = bytes.fromhex(th["msg"])
    parts = [bytes.fromhex(p) for p in th["partials"]]
    rng = random.Random(256)
    batch = []
    for rep in range(4):
        p = list(parts)
        rng.shuffle(p)
        batch += p
    batch[0] = batch[0][:50] + bytes([batch[0][50] ^ 4]) + batch[0][51:]
    batch[17] = batch[17][:2] + bytes.fromhex(golden["mixed"]["sigs"][MIXED["not_in_subgroup"]])
    other = int.from_bytes(batch[40][:2], "big")
    batch[40] = ((other + 1) % th["n"]).to_bytes(2, "big") + batch[40][2:]  # share under another index
    batch[128] = (th["n"] + 3).to_bytes(2, "big") + batch[128][2:]  # index >= n
    batch[255] = bytes.fromhex(th["partials_v2"][0])  # the V2 share: signs MessageV2, not msg
    grp = C.Group(commits)
    want = [grp.verify_partial(msg, p) for p in batch]
    assert sum(1 for c in want if c) == 5
    engine.set_group(commits, th["n"])
    d, b, l = _routes(engine, lambda: engine.verify_partials(msg, batch), len(batch))
    assert d == b == l
    ok, cls = d
    # an index >= n is no error of its own in tbls VerifyPartial (PubPoly.Eval(i) at any i): the
    # share simply fails the pairing check under that index's public share, as in the C oracle
    assert cls == want
    assert ok == [c == 0 for c in cls]


def test_verify_messages_2048(engine, golden, C):
    ch = golden["chained"]
    pk = bytes.fromhex(ch["pk"])
    sk32 = int(ch["sk"], 16).to_bytes(32, "big")
    n = 2048
    msgs = [hashlib.sha256(b"lat-scale %d" % i).digest() for i in range(n)]
    sigs = engine.sign(sk32, msgs)
    pos = [0, 64, 1023, n - 1]
    kinds = list(MIXED) + list(LOCAL)
    touched = {}
    for k, kind in enumerate(kinds):
        i = (pos[k % len(pos)] + 97 * (k // len(pos))) % n
        sigs[i] = _corrupt(kind, sigs, i, golden)
        touched[i] = kind
    want = [C.verify(pk, msgs[i], sigs[i]) if i in touched else 0 for i in range(n)]
    assert len(touched) == len(kinds) and all(want[i] for i in touched)
    d, b, l = _routes(engine, lambda: engine.verify_messages(msgs, sigs, pk48=pk), n)
    assert d.reject_class == b.reject_class == l.reject_class == want
    assert d.first_bad == b.first_bad == l.first_bad == min(touched)
