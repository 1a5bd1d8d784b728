"""blsv_verify_chained_multi: the Go host's multi-GPU shape through the C ABI.

A Go deployment on an 8-GPU node would hold one Engine (context) per GPU and replace the serial
loops of client/verify.go:146-163 and chain/beacon/sync.go:100-119 by one call that splits the range
into contiguous shards, each verified on its own context from its own host thread with the true
previous signature as its halo, and merges the verdicts in host memory (no collective: the shards
share the caller's address space). Here three contexts sit on device i % device_count (all on cuda:0
on the one-GPU test box) and the continuous 2,049-round golden chain (tests/golden/chain2049.bin,
signed by the KAT-pinned C oracle) is split at unaligned boundaries, with corrupted signatures at a
shard's last position (its successor, the next shard's first round, must reject through the halo),
at a shard's first position and in the middle. The merged bitmap, first bad round and classes must
equal one whole-history blsv_verify_chained call and the C oracle's classes, on the latency path and
on the batch pipeline (set_lat_max(0)).
"""
import os

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def chain():
    with open(os.path.join(ROOT, "tests", "golden", "chain2049.bin"), "rb") as f:
        raw = f.read()
    return [raw[i * 96:(i + 1) * 96] for i in range(2049)]


@pytest.fixture(scope="module")
def engines(golden):
    import torch

    from drand_amd.engine import Engine

    ndev = max(torch.cuda.device_count(), 1)
    es = [Engine(i % ndev) for i in range(3)]
    pk = bytes.fromhex(golden["chained"]["pk"])
    for e in es:
        e.set_public_key(pk)
    yield es
    for e in es:
        e.close()


@pytest.fixture(scope="module")
def C():
    from oracle import c_oracle

    c_oracle.load()
    return c_oracle


SPLITS = {"even": None, "ragged": [700, 1, 1348], "empty_middle": [1025, 0, 1024]}


@pytest.mark.parametrize("route", ["lat", "batch"])
@pytest.mark.parametrize("split", list(SPLITS))
def test_multi_context_equals_whole_history(engines, engine, chain, golden, C, split, route):
    from drand_amd.engine import verify_chained_multi

    counts = SPLITS[split]
    n = len(chain)
    cs = counts or [n // 3 + (1 if k < n % 3 else 0) for k in range(3)]
    edges = [sum(cs[:k]) for k in range(1, 3)]
    sigs = list(chain)
    # a shard's last signature (its successor is the next shard's first round: rejects via the halo),
    # a shard's first signature, the middle of the first shard, the last round
    hit = sorted({edges[0] - 1, edges[1], cs[0] // 2, n - 1})
    for i in hit:
        s = bytearray(sigs[i])
        s[50] ^= 0x04
        sigs[i] = bytes(s)
    seed = bytes.fromhex(golden["chained"]["genesis_seed"])
    olds = [e.set_lat_max(0 if route == "batch" else 1536) for e in engines + [engine]]
    try:
        engine.set_public_key(bytes.fromhex(golden["chained"]["pk"]))
        whole = engine.verify_chained(1, seed, sigs)
        multi = verify_chained_multi(engines, 1, seed, sigs, counts)
    finally:
        for e, o in zip(engines + [engine], olds):
            e.set_lat_max(o)
    assert multi.ok == whole.ok
    assert multi.first_bad == whole.first_bad == hit[0] + 1
    assert multi.reject_class == whole.reject_class
    bad = [i for i in range(n) if not multi.ok[i]]
    assert bad == sorted(set(hit) | {i + 1 for i in hit if i + 1 < n})
    # the classes at every rejected round (incl. the halo-linked successor) = the C oracle's
    pk = bytes.fromhex(golden["chained"]["pk"])
    for i in bad:
        prev = seed if i == 0 else sigs[i - 1]
        assert multi.reject_class[i] == C.verify_chained(pk, i + 1, prev, sigs[i])[0], i


def test_multi_context_rejects_bad_arguments(engines, chain, golden):
    from drand_amd.engine import EngineError, verify_chained_multi

    seed = bytes.fromhex(golden["chained"]["genesis_seed"])
    with pytest.raises(EngineError) as e:
        verify_chained_multi([engines[0], engines[0]], 1, seed, chain[:10])
    assert e.value.code == -1
    with pytest.raises(EngineError) as e:
        verify_chained_multi(engines, 1, seed, chain[:10], [3, 3, 3])
    assert e.value.code == -1
    # a context holding another group
    engines[2].set_public_key(bytes.fromhex(golden["kat"]["pk"]))
    try:
        with pytest.raises(EngineError) as e:
            verify_chained_multi(engines, 1, seed, chain[:10])
        assert e.value.code == -1
    finally:
        engines[2].set_public_key(bytes.fromhex(golden["chained"]["pk"]))
