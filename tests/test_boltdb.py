"""drand.db bulk loader (drand_amd/csrc/boltload.cpp) and store verification (drand_amd/boltdb.py).

Fixtures are bbolt files written by tests/support/boltwriter.py in the layout boltStore uses
(chain/boltdb/store.go:21,68-81), holding the 24-round chained golden history. The reference ships
no drand.db, so byte parity with files bbolt itself writes is unpinned; the loader is checked
against the writer and against the golden beacons, and verdicts against the oracle (CPU) and the
HIP engine (GPU).
"""
from __future__ import annotations

import struct

import numpy as np
import pytest

from drand_amd import boltdb, ingest
from drand_amd.callers import Beacon
from tests.support.boltwriter import write_db
from tests.support.oracle_engine import OracleEngine


@pytest.fixture(scope="module")
def chain(golden):
    ch = golden["chained"]
    bs = [Beacon(bytes.fromhex(b["prev"]), b["round"], bytes.fromhex(b["sig"]), bytes.fromhex(b["sig_v2"]))
          for b in ch["beacons"]]
    return bytes.fromhex(ch["pk"]), bytes.fromhex(ch["genesis_seed"]), bs


def _items(beacons):
    return [(struct.pack(">Q", b.round), ingest.beacon_to_json(b)) for b in beacons]


@pytest.mark.parametrize("layout", [dict(per_leaf=5), dict(per_leaf=1), dict(inline=True), dict(page_size=1024, per_leaf=1)])
def test_load_matches_written(tmp_path, chain, layout):
    _, seed, bs = chain
    p = tmp_path / "drand.db"
    write_db(p, _items(bs), **layout)
    sb = boltdb.load_store(p)
    assert len(sb) == 24
    assert sb.rounds.tolist() == list(range(1, 25))
    for i, b in enumerate(bs):
        assert sb.prev[i, :sb.prev_len[i]].tobytes() == b.previous_sig
        assert sb.sigs[i].tobytes() == b.signature and sb.sig_len[i] == 96
        assert sb.sigs_v2[i].tobytes() == b.signature_v2
    assert sb.prev_len[0] == 32 and (sb.prev_len[1:] == 96).all()
    part = boltdb.load_store(p, start=10, max_n=5)
    assert part.rounds.tolist() == list(range(11, 16))
    assert boltdb.linked_runs(sb).tolist() == [0]


def test_meta_selection_and_errors(tmp_path, chain):
    _, _, bs = chain
    p = tmp_path / "a.db"
    # the meta page with the larger txid wins; a bad checksum falls back to the other one
    write_db(p, _items(bs), txids=(5, 9), corrupt_meta1=True)
    assert len(boltdb.load_store(p)) == 24
    write_db(p, _items(bs), txids=(5, 9), corrupt_meta1=False)
    assert len(boltdb.load_store(p)) == 24
    # empty bucket
    write_db(p, [], inline=True)
    assert len(boltdb.load_store(p)) == 0
    # key round != value round
    items = _items(bs[:3])
    items[1] = (struct.pack(">Q", 7), items[1][1])
    write_db(p, items)
    with pytest.raises(boltdb.StoreError, match="key round 7"):
        boltdb.load_store(p)
    # malformed value
    write_db(p, [(struct.pack(">Q", 1), b'{"Round":1,"Signature":"zz"}')])
    with pytest.raises(boltdb.StoreError, match="malformed"):
        boltdb.load_store(p)
    # a Round that overflows uint64 is a json.Unmarshal error, not a silent wrap
    write_db(p, [(struct.pack(">Q", 1), b'{"Round":18446744073709551617,"Signature":"00"}')])
    with pytest.raises(boltdb.StoreError, match="malformed"):
        boltdb.load_store(p)
    # field names match case-insensitively, as encoding/json (hexjson) does
    b0 = bs[0]
    write_db(p, [(struct.pack(">Q", 1), b'{"previoussig":"%s","ROUND":1,"signature":"%s"}'
                  % (b0.previous_sig.hex().encode(), b0.signature.hex().encode()))])
    sb = boltdb.load_store(p)
    assert sb.rounds.tolist() == [1] and sb.sigs[0].tobytes() == b0.signature and sb.prev_len[0] == 32
    # not a bbolt file
    p.write_bytes(b"\0" * 8192)
    with pytest.raises(boltdb.StoreError, match="meta"):
        boltdb.load_store(p)


def _tampered(bs):
    out = list(bs)
    out[9] = Beacon(bs[9].previous_sig, 10, bs[8].signature, bs[9].signature_v2)      # bad sig: 10 and 11 fail
    out[15] = Beacon(bs[15].previous_sig, 16, b"\x01\x02\x03")                          # 3-byte sig: 16 fails
    del out[20]                                                                        # gap at 21
    return out


def _check_verdicts(eng, tmp_path, chain):
    pk, _, bs = chain
    p = tmp_path / "v.db"
    write_db(p, _items(bs), per_leaf=3)
    v = boltdb.verify_store(eng, pk, boltdb.load_store(p))
    assert v.ok.all() and v.first_bad is None and v.runs == 1
    assert boltdb.round_runs(boltdb.load_store(p)).tolist() == [0]
    tb = _tampered(bs)
    write_db(p, _items(tb), per_leaf=4)
    sb = boltdb.load_store(p)
    v = boltdb.verify_store(eng, pk, sb)
    bad_rounds = sb.rounds[~v.ok].tolist()
    # round 11 stores the true prev (= real sig 10), so it still verifies: only the tampered rows fail,
    # plus round 17 whose stored prev is the real sig 16 -> verifies too (VerifyBeacon reads stored prev)
    assert bad_rounds == [10, 16]
    assert v.first_bad == 10
    # verdicts equal the per-beacon oracle answer
    from oracle import c_oracle
    import hashlib
    for i in range(len(sb)):
        r = int(sb.rounds[i])
        prev = sb.prev[i, :sb.prev_len[i]].tobytes()
        sig = sb.sigs[i, :min(96, sb.sig_len[i])].tobytes()
        exp = c_oracle.verify(pk, hashlib.sha256(prev + r.to_bytes(8, "big")).digest(), sig) == 0 \
            if len(sig) == 96 else False
        assert bool(v.ok[i]) == exp, r


def test_verify_store_cpu(tmp_path, chain):
    _check_verdicts(OracleEngine(), tmp_path, chain)


@pytest.mark.gpu
def test_verify_store_gpu(tmp_path, chain, engine):
    _check_verdicts(engine, tmp_path, chain)


def _genesis_item(group_hash):
    # chain.GenesisBeacon (chain/store.go:234-238) as Put at node start (chain/beacon/node.go:69):
    # Round 0, nil PreviousSig (hexjson null), Signature = GroupHash (32 bytes)
    return (struct.pack(">Q", 0), b'{"PreviousSig":null,"Round":0,"Signature":"%s"}' % group_hash.hex().encode())


@pytest.mark.parametrize("tamper", [False, True])
def test_genesis_row_is_trusted_root(tmp_path, chain, tamper):
    """every real drand.db starts with the round-0 genesis beacon; it is never verified
    (sync starts at last+1, the client walk at round 1), so it must not become first_bad."""
    pk, seed, bs = chain
    bs = _tampered(bs) if tamper else bs
    p = tmp_path / "g.db"
    write_db(p, [_genesis_item(seed)] + _items(bs), per_leaf=3)
    sb = boltdb.load_store(p)
    assert sb.rounds[0] == 0 and sb.prev_len[0] == 0 and sb.sig_len[0] == 32
    eng = OracleEngine()
    v = boltdb.verify_store(eng, pk, sb, group_hash=seed)
    assert v.ok[0]
    assert all(c[1] != 0 for c in eng.calls)  # round 0 never reaches the engine
    assert v.first_bad == (10 if tamper else None)
    assert sorted(sb.rounds[~v.ok].tolist()) == ([10, 16] if tamper else [])
    v = boltdb.verify_store(eng, pk, sb)  # no GroupHash given: trusted as is
    assert v.ok[0] and v.first_bad == (10 if tamper else None)
    v = boltdb.verify_store(eng, pk, sb, group_hash=bytes(32))  # wrong GroupHash: flagged, not first_bad
    assert not v.ok[0] and v.first_bad == (10 if tamper else None)


def test_parallel_decode_reports_lowest_bad_entry(tmp_path, chain, monkeypatch):
    _, _, bs = chain
    items = _items(bs) * 2
    items = [(struct.pack(">Q", i + 1), ingest.beacon_to_json(Beacon(b.previous_sig, i + 1, b.signature)))
             for i, (_, v) in enumerate(items) for b in [ingest.beacon_from_json(v)]]
    items[35] = (items[35][0], b'{"Round":36,"Signature":"0g"}')
    items[30] = (items[30][0], b'{"Round":31,"PreviousSig":"abc"}')
    p = tmp_path / "par.db"
    write_db(p, items, per_leaf=2)
    monkeypatch.setenv("DL_THREADS", "4")
    with pytest.raises(boltdb.StoreError, match="entry 30"):
        boltdb.load_store(p)
    monkeypatch.setenv("DL_THREADS", "3")
    sb = boltdb.load_store(p, start=0, max_n=30)
    assert sb.rounds.tolist() == list(range(1, 31))


def _sharded_worker(rank, world, port, path, pk, q):
    import os
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fb, ok = boltdb.verify_store_sharded(OracleEngine(), pk, path)
        q.put((rank, fb, ok.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_verify_store_sharded_gloo(tmp_path, chain, world):
    """Row (e) over row (f): ranks split the stored entries, combine with one SUM all-reduce (gloo)."""
    import multiprocessing as mp
    import socket
    pk, _, bs = chain
    p = tmp_path / "s.db"
    tb = _tampered(bs)
    write_db(p, _items(tb), per_leaf=4)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, str(p), pk, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    rounds = [b.round for b in tb]
    want = [r not in (10, 16) for r in rounds]
    for _, fb, ok in res:
        assert fb == 10 and ok == want


def device_history_items(engine, golden, n, seg=64):
    """A device-generated chained history (bench.py's layout) as drand.db items: rows carry the
    PreviousSig the generator used (the segment seed at segment starts, else the previous sig)."""
    import torch
    g = golden["chained"]
    dev = torch.device("cuda", 0)
    engine.set_public_key(bytes.fromhex(g["pk"]))
    gen = torch.Generator(device=dev)
    gen.manual_seed(77)
    n_seg = (n + seg - 1) // seg
    seeds = torch.randint(0, 256, (n_seg * 96,), dtype=torch.uint8, device=dev, generator=gen)
    sigs = torch.empty(n * 96, dtype=torch.uint8, device=dev)
    engine.generate_chained_dev(int(g["sk"], 16).to_bytes(32, "big"), 1, seg, seeds.data_ptr(), 32, sigs.data_ptr(),
                                n, torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    S, Q = sigs.cpu().numpy().reshape(n, 96), seeds.cpu().numpy().reshape(n_seg, 96)
    items = []
    for i in range(n):
        if i % seg == 0:
            prev = Q[i // seg, :32 if i == 0 else 96].tobytes()
        else:
            prev = S[i - 1].tobytes()
        items.append((struct.pack(">Q", i + 1), ingest.beacon_to_json(Beacon(prev, i + 1, S[i].tobytes()))))
    return items


@pytest.mark.gpu
def test_verify_store_gpu_scale(tmp_path, golden, engine):
    """65,536 stored rounds (1,024 broken-linkage segments) in ONE device pass; then corruptions."""
    n = 65536
    items = device_history_items(engine, golden, n)
    p = tmp_path / "big.db"
    write_db(p, items, per_leaf=5)
    pk = bytes.fromhex(golden["chained"]["pk"])
    sb = boltdb.load_store(p)
    assert len(sb) == n and len(boltdb.linked_runs(sb)) == n // 64 and boltdb.round_runs(sb).tolist() == [0]
    v = boltdb.verify_store(engine, pk, sb)
    assert v.ok.all() and v.first_bad is None and v.runs == 1
    # corrupt rows in memory: a flipped bit, a cleared flag, a wrong stored prev; rows after them keep
    # their own (unchanged) stored prev, so only the tampered rows reject
    sb.sigs[1000, 50] ^= 1
    sb.sigs[40000, 0] &= 0x7F
    sb.prev[50001, 7] ^= 0x80
    sb.sig_len[60000] = 95
    v = boltdb.verify_store(engine, pk, sb)
    assert np.flatnonzero(~v.ok).tolist() == [1000, 40000, 50001, 60000] and v.first_bad == 1001
