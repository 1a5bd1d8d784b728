"""Measurements for BASELINE.json configs[2] and configs[4] on one MI355X (bench.py covers configs[1]).

configs[2] threshold round: n = 64 / t = 33 partials of the golden threshold fixture. One aggregator
round of chain/beacon/chain.go:119-166 = verify all 64 partials (node.go:112) + Recover from 33 +
VerifyRecovered of the group signature. Reports the median wall-clock latency per round.

configs[4] mixed batch: a device-generated 1M-round chained history (bench.py's layout: segments of
64 rounds, golden key) with a seeded 0.1 % of signatures corrupted on device (bit flip in x, cleared
compression flag, infinity encoding, x >= p, a valid signature of another round, an on-curve point
outside G2 and an x with no point on the curve -- the last two taken from the golden mixed batch). The verdict
bitmap must equal the expectation exactly: a corrupted sig_i rejects round i and, inside its
segment, round i + 1 (whose message hashes the corrupted bytes); first_bad = the minimum. Reports
beacons/s over the mixed batch.

Prints one JSON line. Usage: python tools/config_bench.py [--n 1000000] [--reps 20]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)  # bench.host_cores, oracle.c_oracle (CPU baseline leg)


def threshold_round(eng, th, reps):
    commits = [bytes.fromhex(c) for c in th["commits"]]
    msg = bytes.fromhex(th["msg"])
    partials = [bytes.fromhex(p) for p in th["partials"]]
    sub = [bytes.fromhex(p) for p in th["recover_subset"]]
    eng.set_group(commits, th["n"])
    lat = []
    for k in range(reps + 2):
        t0 = time.perf_counter()
        ok, _ = eng.verify_partials(msg, partials)
        sig = eng.recover(msg, sub, th["t"], th["n"])
        res = eng.verify_messages([msg], [sig])
        dt = time.perf_counter() - t0
        assert all(ok) and res.ok == [True] and sig.hex() == th["group_sig"]
        if k >= 2:
            lat.append(dt * 1e3)
    fused = []
    for k in range(reps + 2):
        t0 = time.perf_counter()
        ok, _, sig, gok = eng.aggregate(msg, partials, th["t"], th["n"])
        dt = time.perf_counter() - t0
        assert all(ok) and gok and sig.hex() == th["group_sig"]
        if k >= 2:
            fused.append(dt * 1e3)
    return {"n": th["n"], "t": th["t"], "median_ms_per_round": round(statistics.median(lat), 3),
            "min_ms": round(min(lat), 3), "reps": reps, "bit_exact_group_sig": True,
            "three_calls": "verify_partials + recover + verify_messages",
            "fused_blsv_aggregate_median_ms": round(statistics.median(fused), 3),
            "cpu_baseline": threshold_round_cpu(th, reps=3)}


def threshold_round_cpu(th, reps):
    """The same round on the host: the C oracle (oracle/c/bls_oracle.c, kind "port") with the 64
    VerifyPartial calls (node.go:112, PubPoly.Eval per call as kyber tbls does) spread over all usable
    cores, then tbls.Recover (which re-verifies shares one by one until t are valid, as kyber's does)
    and VerifyRecovered on one core. Bench-side baseline only; never on the product path."""
    from concurrent.futures import ThreadPoolExecutor

    from bench import host_cores
    from oracle import c_oracle  # CPU baseline leg only

    cores, host = host_cores()
    commits = [bytes.fromhex(c) for c in th["commits"]]
    msg = bytes.fromhex(th["msg"])
    partials = [bytes.fromhex(p) for p in th["partials"]]
    sub = [bytes.fromhex(p) for p in th["recover_subset"]]
    pk = commits[0]
    g = c_oracle.Group(commits)
    lat = []
    with ThreadPoolExecutor(cores) as ex:
        for _ in range(reps):
            t0 = time.perf_counter()
            cls = list(ex.map(lambda p: g.verify_partial(msg, p), partials))
            sig = g.recover(msg, sub, th["t"], th["n"])
            ok = c_oracle.verify(pk, msg, sig)
            lat.append((time.perf_counter() - t0) * 1e3)
            assert cls == [0] * len(partials) and sig.hex() == th["group_sig"] and ok == 0
    g.close()
    return {"median_ms_per_round": round(statistics.median(lat), 1), "cores": cores, "kind": "port",
            "host": host, "steps": "64 VerifyPartial over %d threads + Recover(33, re-verifying) + VerifyRecovered"
            % cores}


def mixed_batch(eng, g, mixed, n, seg, steps):
    import torch
    dev = torch.device("cuda", 0)
    sk32 = int(g["sk"], 16).to_bytes(32, "big")
    eng.set_public_key(bytes.fromhex(g["pk"]))
    n_seg = (n + seg - 1) // seg
    gen = torch.Generator(device=dev)
    gen.manual_seed(0x5EED5)
    seeds = torch.randint(0, 256, (n_seg * 96,), dtype=torch.uint8, device=dev, generator=gen)
    sigs = torch.empty(n * 96, dtype=torch.uint8, device=dev)
    bitmap = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
    first_bad = torch.empty(1, dtype=torch.int64, device=dev)
    sp = torch.cuda.current_stream(dev).cuda_stream
    eng.generate_chained_dev(sk32, 1, seg, seeds.data_ptr(), 32, sigs.data_ptr(), n, sp)
    torch.cuda.synchronize(dev)

    rng = torch.Generator()
    rng.manual_seed(1234)
    k = max(1, n // 1000)
    idx = torch.randperm(n, generator=rng)[:k].sort().values
    s2 = sigs.view(n, 96)
    p_bytes = bytes.fromhex("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab")
    p_t = torch.tensor(list(p_bytes), dtype=torch.uint8, device=dev)
    def golden_of_class(c):  # a signature of the golden mixed batch with reject class c
        return torch.tensor(list(bytes.fromhex(mixed["sigs"][mixed["expect_class"].index(c)])), dtype=torch.uint8,
                            device=dev)

    not_in_g2, not_on_curve = golden_of_class(6), golden_of_class(5)
    kinds = {}
    kind_of = {}
    for j, i in enumerate(idx.tolist()):
        kind = j % 7
        kinds[kind] = kinds.get(kind, 0) + 1
        kind_of[i] = kind
        if kind == 0:                                       # bit flip in x
            s2[i, 60] ^= 0x10
        elif kind == 1:                                     # compression flag cleared
            s2[i, 0] &= 0x7F
        elif kind == 2:                                     # infinity encoding (valid point, fails pairing)
            s2[i].zero_()
            s2[i, 0] = 0xC0
        elif kind == 3:                                     # x.c0 = p (non-canonical)
            s2[i, 48:96] = p_t
        elif kind == 4:                                     # a valid signature of another round
            s2[i] = s2[(i + 7) % n].clone()
        elif kind == 5:                                     # on the curve, outside G2 (subgroup check)
            s2[i] = not_in_g2
        else:                                               # x with no curve point
            s2[i] = not_on_curve
    torch.cuda.synchronize(dev)
    bad = set(idx.tolist())
    expect_bad = set(bad)
    for i in bad:
        if i + 1 < n and (i + 1) % seg != 0:
            expect_bad.add(i + 1)

    cls = torch.empty(n, dtype=torch.uint8, device=dev)
    eng.verify_chained_dev(1, seg, seeds.data_ptr(), 32, sigs.data_ptr(), n, bitmap.data_ptr(),
                           first_bad.data_ptr(), cls.data_ptr(), sp)
    torch.cuda.synchronize(dev)
    # reject class per injected kind (include/blsverify.h BLSV_REJ_*); a bit flip lands on any class
    want_cls = {1: 2, 2: 7, 3: 4, 4: 7, 5: 6, 6: 5}
    cl = cls.cpu().numpy()
    for i, kind in kind_of.items():
        if kind in want_cls and not (kind == 4 and (i + 7) % n < i):  # a wrapped copy may be corrupted itself
            assert cl[i] == want_cls[kind], (i, kind, int(cl[i]))
        else:
            assert cl[i] != 0, (i, kind)
    for i in expect_bad - bad:
        assert cl[i] == 7, (i, int(cl[i]))  # the successor's message hashes the corrupted bytes

    def step():
        eng.verify_chained_dev(1, seg, seeds.data_ptr(), 32, sigs.data_ptr(), n, bitmap.data_ptr(),
                               first_bad.data_ptr(), None, sp)

    step()
    torch.cuda.synchronize(dev)
    bm = bitmap.cpu().numpy().view("uint64")
    import numpy as np
    bits = np.unpackbits(bm.view(np.uint8), bitorder="little")[:n]
    got_bad = set(np.flatnonzero(bits == 0).tolist())
    assert got_bad == expect_bad, (len(got_bad), len(expect_bad))
    fb = int(first_bad.item()) & (2 ** 64 - 1)
    assert fb == min(expect_bad) + 1, (fb, min(expect_bad) + 1)   # first_bad is a ROUND (round = index + 1)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    return {"n": n, "segment_len": seg, "corrupted": k, "rejected": len(expect_bad), "kinds": kinds,
            "bitmap_exact": True, "reject_classes_exact": True, "first_bad_round": fb, "beacons_per_s": round(n * steps / dt, 1),
            "ms_per_batch": round(dt * 1e3 / steps, 3)}


def store_check(eng, golden, n, path):
    """§8f rank 2 end to end: a drand.db of n device-generated rounds (segments of 64, so linkage
    breaks every 64 rounds) is loaded by libboltload and verified by blsv_verify_prevs in one pass.
    The file is written outside the timed region (fixture creation)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from drand_amd import boltdb
    from support.boltwriter import write_db
    from test_boltdb import device_history_items
    t0 = time.perf_counter()
    write_db(path, device_history_items(eng, golden, n), per_leaf=5)
    t_write = time.perf_counter() - t0
    pk = bytes.fromhex(golden["chained"]["pk"])
    boltdb.verify_store(eng, pk, boltdb.load_store(path, max_n=4096))   # warm-up
    t0 = time.perf_counter()
    sb = boltdb.load_store(path)
    t_load = time.perf_counter() - t0
    t0 = time.perf_counter()
    v = boltdb.verify_store(eng, pk, sb)
    t_verify = time.perf_counter() - t0
    assert v.ok.all() and v.runs == 1 and len(sb) == n
    os.remove(path)
    return {"n": n, "file_mb": None, "write_s": round(t_write, 2), "load_s": round(t_load, 3),
            "verify_s": round(t_verify, 3), "load_threads": min(16, os.cpu_count() or 1),
            "beacons_per_s_end_to_end": round(n / (t_load + t_verify), 1),
            "note": "verify includes the host->device copy of prev+sig rows (192 B/beacon)"}


def partials_many_rounds(eng, golden, n):
    """Partials of n different rounds in one blsv_verify_partials_multi pass (t = 1 group of the
    golden key; partials signed on device by blsv_sign with share index 0)."""
    import hashlib
    g = golden["chained"]
    sk32 = int(g["sk"], 16).to_bytes(32, "big")
    eng.set_group([bytes.fromhex(g["pk"])], 1)
    msgs = [hashlib.sha256(r.to_bytes(8, "big")).digest() for r in range(1, n + 1)]
    parts = eng.sign(sk32, msgs, index=0)
    ok, _ = eng.verify_partials_multi(msgs[:1024], parts[:1024])   # warm-up
    t0 = time.perf_counter()
    ok, _ = eng.verify_partials_multi(msgs, parts)
    dt = time.perf_counter() - t0
    assert all(ok)
    return {"n": n, "partials_per_s": round(n / dt, 1), "s": round(dt, 3),
            "note": "host-buffer entry point: includes staging copies and ctypes packing"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--seg-len", type=int, default=64)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--partials-n", type=int, default=262144, help="partials in the many-rounds leg (0 = skip)")
    ap.add_argument("--store-n", type=int, default=1_000_000, help="rounds in the drand.db leg (0 = skip)")
    args = ap.parse_args()
    from drand_amd.engine import Engine
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        golden = json.load(f)
    eng = Engine(0)
    out = {"configs[2]_threshold_round": threshold_round(eng, golden["threshold"], args.reps),
           "configs[4]_mixed_batch": mixed_batch(eng, golden["chained"], golden["mixed"], args.n, args.seg_len,
                                                  args.steps)}
    if args.partials_n:
        out["configs[2]_partials_many_rounds"] = partials_many_rounds(eng, golden, args.partials_n)
    if args.store_n:
        out["configs[f2]_store_check"] = store_check(eng, golden, args.store_n, "/tmp/drand_amd_bench.db")
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
