"""Latency of the per-arrival callers on one MI355X:

  lone VerifyRecovered  (chain.VerifyBeacon of one beacon, node.go / validator.go arrival path)
  lone VerifyPartial    (one partial of a round, chain/beacon/node.go:112,125)
  64 VerifyPartial      (one round's partials in one call)
  aggregator round      (blsv_aggregate: 64 partials, Recover from 33, VerifyRecovered)

Each is the median wall clock over `reps` calls from the host API, plus the per-stage GPU time of
one call (HIP events on the launch stream, blsv_profile_*) and, for the lone verify, the phase marks
of the latency kernel (blsv_lat_trace). Inputs are the committed golden vectors
(tests/golden/golden.json); every result is checked against them. The C oracle's single-thread lone
verify of the same beacon is timed on the same host as the CPU baseline.

--sweep N1,N2,..: also time blsv_verify_messages of N distinct device-signed messages through the
latency path and through the batch pipeline (the BLSV_LAT_MAX cutover is where they cross).

usage: python tools/latency_bench.py [--reps 20] [--out profiles/r02_latency.json] [--sweep 64,512]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed(fn, reps):
    lat = []
    for k in range(reps + 2):
        t0 = time.perf_counter()
        fn()
        dt = (time.perf_counter() - t0) * 1e3
        if k >= 2:
            lat.append(dt)
    return round(statistics.median(lat), 3), round(min(lat), 3)


def stages(eng, fn):
    eng.profile(True)
    eng.profile_read()
    fn()
    eng.synchronize()
    got = eng.profile_read()
    eng.profile(False)
    return {k: round(v[0], 3) for k, v in got.items() if v[1]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--out", default=None)
    ap.add_argument("--lat-max", type=int, default=None,
                    help="latency-path cutover for this run (0 = batch pipeline only; default: the library's)")
    ap.add_argument("--sweep", default="", help="batch sizes for the latency-vs-batch crossover")
    ap.add_argument("--agg-only", type=int, default=0,
                    help="run only the aggregator round this many times (under rocprofv3 --kernel-trace)")
    a = ap.parse_args()
    from drand_amd.engine import Engine

    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        g = json.load(f)
    ch, th = g["chained"], g["threshold"]
    sigs = [bytes.fromhex(b["sig"]) for b in ch["beacons"]]
    seed = bytes.fromhex(ch["genesis_seed"])
    commits = [bytes.fromhex(c) for c in th["commits"]]
    msg = bytes.fromhex(th["msg"])
    partials = [bytes.fromhex(p) for p in th["partials"]]
    out = {}
    with Engine(0) as eng:
        if a.lat_max is not None:
            eng.set_lat_max(a.lat_max)
        cur = eng.set_lat_max(0)
        eng.set_lat_max(cur)
        out["lat_max"] = cur
        eng.set_public_key(bytes.fromhex(ch["pk"]))
        if a.agg_only:
            eng.set_group(commits, th["n"])
            for _ in range(a.agg_only):
                ok, _, sig, gok = eng.aggregate(msg, partials, th["t"], th["n"])
                assert all(ok) and gok and sig.hex() == th["group_sig"]
            print("aggregate rounds:", a.agg_only)
            return

        def lone_beacon():
            r = eng.verify_chained(2, sigs[0], [sigs[1]])
            assert r.ok == [True]

        med, mn = timed(lone_beacon, a.reps)
        out["lone_verify_beacon"] = {"median_ms": med, "min_ms": mn, "stages_ms": stages(eng, lone_beacon)}
        eng.lat_trace_enable(True)
        eng.lat_trace(clear=True)
        lone_beacon()
        out["lone_verify_beacon"]["phases_us"] = {k: round(v, 1) for k, v in eng.lat_trace().items()}
        eng.lat_trace_enable(False)

        eng.set_group(commits, th["n"])

        def lone_partial():
            ok, _ = eng.verify_partials(msg, partials[:1])
            assert ok == [True]

        med, mn = timed(lone_partial, a.reps)
        out["lone_verify_partial"] = {"median_ms": med, "min_ms": mn, "stages_ms": stages(eng, lone_partial)}

        def round_partials():
            ok, _ = eng.verify_partials(msg, partials)
            assert all(ok)

        med, mn = timed(round_partials, a.reps)
        out["verify_partials_64"] = {"median_ms": med, "min_ms": mn, "stages_ms": stages(eng, round_partials)}

        def agg():
            ok, _, sig, gok = eng.aggregate(msg, partials, th["t"], th["n"])
            assert all(ok) and gok and sig.hex() == th["group_sig"]

        med, mn = timed(agg, a.reps)
        out["aggregate_round_n64_t33"] = {"median_ms": med, "min_ms": mn, "stages_ms": stages(eng, agg)}
        if a.sweep:
            import hashlib
            sk32 = int(ch["sk"], 16).to_bytes(32, "big")
            pk = bytes.fromhex(ch["pk"])
            cur = eng.set_lat_max(0)
            eng.set_lat_max(cur)
            sweep = []
            for n in [int(x) for x in a.sweep.split(",")]:
                msgs = [hashlib.sha256(b"sweep %d" % i).digest() for i in range(n)]
                msigs = eng.sign(sk32, msgs)
                row = {"n": n}
                for name, lm in (("lat_ms", 1 << 40), ("batch_ms", 0)):
                    eng.set_lat_max(lm)

                    def call():
                        r = eng.verify_messages(msgs, msigs, pk48=pk)
                        assert all(r.ok)

                    row[name] = timed(call, 3)[0]
                sweep.append(row)
                print(json.dumps(row), flush=True)
            eng.set_lat_max(cur)
            out["cutover_sweep"] = sweep
    # CPU baseline of the same lone call: the C oracle (oracle/c/bls_oracle.c, a plain-C port of the
    # kilic algorithms without its assembly) on ONE host thread -- what one kyber verify per arrival
    # costs a core, to set beside the GPU's per-arrival latency
    from oracle import c_oracle  # checker / baseline only
    c_oracle.load()
    pk48 = bytes.fromhex(ch["pk"])

    def cpu_lone():
        assert c_oracle.verify_chained(pk48, 2, sigs[0], sigs[1]) == [0]

    med, mn = timed(cpu_lone, max(3, a.reps // 2))
    out["cpu_lone_verify_beacon"] = {"median_ms": med, "min_ms": mn, "threads": 1, "kind": "port (C oracle)"}
    line = json.dumps(out)
    print(line)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
