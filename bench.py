"""Benchmark: drand chained-beacon batch verification (chain.VerifyBeacon semantics) on MI355X.

Metric (BASELINE.json): beacons verified/s (batch chain verify) at 1/2/4/8 MI355X vs host-CPU.
Workload at N=1 = BASELINE.json configs[1]: a 1,000,000-round synthetic chained beacon history
verified on one MI355X, one pairing-product check per round. Per rank the history is generated on
the device (client/test/result/mock/result.go:98-132 recipe: single key, seeded prev) as
independently seeded chained segments of --seg-len rounds (a continuous 1M chain is
inherently sequential to SIGN; verification work per round is identical either way).

One step = one blsv_verify_chained_dev call over the rank's whole HBM-resident shard (hash-to-G2,
decompress + subgroup, 2-pair Miller loop, final exponentiation, verdict bitmap + first bad round),
followed for N>1 by the north_star's exchange: an all-reduce MIN of first_bad and an all-gather of
the per-shard verdict bitmaps over RCCL. Weak scaling: each rank verifies its own --n rounds of a
contiguous round range.

Usage: python bench.py [--gpus N --steps K --warmup W --n BEACONS_PER_GPU]
       (N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

LIMB_PRODUCTS_PER_FP_MUL = 288  # algorithmic unit: 12x32-bit Montgomery = 144 (a*b) + 144 (m*p) limb products
PMC_FILE = "r01_pmc_traffic.json"


def load_json(rel):
    with open(os.path.join(ROOT, rel)) as f:
        return json.load(f)


def cpu_baseline(pk48, segments, workers):
    """Time the C oracle (oracle/c/bls_oracle.c: the plain-C restatement of kyber/kilic
    verification -- the reference's Go verifier cannot run in this image) over `segments`, a list
    of (first_round, prev0, sigs) chained segments, spread over `workers` host threads (ctypes
    releases the GIL). Returns (beacons/s, number verified OK, number of beacons)."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import c_oracle  # cpu_baseline leg only

    c_oracle.load()
    jobs = [segments[w::workers] for w in range(workers)]

    def run(job):
        ok = 0
        for first_round, prev0, sigs in job:
            ok += sum(c == 0 for c in c_oracle.verify_chained(pk48, first_round, prev0, sigs))
        return ok

    n = sum(len(s[2]) // 96 for s in segments)
    with ThreadPoolExecutor(workers) as ex:
        t0 = time.perf_counter()
        oks = list(ex.map(run, jobs))
        dt = time.perf_counter() - t0
    return n / dt, sum(oks), n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=1_000_000, help="beacons per GPU (configs[1]: 1M)")
    ap.add_argument("--seg-len", type=int, default=64, help="rounds per independently seeded chained segment")
    ap.add_argument("--cpu-per-worker", type=int, default=384, help="C-oracle beacons per host thread (0 = skip)")
    ap.add_argument("--cpu-workers", type=int, default=16)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from drand_amd import shard
    from drand_amd.engine import Engine

    g = load_json("tests/golden/golden.json")["chained"]  # fixed test key (sk, pk) of the golden chain
    sk32 = int(g["sk"], 16).to_bytes(32, "big")
    pk48 = bytes.fromhex(g["pk"])
    opc = load_json("profiles/opcount.json")["fp_mul"]

    n = args.n
    seg = args.seg_len
    n_seg = (n + seg - 1) // seg
    first_round = rank * n + 1  # contiguous round range per rank
    seed0_len = 32 if rank == 0 else 96  # round 1 hashes the 32-byte genesis seed (client/verify.go:122)
    gen = torch.Generator(device=dev)
    gen.manual_seed(0xD7A4D + rank)
    seeds = torch.randint(0, 256, (n_seg * 96,), dtype=torch.uint8, device=dev, generator=gen)
    sigs = torch.empty(n * 96, dtype=torch.uint8, device=dev)
    words = (n + 63) // 64
    bitmap = torch.zeros(words, dtype=torch.int64, device=dev)
    first_bad = torch.empty(1, dtype=torch.int64, device=dev)

    eng = Engine(local)
    eng.set_public_key(pk48)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    t_gen = time.perf_counter()
    eng.generate_chained_dev(sk32, first_round, seg, seeds.data_ptr(), seed0_len, sigs.data_ptr(), n, sp)
    torch.cuda.synchronize(dev)
    t_gen = time.perf_counter() - t_gen

    def step():
        eng.verify_chained_dev(first_round, seg, seeds.data_ptr(), seed0_len, sigs.data_ptr(), n,
                               bitmap.data_ptr(), first_bad.data_ptr(), None, sp)
        if world > 1:
            # per-shard first bad ROUND -> global min; per-shard bitmaps -> every rank (RCCL over xGMI)
            return shard.combine(first_bad, bitmap, n, to_host=False)
        return first_bad, bitmap

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    # correctness gate: every generated round must verify
    fb, bm = step()
    torch.cuda.synchronize(dev)
    ones = int(sum(bin(int(x) & (2 ** 64 - 1)).count("1") for x in bm.cpu().tolist()))
    fbv = int(fb.item()) & (2 ** 64 - 1)
    assert fbv in (2 ** 64 - 1, shard.NONE_I64) and ones == n * world, \
        f"verification failed: first_bad={fbv} ones={ones}"

    eng.profile(True)
    eng.profile_read()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    prof = eng.profile_read()
    eng.profile(False)
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    total = n * world * args.steps
    value = total / dt
    ms_per_step = dt * 1e3 / args.steps

    # roofline of the dominant kernel: algorithmic limb products per launch / mean launch time
    try:
        peak_info = load_json("profiles/intrate.json")
    except FileNotFoundError:
        peak_info = {"peak_mad_u64_u32_per_s": float("nan")}
    stages = {}
    for s, (ms, launches, items) in prof.items():
        if launches:
            stages[s] = {"ms_per_launch": ms / launches, "launches": launches, "items_per_launch": items / launches}
    dom = max((s for s in stages if s in opc), key=lambda s: stages[s]["ms_per_launch"])
    d = stages[dom]
    achieved = opc[dom] * LIMB_PRODUCTS_PER_FP_MUL * d["items_per_launch"] / (d["ms_per_launch"] * 1e-3) / 1e12
    peak = peak_info["peak_mad_u64_u32_per_s"] / 1e12
    try:  # HBM bytes per beacon of each stage from the committed PMC passes (tools/pmc_traffic.py)
        tb = load_json("profiles/" + PMC_FILE)["bytes_per_beacon"][dom]["total"]
        traffic = round(tb * d["items_per_launch"])
    except (FileNotFoundError, KeyError):
        traffic = None
    per_beacon_fp_mul = sum(opc.values())

    out = {
        "metric": "beacons verified/s (batch chain verify)",
        "value": round(value, 1),
        "unit": "beacons/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32 (381-bit Montgomery, 12x32-bit limbs)",
        "data": "synthetic (device-generated chained beacons, seeded key = golden fixture key)",
        "config": {"workload": "configs[1]: %d-round chained beacon history per GPU, chain.VerifyBeacon per round"
                               % n, "beacons_per_gpu": n, "segment_len": seg, "parallelism": "range-shard x%d" % world},
        "roofline": {"bound": "valu", "kernel": dom, "achieved": round(achieved, 3), "peak": round(peak, 3),
                     "unit": "T limb-products/s (v_mad_u64_u32)", "frac": round(achieved / peak, 4),
                     "traffic": traffic,
                     "traffic_unit": "bytes per launch (rocprofv3 PMC, profiles/%s)" % PMC_FILE if traffic else None,
                     "algorithmic_limb_products_per_beacon": per_beacon_fp_mul * LIMB_PRODUCTS_PER_FP_MUL,
                     "whole_pipeline_frac": round(value / world * per_beacon_fp_mul * LIMB_PRODUCTS_PER_FP_MUL
                                                  / (peak * 1e12), 4)},
        "stages_ms_per_launch": {s: round(v["ms_per_launch"], 3) for s, v in stages.items()},
        "generate_s": round(t_gen, 2),
    }
    if rank == 0 and world == 1 and args.cpu_per_worker > 0:  # CPU baseline: rank 0 at N=1 only
        # bounded sample of the same workload: the first whole segments of the rank-0 shard
        workers = max(1, min(args.cpu_workers, os.cpu_count() or 1))
        n_seg_cpu = min(n_seg, max(1, (workers * args.cpu_per_worker + seg - 1) // seg))
        m = min(n, n_seg_cpu * seg)
        sh = sigs[: m * 96].cpu().numpy().tobytes()
        sd = seeds[: n_seg_cpu * 96].cpu().numpy().tobytes()
        segments = []
        for s_i in range(n_seg_cpu):
            lo, hi = s_i * seg, min(m, (s_i + 1) * seg)
            prev0 = sd[s_i * 96: s_i * 96 + (seed0_len if s_i == 0 else 96)]
            segments.append((first_round + lo, prev0, sh[lo * 96: hi * 96]))
        rate, ok, cnt = cpu_baseline(pk48, segments, workers)
        assert ok == cnt, "C oracle rejected device-generated beacons"
        out["cpu_baseline"] = {"value": round(rate, 1), "unit": "beacons/s", "cores": workers, "kind": "port",
                               "sample": "%d chained beacons (first %d segments of the rank-0 shard) verified by the C "
                                         "oracle (oracle/c/bls_oracle.c, kilic algorithms) on %d host threads"
                                         % (cnt, n_seg_cpu, workers)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
