"""Benchmark: drand chained-beacon batch verification (chain.VerifyBeacon semantics) on MI355X.

Metric (BASELINE.json): beacons verified/s (batch chain verify) at 1/2/4/8 MI355X vs host-CPU.

Default workload at N=1 = BASELINE.json configs[1]: a 1,000,000-round synthetic chained beacon
history verified on one MI355X, one pairing-product check per round. Per rank the history is
generated on the device (client/test/result/mock/result.go:98-132 recipe: single key, seeded prev)
as independently seeded chained segments of --seg-len rounds (a continuous 1M chain
is inherently sequential to SIGN; verification work per round is identical either way). With N>1
each rank verifies its own --n rounds (weak scaling).

--total-rounds T = configs[3] (strong scaling): ONE T-round history (same segment layout, segment
seeds drawn from one fixed generator, identical on every rank) split into contiguous shard ranges
(drand_amd/shard.py shard_range, NOT 64-aligned in general). Each rank generates its range plus the
head of the segment it starts in, so the halo it hands the verifier as seeds[0] (seg_phase) is the
true previous signature of its first round. --slice R/W runs rank R of a W-way split in a single
process (the 12.5M-round slice of configs[3] on one GPU).

One step = one blsv_verify_chained_dev call over the rank's whole HBM-resident shard (hash-to-G2,
decompress + subgroup, 2-pair Miller loop, final exponentiation, verdict bitmap + first bad round),
followed for N>1 by the exchange: ONE SUM all-reduce over RCCL of a zero-initialised buffer holding
the verdict bits at global positions plus one first-bad-round slot per rank (shard.combine).

Ranks: with --gpus N > 1 and no WORLD_SIZE in the environment, this process starts the N ranks
itself as a child `python -m torch.distributed.run --nproc-per-node N ...` (before anything here
touches the GPU) and exits with its status; every rank asserts world_size == --gpus. With
--dist-backend gloo the exchange runs through host copies and ranks may share a GPU (rank r on
cuda:(r mod device_count)) -- the -m gpu test runs 2 ranks on one MI355X that way.

Correctness gate before timing: every round verifies, then a negative control -- one signature per
rank corrupted (bit flip in x) must make exactly that round and the next one reject, with first_bad
= the lowest corrupted round over all ranks.

Usage: python bench.py [--gpus N --steps K --warmup W --n BEACONS_PER_GPU]
       python bench.py --gpus 8 --total-rounds 100000000          (configs[3], 8 ranks over RCCL)
       python bench.py --total-rounds 100000000 --slice 7/8      (one shard of it in one process)
       (or launched per rank: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

LIMB_PRODUCTS_PER_FP_MUL = 288  # algorithmic unit: 12x32-bit Montgomery = 144 (a*b) + 144 (m*p) limb products
PMC_FILE = "r06z_pmc_traffic.json"


def load_json(rel):
    with open(os.path.join(ROOT, rel)) as f:
        return json.load(f)


def host_cores():
    """Host cores this process may actually use: the CPUs in its affinity mask, capped by the cgroup
    CPU quota (the GPU box pins a 16-CPU quota on a many-core host: threads beyond it only queue).
    Returns (cores, facts) with the nproc / affinity / quota / model behind the choice."""
    affinity = len(os.sched_getaffinity(0))
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(path) as f:
                q, per = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
        except (OSError, ValueError):
            pass
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    cores = affinity if quota is None else max(1, min(affinity, int(quota + 0.999)))
    return cores, {"nproc": os.cpu_count(), "affinity": affinity, "cgroup_cpu_quota": quota, "cpu_model": model}


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


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """Start n ranks of this script under torch.distributed.run as a CHILD process (never an exec:
    this process has not touched the GPU, and the ranks must each initialise their own) and return
    its exit status."""
    port = free_port()
    # torch.distributed.run's parser would take "--n" as an abbreviation of its own options
    argv = ["--beacons-per-gpu" if a == "--n" else "--beacons-per-gpu=" + a[4:] if a.startswith("--n=") else a
            for a in sys.argv[1:]]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % n,
           "--master-addr=127.0.0.1", "--master-port=%d" % port, os.path.abspath(__file__)] + argv
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL (the box's driver)
    return subprocess.call(cmd, env=env)


def launch_check(args, world, rank):
    """--launch-check: the N-rank plumbing without a GPU (gloo on host tensors): process group of
    --gpus ranks, then one shard.combine exchange of a synthetic verdict bitmap with one rejected
    round in the last rank's shard."""
    import torch
    import torch.distributed as dist

    from drand_amd import shard

    if world > 1:
        dist.init_process_group("gloo")
        assert dist.get_world_size() == args.gpus
    total = args.total_rounds or args.n * world
    counts = [shard.shard_range(total, world, r).count for r in range(world)] if args.total_rounds else [args.n] * world
    n = counts[rank]
    bad = total - 2  # global index of the rejected round
    start = sum(counts[:rank])
    ok = [start + i != bad for i in range(n)]
    words = [0] * ((n + 63) // 64)
    for i, v in enumerate(ok):
        words[i // 64] |= v << (i % 64)
    w = torch.tensor([x - (1 << 64) if x >= 1 << 63 else x for x in words], dtype=torch.int64)
    fb = start + 1 + ok.index(False) if False in ok else shard.NONE_U64
    if world > 1:
        fbv, gw = shard.combine(fb, w, n, counts=counts)
    else:
        fbv, gw = fb, words
    print(json.dumps({"rank": rank, "world_size": world, "gpus": args.gpus, "counts": counts,
                      "first_bad": fbv, "rejected": [i for i in range(total) if not (gw[i // 64] >> (i % 64)) & 1]}),
          flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", "--beacons-per-gpu", dest="n", type=int, default=1_000_000,
                    help="beacons per GPU (configs[1]: 1M)")
    ap.add_argument("--total-rounds", type=int, default=0,
                    help="strong scaling (configs[3]): one history of this many rounds split over the ranks")
    ap.add_argument("--slice", default="", help="R/W: verify shard R of a W-way split in this one process")
    ap.add_argument("--seg-len", type=int, default=64, help="rounds per independently seeded chained segment")
    ap.add_argument("--cpu-per-worker", type=int, default=384, help="C-oracle beacons per host thread (0 = skip)")
    ap.add_argument("--cpu-workers", type=int, default=0, help="host threads for the CPU baseline (0 = all usable cores)")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="exchange backend for N>1: nccl (= RCCL over xGMI, one GPU per rank) or gloo (host "
                         "copies; ranks may share a GPU)")
    ap.add_argument("--force-pg", action="store_true",
                    help="form the --dist-backend process group and run the exchange (shard.combine) even at one "
                         "rank: executes the RCCL branch on a one-GPU box (world size 1)")
    ap.add_argument("--launch-check", action="store_true",
                    help="start the ranks, form the process group, run one exchange on host tensors and print "
                         "one JSON line per rank, without touching a GPU (CPU test of the N-rank launch)")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))

    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: every rank must run with --gpus = "
                         "the number of ranks")
    if args.launch_check:
        return launch_check(args, world, rank)
    ndev = torch.cuda.device_count()  # does not initialise the GPU on this image
    if world > 1 and args.dist_backend == "nccl" and ndev < world:
        raise SystemExit(f"bench.py: {world} RCCL ranks need {world} GPUs, this node shows {ndev} "
                         "(--dist-backend gloo lets ranks share a GPU)")
    dev_idx = local % max(ndev, 1)
    use_pg = world > 1 or args.force_pg
    if use_pg:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1:  # --force-pg without a launcher: a one-rank group by env init
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
            os.environ.setdefault("MASTER_PORT", str(free_port()))
        torch.cuda.set_device(dev_idx)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_idx))
        else:
            dist.init_process_group("gloo")
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)
    else:
        torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)
    # One explicit stream for the engine AND the torch ops around it (the exchange's placement and
    # all-reduce): the C ABI's NULL stream means the context's own non-blocking stream, which torch's
    # default stream does not wait for.
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    assert sp, "the engine stream must be an explicit stream"

    from drand_amd import shard
    from drand_amd.engine import Engine

    g = load_json("tests/golden/golden.json")["chained"]  # fixed test key (sk, pk) of the golden chain
    sk32 = int(g["sk"], 16).to_bytes(32, "big")
    pk48 = bytes.fromhex(g["pk"])
    opc = load_json("profiles/opcount.json")["fp_mul"]
    seg = args.seg_len

    strong = args.total_rounds > 0
    if args.slice:
        s_rank, s_world = (int(x) for x in args.slice.split("/"))
        assert world == 1 and strong and 0 <= s_rank < s_world, "--slice R/W needs --total-rounds and one process"
    else:
        s_rank, s_world = rank, world
    if strong:
        sl = shard.segmented_slice(args.total_rounds, s_world, s_rank, seg)
        counts = [shard.shard_range(args.total_rounds, s_world, r).count for r in range(s_world)]
        n = sl.shard.count
        first_round = sl.shard.first_round
        gen_first_round = sl.gen_start + 1
        # every rank draws the SAME global seed table and keeps its segments' rows
        n_seg_total = (args.total_rounds + seg - 1) // seg
        gen = torch.Generator(device=dev)
        gen.manual_seed(0xD7A4D)
        all_seeds = torch.randint(0, 256, (n_seg_total, 96), dtype=torch.uint8, device=dev, generator=gen)
        gen_seeds = all_seeds[sl.seg_first:sl.seg_first + sl.n_seg].contiguous()
        del all_seeds
        gen_seed0_len = 32 if sl.seg_first == 0 else 96
        gen_n = sl.gen_count
        phase = sl.phase
    else:
        n = args.n
        counts = [n] * world
        first_round = gen_first_round = rank * n + 1  # contiguous round range per rank
        gen_seed0_len = 32 if rank == 0 else 96  # round 1 hashes the 32-byte genesis seed (client/verify.go:122)
        gen = torch.Generator(device=dev)
        gen.manual_seed(0xD7A4D + rank)
        gen_seeds = torch.randint(0, 256, ((n + seg - 1) // seg, 96), dtype=torch.uint8, device=dev, generator=gen)
        gen_n = n
        phase = 0
    seed0_len = 32 if first_round == 1 else 96
    gen_sigs = torch.empty((max(gen_n, 1), 96), dtype=torch.uint8, device=dev)
    words = (n + 63) // 64
    bitmap = torch.zeros(words, dtype=torch.int64, device=dev)
    first_bad = torch.empty(1, dtype=torch.int64, device=dev)

    eng = Engine(dev_idx)
    eng.set_public_key(pk48)
    t_gen = time.perf_counter()
    eng.generate_chained_dev(sk32, gen_first_round, seg, gen_seeds.data_ptr(), gen_seed0_len, gen_sigs.data_ptr(),
                             gen_n, sp)
    torch.cuda.synchronize(dev)
    t_gen = time.perf_counter() - t_gen
    sigs = gen_sigs[phase:phase + n]  # the rank's shard (phase = 0 in weak mode)
    seeds = shard.local_seeds(sl, gen_seeds, gen_sigs) if strong else gen_seeds

    def step():
        eng.verify_chained_dev(first_round, seg, seeds.data_ptr(), seed0_len, sigs.data_ptr(), n,
                               bitmap.data_ptr(), first_bad.data_ptr(), None, sp, seg_phase=phase)
        if use_pg:
            # ONE SUM all-reduce: global-position bitmap + per-rank first bad ROUND slots (RCCL over xGMI)
            return shard.combine(first_bad, bitmap, n, to_host=False, counts=counts)
        return first_bad, bitmap

    def verdicts():
        fb, bm = step()
        torch.cuda.synchronize(dev)
        total = sum(counts) if use_pg else n
        ok = np.unpackbits(bm.cpu().numpy().view(np.uint8), bitorder="little")[:total].astype(bool)
        fbv = int(fb.item()) & (2 ** 64 - 1)
        return (None if fbv in (2 ** 64 - 1, shard.NONE_I64) else fbv), ok

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    # correctness gate 1: every generated round verifies
    fbv, ok = verdicts()
    assert fbv is None and ok.all(), f"verification failed: first_bad={fbv} rejected={int((~ok).sum())}"
    # gate 2 (negative control): one corrupted signature per rank -> exactly it and its successor reject
    def bad_index(count, ph):  # a round whose successor is in the same segment (its prev = the bad sig)
        b = count // 2
        return b - 1 if b > 0 and (b + 1 + ph) % seg == 0 else b

    if strong:
        phases = [shard.segmented_slice(args.total_rounds, s_world, r, seg).phase for r in range(s_world)]
    else:
        phases = [0] * world
    bad_i = bad_index(n, phase)
    saved = sigs[bad_i].clone()
    sigs[bad_i, 50] ^= 1  # bit flip in x.c0
    fbv, ok = verdicts()
    sigs[bad_i].copy_(saved)
    gate = list(zip(counts, phases)) if use_pg else [(n, phase)]
    want = np.ones(len(ok), bool)
    for r, (c, ph) in enumerate(gate):
        off, b = sum(x[0] for x in gate[:r]), bad_index(c, ph)
        want[off + b] = False
        if b + 1 < c:
            want[off + b + 1] = False
    want_fb = (first_round - (sum(counts[:rank]) if use_pg else 0)) + bad_index(*gate[0])
    assert (ok == want).all() and fbv == want_fb, f"negative control failed: first_bad={fbv} want {want_fb} " \
        f"rejected={np.flatnonzero(~ok)[:8].tolist()}"

    eng.profile(True)
    eng.profile_read()
    if use_pg:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if use_pg:
        dist.barrier()
    dt = time.perf_counter() - t0
    prof = eng.profile_read()
    eng.profile(False)
    if use_pg:  # the job's time is the slowest rank's
        t = torch.tensor([dt], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    total = (sum(counts) if use_pg else n) * args.steps
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

    if strong:
        workload = {"workload": "configs[3]: one %d-round chained history split in %d contiguous range shards%s, "
                                "chain.VerifyBeacon per round, true previous-signature halo per shard"
                                % (args.total_rounds, s_world, " (this process: shard %d, rounds %d..%d)"
                                   % (s_rank, first_round, first_round + n - 1) if args.slice else ""),
                    "total_rounds": args.total_rounds, "shard_rounds": n, "segment_len": seg, "seg_phase": phase,
                    "parallelism": "range-shard x%d" % s_world}
    else:
        workload = {"workload": "configs[1]: %d-round chained beacon history per GPU, chain.VerifyBeacon per round"
                                % n, "beacons_per_gpu": n, "segment_len": seg, "parallelism": "range-shard x%d" % world}
    out = {
        "metric": "beacons verified/s (batch chain verify)",
        "value": round(value, 1),
        "unit": "beacons/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "u32 (381-bit Montgomery, 12x32-bit limbs)",
        "data": "synthetic (device-generated chained beacons, seeded key = golden fixture key)",
        "config": workload,
        "roofline": {"bound": "valu", "kernel": dom, "achieved": round(achieved, 3), "peak": round(peak, 3),
                     "unit": "T limb-products/s (v_mad_u64_u32)", "frac": round(achieved / peak, 4),
                     "traffic": traffic,
                     "traffic_unit": "bytes per launch (rocprofv3 PMC, profiles/%s)" % PMC_FILE if traffic else None,
                     "algorithmic_limb_products_per_beacon": per_beacon_fp_mul * LIMB_PRODUCTS_PER_FP_MUL,
                     "whole_pipeline_frac": round(value / world * per_beacon_fp_mul * LIMB_PRODUCTS_PER_FP_MUL
                                                  / (peak * 1e12), 4)},
        "stages_ms_per_launch": {s: round(v["ms_per_launch"], 3) for s, v in stages.items()},
        "generate_s": round(t_gen, 2),
        "gate": "all rounds accept; negative control (one bit-flipped signature per rank) rejects exactly it and "
                "the next round, first_bad = lowest corrupted round",
    }
    if use_pg:  # what the process group actually initialised (the exchange runs over it)
        devs = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        if args.dist_backend == "gloo":
            dist.all_gather(devs, torch.tensor([dev_idx]))
        out["dist"] = {"backend": str(dist.get_backend()), "world_size": dist.get_world_size(),
                       "rank_counts": counts, "ranks_verified_rounds": sum(counts),
                       "exchange": "one all_reduce(SUM) of %d int64 words: the verdict bitmap at global bit "
                                   "positions (disjoint bits: SUM = OR) + %d first-bad-round slots"
                                   % ((sum(counts) + 63) // 64 + world, world),
                       "gate": "passed"}
        if args.dist_backend == "gloo":
            out["dist"]["devices"] = [int(d) for d in devs]
            if len({int(d) for d in devs}) < world:
                out["dist"]["note"] = "ranks share a GPU: a correctness run of the N-rank path, not a scaling number"
    if rank == 0 and world == 1 and args.cpu_per_worker > 0 and not strong:  # CPU baseline: rank 0 at N=1 only
        # bounded sample of the same workload: the first whole segments of the rank-0 shard
        cores, host = host_cores()
        workers = args.cpu_workers or cores
        n_seg_cpu = min(len(seeds), max(1, (workers * args.cpu_per_worker + seg - 1) // seg))
        m = min(n, n_seg_cpu * seg)
        sh = sigs[:m].cpu().numpy().tobytes()
        sd = seeds[:n_seg_cpu].cpu().numpy().tobytes()
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
                                         % (cnt, n_seg_cpu, workers),
                               "host": dict(host, usable_cores=cores)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if use_pg:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
