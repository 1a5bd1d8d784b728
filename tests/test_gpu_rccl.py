"""The RCCL branch of the sharded exchange, executed on the one-GPU test box.

north_star's multi-GPU shape is one contiguous round range per GPU and ONE RCCL all-reduce of the
failure bitmap + first-bad slots (shard.combine). The 8-GPU run is the driver's; here a world-size-1
"nccl" process group executes exactly that branch -- the device-tensor all_reduce queued on the
engine's explicit stream behind blsv_verify_chained_dev -- and the exchanged bitmap and first bad
round must equal the single-process verdicts (and the corruption rule: a bad sig_i rejects round i
and round i + 1 unless i + 1 starts a segment). bench.py --force-pg runs the same branch inside the
bench's own gate and records dist.backend = nccl.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        env["MASTER_PORT"] = str(s.getsockname()[1])
    env["MASTER_ADDR"] = "127.0.0.1"
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def test_rccl_world1_exchange_equals_local_verdicts():
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "support", "rccl_world1.py")], cwd=ROOT,
                       env=_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    out = json.loads(r.stdout.strip().splitlines()[-1])
    print({k: out[k] for k in ("backend", "world_size", "rounds", "collective_words", "exchanged_first_bad")})
    assert out["backend"] == "nccl" and out["world_size"] == 1
    seg, n = out["seg_len"], out["rounds"]
    want = sorted({i for i in out["hit"]} | {i + 1 for i in out["hit"] if i + 1 < n and (i + 1) % seg})
    assert out["local_rejected"] == want
    assert out["exchanged_rejected"] == want
    assert out["local_first_bad"] == 1 and out["exchanged_first_bad"] == 1
    assert out["first_zero_bit"] == 0


def test_bench_force_pg_nccl():
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "1", "--dist-backend", "nccl",
                        "--force-pg", "--n", "65536", "--steps", "1", "--warmup", "0", "--cpu-per-worker", "0"],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    recs = [json.loads(x) for x in r.stdout.splitlines() if x.startswith('{"metric"')]
    assert len(recs) == 1
    d = recs[0]["dist"]
    assert d["backend"] == "nccl" and d["world_size"] == 1 and d["gate"] == "passed"
    assert d["ranks_verified_rounds"] == 65536
