"""bench.py's N-rank path on the GPU: `bench.py --gpus 2 --dist-backend gloo` starts two ranks
itself (torch.distributed.run as a child), both on cuda:0 of the one-GPU test box, each verifying its
shard with the HIP engine and exchanging verdicts through shard.combine (one SUM all-reduce; gloo
through host copies here, RCCL on the 8-GPU node). Weak mode (--n per rank) and strong mode (one
unaligned --total-rounds history split in contiguous ranges with the true previous-signature halo).
The bench's own gate must pass on every rank: all rounds accept, then one corrupted signature per
rank rejects exactly it and its successor, first_bad = the lowest corrupted round over the ranks."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("mode", [["--n", "65536"], ["--total-rounds", "131075"]], ids=["weak", "strong"])
def test_bench_two_ranks_one_gpu(mode):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                        "--steps", "1", "--warmup", "0", "--cpu-per-worker", "0"] + mode,
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    recs = [json.loads(x) for x in r.stdout.splitlines() if x.startswith('{"metric"')]
    assert len(recs) == 1, r.stdout[-3000:]  # rank 0 prints the one line
    out = recs[0]
    d = out["dist"]
    assert out["n_gpus"] == 2 and d["world_size"] == 2 and d["backend"] == "gloo"
    assert d["gate"] == "passed" and d["devices"] == [0, 0]
    assert "one all_reduce(SUM)" in d["exchange"]
    want = 2 * 65536 if mode[0] == "--n" else 131075
    assert d["ranks_verified_rounds"] == sum(d["rank_counts"]) == want
    if mode[0] == "--total-rounds":
        assert out["scaling"] == "strong" and d["rank_counts"] == [65538, 65537]
    else:
        assert out["scaling"] == "weak"
    assert out["value"] > 0
