"""bench.py's N-rank plumbing on the CPU (no GPU touched): `--gpus N` with no WORLD_SIZE starts N
ranks itself through torch.distributed.run as a child process, every rank asserts world_size ==
--gpus, and one shard.combine exchange (gloo) gives every rank the same global verdicts. The GPU
form of the same run is tests/test_gpu_bench_dist.py."""
import json
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=240)


@pytest.mark.parametrize("gpus,extra", [(2, ["--n", "100"]), (3, ["--total-rounds", "1001"])])
def test_bench_launches_n_ranks(gpus, extra):
    r = _run(["--gpus", str(gpus), "--launch-check", "--dist-backend", "gloo"] + extra)
    assert r.returncode == 0, r.stderr[-2000:]
    # ranks share one stdout (and gloo's own log lines): pick the rank records out of the stream
    lines = [json.loads(x) for x in re.findall(r'\{"rank": .*?\]\}', r.stdout)]
    assert sorted(x["rank"] for x in lines) == list(range(gpus))
    total = sum(lines[0]["counts"])
    for x in lines:
        assert x["world_size"] == gpus == x["gpus"]
        assert x["rejected"] == [total - 2] and x["first_bad"] == total - 1


def test_bench_refuses_world_mismatch():
    r = _run(["--gpus", "2", "--launch-check"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "--gpus" in (r.stderr + r.stdout)
