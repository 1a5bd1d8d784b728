"""The RCCL ("nccl") branch of shard.combine on a one-GPU box: a world-size-1 nccl process group on
cuda:0, the engine verifying a corrupted 9,001-round segmented history on an explicit stream, and the
exchange (ONE SUM all-reduce) queued right behind it on the same stream with no host synchronisation
in between -- the ordering that broke the gloo path once. Prints one JSON line with the
single-process verdicts and the exchanged ones; tests/test_gpu_rccl.py compares them. Run as its own
process (the process group must not outlive it)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist

    from drand_amd import shard
    from drand_amd.engine import Engine

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    assert "MASTER_PORT" in os.environ
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", device_id=dev)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream

    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        g = json.load(f)["chained"]
    sk32 = int(g["sk"], 16).to_bytes(32, "big")
    n, seg = 9001, 64
    gen = torch.Generator(device=dev)
    gen.manual_seed(0x5CC1)
    seeds = torch.randint(0, 256, ((n + seg - 1) // seg, 96), dtype=torch.uint8, device=dev, generator=gen)
    sigs = torch.empty((n, 96), dtype=torch.uint8, device=dev)
    eng = Engine(0)
    eng.set_public_key(bytes.fromhex(g["pk"]))
    eng.generate_chained_dev(sk32, 1, seg, seeds.data_ptr(), 32, sigs.data_ptr(), n, sp)
    torch.cuda.synchronize(dev)
    hit = [0, 63, 64, 4095, 4999, n - 1]
    for i in hit:
        sigs[i, 50] ^= 1
    words = (n + 63) // 64
    bm = torch.zeros(words, dtype=torch.int64, device=dev)
    fb = torch.empty(1, dtype=torch.int64, device=dev)
    # engine launch and exchange on ONE stream, nothing synchronised in between
    eng.verify_chained_dev(1, seg, seeds.data_ptr(), 32, sigs.data_ptr(), n, bm.data_ptr(), fb.data_ptr(), None, sp)
    fb_all, gbm = shard.combine(fb, bm, n, to_host=False, counts=[n])
    collective_words = words + 1
    torch.cuda.synchronize(dev)
    local = [w & shard.NONE_U64 for w in bm.cpu().tolist()]
    if n % 64:
        local[-1] &= (1 << (n % 64)) - 1
    out = {
        "backend": str(dist.get_backend()),
        "world_size": dist.get_world_size(),
        "rounds": n,
        "collective_words": collective_words,
        "local_first_bad": int(fb.item()) & shard.NONE_U64,
        "exchanged_first_bad": int(fb_all.item()),
        "local_rejected": [i for i in range(n) if not (local[i // 64] >> (i % 64)) & 1],
        "exchanged_rejected": [i for i in range(n) if not (int(gbm[i // 64]) >> (i % 64)) & 1],
        "first_zero_bit": shard.first_zero_bit(gbm, n),
        "hit": hit,
        "seg_len": seg,
    }
    eng.close()
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
