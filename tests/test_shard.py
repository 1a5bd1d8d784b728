"""Multi-GPU sharding logic on the CPU: contiguous round ranges, the one-signature
halo, and the exchange step (MIN of first bad round + bitmap all-gather) over torch.distributed with
the gloo backend at world_size 2 and 3 -- the same code bench.py runs over RCCL."""
import os
import random
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from drand_amd import shard


def test_shard_range_partitions():
    for n in (0, 1, 63, 64, 65, 1000, 1_000_003):
        for world in (1, 2, 3, 8):
            parts = [shard.shard_range(n, world, r) for r in range(world)]
            assert sum(p.count for p in parts) == n
            pos = 0
            for p in parts:
                assert p.start == pos
                pos += p.count
            assert max(p.count for p in parts) - min(p.count for p in parts) <= 1
    with pytest.raises(ValueError):
        shard.shard_range(10, 2, 2)


def test_halo_is_previous_signature_or_genesis():
    sigs = bytes(range(256)) * 3  # 768 B = 8 signatures
    seed = b"\x07" * 32
    s0 = shard.shard_range(8, 2, 0)
    s1 = shard.shard_range(8, 2, 1)
    assert shard.halo(s0, sigs, seed) == seed  # round 1: GroupHash (client/verify.go:122-124)
    assert shard.halo(s1, sigs, seed) == sigs[3 * 96:4 * 96]
    assert s1.first_round == 5


def _bits_to_words(bits):
    words = [0] * ((len(bits) + 63) // 64)
    for i, b in enumerate(bits):
        if b:
            words[i // 64] |= 1 << (i % 64)
    return words


def test_assemble_bitmap_unaligned():
    rng = random.Random(3)
    counts = [70, 1, 129, 64]
    bits = [rng.random() < 0.7 for _ in range(sum(counts))]
    stride = max((c + 63) // 64 for c in counts)
    words, pos = [], 0
    for c in counts:
        w = _bits_to_words(bits[pos:pos + c])
        w += [0xFFFFFFFFFFFFFFFF] * (stride - len(w))  # garbage beyond the shard must be masked
        words += w
        pos += c
    assert shard.assemble_bitmap(words, counts, stride) == _bits_to_words(bits)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _to_i64(words):
    return torch.tensor([w - (1 << 64) if w >= 1 << 63 else w for w in words], dtype=torch.int64)


def _worker(rank, world, port, n, bad, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sh = shard.shard_range(n, world, rank)
        bits = [(sh.start + i) not in bad for i in range(sh.count)]
        local_bad = [sh.first_round + i for i, b in enumerate(bits) if not b]
        fb = min(local_bad) if local_bad else shard.NONE_U64
        words = _to_i64(_bits_to_words(bits)) if bits else torch.zeros(0, dtype=torch.int64)
        g_fb, g_words = shard.combine(fb, words, sh.count)
        # device form (the bench path), as the kernels write it: UINT64_MAX = -1 in an int64 tensor
        fb_t = torch.tensor([-1 if fb == shard.NONE_U64 else fb], dtype=torch.int64)
        d_fb, d_words = shard.combine(fb_t, words, sh.count, to_host=False)
        q.put((rank, g_fb, g_words, int(d_fb.item()), [w & shard.NONE_U64 for w in d_words.tolist()]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,bad", [(2, 1000, {5, 6, 777}), (2, 128, set()), (3, 1001, {1000}),
                                         (2, 256, {200, 201})])
def test_combine_gloo(world, n, bad):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, bad, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want_words = _bits_to_words([i not in bad for i in range(n)])
    want_fb = min(bad) + 1 if bad else shard.NONE_U64  # ROUND = index + 1
    aligned = all(shard.shard_range(n, world, r).count % 64 == 0 for r in range(world - 1))
    for rank, g_fb, g_words, d_fb, d_words in res:
        assert g_fb == want_fb
        assert g_words == want_words
        assert d_fb == (shard.NONE_I64 if not bad else want_fb)  # the regression the MIN mapping fixes
        if aligned:
            assert d_words[:len(want_words)] == want_words
