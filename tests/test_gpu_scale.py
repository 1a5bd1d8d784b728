"""GPU parity at scale: device-generated chained histories (the bench workload, BASELINE.json
configs[1]/[4]) checked through size-independent properties, with samples cross-checked by the C
oracle (oracle/c/bls_oracle.c, pinned to the reference KAT in tests/test_oracle_c.py):

  * every generated round verifies (bitmap all ones, first_bad = none), also across pipeline-chunk
    boundaries and for ragged sizes;
  * a corrupted signature i rejects exactly rounds i and i+1 (chain.VerifyBeacon hashes the given
    PreviousSig bytes, chain/beacon.go:87-108) unless i+1 starts a new segment; first_bad is the
    smallest rejected ROUND; reject classes match the C oracle;
  * V2 (unchained) batches signed on device verify, wrong rounds reject.
"""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NONE = (1 << 64) - 1


@pytest.fixture(scope="module")
def C():
    from oracle import c_oracle

    if not os.path.exists(c_oracle.LIB_PATH):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    c_oracle.load()
    return c_oracle


def _history(engine, golden, n, seg, first_round=1, seed=7):
    import torch

    ch = golden["chained"]
    engine.set_public_key(bytes.fromhex(ch["pk"]))
    sk32 = int(ch["sk"], 16).to_bytes(32, "big")
    n_seg = (n + seg - 1) // seg
    g = torch.Generator(device="cuda:0")
    g.manual_seed(seed)
    seeds = torch.randint(0, 256, (n_seg * 96,), dtype=torch.uint8, device="cuda:0", generator=g)
    sigs = torch.empty(n * 96, dtype=torch.uint8, device="cuda:0")
    seed0_len = 32 if first_round == 1 else 96
    engine.generate_chained_dev(sk32, first_round, seg, seeds.data_ptr(), seed0_len, sigs.data_ptr(), n)
    torch.cuda.synchronize()
    return seeds, sigs, seed0_len


def _verify(engine, first_round, seg, seeds, seed0_len, sigs, n):
    import torch

    words = (n + 63) // 64
    bitmap = torch.zeros(words, dtype=torch.int64, device="cuda:0")
    fb = torch.empty(1, dtype=torch.int64, device="cuda:0")
    cls = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    engine.verify_chained_dev(first_round, seg, seeds.data_ptr(), seed0_len, sigs.data_ptr(), n, bitmap.data_ptr(),
                              fb.data_ptr(), cls.data_ptr())
    torch.cuda.synchronize()
    bm = [w & NONE for w in bitmap.cpu().tolist()]
    ok = [(bm[i // 64] >> (i % 64)) & 1 == 1 for i in range(n)]
    return ok, int(fb.item()) & NONE, cls.cpu().tolist()


def _segments(seeds, sigs, seed0_len, seg, first_round, idx):
    """(first_round, prev0, sigs) chained pieces covering the segments that contain the indices idx"""
    sh = sigs.cpu().numpy().tobytes()
    sd = seeds.cpu().numpy().tobytes()
    n = len(sh) // 96
    out = []
    for s in sorted({i // seg for i in idx}):
        lo, hi = s * seg, min(n, (s + 1) * seg)
        prev0 = sd[s * 96: s * 96 + (seed0_len if s == 0 else 96)]
        out.append((lo, first_round + lo, prev0, sh[lo * 96: hi * 96]))
    return out


@pytest.mark.parametrize("n,seg", [(4099, 64), (1 << 20 | 4099, 64)])
def test_generated_history_all_accept(engine, golden, C, n, seg):
    seeds, sigs, s0 = _history(engine, golden, n, seg)
    ok, fb, cls = _verify(engine, 1, seg, seeds, s0, sigs, n)
    assert all(ok) and fb == NONE and not any(cls)
    # the generator agrees with the C oracle: first segment, one across the 2^20 chunk edge, last
    pk48 = bytes.fromhex(golden["chained"]["pk"])
    for lo, fr, prev0, sg in _segments(seeds, sigs, s0, seg, 1, [0, min(n - 1, (1 << 20) - 1), n - 1]):
        assert C.verify_chained(pk48, fr, prev0, sg[: 8 * 96]) == [0] * min(8, len(sg) // 96)


def test_lat_max_clamped_to_one_chunk(engine, golden):
    """A cut-over above one pipeline chunk is clamped to 2^20 (blsv_set_lat_max, BLSV_LAT_MAX): a
    call of more items never reaches the latency kernels, whose class buffer is chunk-sized; with the
    cut-over set huge a 2^20 + 4099-round history still verifies, through the chunked pipeline."""
    prev = engine.set_lat_max(1 << 40)
    try:
        assert engine.set_lat_max(1 << 40) == 1 << 20
        n, seg = 1 << 20 | 4099, 64
        seeds, sigs, s0 = _history(engine, golden, n, seg, seed=5)
        ok, fb, cls = _verify(engine, 1, seg, seeds, s0, sigs, n)
        assert all(ok) and fb == NONE and not any(cls)
    finally:
        engine.set_lat_max(prev)


def test_corrupted_history_rejects_exactly(engine, golden, C):
    import torch

    n, seg = 20000, 64
    seeds, sigs, s0 = _history(engine, golden, n, seg, seed=11)
    bad = [5, 127, 128, 4000, 12345, n - 1]  # 127: next round starts a segment; 128: a segment start
    host = sigs.cpu()
    for k, i in enumerate(bad):
        host[i * 96 + 40 + k] ^= 0x10  # flip a bit of x (c1)
    sigs.copy_(host.to("cuda:0"))
    ok, fb, cls = _verify(engine, 1, seg, seeds, s0, sigs, n)
    want = set(bad) | {i + 1 for i in bad if i + 1 < n and (i + 1) % seg != 0}
    assert {i for i, v in enumerate(ok) if not v} == want
    assert fb == 1 + min(want)
    pk48 = bytes.fromhex(golden["chained"]["pk"])
    for lo, fr, prev0, sg in _segments(seeds, sigs, s0, seg, 1, sorted(want)):
        want_cls = C.verify_chained(pk48, fr, prev0, sg)
        assert cls[lo: lo + len(want_cls)] == want_cls


def test_unchained_batch_signed_on_device(engine, golden):
    ch = golden["chained"]
    engine.set_public_key(bytes.fromhex(ch["pk"]))
    sk32 = int(ch["sk"], 16).to_bytes(32, "big")
    import hashlib

    n, first = 3000, 1_000_000
    msgs = [hashlib.sha256((first + i).to_bytes(8, "big")).digest() for i in range(n)]  # chain.MessageV2
    sigs = engine.sign(sk32, msgs)
    res = engine.verify_unchained(sigs, first_round=first)
    assert all(res.ok) and res.first_bad is None
    res = engine.verify_unchained(sigs, first_round=first + 1)
    assert not any(res.ok) and res.first_bad == first + 1


def test_sharded_slices_with_phase_match_whole(engine, golden):
    """configs[3] path on one GPU: one segmented history verified whole, then as 3 and 5 contiguous
    shards that start mid-segment (seg_phase, halo = the true previous signature as seeds[0], exactly
    what bench.py --total-rounds does per rank); the re-assembled verdicts equal the whole-history
    verdicts, including a corrupted signature just before a shard boundary (its successor, the next
    shard's first round, must reject through the halo)."""
    import torch

    from drand_amd import shard

    n, seg = 9001, 64
    seeds, sigs, s0 = _history(engine, golden, n, seg, seed=21)
    S = sigs.view(n, 96)
    Q = seeds.view(-1, 96)
    for world in (3, 5):
        cut = shard.shard_range(n, world, 1).start - 1  # last round of shard 0
        host = sigs.cpu()
        host[cut * 96 + 50] ^= 1
        bad_sigs = host.to("cuda:0")
        ok_whole, fb_whole, _ = _verify(engine, 1, seg, seeds, s0, bad_sigs, n)
        assert fb_whole == cut + 1
        S = bad_sigs.view(n, 96)
        got = []
        for r in range(world):
            sl = shard.segmented_slice(n, world, r, seg)
            gen_sigs = S[sl.gen_start:sl.gen_start + sl.gen_count]
            loc = shard.local_seeds(sl, Q[sl.seg_first:sl.seg_first + sl.n_seg], gen_sigs)
            mine = S[sl.shard.start:sl.shard.start + sl.shard.count].contiguous()
            c = sl.shard.count
            bitmap = torch.zeros((c + 63) // 64, dtype=torch.int64, device="cuda:0")
            fb = torch.empty(1, dtype=torch.int64, device="cuda:0")
            engine.verify_chained_dev(sl.shard.first_round, seg, loc.data_ptr(), 32 if sl.shard.start == 0 else 96,
                                      mine.data_ptr(), c, bitmap.data_ptr(), fb.data_ptr(), None, None,
                                      seg_phase=sl.phase)
            torch.cuda.synchronize()
            bm = [w & NONE for w in bitmap.cpu().tolist()]
            got += [(bm[i // 64] >> (i % 64)) & 1 == 1 for i in range(c)]
        assert got == ok_whole
        assert not got[cut] and (not got[cut + 1] or (cut + 1) % seg == 0)


def test_configs3_shard_7_of_8_full_size(engine, golden, C):
    """BASELINE.json configs[3] at full per-GPU size: rank 7 of a 100,000,000-round history split 8
    ways (12,500,000 rounds, first round 87,500,001, seg_phase 32 -- the shard starts mid-segment and
    is not 64-aligned), generated on the device from its segment's start and verified through
    shard.segmented_slice / local_seeds / verify_chained_dev exactly as bench.py --total-rounds does
    per rank. All rounds accept; the C oracle re-verifies the halo segment (true previous signature
    of the first round, generated by rank 6's range), the last segment and samples in between; a
    corrupted halo must reject the shard's first round and only it; a corrupted signature inside the
    shard rejects it and its successor (client/verify.go:146-163 linkage)."""
    import torch

    from drand_amd import shard

    total, world, rank, seg = 100_000_000, 8, 7, 64
    sl = shard.segmented_slice(total, world, rank, seg)
    n = sl.shard.count
    assert n == 12_500_000 and sl.shard.first_round == 87_500_001 and sl.phase == 32
    ch = golden["chained"]
    pk48 = bytes.fromhex(ch["pk"])
    engine.set_public_key(pk48)
    sk32 = int(ch["sk"], 16).to_bytes(32, "big")
    g = torch.Generator(device="cuda:0")
    g.manual_seed(0xC0F3)
    seg_seeds = torch.randint(0, 256, (sl.n_seg, 96), dtype=torch.uint8, device="cuda:0", generator=g)
    gen_sigs = torch.empty((sl.gen_count, 96), dtype=torch.uint8, device="cuda:0")
    engine.generate_chained_dev(sk32, sl.gen_start + 1, seg, seg_seeds.data_ptr(), 96, gen_sigs.data_ptr(),
                                sl.gen_count)
    torch.cuda.synchronize()
    loc = shard.local_seeds(sl, seg_seeds, gen_sigs)
    mine = gen_sigs[sl.phase:sl.phase + n]
    words = (n + 63) // 64
    bitmap = torch.zeros(words, dtype=torch.int64, device="cuda:0")
    fb = torch.empty(1, dtype=torch.int64, device="cuda:0")

    import numpy as np

    def verify():
        bitmap.zero_()
        engine.verify_chained_dev(sl.shard.first_round, seg, loc.data_ptr(), 96, mine.data_ptr(), n,
                                  bitmap.data_ptr(), fb.data_ptr(), None, None, seg_phase=sl.phase)
        torch.cuda.synchronize()
        bits = np.unpackbits(bitmap.cpu().numpy().view(np.uint8), bitorder="little")[:n]
        return set(np.flatnonzero(bits == 0).tolist()), int(fb.item()) & NONE

    rejected, f = verify()
    assert not rejected and f == NONE
    # the C oracle on the halo segment (the 32 rounds up to the first segment boundary), samples in
    # between and the last rounds
    host = mine.cpu().numpy()
    halo = bytes(loc[0].cpu().numpy())
    first = sl.shard.first_round
    head = seg - sl.phase
    assert C.verify_chained(pk48, first, halo, host[:head].tobytes()) == [0] * head
    for lo in (head + seg * 1000 + 5, head + seg * 97_000 + 10, n - 8):  # none at a segment start
        assert C.verify_chained(pk48, first + lo, bytes(host[lo - 1]), host[lo:lo + 8].tobytes()) == [0] * 8
    # negative controls: a corrupted halo rejects the shard's first round and only it ...
    bad_halo = halo[:50] + bytes([halo[50] ^ 1]) + halo[51:]
    assert C.verify_chained(pk48, first, bad_halo, host[:1].tobytes()) == [7]
    loc[0, 50] ^= 1
    rejected, f = verify()
    loc[0, 50] ^= 1
    assert rejected == {0} and f == first
    # ... and a corrupted signature inside the shard rejects it and its successor
    i = 6_250_001  # (i + phase) % seg = 49: the successor is in the same segment
    mine[i, 60] ^= 0x10
    rejected, f = verify()
    mine[i, 60] ^= 0x10
    assert rejected == {i, i + 1} and f == first + i
