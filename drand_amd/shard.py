"""Round-range sharding of a beacon history across the GPUs of one node.

Each rank verifies a contiguous range of rounds. A beacon's verdict depends only on (round,
PreviousSig bytes, Signature, pk) -- chain.VerifyBeacon, chain/beacon.go:87-92 -- so the only data
a shard needs from outside its range is a one-signature halo: the signature of the round just
before it, or the genesis seed (GroupHash, client/verify.go:122-124) for the shard that starts at
round 1. After the local verification ONE collective combines the results (torch.distributed;
the "nccl" backend is RCCL over xGMI on MI355X, "gloo" in the CPU tests): a SUM all-reduce of a
zero-initialised buffer holding the global-position verdict bitmap plus one first-bad-round slot per
rank (``combine``).
"""
from __future__ import annotations

from dataclasses import dataclass

NONE_U64 = (1 << 64) - 1
NONE_I64 = (1 << 63) - 1


@dataclass(frozen=True)
class Shard:
    rank: int
    start: int  # index of the first beacon of this shard in the history (0-based)
    count: int

    @property
    def first_round(self) -> int:
        return self.start + 1  # histories start at round 1 (chain/store.go:234-238)


def shard_range(n_total: int, world: int, rank: int) -> Shard:
    """Contiguous split: the first n_total % world ranks get one extra beacon."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    base, extra = divmod(n_total, world)
    start = rank * base + min(rank, extra)
    return Shard(rank, start, base + (1 if rank < extra else 0))


def halo(shard: Shard, sigs, genesis_seed: bytes) -> bytes:
    """PreviousSig of the shard's first beacon: the genesis seed at round 1, else the previous
    round's signature (sigs: the full history as a bytes-like of n x 96)."""
    if shard.start == 0:
        return bytes(genesis_seed)
    return bytes(sigs[(shard.start - 1) * 96: shard.start * 96])


@dataclass(frozen=True)
class SegmentedSlice:
    """What one rank generates and verifies of a history built from independently seeded chained
    segments of ``seg_len`` rounds (bench.py's synthetic layout; SURVEY.md §7 / mock/result.go:98-132).

    The rank verifies ``shard`` = [start, start + count). It must generate from the start of the
    segment holding ``start`` (``gen_start``) so that it holds the true previous signature of its
    first round; ``phase`` = start - gen_start is that round's position inside its segment and the
    halo is ``sigs[phase - 1]`` of the generated range (or the segment seed when phase == 0)."""
    shard: Shard
    gen_start: int
    seg_first: int
    phase: int
    n_seg: int

    @property
    def gen_count(self) -> int:
        return self.shard.start + self.shard.count - self.gen_start


def segmented_slice(n_total: int, world: int, rank: int, seg_len: int) -> SegmentedSlice:
    sh = shard_range(n_total, world, rank)
    seg_first = sh.start // seg_len
    gen_start = seg_first * seg_len
    end = sh.start + sh.count
    n_seg = max(1, (end - gen_start + seg_len - 1) // seg_len)
    return SegmentedSlice(sh, gen_start, seg_first, sh.start - gen_start, n_seg)


def to_i64_first_bad(v: int) -> int:
    return NONE_I64 if v == NONE_U64 or v < 0 else v


def from_i64_first_bad(v: int) -> int:
    return NONE_U64 if v == NONE_I64 else v


def combine(first_bad, bitmap_words, count: int, group=None, to_host: bool = True, counts=None):
    """Exchange step of the sharded verification (call on every rank): ONE all-reduce.

    Every rank writes its verdict bits at their GLOBAL positions into a zero-initialised buffer of
    ceil(total/64) words, followed by one slot per rank holding that rank's first bad round
    (INT64_MAX = none) and zeros in the other ranks' slots. One SUM all-reduce of that buffer then
    gives every rank the whole bitmap and every shard's first bad round: the shards' bits are
    disjoint (a word shared by two shards at an unaligned boundary gets bits from both), and adding
    integers with disjoint set bits never carries, so SUM is exactly OR (RCCL has no bitwise OR).
    The global first bad round is the MIN over the slots, taken locally.

    first_bad: this shard's first rejected ROUND -- a Python int (NONE_U64 = none) or a 1-element
      int64 device tensor as written by blsv_verify_chained_dev (UINT64_MAX reads back as -1).
    bitmap_words: this shard's verdict bitmap, a 1-D int64 tensor of >= ceil(count/64) words (bit i
      = the shard's i-th beacon, LSB first; bits past ``count`` are ignored).
    counts: every rank's shard length when the caller knows them (shard_range); else one small
      all-gather of the lengths first (not on the bench path).
    With the gloo backend and a device tensor (two ranks sharing one GPU in the tests) the buffer is
    all-reduced through a host copy.
    Cost on the RCCL ("nccl") branch -- unmeasured here, run only by the driver's 8-GPU scaling job
    (this repository's GPU boxes have one GPU; the tests run the gloo branch): a ring all-reduce moves
    2(N-1)/N of the buffer per rank, about twice what a bitmap all-gather would, i.e. ~22 MB per rank
    for configs[3]'s 100M rounds at N = 8 (12.5 MB buffer), an estimated ~0.2-0.3 ms over xGMI against
    ~6 s of verification per 12.5M-round shard.
    Returns (first_bad, bitmap):
      to_host=True : (global first bad round or NONE_U64, list of 64-bit words at global positions)
      to_host=False: (1-element int64 tensor, INT64_MAX = none; int64 words at global bit positions),
                     on bitmap_words' device.
    """
    import torch
    import torch.distributed as dist

    dev = bitmap_words.device
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if counts is None:
        c_t = torch.tensor([count], dtype=torch.int64)
        all_counts = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        if dist.get_backend(group) == "gloo":
            dist.all_gather(all_counts, c_t, group=group)
        else:
            gathered = torch.empty(world, dtype=torch.int64, device=dev)
            dist.all_gather_into_tensor(gathered, c_t.to(dev), group=group)
            all_counts = gathered.cpu().split(1)
        counts = [int(c) for c in all_counts]
    counts = list(counts)
    if len(counts) != world or counts[rank] != count:
        raise ValueError(f"counts {counts} do not match world {world} / this shard's count {count}")
    total = sum(counts)
    tw = (total + 63) // 64
    buf = torch.zeros(tw + world, dtype=torch.int64, device=dev)
    place_words(buf, bitmap_words, count, sum(counts[:rank]))
    if isinstance(first_bad, int):
        buf[tw + rank] = to_i64_first_bad(first_bad)
    else:
        fb = first_bad.reshape(1).to(torch.int64)
        buf[tw + rank:tw + rank + 1] = torch.where(fb < 0, torch.full_like(fb, NONE_I64), fb)
    if dist.get_backend(group) == "gloo" and buf.device.type != "cpu":
        host = buf.cpu()
        dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
        buf.copy_(host)
    else:
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
    fb_all = buf[tw:].min().reshape(1)
    if not to_host:
        return fb_all, buf[:tw]
    return from_i64_first_bad(int(fb_all.item())), [w & NONE_U64 for w in buf[:tw].cpu().tolist()]


def first_zero_bit(words, total: int):
    """Index of the first 0 bit among the first ``total`` bits of an int64 word tensor, or None (a
    check of the exchanged bitmap against the exchanged first bad round: for a history starting at
    round 1 the first bad round is this index + 1)."""
    import torch

    nw = (total + 63) // 64
    if nw == 0:
        return None
    w = words[:nw].clone()
    if total % 64:
        w[-1] |= -(1 << (total % 64))  # bits past the history count as accepted
    bad = torch.nonzero(w != -1)
    if bad.numel() == 0:
        return None
    q = int(bad[0, 0])
    inv = (~int(w[q])) & NONE_U64
    return 64 * q + ((inv & -inv).bit_length() - 1)


def assemble_bitmap(words, counts, stride):
    """Host reference of the exchange's bit placement: per-shard bitmaps (shard r's words at
    words[r*stride:]) concatenated at global bit offsets."""
    total = sum(counts)
    out = [0] * ((total + 63) // 64)
    pos = 0
    for r, c in enumerate(counts):
        for i in range((c + 63) // 64):
            w = words[r * stride + i]
            nb = min(64, c - 64 * i)
            w &= (1 << nb) - 1
            q, s = divmod(pos + 64 * i, 64)
            out[q] |= (w << s) & NONE_U64
            if s and q + 1 < len(out):
                out[q + 1] |= w >> (64 - s)
        pos += c
    return out


def place_words(out, words, count: int, pos: int):
    """OR the first ``count`` bits of ``words`` (int64 tensor, LSB first) into ``out`` (int64 tensor
    on the same device) starting at global bit ``pos``: word-level shifts with torch ops on the
    device, O(words), no per-bit temporaries (a 100M-round bitmap is 1.56M words)."""
    import torch

    nw = (count + 63) // 64
    if nw == 0:
        return out
    w = words[:nw].to(out.device).clone()
    nb = count - 64 * (nw - 1)
    if nb < 64:
        w[-1] &= (1 << nb) - 1  # bits past the shard's last beacon
    q, s = divmod(pos, 64)
    if not s:
        out[q:q + nw] |= w
        return out
    out[q:q + nw] |= w << s
    spill = (w >> (64 - s)) & ((1 << s) - 1)  # logical shift of the int64 words
    hi = min(nw, out.numel() - q - 1)
    if hi > 0:
        out[q + 1:q + 1 + hi] |= spill[:hi]
    return out


def local_seeds(sl: SegmentedSlice, seg_seeds, gen_sigs):
    """Seed rows for ``blsv_verify_chained_dev(seg_phase=sl.phase)`` over the rank's shard (torch
    uint8 tensors on the device). seg_seeds: (sl.n_seg, 96) seeds of the segments the rank
    generated; gen_sigs: (sl.gen_count, 96) signatures from ``sl.gen_start``. Row 0 is the halo --
    the true PreviousSig of the shard's first round: its segment seed when the shard starts a
    segment, else the signature just before it -- and rows 1.. are the seeds of the segments that
    start inside the shard."""
    import torch

    halo = seg_seeds[0:1] if sl.phase == 0 else gen_sigs[sl.phase - 1:sl.phase]
    return torch.cat([halo, seg_seeds[1:]]).contiguous()


def chained_prev(i: int, phase: int, seg_len: int, seeds, sigs, seed0_len: int) -> bytes:
    """Host restatement of the device seed rule (drand_amd/csrc/kernels.h ChainedSrc): the
    PreviousSig of local item i; seeds/sigs are lists of 96-byte rows."""
    s = (i + phase) // seg_len
    if i == 0 or (i + phase) % seg_len == 0:
        return bytes(seeds[s][:seed0_len if s == 0 else 96])
    return bytes(sigs[i - 1])
