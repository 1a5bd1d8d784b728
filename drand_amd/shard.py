"""Round-range sharding of a beacon history across the GPUs of one node.

Each rank verifies a contiguous range of rounds. A beacon's verdict depends only on (round,
PreviousSig bytes, Signature, pk) -- chain.VerifyBeacon, chain/beacon.go:87-92 -- so the only data
a shard needs from outside its range is a one-signature halo: the signature of the round just
before it, or the genesis seed (GroupHash, client/verify.go:122-124) for the shard that starts at
round 1. After the local verification one exchange combines the results (torch.distributed; the
"nccl" backend is RCCL over xGMI on MI355X, "gloo" in the CPU tests):

  * all-reduce MIN of the per-shard first bad ROUND (UINT64_MAX = none is mapped to INT64_MAX so
    that signed MIN is correct);
  * all-gather of the per-shard verdict bitmaps (RCCL has no bitwise OR; shards are disjoint, so
    gathering is exact), re-packed to global bit positions when a shard is not 64-aligned.
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
    """Exchange step of the sharded verification (call on every rank).

    first_bad: this shard's first rejected ROUND -- a Python int (NONE_U64 = none) or a 1-element
      int64 device tensor as written by blsv_verify_chained_dev (UINT64_MAX reads back as -1).
    bitmap_words: this shard's verdict bitmap, a 1-D int64 tensor of ceil(count/64) words (bit i =
      the shard's i-th beacon, LSB first) on the device the process group uses.
    counts: every rank's shard length, when the caller knows them (shard_range); else one extra
      all-gather of the lengths.
    Returns (first_bad, bitmap):
      to_host=True : (global first bad round or NONE_U64, list of 64-bit words at global positions)
      to_host=False: (1-element int64 device tensor, INT64_MAX = none; device words at global bit
                     positions). Shards whose lengths are multiples of 64 (all but the last) are
                     concatenated as is; otherwise the words are re-packed on the device.
    """
    import torch
    import torch.distributed as dist

    dev = bitmap_words.device
    world = dist.get_world_size(group)
    if isinstance(first_bad, int):
        fb = torch.tensor([to_i64_first_bad(first_bad)], dtype=torch.int64, device=dev)
    else:
        fb = first_bad.reshape(1).to(torch.int64)
        fb = torch.where(fb < 0, torch.full_like(fb, NONE_I64), fb)
    dist.all_reduce(fb, op=dist.ReduceOp.MIN, group=group)
    words = (count + 63) // 64
    if not to_host and counts is not None and all(c % 64 == 0 for c in counts[:-1]) \
            and len({(c + 63) // 64 for c in counts}) == 1:
        # the bench path: every shard covers the same whole number of words
        gathered = torch.empty(world * words, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(gathered, bitmap_words[:words].contiguous(), group=group)
        return fb, gathered
    if counts is None:
        c_t = torch.tensor([count], dtype=torch.int64, device=dev)
        all_counts = torch.empty(world, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(all_counts, c_t, group=group)
        counts = [int(c) for c in all_counts.cpu().tolist()]
    counts_l = list(counts)
    wmax = max((c + 63) // 64 for c in counts_l)
    padded = torch.zeros(wmax, dtype=torch.int64, device=dev)
    padded[:words] = bitmap_words[:words]
    gathered = torch.empty(world * wmax, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(gathered, padded, group=group)
    if not to_host:
        return fb, repack_words(gathered, counts_l, wmax)
    host_words = [w & NONE_U64 for w in gathered.cpu().tolist()]
    return from_i64_first_bad(int(fb.item())), assemble_bitmap(host_words, counts_l, wmax)


def assemble_bitmap(words, counts, stride):
    """Concatenate per-shard bitmaps (shard r's words at words[r*stride:]) at global bit offsets."""
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


def repack_words(gathered, counts, stride):
    """Device form of assemble_bitmap: per-shard words (shard r at gathered[r*stride:]) -> one
    bitmap at global bit offsets. Word-level bit-offset shifts with torch ops on the tensor's device:
    shard r, starting at global bit pos = 64 q + s, ORs (w << s) into words q.. and the spill
    (w >>> (64 - s)) into words q+1..; O(words) per shard, no per-bit temporaries (a 100M-round
    bitmap is 1.56M words)."""
    import torch

    dev = gathered.device
    total = int(sum(counts))
    out = torch.zeros(max(1, (total + 63) // 64), dtype=torch.int64, device=dev)
    pos = 0
    for r, c in enumerate(counts):
        nw = (c + 63) // 64
        if nw == 0:
            continue
        w = gathered[r * stride: r * stride + nw].clone()
        nb = c - 64 * (nw - 1)
        if nb < 64:
            w[-1] &= (1 << nb) - 1  # bits past the shard's last beacon
        q, s = divmod(pos, 64)
        out[q:q + nw] |= w << s if s else w
        if s:
            spill = (w >> (64 - s)) & ((1 << s) - 1)  # logical shift of the int64 words
            hi = min(nw, out.numel() - q - 1)
            if hi > 0:
                out[q + 1:q + 1 + hi] |= spill[:hi]
        pos += c
    return out[:(total + 63) // 64]


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
