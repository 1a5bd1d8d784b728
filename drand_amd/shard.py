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


def to_i64_first_bad(v: int) -> int:
    return NONE_I64 if v == NONE_U64 or v < 0 else v


def from_i64_first_bad(v: int) -> int:
    return NONE_U64 if v == NONE_I64 else v


def combine(first_bad, bitmap_words, count: int, group=None, to_host: bool = True):
    """Exchange step of the sharded verification (call on every rank).

    first_bad: this shard's first rejected ROUND -- a Python int (NONE_U64 = none) or a 1-element
      int64 device tensor as written by blsv_verify_chained_dev (UINT64_MAX reads back as -1).
    bitmap_words: this shard's verdict bitmap, a 1-D int64 tensor of ceil(count/64) words (bit i =
      the shard's i-th beacon, LSB first) on the device the process group uses.
    Returns (first_bad, bitmap):
      to_host=True : (global first bad round or NONE_U64, list of 64-bit words at global positions)
      to_host=False: (1-element int64 device tensor, INT64_MAX = none; gathered device words) --
                     the device form needs every shard but the last to be a multiple of 64 long.
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
    if not to_host:
        gathered = torch.empty(world * words, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(gathered, bitmap_words[:words].contiguous(), group=group)
        return fb, gathered
    counts = torch.tensor([count], dtype=torch.int64, device=dev)
    all_counts = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(all_counts, counts, group=group)
    counts_l = [int(c) for c in all_counts.cpu().tolist()]
    wmax = max((c + 63) // 64 for c in counts_l)
    padded = torch.zeros(wmax, dtype=torch.int64, device=dev)
    padded[:words] = bitmap_words[:words]
    gathered = torch.empty(world * wmax, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(gathered, padded, group=group)
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
