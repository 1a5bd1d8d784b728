"""Offline verification of a node's stored history: drand.db → SoA → batched GPU verify.

SURVEY.md §8f rank 2. ``libboltload.so`` (drand_amd/csrc/boltload.cpp, include/boltload.h) walks
bucket "beacons" of the bbolt file (chain/boltdb/store.go:21,68-81) and decodes every hexjson
``chain.Beacon`` straight into round / prev / signature arrays. ``verify_store`` hands each run of
consecutive rounds to ``Engine.verify_prevs`` (one device pass, every row hashing its own stored
PreviousSig); each beacon's verdict is ``chain.VerifyBeacon`` (chain/beacon.go:87-92) on its own
stored fields. ``linked_runs`` reports the ``appendStore.Put`` linkage rule
(chain/beacon/store.go:43-48: round + 1 and ``PreviousSig == previous Signature``).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

from .callers import _verify_run

LIB_PATH = os.environ.get("DRAND_AMD_BOLTLOAD_LIB",
                          os.path.join(os.path.dirname(os.path.abspath(__file__)), "libboltload.so"))
_lib = None


class StoreError(RuntimeError):
    pass


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise StoreError(f"{LIB_PATH} not found: build with make -C drand_amd/csrc")
        lib = ctypes.CDLL(LIB_PATH)
        vp, sz, u8 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p
        lib.dl_open.argtypes = [ctypes.c_char_p, ctypes.POINTER(vp)]
        lib.dl_open.restype = ctypes.c_int
        lib.dl_count.argtypes = [vp]
        lib.dl_count.restype = ctypes.c_int64
        lib.dl_load.argtypes = [vp, sz, sz, u8, u8, u8, u8, u8, u8, u8, ctypes.POINTER(sz)]
        lib.dl_load.restype = ctypes.c_int
        lib.dl_last_error.argtypes = [vp]
        lib.dl_last_error.restype = ctypes.c_char_p
        lib.dl_close.argtypes = [vp]
        lib.dl_close.restype = None
        _lib = lib
    return _lib


@dataclass
class StoredBeacons:
    """SoA view of bucket "beacons": n rows in round order. Byte fields are zero-padded to 96;
    ``*_len`` give the stored lengths (255 = longer than 96)."""
    rounds: np.ndarray      # uint64[n]
    prev: np.ndarray        # uint8[n, 96]
    prev_len: np.ndarray    # uint8[n]
    sigs: np.ndarray        # uint8[n, 96]
    sig_len: np.ndarray     # uint8[n]
    sigs_v2: np.ndarray     # uint8[n, 96]
    v2_len: np.ndarray      # uint8[n]

    def __len__(self):
        return len(self.rounds)


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def load_store(path, start=0, max_n=None) -> StoredBeacons:
    """Read entries [start, start + max_n) of bucket "beacons" (all of them by default)."""
    lib = _load()
    h = ctypes.c_void_p()
    rc = lib.dl_open(os.fsencode(path), ctypes.byref(h))
    try:
        if rc != 0:
            raise StoreError(lib.dl_last_error(h).decode() if h.value else "dl_open failed")
        total = lib.dl_count(h)
        n = max(0, total - start) if max_n is None else max(0, min(max_n, total - start))
        out = StoredBeacons(np.zeros(n, np.uint64), np.zeros((n, 96), np.uint8), np.zeros(n, np.uint8),
                            np.zeros((n, 96), np.uint8), np.zeros(n, np.uint8), np.zeros((n, 96), np.uint8),
                            np.zeros(n, np.uint8))
        got = ctypes.c_size_t()
        if n:
            rc = lib.dl_load(h, start, n, _ptr(out.rounds), _ptr(out.prev), _ptr(out.prev_len), _ptr(out.sigs),
                             _ptr(out.sig_len), _ptr(out.sigs_v2), _ptr(out.v2_len), ctypes.byref(got))
            if rc != 0:
                raise StoreError(lib.dl_last_error(h).decode())
        return out
    finally:
        if h.value:
            lib.dl_close(h)


def linked_runs(sb: StoredBeacons):
    """Start indices of maximal runs that ``blsv_verify_chained`` can take in one call."""
    n = len(sb)
    if n == 0:
        return np.zeros(0, np.int64)
    link = np.zeros(n, bool)
    if n > 1:
        link[1:] = ((sb.rounds[1:] == sb.rounds[:-1] + 1) & (sb.prev_len[1:] == 96) & (sb.sig_len[:-1] == 96)
                    & (sb.sig_len[1:] == 96) & np.all(sb.prev[1:] == sb.sigs[:-1], axis=1))
    return np.flatnonzero(~link)


@dataclass
class StoreVerdict:
    ok: np.ndarray              # bool[n], in stored (round) order
    first_bad: int | None       # lowest failing round, None if every beacon verifies
    runs: int                   # engine calls made for the linked runs


def round_runs(sb: StoredBeacons):
    """Start indices of maximal runs of consecutive rounds in which every row but the first has a
    96-byte PreviousSig: each is one device pass (``Engine.verify_prevs``), whatever the linkage."""
    n = len(sb)
    if n == 0:
        return np.zeros(0, np.int64)
    cont = np.zeros(n, bool)
    if n > 1:
        cont[1:] = (sb.rounds[1:] == sb.rounds[:-1] + 1) & (sb.prev_len[1:] == 96)
    return np.flatnonzero(~cont)


def verify_store(engine, public_key: bytes, sb: StoredBeacons, group_hash: bytes | None = None) -> StoreVerdict:
    """``chain.VerifyBeacon`` for every stored beacon on its own stored fields: one device pass per
    run of consecutive rounds (a whole drand.db is normally one run). Each row hashes its own
    stored PreviousSig, so broken linkage costs nothing extra; ``linked_runs`` reports linkage.

    Round 0 is the genesis beacon every node stores at startup (chain/beacon/node.go:69,
    core/drand_control.go:838: ``Put(chain.GenesisBeacon(info))``): no PreviousSig and a 32-byte
    Signature = GroupHash (chain/store.go:234-238). The reference never verifies it (sync starts at
    last+1, sync.go:91; the client walk starts at round 1, client/verify.go:122), so it is the
    trusted root here too: never handed to the engine and never a ``first_bad``. With
    ``group_hash`` given, its ok bit says whether the stored Signature equals it."""
    engine.set_public_key(public_key)
    n = len(sb)
    ok = np.zeros(n, bool)
    genesis = sb.rounds == 0
    starts = round_runs(sb)
    ends = np.append(starts[1:], n)
    for s, e in zip(starts.tolist(), ends.tolist()):
        if genesis[s]:  # a genesis row always ends its run: the next row's prev is 32 bytes
            s += 1
            if s >= e:
                continue
        plen = int(sb.prev_len[s])
        s0 = s
        if plen not in (32, 96):
            # An odd-length stored prev is still a well-defined message: message-form call for that
            # row. A prev longer than 96 bytes is not kept by the loader and is reported as a reject
            # (documented deviation: no drand writer produces one).
            if plen < 96 and int(sb.sig_len[s]) == 96:
                ok[s] = _verify_run(engine, int(sb.rounds[s]), sb.prev[s, :plen].tobytes(),
                                    [sb.sigs[s].tobytes()]) is None
            s0, plen = s + 1, 96
        if s0 < e:
            res = engine.verify_prevs(int(sb.rounds[s0]), plen, np.ascontiguousarray(sb.prev[s0:e]),
                                      np.ascontiguousarray(sb.sigs[s0:e]), e - s0)
            ok[s0:e] = np.asarray(res.ok, bool)
    ok &= sb.sig_len == 96          # kyber rejects any signature that is not 96 bytes
    if genesis.any():
        gi = np.flatnonzero(genesis)
        if group_hash is None:
            ok[gi] = True
        else:
            gh = bytes(group_hash)
            ok[gi] = [int(sb.sig_len[i]) == len(gh) and sb.sigs[i, :len(gh)].tobytes() == gh for i in gi]
    bad = np.flatnonzero(~ok & ~genesis)
    return StoreVerdict(ok, int(sb.rounds[bad[0]]) if len(bad) else None, len(starts))


def store_count(path) -> int:
    """Entries in bucket "beacons" (boltStore.Len, chain/boltdb/store.go:47-58)."""
    lib = _load()
    h = ctypes.c_void_p()
    try:
        if lib.dl_open(os.fsencode(path), ctypes.byref(h)) != 0:
            raise StoreError(lib.dl_last_error(h).decode() if h.value else "dl_open failed")
        return int(lib.dl_count(h))
    finally:
        if h.value:
            lib.dl_close(h)


def _words(ok: np.ndarray) -> np.ndarray:
    """bool[n] -> int64 words, bit i = ok[i], LSB first (the kernels' bitmap layout)."""
    n = len(ok)
    padded = np.zeros(((n + 63) // 64) * 64, np.uint8)
    padded[:n] = ok
    return np.packbits(padded, bitorder="little").view(np.int64)


def verify_store_sharded(engine, public_key: bytes, path, device=None, group=None, group_hash=None):
    """Multi-GPU offline check of one store (SURVEY.md §8e applied to §8f rank 2).

    Each rank loads and verifies a contiguous slice of the stored entries (``shard.shard_range``).
    No halo is needed: every stored beacon carries its own PreviousSig. The exchange is
    ``shard.combine``: one SUM all-reduce of the global-position bitmap and the per-rank first bad rounds.
    Returns (global first bad round or None, global ok bool array in stored order)."""
    import torch
    import torch.distributed as dist

    from . import shard

    world, rank = dist.get_world_size(group), dist.get_rank(group)
    sh = shard.shard_range(store_count(path), world, rank)
    sb = load_store(path, start=sh.start, max_n=sh.count)
    v = verify_store(engine, public_key, sb, group_hash)
    words = torch.from_numpy(_words(v.ok).copy())
    if device is not None:
        words = words.to(device)
    fb, gwords = shard.combine(shard.NONE_U64 if v.first_bad is None else v.first_bad, words, sh.count,
                               group=group)
    total = sum(shard.shard_range(store_count(path), world, r).count for r in range(world))
    bits = np.unpackbits(np.array(gwords, dtype=np.uint64).view(np.uint8), bitorder="little")[:total]
    return (None if fb == shard.NONE_U64 else fb), bits.astype(bool)
