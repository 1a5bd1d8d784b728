"""ctypes loader of the C oracle (oracle/c/bls_oracle.c -> oracle/c/build/libbls_oracle.so).

CPU ORACLE, test infrastructure only: loaded by tests/ and bench.py's cpu_baseline leg, never by
the product path (drand_amd/). Build: make -C oracle (also run by __graft_entry__.build()).
"""
from __future__ import annotations

import ctypes
import os

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c", "build", "libbls_oracle.so")
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FileNotFoundError(f"{LIB_PATH} missing: run `make -C oracle`")
        lib = ctypes.CDLL(LIB_PATH)
        c_u8p = ctypes.c_char_p
        lib.bo_init.restype = ctypes.c_int
        lib.bo_verify.argtypes = [c_u8p, c_u8p, ctypes.c_size_t, c_u8p, ctypes.c_size_t]
        lib.bo_verify.restype = ctypes.c_int
        lib.bo_verify_chained.argtypes = [c_u8p, ctypes.c_uint64, c_u8p, ctypes.c_size_t, c_u8p, ctypes.c_size_t,
                                          ctypes.c_void_p]
        lib.bo_verify_chained.restype = ctypes.c_long
        lib.bo_hash_to_g2.argtypes = [c_u8p, ctypes.c_size_t, ctypes.c_char_p]
        lib.bo_sign.argtypes = [c_u8p, c_u8p, ctypes.c_size_t, ctypes.c_char_p]
        lib.bo_g2_decode_class.argtypes = [c_u8p, ctypes.c_size_t]
        lib.bo_group_new.argtypes = [c_u8p, ctypes.c_int]
        lib.bo_group_new.restype = ctypes.c_void_p
        lib.bo_group_free.argtypes = [ctypes.c_void_p]
        lib.bo_tbls_verify_partial.argtypes = [ctypes.c_void_p, c_u8p, ctypes.c_size_t, c_u8p, ctypes.c_size_t]
        lib.bo_tbls_recover.argtypes = [ctypes.c_void_p, c_u8p, ctypes.c_size_t, c_u8p, ctypes.c_void_p,
                                        ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_char_p]
        lib.bo_init()  # constants; must precede any multi-threaded use
        _lib = lib
    return _lib


def verify(pk48: bytes, msg: bytes, sig: bytes) -> int:
    """kyber bls.Verify -> reject class (0 = accept, -1 = pk does not decode)."""
    return load().bo_verify(pk48, msg, len(msg), sig, len(sig))


def verify_chained(pk48: bytes, first_round: int, prev0: bytes, sigs: bytes):
    """chain.VerifyBeacon over a chained range -> list of reject classes."""
    n = len(sigs) // 96
    cls = (ctypes.c_uint8 * max(n, 1))()
    rc = load().bo_verify_chained(pk48, first_round, prev0, len(prev0), sigs, n, ctypes.cast(cls, ctypes.c_void_p))
    if rc < 0:
        raise ValueError("public key does not decode")
    return list(cls)[:n]


def hash_to_g2(msg: bytes) -> bytes:
    out = ctypes.create_string_buffer(96)
    load().bo_hash_to_g2(msg, len(msg), out)
    return out.raw


def sign(sk: int, msg: bytes) -> bytes:
    out = ctypes.create_string_buffer(96)
    load().bo_sign(sk.to_bytes(32, "big"), msg, len(msg), out)
    return out.raw


def g2_decode_class(sig: bytes) -> int:
    return load().bo_g2_decode_class(sig, len(sig))


class Group:
    """share.PubPoly of t G1 commitments (decoded once), for tbls VerifyPartial / Recover."""

    def __init__(self, commits48):
        self._h = load().bo_group_new(b"".join(commits48), len(commits48))
        if not self._h:
            raise ValueError("a commitment does not decode")

    def close(self):
        if self._h:
            load().bo_group_free(self._h)
            self._h = None

    __del__ = close

    def verify_partial(self, msg: bytes, partial: bytes) -> int:
        """tbls.VerifyPartial -> reject class (0 = accept)."""
        return load().bo_tbls_verify_partial(self._h, msg, len(msg), partial, len(partial))

    def recover(self, msg: bytes, partials, t: int, n: int):
        """tbls.Recover -> 96-byte group signature, or None (not enough good shares)."""
        lens = (ctypes.c_size_t * max(len(partials), 1))(*[len(p) for p in partials])
        out = ctypes.create_string_buffer(96)
        rc = load().bo_tbls_recover(self._h, msg, len(msg), b"".join(partials), ctypes.cast(lens, ctypes.c_void_p),
                                    len(partials), t, n, out)
        return out.raw if rc == 0 else None
