"""ctypes binding of libblsverify.so (the C ABI declared in include/blsverify.h).

There is no CPU fallback: if the HIP library is missing or fails to load, every entry point raises.
The library is built in-tree by `python __graft_entry__.py` / `make -C drand_amd/csrc`.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DRAND_AMD_LIB", os.path.join(_HERE, "libblsverify.so"))

BLSV_OK = 0
BLSV_EINVAL = -1
BLSV_EHIP = -2
BLSV_ENOGROUP = -3
BLSV_ENOTENOUGH = -4

AGG_OK = 0
AGG_OK_V2 = 1
AGG_V1_RECOVER_FAIL = 2
AGG_V1_INVALID = 3
AGG_V2_RECOVER_FAIL = 4

REJ_OK = 0
REJ_LENGTH = 1
REJ_FLAG = 2
REJ_INF_NONZERO = 3
REJ_X_GE_P = 4
REJ_NOT_ON_CURVE = 5
REJ_NOT_IN_SUBGROUP = 6
REJ_PAIRING = 7
REJ_SHARE_INDEX = 8

REJ_NAMES = {
    REJ_OK: "ok",
    REJ_LENGTH: "bad length",
    REJ_FLAG: "bad compression flag",
    REJ_INF_NONZERO: "infinity with non-zero bits",
    REJ_X_GE_P: "coordinate >= p",
    REJ_NOT_ON_CURVE: "point is not on curve",
    REJ_NOT_IN_SUBGROUP: "point is not on correct subgroup",
    REJ_PAIRING: "bls: invalid signature",
    REJ_SHARE_INDEX: "tbls: invalid signature share",
}

u8p = ctypes.POINTER(ctypes.c_uint8)
u32p = ctypes.POINTER(ctypes.c_uint32)
u64p = ctypes.POINTER(ctypes.c_uint64)
vp = ctypes.c_void_p
sz = ctypes.c_size_t

# name -> (restype, argtypes); exactly the symbols of include/blsverify.h + blsverify_testing.h
SIGNATURES = {
    "blsv_version": (ctypes.c_char_p, []),
    "blsv_device_count": (ctypes.c_int, []),
    "blsv_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(vp)]),
    "blsv_destroy": (None, [vp]),
    "blsv_last_error": (ctypes.c_char_p, [vp]),
    "blsv_synchronize": (ctypes.c_int, [vp]),
    "blsv_set_group": (ctypes.c_int, [vp, u8p, sz, sz]),
    "blsv_verify_chained": (ctypes.c_int, [vp, ctypes.c_uint64, u8p, sz, u8p, sz, u8p, u64p, u8p]),
    "blsv_verify_chained_multi": (ctypes.c_int, [ctypes.POINTER(vp), sz, ctypes.POINTER(sz), ctypes.c_uint64, u8p, sz,
                                                  u8p, sz, u8p, u64p, u8p]),
    "blsv_verify_prevs": (ctypes.c_int, [vp, ctypes.c_uint64, u8p, sz, u8p, sz, u8p, u64p, u8p]),
    "blsv_verify_unchained": (ctypes.c_int, [vp, u64p, ctypes.c_uint64, u8p, sz, u8p, u64p, u8p]),
    "blsv_verify_messages": (ctypes.c_int, [vp, u8p, u8p, u32p, sz, u8p, u8p, u64p, u8p]),
    "blsv_verify_partials": (ctypes.c_int, [vp, u8p, sz, u8p, sz, sz, u8p, u8p]),
    "blsv_verify_partials_multi": (ctypes.c_int, [vp, u8p, u32p, u8p, sz, sz, u8p, u8p]),
    "blsv_recover": (ctypes.c_int, [vp, u8p, sz, u8p, sz, sz, sz, sz, u8p]),
    "blsv_aggregate": (ctypes.c_int, [vp, u8p, sz, u8p, sz, sz, sz, sz, u8p, u8p, u8p, u8p]),
    "blsv_aggregate_round": (ctypes.c_int, [vp, u8p, sz, u8p, sz, u8p, sz, u8p, sz, sz, sz, sz, u8p, u8p, u8p, u8p,
                                             ctypes.POINTER(ctypes.c_int32), u8p]),
    "blsv_sign": (ctypes.c_int, [vp, u8p, ctypes.c_int32, u8p, u32p, sz, u8p]),
    "blsv_verify_chained_dev": (ctypes.c_int, [vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, vp, sz, vp, sz,
                                                vp, vp, vp, vp]),
    "blsv_generate_chained_dev": (ctypes.c_int, [vp, u8p, ctypes.c_uint64, ctypes.c_uint64, vp, sz, vp, sz, vp]),
    "blsv_profile_enable": (ctypes.c_int, [vp, ctypes.c_int]),
    "blsv_profile_read": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_double), u64p, u64p, ctypes.c_int]),
    "blsv_lat_trace": (ctypes.c_int, [vp, u64p, ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.c_int]),
    "blsv_test_fp_mul": (ctypes.c_int, [vp, u32p, u32p, sz, u32p]),
    "blsv_test_pairing": (ctypes.c_int, [vp, u32p, u32p, sz, u32p]),
    "blsv_test_hash_to_g2": (ctypes.c_int, [vp, u8p, u32p, sz, u32p, u8p]),
    "blsv_test_final_exp": (ctypes.c_int, [vp, u32p, sz, u32p, u32p]),
    "blsv_set_lat_max": (sz, [vp, sz]),
    "blsv_set_chunk": (sz, [vp, sz]),
    "blsv_workspace_bytes": (sz, [vp]),
    "blsv_lat_trace_enable": (ctypes.c_int, [vp, ctypes.c_int]),
    "blsv_test_generic_chains": (ctypes.c_int, [vp, ctypes.c_int]),
    "blsv_test_spec_stats": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    "blsv_test_lagrange": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint32), ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint32)]),
    "blsv_service_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(vp)]),
    "blsv_service_destroy": (None, [vp]),
    "blsv_service_verify_partial": (ctypes.c_int, [vp, u8p, sz, sz, u8p, sz, u8p, sz, u8p, u8p]),
    "blsv_service_verify_recovered": (ctypes.c_int, [vp, u8p, u8p, sz, u8p, u8p, u8p]),
    "blsv_service_stats": (ctypes.c_int, [vp, u64p, u64p, u64p]),
    "blsv_test_service_limits": (ctypes.c_int, [vp, sz, sz, sz, u64p]),
}

_lib = None


class EngineUnavailable(RuntimeError):
    """The HIP engine library could not be loaded (no silent fallback exists)."""


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise EngineUnavailable(
            f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(make -C drand_amd/csrc); drand_amd has no CPU fallback")
    try:
        lib = ctypes.CDLL(LIB_PATH)
    except OSError as e:
        raise EngineUnavailable(f"cannot load {LIB_PATH}: {e}") from e
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def buf(data):
    """bytes-like -> (ctypes uint8 array, keepalive)."""
    if data is None:
        return None
    b = bytes(data)
    arr = (ctypes.c_uint8 * max(len(b), 1)).from_buffer_copy(b if b else b"\0")
    return arr


def out_buf(n):
    return (ctypes.c_uint8 * max(n, 1))()
