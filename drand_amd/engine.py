"""Python handle on one engine context (one HIP device, one stream): thin wrappers over the C ABI.

Every method runs the HIP kernels; nothing here computes a verdict on the CPU.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

from . import _lib
from ._lib import u8p, u32p, u64p


class EngineError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"blsverify error {code}: {msg}")
        self.code = code


@dataclass
class BatchResult:
    """Outcome of a batch verify: ok[i] per item, first_bad (round or index, None if all ok),
    reject classes (REJ_*) per item."""
    ok: list
    first_bad: int | None
    reject_class: list

    @property
    def all_ok(self):
        return self.first_bad is None

    def bitmap(self):
        out = bytearray((len(self.ok) + 7) // 8)
        for i, v in enumerate(self.ok):
            if v:
                out[i // 8] |= 1 << (i % 8)
        return bytes(out)


def _bits(bitmap, n):
    import numpy as np
    if n == 0:
        return []
    return np.unpackbits(np.frombuffer(bytes(bitmap), np.uint8), bitorder="little")[:n].astype(bool).tolist()


class Engine:
    """One blsv_ctx. Not thread-safe (like the C context); create one per thread."""

    def __init__(self, device: int = 0, init_torch: bool = True):
        if init_torch:
            # torch ships its own HIP runtime next to /opt/rocm's. The order bench.py uses is the
            # one that works on the MI355X boxes: torch's runtime is up (a first allocation) before
            # libblsverify.so is loaded, and device buffers from torch are passed to the *_dev and
            # verify_prevs entry points.
            try:
                import torch
            except ImportError:
                torch = None
            if torch is not None:
                torch.cuda.set_device(int(device))
                torch.zeros(1, device=torch.device("cuda", int(device)))
        self.lib = _lib.load()
        h = ctypes.c_void_p()
        rc = self.lib.blsv_create(int(device), ctypes.byref(h))
        if rc != 0:
            raise EngineError(rc, f"blsv_create(device={device}) failed")
        self._h = h
        self.device = device

    # ------------------------------------------------------------------ lifecycle
    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self.lib.blsv_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, rc):
        if rc != 0:
            raise EngineError(rc, self.lib.blsv_last_error(self._h).decode())
        return rc

    @property
    def handle(self):
        return self._h

    def synchronize(self):
        self._check(self.lib.blsv_synchronize(self._h))

    # ------------------------------------------------------------------ group
    def set_group(self, commits, n=None):
        """commits: list of 48-byte compressed G1 points (commits[0] = group public key)."""
        commits = [bytes(c) for c in commits]
        if any(len(c) != 48 for c in commits):
            raise ValueError("commitments must be 48 bytes")
        t = len(commits)
        self._check(self.lib.blsv_set_group(self._h, _lib.buf(b"".join(commits)), t, n if n is not None else t))

    def set_public_key(self, pk48):
        self.set_group([pk48], 1)

    # ------------------------------------------------------------------ verification
    def verify_chained(self, first_round, prev0, sigs):
        n = len(sigs)
        sigb = b"".join(bytes(s) for s in sigs)
        if any(len(s) != 96 for s in sigs):
            raise ValueError("chained signatures must be 96 bytes (reject wrong lengths host-side)")
        bm = _lib.out_buf((n + 7) // 8)
        fb = ctypes.c_uint64()
        cls = _lib.out_buf(n)
        self._check(self.lib.blsv_verify_chained(self._h, first_round, _lib.buf(prev0), len(prev0), _lib.buf(sigb), n,
                                                 bm, ctypes.byref(fb), cls))
        return BatchResult(_bits(bm, n), None if fb.value == 2 ** 64 - 1 else fb.value, list(cls)[:n])

    def verify_chained_packed(self, first_round, prev0, sigs96, n):
        """``verify_chained`` over n signatures already packed as n*96 contiguous bytes (any object
        with the buffer protocol, e.g. a numpy slice of the bulk loader's SoA array)."""
        mv = memoryview(sigs96).cast("B")
        if len(mv) != 96 * n:
            raise ValueError("packed signatures must be n*96 bytes")
        bm = _lib.out_buf((n + 7) // 8)
        fb = ctypes.c_uint64()
        cls = _lib.out_buf(n)
        src = (ctypes.c_uint8 * max(len(mv), 1)).from_buffer_copy(mv) if len(mv) else None
        self._check(self.lib.blsv_verify_chained(self._h, first_round, _lib.buf(prev0), len(prev0), src, n, bm,
                                                 ctypes.byref(fb), cls))
        return BatchResult(_bits(bm, n), None if fb.value == 2 ** 64 - 1 else fb.value, list(cls)[:n])

    def verify_prevs(self, first_round, prev0_len, prevs96, sigs96, n):
        """``chain.VerifyBeacon`` for n consecutive rounds, each with its own stored PreviousSig
        (``blsv_verify_prevs``): prevs96 / sigs96 are n*96 packed bytes (row 0's prev uses its first
        prev0_len = 32 or 96 bytes, every other row all 96). One device pass (drand.db ranges).
        Bulk form: ``ok`` and ``reject_class`` come back as numpy arrays, and the inputs are passed
        to the library without a host copy when they are contiguous numpy arrays."""
        import numpy as np
        p = np.ascontiguousarray(np.frombuffer(memoryview(prevs96).cast("B"), np.uint8))
        q = np.ascontiguousarray(np.frombuffer(memoryview(sigs96).cast("B"), np.uint8))
        if len(p) != 96 * n or len(q) != 96 * n:
            raise ValueError("prevs and sigs must be n*96 bytes")
        bm = np.zeros(max((n + 7) // 8, 1), np.uint8)
        cls = np.zeros(max(n, 1), np.uint8)
        fb = ctypes.c_uint64()
        u8 = ctypes.POINTER(ctypes.c_uint8)
        ptr = lambda a: a.ctypes.data_as(u8) if a.size else None
        self._check(self.lib.blsv_verify_prevs(self._h, first_round, ptr(p), prev0_len, ptr(q), n, ptr(bm),
                                               ctypes.byref(fb), ptr(cls)))
        ok = np.unpackbits(bm, bitorder="little")[:n].astype(bool)
        return BatchResult(ok, None if fb.value == 2 ** 64 - 1 else fb.value, cls[:n])

    def verify_unchained(self, sigs, first_round=None, rounds=None):
        n = len(sigs)
        if any(len(s) != 96 for s in sigs):
            raise ValueError("signatures must be 96 bytes (reject wrong lengths host-side)")
        sigb = b"".join(bytes(s) for s in sigs)
        rr = None
        if rounds is not None:
            rr = (ctypes.c_uint64 * max(n, 1))(*rounds)
        bm = _lib.out_buf((n + 7) // 8)
        fb = ctypes.c_uint64()
        cls = _lib.out_buf(n)
        self._check(self.lib.blsv_verify_unchained(self._h, rr, first_round or 0, _lib.buf(sigb), n, bm,
                                                   ctypes.byref(fb), cls))
        return BatchResult(_bits(bm, n), None if fb.value == 2 ** 64 - 1 else fb.value, list(cls)[:n])

    def verify_messages(self, msgs, sigs, pk48=None):
        n = len(msgs)
        assert len(sigs) == n
        if any(len(s) != 96 for s in sigs):
            raise ValueError("signatures must be 96 bytes (reject wrong lengths host-side)")
        lens = (ctypes.c_uint32 * max(n, 1))(*[len(m) for m in msgs])
        bm = _lib.out_buf((n + 7) // 8)
        fb = ctypes.c_uint64()
        cls = _lib.out_buf(n)
        self._check(self.lib.blsv_verify_messages(self._h, _lib.buf(pk48) if pk48 is not None else None,
                                                  _lib.buf(b"".join(bytes(m) for m in msgs)), lens, n,
                                                  _lib.buf(b"".join(bytes(s) for s in sigs)), bm, ctypes.byref(fb),
                                                  cls))
        return BatchResult(_bits(bm, n), None if fb.value == 2 ** 64 - 1 else fb.value, list(cls)[:n])

    def verify_partials(self, msg, partials):
        k = len(partials)
        plen = len(partials[0]) if k else 98
        if any(len(p) != plen for p in partials):
            raise ValueError("partials of one call must share a length")
        ok = _lib.out_buf(k)
        cls = _lib.out_buf(k)
        self._check(self.lib.blsv_verify_partials(self._h, _lib.buf(msg), len(msg),
                                                  _lib.buf(b"".join(bytes(p) for p in partials)), plen, k, ok, cls))
        return [bool(x) for x in list(ok)[:k]], list(cls)[:k]

    def verify_partials_multi(self, msgs, partials):
        """Partials of many rounds in one pass: partial i signs msgs[i] (blsv_verify_partials_multi)."""
        k = len(partials)
        assert len(msgs) == k
        plen = len(partials[0]) if k else 98
        if any(len(p) != plen for p in partials):
            raise ValueError("partials of one call must share a length")
        lens = (ctypes.c_uint32 * max(k, 1))(*[len(m) for m in msgs])
        ok = _lib.out_buf(k)
        cls = _lib.out_buf(k)
        self._check(self.lib.blsv_verify_partials_multi(self._h, _lib.buf(b"".join(bytes(m) for m in msgs)), lens,
                                                        _lib.buf(b"".join(bytes(p) for p in partials)), plen, k, ok,
                                                        cls))
        return [bool(x) for x in list(ok)[:k]], list(cls)[:k]

    def recover(self, msg, partials, t, n):
        k = len(partials)
        plen = len(partials[0]) if k else 98
        out = _lib.out_buf(96)
        self._check(self.lib.blsv_recover(self._h, _lib.buf(msg), len(msg),
                                          _lib.buf(b"".join(bytes(p) for p in partials)), plen, k, t, n, out))
        return bytes(out)

    def aggregate(self, msg, partials, t, n):
        """One aggregator round (blsv_aggregate): (ok per partial, reject classes, group sig, group_ok)."""
        k = len(partials)
        plen = len(partials[0]) if k else 98
        if any(len(p) != plen for p in partials):
            raise ValueError("partials of one call must share a length")
        ok = _lib.out_buf(k)
        cls = _lib.out_buf(k)
        out = _lib.out_buf(96)
        gok = _lib.out_buf(1)
        self._check(self.lib.blsv_aggregate(self._h, _lib.buf(msg), len(msg),
                                            _lib.buf(b"".join(bytes(p) for p in partials)), plen, k, t, n, ok, cls,
                                            out, gok))
        return [bool(x) for x in list(ok)[:k]], list(cls)[:k], bytes(out), bool(gok[0])

    def aggregate_round(self, msg1, partials1, msg2, partials2, t, n):
        """The aggregation step of one round cache, V1 + V2 (blsv_aggregate_round, chain.go:131-166):
        returns (status AGG_*, ok1, ok2, sig1, sig2 or None, v2_valid)."""
        # A share of the wrong length cannot parse: kyber's Recover skips it and VerifyPartial rejects
        # it, but it still counts in roundCache.Len()/LenV2() -- the V2 gate `LenV2() >= thr`
        # (chain.go:153) sees it. So it is passed on as a 98-byte share that can never verify (index
        # 0xFFFF >= n, compression flag clear): the C side counts it toward k2 >= t, rejects it
        # (ok = False at its position) and Recover skips it, exactly as kyber does.
        bad_share = b"\xff\xff" + bytes(96)
        partials1 = [p if len(p) == 98 else bad_share for p in (bytes(p) for p in partials1)]
        partials2 = [p if len(p) == 98 else bad_share for p in (bytes(p) for p in partials2)]
        k1, k2 = len(partials1), len(partials2)
        plen = 98
        ok1, ok2 = _lib.out_buf(k1), _lib.out_buf(k2)
        s1, s2 = _lib.out_buf(96), _lib.out_buf(96)
        st = ctypes.c_int32()
        v2 = _lib.out_buf(1)
        self._check(self.lib.blsv_aggregate_round(
            self._h, _lib.buf(msg1), len(msg1), _lib.buf(b"".join(partials1)), k1,
            _lib.buf(msg2), len(msg2), _lib.buf(b"".join(partials2)), k2, plen, t, n, ok1, ok2,
            s1, s2, ctypes.byref(st), v2))
        status = st.value
        sig1 = bytes(s1) if status in (_lib.AGG_OK, _lib.AGG_OK_V2, _lib.AGG_V1_INVALID,
                                       _lib.AGG_V2_RECOVER_FAIL) else None
        sig2 = bytes(s2) if status == _lib.AGG_OK_V2 else None
        r1 = [bool(x) for x in list(ok1)[:k1]]
        r2 = [bool(x) for x in list(ok2)[:k2]]
        return status, r1, r2, sig1, sig2, bool(v2[0])

    def sign(self, sk32, msgs, index=-1):
        n = len(msgs)
        lens = (ctypes.c_uint32 * max(n, 1))(*[len(m) for m in msgs])
        stride = 98 if index >= 0 else 96
        out = _lib.out_buf(n * stride)
        self._check(self.lib.blsv_sign(self._h, _lib.buf(sk32), index, _lib.buf(b"".join(bytes(m) for m in msgs)),
                                       lens, n, out))
        ob = bytes(out)
        return [ob[i * stride:(i + 1) * stride] for i in range(n)]

    # ------------------------------------------------------------------ device-resident batches
    def verify_chained_dev(self, first_round, seg_len, d_seeds, seed0_len, d_sigs, n, d_bitmap, d_first_bad,
                           d_cls=None, stream=None, seg_phase=0):
        self._check(self.lib.blsv_verify_chained_dev(self._h, first_round, seg_len, seg_phase, d_seeds, seed0_len,
                                                     d_sigs, n, d_bitmap, d_first_bad, d_cls, stream))

    def generate_chained_dev(self, sk32, first_round, seg_len, d_seeds, seed0_len, d_sigs, n, stream=None):
        self._check(self.lib.blsv_generate_chained_dev(self._h, _lib.buf(sk32), first_round, seg_len, d_seeds,
                                                       seed0_len, d_sigs, n, stream))

    # ------------------------------------------------------------------ stage profiling
    STAGES = ("hash", "decompress", "miller", "final_exp", "finish", "lat")

    def profile(self, on=True):
        self._check(self.lib.blsv_profile_enable(self._h, 1 if on else 0))

    def profile_read(self):
        """{stage: (summed ms, launches, items)} since the last read (HIP events on the launch stream)."""
        n = len(self.STAGES)
        ms = (ctypes.c_double * n)()
        la = (ctypes.c_uint64 * n)()
        it = (ctypes.c_uint64 * n)()
        rc = self.lib.blsv_profile_read(self._h, ms, la, it, n)
        if rc < 0:
            raise EngineError(rc, self.lib.blsv_last_error(self._h).decode())
        return {s: (ms[k], la[k], it[k]) for k, s in enumerate(self.STAGES)}

    LAT_MARKS = ("start", "hash", "sig_decoded", "sig_miller", "phase_a", "key_miller", "miller_product",
                 "final_exp", "pow1_start", "pow1_end", "xmd_done", "sswu_done", "iso_add_done", "cofactor_done",
                 "sig_sqrt_done", "sig_subgroup_done")

    def lat_trace_enable(self, on=True):
        """Turn the latency kernel's phase marks on or off (a device-global flag, off by default)."""
        self._check(self.lib.blsv_lat_trace_enable(self._h, 1 if on else 0))

    def lat_trace(self, clear=True):
        """Phase marks (microseconds from the first mark) of item 0 of the last latency-path launch
        while marks are enabled (blsv_lat_trace_enable, blsv_lat_trace); marks never stamped are left
        out."""
        n = len(self.LAT_MARKS)
        t = (ctypes.c_uint64 * n)()
        rate = ctypes.c_double()
        got = self.lib.blsv_lat_trace(self._h, t, n, ctypes.byref(rate), 1 if clear else 0)
        if got < 0:
            raise EngineError(got, self.lib.blsv_last_error(self._h).decode())
        t0 = t[0]
        return {k: (t[i] - t0) / rate.value for i, k in enumerate(self.LAT_MARKS[:got]) if t[i] and t0}

    # ------------------------------------------------------------------ testing hooks
    def set_lat_max(self, n):
        """Batches of at most n items take the latency path (one 8-wave workgroup per item; default
        1,536, clamped to the chunk); returns the old cutover."""
        return self.lib.blsv_set_lat_max(self._h, int(n))

    def set_chunk(self, items):
        """Cap the items per pipeline pass (~42.4 KB of HBM staging per item; 0 = the default 2^20);
        returns the previous chunk (blsv_set_chunk)."""
        return self.lib.blsv_set_chunk(self._h, int(items))

    def workspace_bytes(self):
        """HBM bytes of pipeline staging this context holds (blsv_workspace_bytes)."""
        return self.lib.blsv_workspace_bytes(self._h)

    def test_fp_mul(self, a_limbs, b_limbs):
        n = len(a_limbs) // 12
        A = (ctypes.c_uint32 * max(len(a_limbs), 1))(*a_limbs)
        B = (ctypes.c_uint32 * max(len(b_limbs), 1))(*b_limbs)
        O = (ctypes.c_uint32 * max(n * 12, 1))()
        self._check(self.lib.blsv_test_fp_mul(self._h, A, B, n, O))
        return list(O)[:n * 12]

    def test_pairing(self, p_words, q_words):
        n = len(p_words) // 24
        Pp = (ctypes.c_uint32 * max(len(p_words), 1))(*p_words)
        Q = (ctypes.c_uint32 * max(len(q_words), 1))(*q_words)
        O = (ctypes.c_uint32 * max(n * 144, 1))()
        self._check(self.lib.blsv_test_pairing(self._h, Pp, Q, n, O))
        return list(O)[:n * 144]

    def test_final_exp(self, f_words):
        """(production stage, one-lane reference) final exponentiations of n Fp12 (144 raw words each)."""
        n = len(f_words) // 144
        Fw = (ctypes.c_uint32 * max(len(f_words), 1))(*f_words)
        A = (ctypes.c_uint32 * max(n * 144, 1))()
        B = (ctypes.c_uint32 * max(n * 144, 1))()
        self._check(self.lib.blsv_test_final_exp(self._h, Fw, n, A, B))
        return list(A)[:n * 144], list(B)[:n * 144]

    def test_hash_to_g2(self, msgs):
        n = len(msgs)
        lens = (ctypes.c_uint32 * max(n, 1))(*[len(m) for m in msgs])
        O = (ctypes.c_uint32 * max(n * 48, 1))()
        inf = _lib.out_buf(n)
        self._check(self.lib.blsv_test_hash_to_g2(self._h, _lib.buf(b"".join(bytes(m) for m in msgs)), lens, n, O,
                                                  inf))
        return list(O)[:n * 48], list(inf)[:n]

    def spec_stats(self):
        """(kept, recomputed) speculative recoveries of this context (blsv_test_spec_stats)."""
        h, m = ctypes.c_uint64(), ctypes.c_uint64()
        self._check(self.lib.blsv_test_spec_stats(self._h, ctypes.byref(h), ctypes.byref(m)))
        return h.value, m.value

    def test_generic_chains(self, on=True):
        """Every hash's cofactor clearing and every signature's subgroup check through the generic
        formulas (k_hash_cofactor_generic, k_subgroup_g2_generic) instead of only the lanes the
        call-free chains flag; process-global, for the parity tests."""
        self._check(self.lib.blsv_test_generic_chains(self._h, 1 if on else 0))


def verify_chained_multi(engines, first_round, prev0, sigs, counts=None):
    """blsv_verify_chained_multi: the chained range split into contiguous shards over several
    Engines (one per GPU; each holds the same group), verified concurrently (one host thread per
    context inside the library) and merged: the BatchResult of one verify_chained over the whole
    range. counts: shard lengths (None = even split)."""
    if not engines:
        raise ValueError("verify_chained_multi needs at least one engine")
    lib = engines[0].lib
    n = len(sigs)
    if any(len(s) != 96 for s in sigs):
        raise ValueError("chained signatures must be 96 bytes (reject wrong lengths host-side)")
    sigb = b"".join(bytes(s) for s in sigs)
    hs = (ctypes.c_void_p * len(engines))(*[e._h.value for e in engines])
    cs = None if counts is None else (ctypes.c_size_t * len(engines))(*counts)
    bm = _lib.out_buf((n + 7) // 8)
    fb = ctypes.c_uint64()
    cls = _lib.out_buf(n)
    rc = lib.blsv_verify_chained_multi(hs, len(engines), cs, first_round, _lib.buf(prev0), len(prev0), _lib.buf(sigb),
                                       n, bm, ctypes.byref(fb), cls)
    if rc != 0:
        msgs = "; ".join(lib.blsv_last_error(e._h).decode(errors="replace") for e in engines)
        raise EngineError(rc, f"blsv_verify_chained_multi failed: {msgs}")
    return BatchResult(_bits(bm, n), None if fb.value == 2 ** 64 - 1 else fb.value, list(cls)[:n])


class Service:
    """Thread-safe front end (blsv_service_*): any number of threads call verify_partial /
    verify_recovered at once; items that arrive together are verified in one launch. ctypes releases
    the GIL for the duration of each call, so Python threads block in C side by side."""

    def __init__(self, device: int = 0, gap_us: int = 0, max_wait_us: int = 0, init_torch: bool = True):
        if init_torch:
            try:
                import torch
            except ImportError:
                torch = None
            if torch is not None:
                torch.cuda.set_device(int(device))
                torch.zeros(1, device=torch.device("cuda", int(device)))
        self.lib = _lib.load()
        h = ctypes.c_void_p()
        rc = self.lib.blsv_service_create(int(device), int(gap_us), int(max_wait_us), ctypes.byref(h))
        if rc != 0:
            raise EngineError(rc, f"blsv_service_create(device={device}) failed")
        self._h = h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self.lib.blsv_service_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def verify_partial(self, commits, n, msg, partial):
        """key.Scheme.VerifyPartial(pubPoly, msg, partial): (ok, reject class)."""
        cb = b"".join(bytes(c) for c in commits)
        ok, cls = ctypes.c_uint8(), ctypes.c_uint8()
        p = bytes(partial)
        rc = self.lib.blsv_service_verify_partial(self._h, _lib.buf(cb), len(commits), int(n), _lib.buf(msg), len(msg),
                                                  _lib.buf(p), len(p), ctypes.byref(ok), ctypes.byref(cls))
        if rc != 0:
            raise EngineError(rc, "blsv_service_verify_partial failed")
        return bool(ok.value), cls.value

    def prepare_partial(self, commits, n, msg, partial):
        """A zero-argument callable doing exactly the ctypes call of verify_partial, its arguments
        marshalled in advance (so concurrent Python callers hold the GIL only for the call itself)."""
        cb = _lib.buf(b"".join(bytes(c) for c in commits))
        mb, pb = _lib.buf(msg), _lib.buf(bytes(partial))
        t, ml, pl = len(commits), len(msg), len(partial)
        ok, cls = ctypes.c_uint8(), ctypes.c_uint8()
        f, h, pok, pcls = self.lib.blsv_service_verify_partial, self._h, ctypes.byref(ok), ctypes.byref(cls)

        def call():
            rc = f(h, cb, t, n, mb, ml, pb, pl, pok, pcls)
            if rc != 0:
                raise EngineError(rc, "blsv_service_verify_partial failed")
            return bool(ok.value), cls.value

        return call

    def verify_recovered(self, pk48, msg, sig96):
        """key.Scheme.VerifyRecovered(pub, msg, sig): (ok, reject class)."""
        ok, cls = ctypes.c_uint8(), ctypes.c_uint8()
        rc = self.lib.blsv_service_verify_recovered(self._h, _lib.buf(pk48), _lib.buf(msg), len(msg), _lib.buf(sig96),
                                                    ctypes.byref(ok), ctypes.byref(cls))
        if rc != 0:
            raise EngineError(rc, "blsv_service_verify_recovered failed")
        return bool(ok.value), cls.value

    def test_limits(self, chunk=0, lat_max=(1 << 64) - 1, arena_entries=0):
        """blsv_test_service_limits: shrink the dispatcher's pass size / cutover / key arena (tests of
        the multi-pass and arena-overflow paths); returns the device batches run so far."""
        n = ctypes.c_uint64()
        rc = self.lib.blsv_test_service_limits(self._h, int(chunk), int(lat_max), int(arena_entries), ctypes.byref(n))
        if rc != 0:
            raise EngineError(rc, "blsv_test_service_limits failed")
        return n.value

    def stats(self):
        """(launches, items, largest batch) since creation."""
        a, b, c = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        self.lib.blsv_service_stats(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
        return a.value, b.value, c.value


def limbs_of(v, n=12):
    return [(v >> (32 * i)) & 0xFFFFFFFF for i in range(n)]


def int_of(limbs):
    return sum(int(x) << (32 * i) for i, x in enumerate(limbs))
