"""Wire-format ingest into the engine's batch layout.

Three encodings carry beacons into a verifier in the reference:

* ``chain.Beacon`` as hexjson (chain/beacon.go:35-43; github.com/nikkolasg/hexjson = encoding/json
  with ``[]byte`` as lowercase hex): keys ``PreviousSig``, ``Round``, ``Signature`` and, when set,
  ``SignatureV2``. This is also the value stored per round in bbolt (chain/boltdb/store.go:68-81).
* ``client.RandomData`` from the HTTP relay (client/random.go:5-12, decoded with hexjson at
  client/http/http.go:275-279): ``round``, ``randomness``, ``signature``, ``previous_signature``,
  ``signaturev2``, all ``omitempty``.
* protobuf ``BeaconPacket`` (protobuf/drand/protocol.proto:88-92: previous_sig = 1, round = 2,
  signature = 3) on the sync stream and ``PublicRandResponse`` (protobuf/drand/api.proto:46-54:
  round = 1, signature = 2, previous_signature = 3, randomness = 4, signature_v2 = 5).

``segments()`` turns a decoded stream into the chained SoA runs ``Engine.verify_chained`` takes:
contiguous rounds whose ``previous_sig`` links to the prior ``signature``.
"""
from __future__ import annotations

import json
from dataclasses import dataclass

from .callers import Beacon, RandomData


# ---------------------------------------------------------------------------- hexjson
def beacon_from_json(buf) -> Beacon:
    """``Beacon.Unmarshal`` (chain/beacon.go:40-43). Absent byte fields decode as empty."""
    d = json.loads(buf)
    return Beacon(previous_sig=bytes.fromhex(d.get("PreviousSig") or ""), round=int(d.get("Round", 0)),
                  signature=bytes.fromhex(d.get("Signature") or ""),
                  signature_v2=bytes.fromhex(d.get("SignatureV2") or ""))


def beacon_to_json(b: Beacon) -> bytes:
    """``Beacon.Marshal`` (chain/beacon.go:35-38): field order as declared, SignatureV2 omitempty."""
    d = {"PreviousSig": b.previous_sig.hex(), "Round": b.round, "Signature": b.signature.hex()}
    if b.signature_v2:
        d["SignatureV2"] = b.signature_v2.hex()
    return json.dumps(d, separators=(",", ":")).encode()


def random_from_json(buf, v2from=2 ** 64 - 1) -> RandomData:
    """HTTP ``RandomData`` (client/random.go:5-12); ``version`` set as client/verify.go:102-107 does."""
    d = json.loads(buf)
    r = RandomData(round=int(d.get("round", 0)), signature=bytes.fromhex(d.get("signature") or ""),
                   previous_signature=bytes.fromhex(d["previous_signature"]) if d.get("previous_signature") else None,
                   signature_v2=bytes.fromhex(d.get("signaturev2") or ""),
                   randomness=bytes.fromhex(d.get("randomness") or ""))
    r.version = 2 if r.round >= v2from else 1
    return r


# ---------------------------------------------------------------------------- protobuf
class WireError(ValueError):
    pass


def _varint(buf, i):
    v = shift = 0
    while True:
        if i >= len(buf):
            raise WireError("truncated varint")
        c = buf[i]
        i += 1
        v |= (c & 0x7F) << shift
        if not c & 0x80:
            return v & (2 ** 64 - 1), i
        shift += 7
        if shift >= 70:
            raise WireError("varint too long")


def _put_varint(v):
    out = bytearray()
    while True:
        c = v & 0x7F
        v >>= 7
        if v:
            out.append(c | 0x80)
        else:
            out.append(c)
            return bytes(out)


def _fields(buf):
    """Yield (field number, value) for varint and length-delimited fields; skip fixed32/64."""
    buf = bytes(buf)
    i = 0
    while i < len(buf):
        key, i = _varint(buf, i)
        num, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(buf, i)
        elif wt == 2:
            n, i = _varint(buf, i)
            if i + n > len(buf):
                raise WireError("truncated bytes field")
            v, i = buf[i:i + n], i + n
        elif wt == 1:
            v, i = None, i + 8
        elif wt == 5:
            v, i = None, i + 4
        else:
            raise WireError(f"unsupported wire type {wt}")
        if i > len(buf):
            raise WireError("truncated fixed field")
        yield num, v


def beacon_from_packet(buf) -> Beacon:
    """``protoToBeacon`` (chain/beacon/convert.go:8-14) of a serialized ``BeaconPacket``: there is
    no SignatureV2 on this message, so synced beacons carry none."""
    b = Beacon(previous_sig=b"", round=0, signature=b"")
    for num, v in _fields(buf):
        if num == 1 and isinstance(v, bytes):
            b.previous_sig = v
        elif num == 2 and isinstance(v, int):
            b.round = v
        elif num == 3 and isinstance(v, bytes):
            b.signature = v
    return b


def beacon_to_packet(b: Beacon) -> bytes:
    """proto3 encoding of ``BeaconPacket`` (default values are not emitted)."""
    out = bytearray()
    if b.previous_sig:
        out += _put_varint(1 << 3 | 2) + _put_varint(len(b.previous_sig)) + bytes(b.previous_sig)
    if b.round:
        out += _put_varint(2 << 3 | 0) + _put_varint(b.round)
    if b.signature:
        out += _put_varint(3 << 3 | 2) + _put_varint(len(b.signature)) + bytes(b.signature)
    return bytes(out)


def random_from_response(buf, v2from=2 ** 64 - 1) -> RandomData:
    """``PublicRandResponse`` (api.proto:46-54) → ``RandomData``. core/convert.go:15-22 omits
    ``previous_signature`` on the gRPC path, so such results make a V1 client walk the chain."""
    r = RandomData(round=0)
    for num, v in _fields(buf):
        if num == 1 and isinstance(v, int):
            r.round = v
        elif num == 2 and isinstance(v, bytes):
            r.signature = v
        elif num == 3 and isinstance(v, bytes):
            r.previous_signature = v
        elif num == 4 and isinstance(v, bytes):
            r.randomness = v
        elif num == 5 and isinstance(v, bytes):
            r.signature_v2 = v
    r.version = 2 if r.round >= v2from else 1
    return r


# ---------------------------------------------------------------------------- batch layout
@dataclass
class Segment:
    """One chained run for ``blsv_verify_chained``: rounds first_round .. first_round+n-1,
    ``prev0`` = the first beacon's PreviousSig, ``sigs`` = the n signatures in round order."""
    first_round: int
    prev0: bytes
    sigs: list
    start: int   # index of the first beacon in the input stream

    @property
    def n(self):
        return len(self.sigs)


def segments(beacons):
    """Split a beacon stream into maximal chained runs. A run breaks where the round is not the
    previous round + 1, where PreviousSig differs from the previous Signature, or at a signature
    that is not 96 bytes (that beacon becomes a run of its own so the engine rejects it host-side).
    Each beacon's verdict is unchanged by the split: chain.VerifyBeacon (chain/beacon.go:87-92)
    reads only the beacon's own fields."""
    out = []
    cur = None
    prev = None
    for idx, b in enumerate(beacons):
        sig = bytes(b.signature)
        linked = (cur is not None and len(sig) == 96 and b.round == prev.round + 1
                  and bytes(b.previous_sig) == bytes(prev.signature) and len(prev.signature) == 96)
        if linked:
            cur[2].append(sig)
        else:
            if cur is not None:
                out.append(cur)
            cur = (b.round, bytes(b.previous_sig), [sig], idx)
        prev = b
    if cur is not None:
        out.append(cur)
    return [Segment(fr, p0, s, st) for fr, p0, s, st in out]
