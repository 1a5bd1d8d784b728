"""Minimal bbolt (go.etcd.io/bbolt v1.3.4) file writer: TEST INFRASTRUCTURE ONLY.

Writes the layout drand's boltStore produces (chain/boltdb/store.go:21,68-81): a root bucket with
one sub-bucket "beacons", keys = 8-byte BE rounds, values = hexjson chain.Beacon. Pages follow the
published bbolt format (16-byte page header; meta {magic, version 2, pageSize, flags, root bucket,
freelist, pgid, txid, FNV-1a-64 checksum}; branch elements {pos, ksize, pgid}; leaf elements
{flags, pos, ksize, vsize}, pos relative to the element). Used to build fixtures for
drand_amd/boltload; parity with files bbolt itself writes is unpinned (no drand.db in the reference).
"""
from __future__ import annotations

import struct

MAGIC = 0xED0CDAED
BRANCH, LEAF, META, FREELIST = 0x01, 0x02, 0x04, 0x10


def _fnv64a(b):
    h = 0xcbf29ce484222325
    for c in b:
        h ^= c
        h = (h * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return h


def _page(pid, flags, count, body, ps, overflow=0):
    hdr = struct.pack("<QHHI", pid, flags, count, overflow)
    raw = hdr + body
    span = ps * (overflow + 1)
    assert len(raw) <= span, (len(raw), span)
    return raw + b"\0" * (span - len(raw))


def _leaf_body(items, flags_of=lambda k: 0):
    n = len(items)
    elems, data = b"", b""
    for i, (k, v) in enumerate(items):
        pos = 16 * (n - i) + len(data)          # from this element to its key
        elems += struct.pack("<IIII", flags_of(k), pos, len(k), len(v))
        data += k + v
    return elems + data


def _branch_body(children):
    n = len(children)
    elems, data = b"", b""
    for i, (k, pid) in enumerate(children):
        pos = 16 * (n - i) + len(data)
        elems += struct.pack("<IIQ", pos, len(k), pid)
        data += k
    return elems + data


def write_db(path, items, page_size=4096, per_leaf=5, inline=False, txids=(1, 2), corrupt_meta1=False):
    """items: list of (key bytes, value bytes) in key order."""
    pages = {}
    next_id = 4                                  # 0,1 meta; 2 freelist; 3 root bucket leaf
    if inline:
        ip = struct.pack("<QHHI", 0, LEAF, len(items), 0) + _leaf_body(items)   # inline: not page-sized
        bucket_val = struct.pack("<QQ", 0, 0) + ip
    else:
        leaves = []
        for s in range(0, max(len(items), 1), per_leaf):
            chunk = items[s:s + per_leaf]
            body = _leaf_body(chunk)
            ovf = (16 + len(body) - 1) // page_size
            pid = next_id
            next_id += ovf + 1
            pages[pid] = _page(pid, LEAF, len(chunk), body, page_size, ovf)
            leaves.append((chunk[0][0] if chunk else b"", pid))
        level = leaves
        fan = (page_size - 16) // 24               # 8-byte keys: 16-byte element + key
        while len(level) > 1:                      # build branch levels up to a single root
            up = []
            for s in range(0, len(level), fan):
                kids = level[s:s + fan]
                pid = next_id
                next_id += 1
                pages[pid] = _page(pid, BRANCH, len(kids), _branch_body(kids), page_size)
                up.append((kids[0][0], pid))
            level = up
        root = level[0][1]
        bucket_val = struct.pack("<QQ", root, 0)
    rbody = _leaf_body([(b"beacons", bucket_val)], lambda k: 1)
    rovf = (16 + len(rbody) - 1) // page_size
    assert rovf == 0 or inline                   # a page-backed bucket keeps the root page small
    next_id += rovf
    pages[3] = _page(3, LEAF, 1, rbody, page_size, rovf)
    pages[2] = _page(2, FREELIST, 0, b"", page_size)
    for m, tx in enumerate(txids):
        meta = struct.pack("<IIII", MAGIC, 2, page_size, 0) + struct.pack("<QQ", 3, 0) + \
            struct.pack("<QQQ", 2, next_id, tx)
        cs = _fnv64a(meta)
        if corrupt_meta1 and m == 1:
            cs ^= 1
        pages[m] = _page(m, META, 0, meta + struct.pack("<Q", cs), page_size)
    with open(path, "wb") as f:
        for pid in range(next_id):
            if pid in pages:
                f.write(pages[pid])
            elif not any(p < pid < p + len(pages[p]) // page_size for p in pages):
                f.write(b"\0" * page_size)
