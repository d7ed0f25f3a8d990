"""CPU ORACLE — TEST INFRASTRUCTURE ONLY: the reference's index file format.

Pure-Python restatement of what QueryEngine::save_index / load_index
(src/query.rs:282-409) put on disk: gzip(postcard(IndexPersistenceData)),
with IndexPersistenceData / IndexMetadata at query.rs:16-28 and HnswConfig at
config.rs:196-209.  The serializer is the `postcard` crate 1.x (Cargo.toml:14;
not vendored in /root/reference, so its published wire format is restated
here): struct = fields in order, no tags; usize and every length = unsigned
LEB128 varint; String = varint(len) + UTF-8 bytes; Vec<T> / tuples = varint(len)
+ elements / elements in order; f32 = 4 little-endian bytes.  chrono 0.4's
serde `Serialize for DateTime<Utc>` writes the RFC 3339 string (collect_str of
to_rfc3339_opts(SecondsFormat::AutoSi, use_z = true)), so created_at is a
postcard String.  gzip via flate2's GzEncoder (Compression::default() = 6);
only the decompressed bytes are format-defining.

Parity status: pinned to the postcard / chrono specifications above by the
hand-assembled known-answer bytes in tests/test_persist.py (the reference's
own tests do not exercise save/load, and no reference-written index file
ships with it).

Only tests/ may import this module.
"""
from __future__ import annotations

import gzip
import struct
from typing import List, Sequence, Tuple


def varint(v: int) -> bytes:
    """Unsigned LEB128, as postcard encodes usize / u64 / lengths."""
    if v < 0:
        raise ValueError("varint of a negative value")
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def read_varint(b: bytes, pos: int) -> Tuple[int, int]:
    x, sh = 0, 0
    while True:
        c = b[pos]
        pos += 1
        x |= (c & 0x7F) << sh
        if not c & 0x80:
            return x, pos
        sh += 7
        if sh > 63:
            raise ValueError("varint too long")


def encode(dimension: int, total_points: int, created_at: str, config: Sequence[int],
           vectors: Sequence[Tuple[str, Sequence[float]]]) -> bytes:
    """postcard(IndexPersistenceData) (query.rs:16-28)."""
    out = bytearray()
    out += varint(dimension) + varint(total_points)
    ts = created_at.encode()
    out += varint(len(ts)) + ts
    for c in config:  # m, ef_construction, ef_search, max_layers
        out += varint(c)
    out += varint(len(vectors))
    for sid, vec in vectors:
        bid = sid.encode()
        out += varint(len(bid)) + bid
        out += varint(len(vec))
        out += struct.pack(f"<{len(vec)}f", *vec)
    return bytes(out)


def decode(b: bytes):
    """Inverse of encode: (dimension, total_points, created_at, (m, efc, efs, layers), [(id, [f32])])."""
    pos = 0
    dim, pos = read_varint(b, pos)
    tot, pos = read_varint(b, pos)
    n, pos = read_varint(b, pos)
    created = b[pos:pos + n].decode()
    pos += n
    cfg = []
    for _ in range(4):
        v, pos = read_varint(b, pos)
        cfg.append(v)
    cnt, pos = read_varint(b, pos)
    vecs: List[Tuple[str, List[float]]] = []
    for _ in range(cnt):
        n, pos = read_varint(b, pos)
        sid = b[pos:pos + n].decode()
        pos += n
        n, pos = read_varint(b, pos)
        vec = list(struct.unpack_from(f"<{n}f", b, pos))
        pos += 4 * n
        vecs.append((sid, vec))
    if pos != len(b):
        raise ValueError("trailing bytes")
    return dim, tot, created, tuple(cfg), vecs


def write_file(path: str, payload: bytes) -> None:
    with gzip.open(path, "wb", compresslevel=6) as f:
        f.write(payload)


def read_file(path: str) -> bytes:
    with gzip.open(path, "rb") as f:
        return f.read()
