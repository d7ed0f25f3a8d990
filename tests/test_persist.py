"""Index persistence in the reference's on-disk format (query.rs:282-409).

CPU tests: the C-ABI codec (gvdb_persist_*, host-only code in libgvdb.so)
against the pure-Python restatement in oracle/persist_oracle.py, which is
itself pinned to the postcard / chrono wire format by hand-assembled
known-answer bytes below.  The device round trip (export -> file -> add ->
search) is in test_gpu_persist at the end (marked gpu).
"""
import ctypes as C
import gzip
import os
import re
import struct

import numpy as np
import pytest

from oracle import persist_oracle as po


def _lib(gvdb_lib_path):
    from gvdb import _ffi

    return _ffi.lib()


def _meta(dim, total, created="2024-01-02T03:04:05Z", cfg=(16, 200, 100, 16)):
    from gvdb import _ffi

    return _ffi.gvdb_persist_meta(dim, total, *cfg, created.encode())


def _write(L, path, dim, vectors, created="2024-01-02T03:04:05Z", cfg=(16, 200, 100, 16), batch=7, level=-1):
    from gvdb import check

    w = C.c_void_p()
    check(L.gvdb_persist_create(path.encode(), C.byref(_meta(dim, len(vectors), created, cfg)), len(vectors), level,
                                C.byref(w)))
    for b0 in range(0, len(vectors), batch):
        part = vectors[b0:b0 + batch]
        enc = [s.encode() for s, _ in part]
        offs = np.zeros(len(part) + 1, np.uint64)
        offs[1:] = np.cumsum([len(e) for e in enc])
        rows = np.ascontiguousarray(np.array([v for _, v in part], np.float32).reshape(len(part), dim))
        check(L.gvdb_persist_append(w, rows.ctypes.data, len(part), dim, b"".join(enc) or b"\0", offs.ctypes.data))
    check(L.gvdb_persist_close(w))


def _read(L, path, dim_hint=None, batch=5, blob_cap=1 << 12):
    from gvdb import _ffi, check

    m = _ffi.gvdb_persist_meta()
    cnt = C.c_uint64()
    r = C.c_void_p()
    check(L.gvdb_persist_open(path.encode(), C.byref(m), C.byref(cnt), C.byref(r)))
    D = int(m.dimension) if dim_hint is None else dim_hint
    out = []
    try:
        rows = np.zeros((batch, max(D, 1)), np.float32)
        offs = np.zeros(batch + 1, np.uint64)
        blob = C.create_string_buffer(blob_cap)
        got = C.c_uint64()
        while True:
            check(L.gvdb_persist_next(r, rows.ctypes.data, D, batch, blob, blob_cap, offs.ctypes.data, C.byref(got)))
            if got.value == 0:
                break
            raw = blob.raw
            for i in range(got.value):
                out.append((raw[int(offs[i]):int(offs[i + 1])].decode(), rows[i, :D].copy()))
    finally:
        L.gvdb_persist_free(r)
    cfg = (int(m.m), int(m.ef_construction), int(m.ef_search), int(m.max_layers))
    return int(m.dimension), int(m.total_points), m.created_at.decode(), cfg, int(cnt.value), out


# -- the oracle against the wire-format specification ------------------------------
def test_varint_known_answers():
    # unsigned LEB128 as postcard encodes usize
    assert po.varint(0) == b"\x00"
    assert po.varint(1) == b"\x01"
    assert po.varint(127) == b"\x7f"
    assert po.varint(128) == b"\x80\x01"
    assert po.varint(300) == b"\xac\x02"
    assert po.varint(16384) == b"\x80\x80\x01"
    assert po.varint(2**64 - 1) == b"\xff" * 9 + b"\x01"
    for v in (0, 1, 127, 128, 300, 2**32, 2**64 - 1):
        assert po.read_varint(po.varint(v), 0) == (v, len(po.varint(v)))


def test_oracle_known_answer_document():
    # IndexPersistenceData{ metadata: {dimension 2, total_points 1,
    # created_at "2024-01-02T03:04:05Z", config {16, 200, 100, 16}},
    # vectors: [("a", [1.0, -2.0])] } assembled by hand from the spec
    want = (b"\x02" b"\x01" b"\x14" + b"2024-01-02T03:04:05Z" + b"\x10" b"\xc8\x01" b"\x64" b"\x10"
            + b"\x01" + b"\x01a" + b"\x02" + struct.pack("<ff", 1.0, -2.0))
    got = po.encode(2, 1, "2024-01-02T03:04:05Z", (16, 200, 100, 16), [("a", [1.0, -2.0])])
    assert got == want
    assert po.decode(want) == (2, 1, "2024-01-02T03:04:05Z", (16, 200, 100, 16), [("a", [1.0, -2.0])])


def test_created_at_autosi_format():
    from gvdb import utc_now_rfc3339

    s = utc_now_rfc3339()
    assert re.fullmatch(r"\d{4}-\d\d-\d\dT\d\d:\d\d:\d\d(\.(\d{3}|\d{6}|\d{9}))?Z", s), s


# -- the C-ABI codec against the oracle ------------------------------------------
def _random_vectors(rng, n, dim):
    ids = []
    for i in range(n):
        k = i % 5
        if k == 0:
            ids.append(f"doc-{i:06d}")
        elif k == 1:
            ids.append("x" * (120 + i % 20) + str(i))  # length >= 128: 2-byte varint
        elif k == 2:
            ids.append(f"向量-{i}-é")  # multi-byte UTF-8
        elif k == 3:
            ids.append("")  # empty id
        else:
            ids.append(str(rng.integers(0, 2**63)))
    vals = rng.standard_normal((n, dim)).astype(np.float32)
    vals[0, :] = [np.inf, -np.inf, np.nan, 0.0, -0.0, 1e-45][: dim] + [0.0] * max(0, dim - 6)
    return [(ids[i], vals[i]) for i in range(n)]


@pytest.mark.parametrize("dim", [1, 6, 37, 768])
def test_writer_matches_oracle_bytes(gvdb_lib_path, tmp_path, dim):
    L = _lib(gvdb_lib_path)
    rng = np.random.default_rng(dim)
    vecs = _random_vectors(rng, 53, dim)
    path = str(tmp_path / "index.bin")
    _write(L, path, dim, vecs, created="2025-08-24T10:11:12.123456Z", cfg=(32, 400, 64, 8))
    with open(path, "rb") as f:
        assert f.read(2) == b"\x1f\x8b"  # gzip member
    want = po.encode(dim, len(vecs), "2025-08-24T10:11:12.123456Z", (32, 400, 64, 8),
                     [(s, v.tolist()) for s, v in vecs])
    got = po.read_file(path)
    assert got == want  # byte-exact postcard payload


@pytest.mark.parametrize("dim", [3, 768])
def test_reader_reads_oracle_file(gvdb_lib_path, tmp_path, dim):
    L = _lib(gvdb_lib_path)
    rng = np.random.default_rng(100 + dim)
    vecs = _random_vectors(rng, 41, dim)
    path = str(tmp_path / "ref.bin")
    po.write_file(path, po.encode(dim, 41, "2024-01-01T00:00:00Z", (16, 200, 100, 16),
                                  [(s, v.tolist()) for s, v in vecs]))
    d, tot, created, cfg, cnt, out = _read(L, path, batch=4, blob_cap=200)
    assert (d, tot, created, cfg, cnt) == (dim, 41, "2024-01-01T00:00:00Z", (16, 200, 100, 16), 41)
    assert [s for s, _ in out] == [s for s, _ in vecs]
    for (_, a), (_, b) in zip(out, vecs):
        assert a.tobytes() == b.tobytes()  # bit-exact, NaN / -0.0 / denormal included


def test_empty_index_file(gvdb_lib_path, tmp_path):
    L = _lib(gvdb_lib_path)
    path = str(tmp_path / "empty.bin")
    _write(L, path, 0, [], created="2024-01-01T00:00:00Z")
    assert po.read_file(path) == po.encode(0, 0, "2024-01-01T00:00:00Z", (16, 200, 100, 16), [])
    assert _read(L, path)[4:] == (0, [])


def test_errors(gvdb_lib_path, tmp_path):
    from gvdb import DimensionMismatch, InvalidArgument, StorageError, _ffi, check

    L = _lib(gvdb_lib_path)
    m, cnt, r = _ffi.gvdb_persist_meta(), C.c_uint64(), C.c_void_p()
    with pytest.raises(StorageError, match="does not exist"):
        check(L.gvdb_persist_open(str(tmp_path / "missing.bin").encode(), C.byref(m), C.byref(cnt), C.byref(r)))
    # truncated payload
    full = po.encode(4, 3, "t", (1, 2, 3, 4), [("a", [1, 2, 3, 4]), ("b", [5, 6, 7, 8]), ("c", [9, 9, 9, 9])])
    path = str(tmp_path / "trunc.bin")
    po.write_file(path, full[:-5])
    with pytest.raises(StorageError, match="truncated"):
        _read(L, path)
    # not gzip at all
    bad = str(tmp_path / "bad.bin")
    with open(bad, "wb") as f:
        f.write(b"\xff" * 64)
    with pytest.raises(StorageError):
        _read(L, bad)
    # a stored vector of another length (HnswVectorIndex::add_vector would refuse it)
    path2 = str(tmp_path / "ragged.bin")
    po.write_file(path2, po.encode(4, 2, "t", (1, 2, 3, 4), [("a", [1, 2, 3, 4]), ("b", [5, 6, 7])]))
    with pytest.raises(DimensionMismatch):
        _read(L, path2)
    # writer: fewer vectors than declared
    w = C.c_void_p()
    check(L.gvdb_persist_create(str(tmp_path / "short.bin").encode(), C.byref(_meta(2, 2)), 2, -1, C.byref(w)))
    with pytest.raises(InvalidArgument, match="fewer"):
        check(L.gvdb_persist_close(w))


def test_gzip_trailer_is_checked(gvdb_lib_path, tmp_path):
    """A CRC-32 mismatch in the gzip trailer is a zlib error reported as
    Storage (GzDecoder::read_to_end verifies the trailer), not a truncation."""
    from gvdb import StorageError

    L = _lib(gvdb_lib_path)
    path = str(tmp_path / "crc.bin")
    po.write_file(path, po.encode(4, 2, "t", (1, 2, 3, 4), [("a", [1, 2, 3, 4]), ("b", [5, 6, 7, 8])]))
    raw = bytearray(open(path, "rb").read())
    raw[-8] ^= 0xFF  # first byte of the CRC-32
    open(path, "wb").write(bytes(raw))
    with pytest.raises(StorageError) as e:
        _read(L, path)
    assert "truncated" not in str(e.value)


def test_append_checks_header_dimension(gvdb_lib_path, tmp_path):
    from gvdb import DimensionMismatch, check

    L = _lib(gvdb_lib_path)
    w = C.c_void_p()
    check(L.gvdb_persist_create(str(tmp_path / "d.bin").encode(), C.byref(_meta(4, 1)), 1, -1, C.byref(w)))
    rows = np.zeros((1, 3), np.float32)
    offs = np.array([0, 1], np.uint64)
    with pytest.raises(DimensionMismatch):
        check(L.gvdb_persist_append(w, rows.ctypes.data, 1, 3, b"a", offs.ctypes.data))
    L.gvdb_persist_close(w)


def test_large_payload_streams(gvdb_lib_path, tmp_path):
    # > 64 MiB of postcard payload: several writer flushes and reader refills
    L = _lib(gvdb_lib_path)
    dim, n = 768, 24000
    rng = np.random.default_rng(7)
    rows = rng.standard_normal((n, dim)).astype(np.float32)
    vecs = [(f"id{i:07d}", rows[i]) for i in range(n)]
    path = str(tmp_path / "big.bin")
    _write(L, path, dim, vecs, batch=5000, level=1)
    d, tot, _, _, cnt, out = _read(L, path, batch=3000, blob_cap=1 << 16)
    assert (d, tot, cnt, len(out)) == (dim, n, n, n)
    assert np.array_equal(np.stack([v for _, v in out]), rows)
    assert [s for s, _ in out[:3]] == ["id0000000", "id0000001", "id0000002"]
    with gzip.open(path, "rb") as f:
        head = f.read(64)
    assert head[:2] == b"\x80\x06"  # varint(768)


@pytest.mark.gpu
def test_gpu_save_load_round_trip(tmp_path):
    import gvdb

    rng = np.random.default_rng(11)
    D, n = 96, 5000
    rows = rng.standard_normal((n, D)).astype(np.float32)
    ids = [f"v{(i * 7919) % 100003}" for i in range(n)]
    ix = gvdb.GpuVectorIndex(dimension=D)
    ix.add_vectors(list(zip(ids, rows)))
    for i in range(0, n, 97):
        assert ix.remove_vector(ids[i])
    ix.add_vector(ids[5], rows[6])  # overwrite: the new row must persist
    path = str(tmp_path / "sub" / "index.gvdb")
    ix.save_index(path, gvdb.HnswConfig(m=24, ef_construction=300, ef_search=80, max_layers=12),
                  created_at="2025-01-01T00:00:00.5Z")
    want = ix.get_all_vectors()
    # the file is the reference's format, sorted by id (index.rs:131-132)
    d, tot, created, cfg, vecs = po.decode(po.read_file(path))
    assert (d, tot, created, cfg) == (D, len(want), "2025-01-01T00:00:00.5Z", (24, 300, 80, 12))
    assert [s for s, _ in vecs] == sorted(s for s, _ in want)
    assert all(np.array_equal(np.array(v, np.float32), w) for (_, v), (_, w) in zip(vecs, want))
    ix2 = gvdb.GpuVectorIndex(dimension=D)
    meta = ix2.load_index(path)
    assert meta.total_points == len(want) and meta.config.m == 24
    got = ix2.get_all_vectors()
    assert [s for s, _ in got] == [s for s, _ in want]
    assert all(a.tobytes() == b.tobytes() for (_, a), (_, b) in zip(got, want))
    # exact (flat) search is independent of the row order the reload produces
    # (the BQ path's stage-1 tie order is by row, as the reference's is by
    # insertion order, so its top-R can legitimately differ after a reload)
    q = rng.standard_normal((8, D)).astype(np.float32)
    flat = gvdb.SearchParams(mode=gvdb._ffi.GVDB_SEARCH_FLAT)
    i1, s1, n1 = ix.search_batch(q, 10, flat)
    i2, s2, n2 = ix2.search_batch(q, 10, flat)
    names1 = [[ix._str_of[int(u)] for u in row[:n]] for row, n in zip(i1, n1)]
    names2 = [[ix2._str_of[int(u)] for u in row[:n]] for row, n in zip(i2, n2)]
    assert names1 == names2
    assert s1.tobytes() == s2.tobytes()
    with pytest.raises(gvdb.DimensionMismatch):
        gvdb.GpuVectorIndex(dimension=D + 1).load_index(path)


@pytest.mark.gpu
def test_gpu_failed_load_leaves_index_intact(tmp_path):
    """load_index decodes into a staging index: a truncated file raises
    Storage and the index keeps its previous contents (query.rs:355-373 decodes
    the whole file before it touches the index)."""
    import gvdb

    rng = np.random.default_rng(12)
    D = 32
    rows = rng.standard_normal((300, D)).astype(np.float32)
    ix = gvdb.GpuVectorIndex(dimension=D)
    ix.add_vectors([(f"k{i}", rows[i]) for i in range(300)])
    good = str(tmp_path / "good.gvdb")
    ix.save_index(good)
    full = po.read_file(good)
    bad = str(tmp_path / "bad.gvdb")
    po.write_file(bad, full[: len(full) * 2 // 3])
    ix2 = gvdb.GpuVectorIndex(dimension=D)
    ix2.add_vectors([("keep-me", rows[0]), ("and-me", rows[1])])
    before = ix2.get_all_vectors()
    with pytest.raises(gvdb.StorageError):
        ix2.load_index(bad)
    after = ix2.get_all_vectors()
    assert [s for s, _ in after] == [s for s, _ in before] == ["and-me", "keep-me"]
    assert ix2.search(rows[1], 1)[0][0] == "and-me"
    ix2.load_index(good)  # a good file still loads afterwards
    assert ix2.len() == 300
