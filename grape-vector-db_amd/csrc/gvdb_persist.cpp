// gvdb_persist.cpp — index persistence in the reference's on-disk format.
//
// QueryEngine::save_index / load_index (src/query.rs:282-409) write
//   gzip( postcard( IndexPersistenceData { metadata, vectors } ) )
// with (query.rs:16-28, config.rs:196-209)
//   IndexMetadata { dimension: usize, total_points: usize,
//                   created_at: chrono::DateTime<Utc>, config: HnswConfig }
//   HnswConfig    { m, ef_construction, ef_search, max_layers: usize }
//   vectors: Vec<(String, Vec<f32>)>   (sorted by id, index.rs:120-135)
// Postcard 1.x (the `postcard` crate, not vendored here): a struct is its
// fields in order; usize / lengths are unsigned LEB128 varints; String and
// Vec are varint(len) + elements; f32 is 4 little-endian bytes; chrono's
// serde Serialize emits the RFC 3339 string (SecondsFormat::AutoSi, 'Z').
//
// Streaming in both directions (a 10M x 768 index is ~30 GB of payload):
// the writer appends batches of (id, row) pairs behind the count declared at
// create time; the reader returns the metadata then batches of entries.
// Host-only code (zlib's gzFile API); the device side is gvdb_index_export /
// gvdb_index_add.
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <zlib.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/gvdb.h"

namespace gvdb {
gvdb_status report_status(gvdb_status s, const std::string& msg);  // gvdb_capi.hip
}
using gvdb::report_status;

struct gvdb_persist_writer {
    gzFile f = nullptr;
    uint64_t declared = 0, written = 0;
    uint32_t dim = 0;
    std::vector<uint8_t> buf;
};

struct gvdb_persist_reader {
    gzFile f = nullptr;
    gvdb_persist_meta meta{};
    uint64_t count = 0, read = 0;
    std::vector<uint8_t> buf;  // undecoded bytes [pos, buf.size())
    size_t pos = 0;
    bool eof = false;
    std::string zerr;     // a zlib error met while reading (distinct from a clean end of stream)
    bool drained = false; // the stream was read to its end after the last entry (trailer checked)
};

namespace {

void put_varint(std::vector<uint8_t>& b, uint64_t v) {
    while (v >= 0x80) {
        b.push_back((uint8_t)(v | 0x80));
        v >>= 7;
    }
    b.push_back((uint8_t)v);
}

void put_str(std::vector<uint8_t>& b, const char* s, size_t n) {
    put_varint(b, n);
    b.insert(b.end(), (const uint8_t*)s, (const uint8_t*)s + n);
}

gvdb_status flush(gvdb_persist_writer* w) {
    size_t off = 0;
    while (off < w->buf.size()) {
        const unsigned chunk = (unsigned)std::min<size_t>(w->buf.size() - off, 1u << 30);
        if (gzwrite(w->f, w->buf.data() + off, chunk) != (int)chunk) {
            int err = 0;
            const char* m = gzerror(w->f, &err);
            return report_status(GVDB_ERR_STORAGE, std::string("index write failed: ") + (m ? m : "?"));
        }
        off += chunk;
    }
    w->buf.clear();
    return GVDB_OK;
}

// reader: make at least `need` undecoded bytes available (false at EOF)
bool fill(gvdb_persist_reader* r, size_t need) {
    if (r->buf.size() - r->pos >= need) return true;
    if (r->pos) {
        r->buf.erase(r->buf.begin(), r->buf.begin() + (ptrdiff_t)r->pos);
        r->pos = 0;
    }
    while (r->buf.size() < need && !r->eof) {
        const size_t have = r->buf.size();
        const size_t want = std::max<size_t>(need - have, 1u << 22);
        r->buf.resize(have + want);
        const int got = gzread(r->f, r->buf.data() + have, (unsigned)want);
        if (got <= 0) {
            r->eof = true;
            r->buf.resize(have);
            if (got < 0) {
                int err = 0;
                const char* m = gzerror(r->f, &err);
                r->zerr = m ? m : "zlib error";
            }
        } else {
            r->buf.resize(have + (size_t)got);
        }
    }
    return r->buf.size() >= need;
}

gvdb_status truncated(const gvdb_persist_reader* r) {
    if (!r->zerr.empty()) return report_status(GVDB_ERR_STORAGE, "index file: " + r->zerr);
    return report_status(GVDB_ERR_STORAGE, "index file truncated or not in postcard format");
}

// After the last entry: read the gzip stream to its end so the trailer (CRC-32,
// length) is verified, as GzDecoder::read_to_end does (query.rs:355-373).
gvdb_status drain_and_check(gvdb_persist_reader* r) {
    if (r->drained) return GVDB_OK;
    r->drained = true;
    std::vector<uint8_t> sink(1u << 20);
    while (!r->eof) {
        const int got = gzread(r->f, sink.data(), (unsigned)sink.size());
        if (got < 0) {
            int err = 0;
            const char* m = gzerror(r->f, &err);
            r->zerr = m ? m : "zlib error";
        }
        if (got <= 0) r->eof = true;
    }
    if (!r->zerr.empty()) return report_status(GVDB_ERR_STORAGE, "index file: " + r->zerr);
    return GVDB_OK;
}

gvdb_status get_varint(gvdb_persist_reader* r, uint64_t* v) {
    uint64_t x = 0;
    for (int sh = 0; sh < 70; sh += 7) {
        if (!fill(r, 1)) return truncated(r);
        const uint8_t c = r->buf[r->pos++];
        if (sh == 63 && c > 1) return report_status(GVDB_ERR_STORAGE, "varint overflows u64");
        x |= (uint64_t)(c & 0x7f) << sh;
        if (!(c & 0x80)) {
            *v = x;
            return GVDB_OK;
        }
    }
    return report_status(GVDB_ERR_STORAGE, "varint longer than 10 bytes");
}

gvdb_status get_bytes(gvdb_persist_reader* r, size_t n, const uint8_t** p) {
    if (!fill(r, n)) return truncated(r);
    *p = r->buf.data() + r->pos;
    r->pos += n;
    return GVDB_OK;
}

}  // namespace

extern "C" {

gvdb_status gvdb_persist_create(const char* path, const gvdb_persist_meta* meta, uint64_t n_vectors, int32_t level,
                                gvdb_persist_writer** out) {
    if (!path || !meta || !out) return report_status(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    *out = nullptr;
    const size_t tl = strnlen(meta->created_at, sizeof meta->created_at);
    if (tl == sizeof meta->created_at) return report_status(GVDB_ERR_INVALID_ARGUMENT, "created_at not terminated");
    char mode[8];
    snprintf(mode, sizeof mode, "wb%d", level < 0 ? 6 : (level > 9 ? 9 : level));  // flate2 Compression::default() = 6
    gzFile f = gzopen(path, mode);
    if (!f) return report_status(GVDB_ERR_STORAGE, std::string("cannot create index file ") + path);
    auto* w = new gvdb_persist_writer();
    w->f = f;
    w->declared = n_vectors;
    w->dim = (uint32_t)meta->dimension;
    // IndexMetadata, then the Vec length of `vectors`
    put_varint(w->buf, meta->dimension);
    put_varint(w->buf, meta->total_points);
    put_str(w->buf, meta->created_at, tl);
    put_varint(w->buf, meta->m);
    put_varint(w->buf, meta->ef_construction);
    put_varint(w->buf, meta->ef_search);
    put_varint(w->buf, meta->max_layers);
    put_varint(w->buf, n_vectors);
    *out = w;
    return GVDB_OK;
}

gvdb_status gvdb_persist_append(gvdb_persist_writer* w, const float* rows, uint64_t n, uint32_t dim,
                                const char* id_blob, const uint64_t* id_offs) {
    if (!w || (n && (!rows || !id_blob || !id_offs))) return report_status(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    if (w->written + n > w->declared)
        return report_status(GVDB_ERR_INVALID_ARGUMENT, "more vectors appended than declared at create");
    if (n && dim != w->dim)  // the header states w->dim: a row of another length makes an invalid file
        return report_status(GVDB_ERR_DIMENSION_MISMATCH, "appended rows have dimension " + std::to_string(dim) +
                                                              ", the file header states " + std::to_string(w->dim));
    for (uint64_t i = 0; i < n; ++i) {
        if (id_offs[i + 1] < id_offs[i]) return report_status(GVDB_ERR_INVALID_ARGUMENT, "id offsets not ascending");
        put_str(w->buf, id_blob + id_offs[i], (size_t)(id_offs[i + 1] - id_offs[i]));
        put_varint(w->buf, dim);
        const size_t at = w->buf.size();
        w->buf.resize(at + (size_t)dim * 4);
        memcpy(w->buf.data() + at, rows + i * dim, (size_t)dim * 4);  // little-endian host
        if (w->buf.size() >= (64u << 20)) {
            gvdb_status st = flush(w);
            if (st != GVDB_OK) return st;
        }
    }
    w->written += n;
    return GVDB_OK;
}

gvdb_status gvdb_persist_close(gvdb_persist_writer* w) {
    if (!w) return GVDB_OK;
    gvdb_status st = flush(w);
    if (st == GVDB_OK && w->written != w->declared)
        st = report_status(GVDB_ERR_INVALID_ARGUMENT, "fewer vectors appended than declared at create");
    if (gzclose(w->f) != Z_OK && st == GVDB_OK) st = report_status(GVDB_ERR_STORAGE, "index file close failed");
    delete w;
    return st;
}

gvdb_status gvdb_persist_open(const char* path, gvdb_persist_meta* meta, uint64_t* n_vectors,
                              gvdb_persist_reader** out) {
    if (!path || !meta || !n_vectors || !out) return report_status(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    *out = nullptr;
    FILE* probe = fopen(path, "rb");
    if (!probe) return report_status(GVDB_ERR_STORAGE, std::string("index file does not exist: ") + path);
    fclose(probe);
    gzFile f = gzopen(path, "rb");
    if (!f) return report_status(GVDB_ERR_STORAGE, std::string("cannot open index file ") + path);
    gzbuffer(f, 1u << 20);
    auto* r = new gvdb_persist_reader();
    r->f = f;
    gvdb_status st = GVDB_OK;
    uint64_t tl = 0;
    const uint8_t* p = nullptr;
    gvdb_persist_meta& m = r->meta;
    if ((st = get_varint(r, &m.dimension)) || (st = get_varint(r, &m.total_points)) || (st = get_varint(r, &tl)))
        goto bad;
    if (tl >= sizeof m.created_at) {
        st = report_status(GVDB_ERR_STORAGE, "created_at longer than 63 bytes");
        goto bad;
    }
    if ((st = get_bytes(r, (size_t)tl, &p))) goto bad;
    memcpy(m.created_at, p, (size_t)tl);
    m.created_at[tl] = 0;
    if ((st = get_varint(r, &m.m)) || (st = get_varint(r, &m.ef_construction)) || (st = get_varint(r, &m.ef_search)) ||
        (st = get_varint(r, &m.max_layers)) || (st = get_varint(r, &r->count)))
        goto bad;
    *meta = m;
    *n_vectors = r->count;
    *out = r;
    return GVDB_OK;
bad:
    gzclose(r->f);
    delete r;
    return st;
}

gvdb_status gvdb_persist_next(gvdb_persist_reader* r, float* rows, uint32_t dim, uint64_t max_n, char* id_blob,
                              uint64_t blob_cap, uint64_t* id_offs, uint64_t* n_out) {
    if (!r || !n_out || (max_n && (!rows || !id_offs || (blob_cap && !id_blob))))
        return report_status(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    uint64_t n = 0, used = 0;
    if (max_n) id_offs[0] = 0;
    while (n < max_n && r->read < r->count) {
        // peek the id length: stop before an entry whose id does not fit
        // (fill first so the varint below cannot compact the buffer under `save`)
        (void)fill(r, 10);
        const size_t save = r->pos;
        uint64_t il = 0, vl = 0;
        const uint8_t* p = nullptr;
        gvdb_status st = get_varint(r, &il);
        if (st != GVDB_OK) return st;
        if (used + il > blob_cap) {
            if (n == 0) return report_status(GVDB_ERR_INVALID_ARGUMENT, "id blob too small for one id");
            r->pos = save;
            break;
        }
        if ((st = get_bytes(r, (size_t)il, &p)) != GVDB_OK) return st;
        memcpy(id_blob + used, p, (size_t)il);
        used += il;
        id_offs[n + 1] = used;
        if ((st = get_varint(r, &vl)) != GVDB_OK) return st;
        if (vl != dim) {
            // HnswVectorIndex::add_vector (index.rs:187-210) on a row of another length
            return report_status(GVDB_ERR_DIMENSION_MISMATCH, "stored vector length " + std::to_string(vl) +
                                                                  " differs from dimension " + std::to_string(dim));
        }
        if ((st = get_bytes(r, (size_t)vl * 4, &p)) != GVDB_OK) return st;
        memcpy(rows + n * dim, p, (size_t)vl * 4);
        ++n;
        ++r->read;
    }
    *n_out = n;
    if (r->read == r->count) return drain_and_check(r);
    return GVDB_OK;
}

void gvdb_persist_free(gvdb_persist_reader* r) {
    if (!r) return;
    gzclose(r->f);
    delete r;
}

}  // extern "C"
