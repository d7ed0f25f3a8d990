// gvdb.hpp — C++ host mirror of grape-vector-db's vector hot-path API over the
// C ABI (include/gvdb.h).  Header-only; link with -lgvdb.
//
//   gvdb::VectorIndex          trait VectorIndex              src/index.rs:35-62
//   gvdb::GpuVectorIndex       HnswVectorIndex drop-in        src/index.rs:91-310
//   gvdb::IndexStats           IndexStats                     src/index.rs:83-88
//   gvdb::BinaryQuantizationConfig / BinaryVector / BinaryQuantizer
//                                                             src/quantization.rs:10-216
//   gvdb::VectorDbError        VectorDbError                  src/types.rs:859-920
//
// Errors surface as gvdb::VectorDbError (the Result<_, VectorDbError> of the
// reference), String ids stay in this layer (String <-> u64 table).
#pragma once
#include <cstdint>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../include/gvdb.h"

namespace gvdb {

struct VectorDbError : std::runtime_error {
    gvdb_status code;
    uint64_t expected = 0, actual = 0;  // DimensionMismatch detail
    VectorDbError(gvdb_status c, const std::string& m) : std::runtime_error(m), code(c) {}
};

inline void check(gvdb_status s) {
    if (s == GVDB_OK) return;
    VectorDbError e(s, std::string(gvdb_status_string(s)) + ": " + gvdb_last_error());
    if (s == GVDB_ERR_DIMENSION_MISMATCH) gvdb_last_dimension_mismatch(&e.expected, &e.actual);
    throw e;
}

struct IndexStats {
    size_t vector_count, dimension;
    std::string index_type;
    size_t memory_usage;
};

class VectorIndex {
public:
    virtual ~VectorIndex() = default;
    virtual void add_vector(std::string id, std::vector<float> vector) = 0;
    virtual void add_vectors(std::vector<std::pair<std::string, std::vector<float>>> vectors) = 0;
    virtual std::vector<std::pair<std::string, float>> search(const std::vector<float>& query, size_t k) const = 0;
    virtual bool remove_vector(const std::string& id) = 0;
    virtual size_t len() const = 0;
    virtual bool is_empty() const = 0;
    virtual void optimize() = 0;
    virtual void clear() = 0;
    virtual IndexStats get_stats() const = 0;
};

class GpuVectorIndex final : public VectorIndex {
public:
    explicit GpuVectorIndex(int device = 0, gvdb_metric metric = GVDB_METRIC_COSINE, uint64_t rescore_count = 100) {
        gvdb_params p{};
        p.device = device;
        check(gvdb_index_create(&p, &h_));
        sp_.mode = GVDB_SEARCH_BQ_RERANK;
        sp_.metric = metric;
        sp_.rescore_count = rescore_count;
        sp_.rescore_ratio = 0.1f;
    }
    ~GpuVectorIndex() override { gvdb_index_destroy(h_); }
    GpuVectorIndex(const GpuVectorIndex&) = delete;
    GpuVectorIndex& operator=(const GpuVectorIndex&) = delete;

    void add_vector(std::string id, std::vector<float> v) override {
        const uint64_t u = intern(id);
        check(gvdb_index_add(h_, v.data(), 1, (uint32_t)v.size(), &u));
    }
    // index.rs:187-210: rows before a dimension mismatch stay added.  Each run of
    // equal-length rows is ONE gvdb_index_add (one H2D copy); the C ABI checks the
    // run's length, so the first row of another length fails where the reference's
    // per-row check does.
    void add_vectors(std::vector<std::pair<std::string, std::vector<float>>> vs) override {
        for (size_t i = 0; i < vs.size();) {
            const size_t d = vs[i].second.size();
            size_t j = i;
            while (j < vs.size() && vs[j].second.size() == d) ++j;
            std::vector<float> flat;
            flat.reserve((j - i) * d);
            std::vector<uint64_t> ids;
            ids.reserve(j - i);
            for (size_t r = i; r < j; ++r) {
                ids.push_back(intern(vs[r].first));
                flat.insert(flat.end(), vs[r].second.begin(), vs[r].second.end());
            }
            check(gvdb_index_add(h_, flat.data(), j - i, (uint32_t)d, ids.data()));
            i = j;
        }
    }
    std::vector<std::pair<std::string, float>> search(const std::vector<float>& q, size_t k) const override {
        std::vector<uint64_t> ids(k ? k : 1);
        std::vector<float> sc(k ? k : 1);
        uint32_t n = 0;
        check(gvdb_index_search(h_, q.data(), 1, (uint32_t)q.size(), k, &sp_, ids.data(), sc.data(), &n));
        std::vector<std::pair<std::string, float>> out;
        for (uint32_t i = 0; i < n; ++i) out.emplace_back(str_of_[ids[i]], sc[i]);
        return out;
    }
    bool remove_vector(const std::string& id) override {
        auto it = id_of_.find(id);
        if (it == id_of_.end()) return false;
        int32_t removed = 0;
        check(gvdb_index_remove(h_, it->second, &removed));
        return removed != 0;
    }
    size_t len() const override { return (size_t)gvdb_index_len(h_); }
    bool is_empty() const override { return gvdb_index_is_empty(h_) != 0; }
    void optimize() override { check(gvdb_index_optimize(h_)); }
    void clear() override { gvdb_index_clear(h_); }
    IndexStats get_stats() const override {
        gvdb_index_stats s{};
        check(gvdb_index_get_stats(h_, &s));
        return {(size_t)s.vector_count, (size_t)s.dimension, "GPU-BQ", (size_t)s.memory_usage};
    }

private:
    uint64_t intern(const std::string& id) {
        auto it = id_of_.find(id);
        if (it != id_of_.end()) return it->second;
        const uint64_t u = str_of_.size();
        str_of_.push_back(id);
        id_of_.emplace(id, u);
        return u;
    }
    gvdb_index* h_ = nullptr;
    gvdb_search_params sp_{};
    std::unordered_map<std::string, uint64_t> id_of_;
    std::vector<std::string> str_of_;
};

// ---- BinaryQuantizer (quantization.rs) ------------------------------------------
struct BinaryQuantizationConfig {  // quantization.rs:10-31
    float threshold = 0.0f;
    bool enable_simd = true;
    float rescore_ratio = 0.1f;
    bool enable_cache = true;
};

struct BinaryVector {  // quantization.rs:35-63
    std::vector<uint8_t> data;  // BitVec<u8, Msb0> storage
    size_t dimension = 0;
    size_t byte_size() const { return (dimension + 7) / 8; }
    size_t bit_len() const { return dimension; }
};

class BinaryQuantizer {
public:
    explicit BinaryQuantizer(BinaryQuantizationConfig c = {}) : cfg_(c) {}
    BinaryVector quantize(const std::vector<float>& v) const {
        BinaryVector b;
        b.dimension = v.size();
        b.data.assign(b.byte_size(), 0);
        if (!v.empty()) check(gvdb_bq_quantize(v.data(), 1, (uint32_t)v.size(), cfg_.threshold, b.data.data()));
        return b;
    }
    float hamming_distance(const BinaryVector& a, const BinaryVector& b) const {
        if (a.dimension != b.dimension) throw VectorDbError(GVDB_ERR_INVALID_VECTOR_DIMENSION, "dimension differs");
        uint32_t d = 0;
        if (a.byte_size()) check(gvdb_bq_hamming(a.data.data(), b.data.data(), 1, (uint32_t)a.dimension, &d));
        return (float)d;
    }
    float similarity(const BinaryVector& a, const BinaryVector& b) const {
        return 1.0f - (hamming_distance(a, b) / (float)a.dimension);
    }
    std::vector<std::pair<size_t, float>> multi_stage_search(const BinaryVector& qb,
                                                             const std::vector<BinaryVector>& cb,
                                                             const std::vector<float>& q,
                                                             const std::vector<std::vector<float>>& cands) const {
        if (cb.size() != cands.size())
            throw VectorDbError(GVDB_ERR_QUANTIZATION, "Mismatch between binary and original candidate counts");
        const size_t N = cb.size();
        if (N == 0) return {};
        const size_t nb = cb[0].byte_size(), clen = cands[0].size();
        std::vector<uint8_t> bits(N * nb);
        std::vector<float> rows(N * clen);
        for (size_t i = 0; i < N; ++i) {
            std::copy(cb[i].data.begin(), cb[i].data.begin() + nb, bits.begin() + i * nb);
            std::copy(cands[i].begin(), cands[i].end(), rows.begin() + i * clen);
        }
        std::vector<uint64_t> idx(N);
        std::vector<float> cs(N);
        uint64_t n = 0;
        check(gvdb_bq_multi_stage_search(qb.data.data(), (uint32_t)qb.dimension, bits.data(),
                                         (uint32_t)cb[0].dimension, N, q.data(), q.size(), rows.data(), clen,
                                         cfg_.rescore_ratio, idx.data(), cs.data(), &n));
        std::vector<std::pair<size_t, float>> out;
        for (uint64_t i = 0; i < n; ++i) out.emplace_back((size_t)idx[i], cs[i]);
        return out;
    }

private:
    BinaryQuantizationConfig cfg_;
};

}  // namespace gvdb
