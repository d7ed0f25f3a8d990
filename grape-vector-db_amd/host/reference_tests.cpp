// reference_tests.cpp — the reference's own unit tests for the hot path,
// re-run through the C++ host mirror (gvdb.hpp) on the GPU:
//   quantization.rs:361-372 test_binary_quantization
//   quantization.rs:375-386 test_hamming_distance
//   quantization.rs:389-400 test_binary_vector_store (count only: the store is host data)
//   query.rs:428-483        test_query_engine (3-d document, top-1 "test1")
//   index.rs VectorIndex     add / dimension mismatch / remove / clear semantics
#include <cmath>
#include <cstdio>

#include "gvdb.hpp"

static int failures = 0;
#define CHECK(c)                                                        \
    do {                                                                \
        if (!(c)) {                                                     \
            std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);    \
            ++failures;                                                 \
        }                                                               \
    } while (0)

int main() {
    using namespace gvdb;
    {  // test_binary_quantization
        BinaryQuantizer q;
        BinaryVector b = q.quantize({0.5f, -0.3f, 0.8f, -0.1f, 0.2f});
        CHECK(b.dimension == 5);
        CHECK(b.bit_len() == 5);
        CHECK(b.data.size() == 1 && b.data[0] == 0xA8);  // [1,0,1,0,1]
    }
    {  // test_hamming_distance
        BinaryQuantizer q;
        BinaryVector a = q.quantize({1.0f, -1.0f, 1.0f, -1.0f});
        BinaryVector b = q.quantize({1.0f, 1.0f, -1.0f, -1.0f});
        float d = q.hamming_distance(a, b);
        CHECK(d > 0.0f);
        CHECK(d == 2.0f);
        CHECK(q.similarity(a, b) == 0.5f);
        bool threw = false;
        try {
            q.hamming_distance(a, q.quantize({1.0f}));
        } catch (const VectorDbError& e) {
            threw = e.code == GVDB_ERR_INVALID_VECTOR_DIMENSION;
        }
        CHECK(threw);
    }
    {  // test_binary_vector_store
        BinaryQuantizer q;
        std::vector<BinaryVector> store{q.quantize({0.1f, 0.2f, 0.3f})};
        CHECK(store.size() == 1 && store[0].data[0] == 0xE0);
    }
    {  // test_query_engine: vector_search(&[1.0, 0.1, 0.0], 5)[0] == "test1"
        GpuVectorIndex ix;
        ix.add_vector("test1", {1.0f, 0.0f, 0.0f});
        auto r = ix.search({1.0f, 0.1f, 0.0f}, 5);
        CHECK(!r.empty() && r[0].first == "test1");
    }
    {  // VectorIndex semantics
        GpuVectorIndex ix;
        bool nb = false;
        try {
            ix.search({1.0f, 0.0f}, 1);
        } catch (const VectorDbError& e) {
            nb = e.code == GVDB_ERR_INDEX_NOT_BUILT;
        }
        CHECK(nb);
        ix.add_vectors({{"a", {1.0f, 0.0f}}, {"b", {0.0f, 1.0f}}});
        bool dm = false;
        try {
            ix.add_vector("c", {1.0f, 2.0f, 3.0f});
        } catch (const VectorDbError& e) {
            dm = e.code == GVDB_ERR_DIMENSION_MISMATCH && e.expected == 2 && e.actual == 3;
        }
        CHECK(dm);
        CHECK(ix.len() == 2 && !ix.is_empty());
        CHECK(ix.remove_vector("a") && !ix.remove_vector("zz"));
        CHECK(ix.len() == 1);
        auto r = ix.search({1.0f, 0.0f}, 3);
        CHECK(r.size() == 1 && r[0].first == "b");
        ix.clear();
        CHECK(ix.is_empty() && ix.get_stats().dimension == 0);
    }
    {  // multi_stage_search through the mirror: R = (N as f32 * 0.5) as usize
        BinaryQuantizer q(BinaryQuantizationConfig{0.0f, true, 0.5f, true});
        std::vector<std::vector<float>> c{{1, 0, 0, 0}, {0, 1, 0, 0}, {1, 1, 0, 0}, {-1, 0, 0, 0}};
        std::vector<BinaryVector> cb;
        for (auto& v : c) cb.push_back(q.quantize(v));
        std::vector<float> qv{1, 0.2f, 0, 0};
        auto r = q.multi_stage_search(q.quantize(qv), cb, qv, c);
        CHECK(r.size() == 2);
        CHECK(r[0].first == 0);  // cos 0.98 > cand 2's 0.83
    }
    std::printf("%s (%d failures)\n", failures ? "FAILED" : "OK", failures);
    return failures ? 1 : 0;
}
