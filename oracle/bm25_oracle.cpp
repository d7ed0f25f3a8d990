// ============================================================================
// bm25_oracle.cpp — CPU ORACLE (TEST INFRASTRUCTURE ONLY)
//
// A sequential C++ restatement of grape-vector-db's sparse (BM25) search and
// its reciprocal-rank fusion (reference snapshot 2025-08-24, Rust).  It exists
// to CHECK the HIP product path (grape-vector-db_amd/csrc/gvdb_sparse.hip);
// only tests/ and bench legs load it.
//
// Restated (file:line of the reference):
//   * SparseIndex::add_document      src/sparse.rs:71-107
//   * SparseIndex::remove_document   src/sparse.rs:109-149
//   * SparseIndex::search_bm25       src/sparse.rs:151-198
//   * calculate_idf / _bm25_score    src/sparse.rs:200-222 (k1 1.2, b 0.75: 49-53)
//   * HybridSearchEngine::rrf_fusion src/hybrid.rs:422-488
//
// The reference leaves three orders to HashMap iteration (random per process):
//   (1) avgdl = (sum over ALL posting entries of document_length) / N
//       (sparse.rs:96-104, the "avgdl quirk": a document is counted once per
//       distinct term) is an f32 fold in HashMap order; here: slot order,
//       each slot's entries by (term, add order);
//   (2) equal BM25 scores come out of `document_scores.into_iter()` in HashMap
//       order before the stable sort (sparse.rs:192-196);
//   (3) equal RRF scores likewise (hybrid.rs:481-486).
// This restatement (and the GPU path) fix them as: (1) above (slot = first
// add of the id); (2)/(3) ties by slot / by first appearance.  Parity with the reference is
// therefore bit-exact for every score given avgdl, and avgdl itself is one of
// the reference's possible fold orders.  NaN scores (reachable only when
// remove_document leaves df > total_documents, sparse.rs:128-133) sort last.
// ============================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <unordered_map>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

struct Entry {
    uint32_t term;
    float tf, dl;
};
struct Posting {
    uint32_t slot;
    float tf, dl;  // InvertedIndexEntry {term_frequency, document_length} (sparse.rs:19-27)
};

struct Bm25Oracle {
    float k1 = 1.2f, b = 0.75f;
    std::unordered_map<uint64_t, uint32_t> slot_of;
    std::vector<uint64_t> slot_id;
    std::vector<std::vector<Entry>> slot_entries;       // per slot, add order
    std::map<uint32_t, std::vector<Posting>> postings;   // term -> entries, posting order
    std::unordered_map<uint32_t, uint64_t> df;
    uint64_t total_documents = 0;
    float total_length = 0.0f;
    float avgdl = 0.0f;

    void recompute_length() {
        // sparse.rs:96-100: .sum() of f32, folded here in slot order, each
        // slot's entries by (term, add order)
        float t = 0.0f;
        for (const auto& v : slot_entries) {
            std::vector<Entry> s(v);
            std::stable_sort(s.begin(), s.end(), [](const Entry& x, const Entry& y) { return x.term < y.term; });
            for (const Entry& e : s) t = t + e.dl;
        }
        total_length = t;
    }
    void refresh_avgdl() {
        if (total_documents > 0) avgdl = total_length / (float)total_documents;
    }
};

}  // namespace

extern "C" {

void* bm25o_create(float k1, float b) {
    Bm25Oracle* o = new Bm25Oracle();
    o->k1 = k1;
    o->b = b;
    return o;
}

void bm25o_free(void* h) { delete (Bm25Oracle*)h; }

// add_document (sparse.rs:71-107): one posting entry per distinct term.
void bm25o_add(void* h, uint64_t id, const uint32_t* terms, const float* tfs, uint64_t n, float dl) {
    Bm25Oracle* o = (Bm25Oracle*)h;
    auto it = o->slot_of.find(id);
    uint32_t slot;
    const bool fresh = it == o->slot_of.end();
    if (fresh) {
        slot = (uint32_t)o->slot_id.size();
        o->slot_of[id] = slot;
        o->slot_id.push_back(id);
        o->slot_entries.emplace_back();
    } else {
        slot = it->second;
    }
    for (uint64_t i = 0; i < n; ++i) {
        o->slot_entries[slot].push_back({terms[i], tfs[i], dl});
        o->postings[terms[i]].push_back({slot, tfs[i], dl});
        o->df[terms[i]] += 1;
    }
    o->total_documents += 1;
    if (fresh) {
        for (uint64_t i = 0; i < n; ++i) o->total_length = o->total_length + dl;  // new slot = end of the order
    } else {
        o->recompute_length();
    }
    o->refresh_avgdl();
}

// n_docs add_document calls in one (CSR: document d = terms[doc_ptr[d] ..
// doc_ptr[d+1])), for building large baselines without per-call overhead.
void bm25o_add_csr(void* h, const uint64_t* ids, const uint64_t* doc_ptr, const uint32_t* terms, const float* tfs,
                   const float* dls, uint64_t n_docs) {
    for (uint64_t d = 0; d < n_docs; ++d)
        bm25o_add(h, ids[d], terms + doc_ptr[d], tfs + doc_ptr[d], doc_ptr[d + 1] - doc_ptr[d], dls[d]);
}

// remove_document (sparse.rs:109-149): the FIRST entry of the id in every
// posting list goes; df is erased only when a list empties.
int bm25o_remove(void* h, uint64_t id) {
    Bm25Oracle* o = (Bm25Oracle*)h;
    auto it = o->slot_of.find(id);
    if (it == o->slot_of.end()) return 0;
    const uint32_t slot = it->second;
    bool removed = false;
    for (auto& kv : o->postings) {
        auto& v = kv.second;
        auto p = std::find_if(v.begin(), v.end(), [&](const Posting& x) { return x.slot == slot; });
        if (p == v.end()) continue;
        v.erase(p);
        removed = true;
        // the slot's first entry of this term (add order) goes with it
        auto& se = o->slot_entries[slot];
        for (size_t i = 0; i < se.size(); ++i)
            if (se[i].term == kv.first) {
                se.erase(se.begin() + i);
                break;
            }
        if (v.empty()) o->df.erase(kv.first);
    }
    if (removed) {
        o->total_documents = o->total_documents > 0 ? o->total_documents - 1 : 0;
        o->recompute_length();
        if (o->total_documents > 0)
            o->avgdl = o->total_length / (float)o->total_documents;
        else
            o->avgdl = 0.0f;
    }
    return removed ? 1 : 0;
}

void bm25o_stats(void* h, uint64_t* total_documents, float* avgdl, uint64_t* vocabulary_size) {
    Bm25Oracle* o = (Bm25Oracle*)h;
    *total_documents = o->total_documents;
    *avgdl = o->avgdl;
    *vocabulary_size = o->df.size();
}

// search_bm25 (sparse.rs:151-198) for one query: writes up to `limit` (id,
// score) pairs sorted by score descending (ties: slot ascending; NaN last).
uint64_t bm25o_search(void* h, const uint32_t* q_terms, const float* q_vals, uint64_t nq, uint64_t limit,
                      uint64_t* out_ids, float* out_scores) {
    Bm25Oracle* o = (Bm25Oracle*)h;
    if (o->total_documents == 0) return 0;
    std::vector<float> score(o->slot_id.size(), 0.0f);
    std::vector<uint8_t> hit(o->slot_id.size(), 0);
    std::vector<uint32_t> order;
    const float k1 = o->k1, b = o->b;
    for (uint64_t p = 0; p < nq; ++p) {
        auto pl = o->postings.find(q_terms[p]);
        if (pl == o->postings.end()) continue;
        auto d = o->df.find(q_terms[p]);
        const uint64_t dfv = d == o->df.end() ? 1 : d->second;
        // calculate_idf (sparse.rs:200-203)
        const float idf = std::log(((float)o->total_documents - (float)dfv + 0.5f) / ((float)dfv + 0.5f));
        for (const Posting& e : pl->second) {  // posting order
            const uint32_t slot = e.slot;
            // calculate_bm25_score (sparse.rs:206-222)
            const float tfc = (e.tf * (k1 + 1.0f)) / (e.tf + k1 * (1.0f - b + b * (e.dl / o->avgdl)));
            const float s = q_vals[p] * tfc * idf;
            if (!hit[slot]) {
                hit[slot] = 1;
                score[slot] = 0.0f;
                order.push_back(slot);
            }
            score[slot] = score[slot] + s;
        }
    }
    std::sort(order.begin(), order.end());
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t c) {
        const float x = score[a], y = score[c];
        const bool nx = x != x, ny = y != y;
        if (nx || ny) return !nx && ny;  // NaN last
        return x > y;
    });
    const uint64_t n = std::min<uint64_t>(limit, order.size());
    for (uint64_t i = 0; i < n; ++i) {
        out_ids[i] = o->slot_id[order[i]];
        out_scores[i] = score[order[i]];
    }
    return n;
}

// B queries in CSR (q_ptr[B+1]), one query per thread: the CPU baseline's
// throughput leg (concurrent readers, as SparseIndex's RwLock allows).
void bm25o_search_batch(void* h, const uint64_t* q_ptr, const uint32_t* q_terms, const float* q_vals, uint64_t B,
                        uint64_t limit, uint64_t* out_ids, float* out_scores, uint64_t* out_n, int threads) {
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int64_t q = 0; q < (int64_t)B; ++q)
        out_n[q] = bm25o_search(h, q_terms + q_ptr[q], q_vals + q_ptr[q], q_ptr[q + 1] - q_ptr[q], limit,
                                out_ids + q * limit, out_scores + q * limit);
}

// rrf_fusion (hybrid.rs:422-488): ranked id lists -> fused (id, score), all of
// them, sorted by score descending (ties: first appearance).  Also the
// breakdown of each result: its dense / sparse / text raw score (NaN = None).
uint64_t bm25o_rrf(const uint64_t* dense_ids, const float* dense_sc, uint64_t nd, const uint64_t* sparse_ids,
                   const float* sparse_sc, uint64_t ns, const uint64_t* text_ids, const float* text_sc, uint64_t nt,
                   float k, uint64_t* out_ids, float* out_scores, float* out_dense, float* out_sparse, float* out_text) {
    struct Acc {
        uint64_t id;
        float score, dense, sparse, text;
    };
    std::vector<Acc> acc;
    std::unordered_map<uint64_t, size_t> at;
    const float nan = std::nanf("");
    auto put = [&](uint64_t id, float r, int list, float raw) {
        auto f = at.find(id);
        if (f == at.end()) {
            at[id] = acc.size();
            acc.push_back({id, r, nan, nan, nan});
            f = at.find(id);
        } else if (list == 0) {
            acc[f->second].score = r;  // HashMap::insert replaces (hybrid.rs:444)
            acc[f->second].sparse = nan;
            acc[f->second].text = nan;
        } else {
            acc[f->second].score = acc[f->second].score + r;  // *current_score += rrf_score
        }
        Acc& a = acc[f->second];
        (list == 0 ? a.dense : list == 1 ? a.sparse : a.text) = raw;
    };
    for (uint64_t r = 0; r < nd; ++r) put(dense_ids[r], 1.0f / (k + (float)(r + 1)), 0, dense_sc[r]);
    for (uint64_t r = 0; r < ns; ++r) put(sparse_ids[r], 1.0f / (k + (float)(r + 1)), 1, sparse_sc[r]);
    for (uint64_t r = 0; r < nt; ++r) put(text_ids[r], 1.0f / (k + (float)(r + 1)), 2, text_sc[r]);
    std::vector<size_t> idx(acc.size());
    for (size_t i = 0; i < idx.size(); ++i) idx[i] = i;
    std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t c) { return acc[a].score > acc[c].score; });
    for (size_t i = 0; i < idx.size(); ++i) {
        out_ids[i] = acc[idx[i]].id;
        out_scores[i] = acc[idx[i]].score;
        if (out_dense) out_dense[i] = acc[idx[i]].dense;
        if (out_sparse) out_sparse[i] = acc[idx[i]].sparse;
        if (out_text) out_text[i] = acc[idx[i]].text;
    }
    return idx.size();
}

}  // extern "C"
