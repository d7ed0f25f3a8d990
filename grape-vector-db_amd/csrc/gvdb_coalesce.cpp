// gvdb_coalesce.cpp — batch-1 request coalescing for concurrent readers
// (include/gvdb.h, gvdb_coalescer_*).  Host code only: it drives the library's
// own gvdb_index_search.
//
// The reference serves many concurrent single-query searches through
// Arc<RwLock<dyn VectorIndex>> (src/lib.rs:238): every reader runs its own
// HnswVectorIndex::search(q, k) (src/index.rs:212-231).  On the GPU a
// batch-1 search is bound by reading the whole code array once (~0.15 ms at
// 10M x 768); B queries in one batch read it once as well.  So concurrent
// single-query callers are coalesced: a caller's query joins the pending
// list; whenever no batch is executing, the first caller to notice takes the
// whole pending list (up to max_batch) and runs it as ONE gvdb_index_search,
// then hands every caller its own k results.  No timer: requests arriving
// while a batch executes form the next batch ("batch while busy"), so a lone
// caller pays no added latency and batches grow with the load.
//
// Results are those of a serial gvdb_index_search per query: every search
// mode of the library is exact (certified stage 1 + exact rerank), so a
// query's answer does not depend on the batch it ran in (tests:
// tests/test_gpu_coalesce.py, bit-equal to serial calls).
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <condition_variable>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/gvdb.h"

namespace gvdb {
gvdb_status report_status(gvdb_status s, const std::string& msg);  // gvdb_capi.hip
}
using gvdb::report_status;

namespace {
struct Req {
    const float* q;
    uint64_t* ids;
    float* scores;
    uint32_t* n;
    gvdb_status st = GVDB_OK;
    std::string err;
    bool taken = false;
    bool done = false;
};
}  // namespace

struct gvdb_coalescer {
    const gvdb_index* ix;
    uint32_t dim;
    uint64_t k;
    gvdb_search_params sp;
    uint32_t max_batch;
    uint32_t max_exec;
    std::mutex mu;
    std::condition_variable cv;
    std::vector<Req*> pending;
    uint32_t executing = 0;
    uint64_t n_batches = 0, n_queries = 0, max_seen = 0;
};

namespace {
// one batch: the queries copied into one contiguous block, one library search,
// the results scattered back to the callers' buffers
void run_batch(gvdb_coalescer* c, const std::vector<Req*>& reqs) {
    const size_t B = reqs.size();
    std::vector<float> q(B * (size_t)c->dim);
    for (size_t i = 0; i < B; ++i) memcpy(q.data() + i * c->dim, reqs[i]->q, (size_t)c->dim * 4);
    std::vector<uint64_t> ids(B * c->k);
    std::vector<float> sc(B * c->k);
    std::vector<uint32_t> n(B);
    const gvdb_status st =
        gvdb_index_search(c->ix, q.data(), B, c->dim, c->k, &c->sp, ids.data(), sc.data(), n.data());
    const std::string err = st == GVDB_OK ? std::string() : std::string(gvdb_last_error());
    // A NaN score fails only the queries it poisoned: gvdb_index_search has
    // downloaded every query's results and counts before it reports
    // GVDB_ERR_QUANTIZATION, and each caller gets exactly its own serial result.
    const bool per_query = st == GVDB_ERR_QUANTIZATION;
    for (size_t i = 0; i < B; ++i) {
        Req* r = reqs[i];
        const bool ok = st == GVDB_OK || (per_query && n[i] != GVDB_N_POISONED);
        r->st = ok ? GVDB_OK : st;
        r->err = ok ? std::string() : err;
        if (ok) {
            memcpy(r->ids, ids.data() + i * c->k, c->k * 8);
            memcpy(r->scores, sc.data() + i * c->k, c->k * 4);
            if (r->n) *r->n = n[i];
        }
    }
}
}  // namespace

extern "C" {

gvdb_status gvdb_coalescer_create(const gvdb_index* index, uint32_t dim, uint64_t k, const gvdb_search_params* sp,
                                  uint32_t max_batch, uint32_t max_inflight, gvdb_coalescer** out) {
    if (!index || !out) return report_status(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    *out = nullptr;
    if (k == 0 || dim == 0) return report_status(GVDB_ERR_INVALID_ARGUMENT, "coalescer: k and dim must be > 0");
    auto* c = new gvdb_coalescer();
    c->ix = index;
    c->dim = dim;
    c->k = k;
    if (sp) {
        c->sp = *sp;
    } else {
        memset(&c->sp, 0, sizeof(c->sp));
        c->sp.mode = GVDB_SEARCH_BQ_RERANK;
        c->sp.metric = GVDB_METRIC_COSINE;
        c->sp.rescore_ratio = 0.1f;
    }
    c->max_batch = max_batch ? std::min<uint32_t>(max_batch, 4096u) : 256u;
    c->max_exec = max_inflight ? max_inflight : 1u;
    *out = c;
    return GVDB_OK;
}

gvdb_status gvdb_coalescer_search(gvdb_coalescer* c, const float* query, uint64_t* out_ids, float* out_scores,
                                  uint32_t* out_n) {
    if (!c || !query || !out_ids || !out_scores) return report_status(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    Req r;
    r.q = query;
    r.ids = out_ids;
    r.scores = out_scores;
    r.n = out_n;
    std::unique_lock<std::mutex> lk(c->mu);
    c->pending.push_back(&r);
    while (!r.done) {
        if (!r.taken && c->executing < c->max_exec && !c->pending.empty()) {
            // this caller leads the next batch: the oldest pending requests (its own included)
            const size_t m = std::min<size_t>(c->pending.size(), c->max_batch);
            std::vector<Req*> mine(c->pending.begin(), c->pending.begin() + m);
            c->pending.erase(c->pending.begin(), c->pending.begin() + m);
            for (Req* x : mine) x->taken = true;
            c->executing += 1;
            c->n_batches += 1;
            c->n_queries += m;
            c->max_seen = std::max<uint64_t>(c->max_seen, m);
            lk.unlock();
            run_batch(c, mine);
            lk.lock();
            c->executing -= 1;
            for (Req* x : mine) x->done = true;
            c->cv.notify_all();
        } else {
            c->cv.wait(lk);
        }
    }
    lk.unlock();
    if (r.st != GVDB_OK) return report_status(r.st, r.err);
    return GVDB_OK;
}

gvdb_status gvdb_coalescer_stats(gvdb_coalescer* c, uint64_t* batches, uint64_t* queries, uint64_t* max_batch) {
    if (!c) return report_status(GVDB_ERR_INVALID_ARGUMENT, "null coalescer");
    std::lock_guard<std::mutex> lk(c->mu);
    if (batches) *batches = c->n_batches;
    if (queries) *queries = c->n_queries;
    if (max_batch) *max_batch = c->max_seen;
    return GVDB_OK;
}

void gvdb_coalescer_destroy(gvdb_coalescer* c) {
    if (!c) return;
    {
        // callers still inside gvdb_coalescer_search would be a caller bug; wait for them anyway
        std::unique_lock<std::mutex> lk(c->mu);
        c->cv.wait(lk, [c] { return c->executing == 0 && c->pending.empty(); });
    }
    delete c;
}

}  // extern "C"
