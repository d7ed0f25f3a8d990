// ============================================================================
// hnsw_oracle.cpp — CPU HNSW BASELINE (TEST / BENCH INFRASTRUCTURE ONLY)
//
// A C++ restatement of the graph index behind the reference's
// HnswVectorIndex (src/index.rs:140-154 build, 212-231 search), which calls
// the third-party crate instant-distance 0.6.1 (Cargo.lock:1609; not vendored
// under /root/reference and not fetchable here).  Only tests/ and bench /
// scripts CPU-baseline legs load it; nothing in grape-vector-db_amd/ does.
//
// What is restated (instant-distance 0.6.1 as used with Builder::default()):
//   * distance = VectorPoint::distance (index.rs:64-79): sqrt of the strict
//     left-to-right f32 sum of (x-y)^2, folded from -0.0;
//   * M = 32 links on upper layers, 2M = 64 on layer 0; ml = 1/ln(M);
//     ef_construction = ef_search = 100 (Builder::default);
//   * layer sizes are fixed by ml (the crate sizes layers geometrically:
//     next = (num as f32 * ml) as usize until next < M) and a seeded random
//     permutation decides which point lands where; the entry point is the
//     first point of the top layer;
//   * insertion: greedy descent (ef = 1) through the layers above the point's
//     own, then an ef_construction beam per own layer, neighbours chosen by
//     the paper's heuristic with keep_pruned = true, extend_candidates =
//     false (the crate's default Heuristic); a node's links are kept sorted by
//     distance in a fixed-size array, and a reverse link into a full array
//     replaces the farthest one when it is nearer (sorted insert);
//   * search: greedy descent to layer 1, an ef_search beam on layer 0, results
//     ascending by distance, take(k) (index.rs:216-217).
//
// Parity status: NOT bit-comparable.  The crate builds its layers with rayon
// in parallel (graph depends on thread timing) from an OS-random seed, so no
// two reference builds agree either.  Parity for this component is by
// recall@10 against exact ground truth only — "parity
// unpinned" for graph identity.  The reference-faithful O(N*k) id remap of
// index.rs:219-228 is deliberately NOT reproduced here ("ref-algorithmic"
// baseline); bench notes say so.
// ============================================================================
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <queue>
#include <thread>
#include <vector>

namespace {

float l2(const float* a, const float* b, uint32_t d) {
    float s = -0.0f;
    for (uint32_t i = 0; i < d; ++i) {
        const float t = a[i] - b[i];
        s = s + t * t;
    }
    return std::sqrt(s);
}

// Four independent distances with their folds interleaved: each sum is still
// the strict left-to-right fold of l2() (bit-identical), but the four
// dependency chains overlap, so a beam step costs ~1/4 of four l2() calls.
// (A CPU-side optimisation the reference does not have: it only makes the
// baseline faster, never different.)
void l2x4(const float* q, const float* const* r, uint32_t d, float* out) {
    float s0 = -0.0f, s1 = -0.0f, s2 = -0.0f, s3 = -0.0f;
    const float *a = r[0], *b = r[1], *c = r[2], *e = r[3];
    for (uint32_t i = 0; i < d; ++i) {
        const float x = q[i];
        const float t0 = x - a[i], t1 = x - b[i], t2 = x - c[i], t3 = x - e[i];
        s0 = s0 + t0 * t0;
        s1 = s1 + t1 * t1;
        s2 = s2 + t2 * t2;
        s3 = s3 + t3 * t3;
    }
    out[0] = std::sqrt(s0);
    out[1] = std::sqrt(s1);
    out[2] = std::sqrt(s2);
    out[3] = std::sqrt(s3);
}

// "fast" distances (opt-in, hnsw_build2 / hnsw_set_fast): the same L2 with the
// sum split over 32 partial sums (AVX2 lanes), i.e. re-associated -- results
// differ from the strict fold in the last bits.  Used to BUILD the 10M-row
// graph in reasonable time (the graph is random anyway: the crate builds it in
// parallel from an OS seed) and as the optimised-CPU point of the baseline;
// the reference-faithful strict fold stays the default.
typedef float v8f __attribute__((vector_size(32)));
__attribute__((target("avx2"))) float l2_fast(const float* a, const float* b, uint32_t d) {
    v8f s0 = {0, 0, 0, 0, 0, 0, 0, 0}, s1 = s0, s2 = s0, s3 = s0;
    uint32_t i = 0;
    for (; i + 32 <= d; i += 32) {
        v8f x0, x1, x2, x3, y0, y1, y2, y3;
        std::memcpy(&x0, a + i, 32);
        std::memcpy(&x1, a + i + 8, 32);
        std::memcpy(&x2, a + i + 16, 32);
        std::memcpy(&x3, a + i + 24, 32);
        std::memcpy(&y0, b + i, 32);
        std::memcpy(&y1, b + i + 8, 32);
        std::memcpy(&y2, b + i + 16, 32);
        std::memcpy(&y3, b + i + 24, 32);
        x0 -= y0;
        x1 -= y1;
        x2 -= y2;
        x3 -= y3;
        s0 += x0 * x0;
        s1 += x1 * x1;
        s2 += x2 * x2;
        s3 += x3 * x3;
    }
    const v8f t = (s0 + s1) + (s2 + s3);
    float s = ((t[0] + t[1]) + (t[2] + t[3])) + ((t[4] + t[5]) + (t[6] + t[7]));
    for (; i < d; ++i) {
        const float u = a[i] - b[i];
        s = s + u * u;
    }
    return std::sqrt(s);
}

uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

struct Cand {
    float d;
    uint32_t id;
    bool operator<(const Cand& o) const { return d < o.d || (d == o.d && id < o.id); }
    bool operator>(const Cand& o) const { return o < *this; }
};

struct Hnsw {
    const float* rows = nullptr;  // caller-owned, n x d row-major (not copied)
    uint64_t n = 0;
    uint32_t d = 0, M = 32, ef_c = 100;
    std::vector<uint32_t> order;        // insertion order (shuffled point ids)
    std::vector<uint8_t> level;         // top layer of each point
    uint32_t top = 0;
    uint32_t entry = 0;
    // layer 0: fixed 2M slots per node; upper layers: M slots, sparse map by rank
    std::vector<uint32_t> l0, l0n;
    std::vector<float> l0d;                      // link distances (lists sorted ascending)
    std::vector<std::vector<uint32_t>> up, upn;  // [layer-1][slot index]
    std::vector<std::vector<float>> upd;
    std::vector<uint32_t> upslot;               // point -> slot in upper layers (or ~0)
    std::vector<std::mutex> locks;
    bool fast = false;  // l2_fast instead of the strict fold

    void dist4(const float* q, const float* const* r4, float* out) const {
        if (fast) {
            for (int t = 0; t < 4; ++t) out[t] = l2_fast(q, r4[t], d);
        } else {
            l2x4(q, r4, d, out);
        }
    }
    float dist_rows(const float* a, const float* b) const { return fast ? l2_fast(a, b, d) : l2(a, b, d); }

    uint32_t cap(uint32_t layer) const { return layer == 0 ? 2 * M : M; }
    uint32_t* links(uint32_t p, uint32_t layer, uint32_t*& cnt, float** ds = nullptr) {
        if (layer == 0) {
            cnt = &l0n[p];
            if (ds) *ds = &l0d[(uint64_t)p * 2 * M];
            return &l0[(uint64_t)p * 2 * M];
        }
        const uint32_t s = upslot[p];
        cnt = &upn[layer - 1][s];
        if (ds) *ds = &upd[layer - 1][(uint64_t)s * M];
        return &up[layer - 1][(uint64_t)s * M];
    }
    float dist(const float* q, uint32_t p) const { return dist_rows(q, rows + (uint64_t)p * d); }

    // ef-beam on one layer from the given entry set; returns ascending results
    std::vector<Cand> beam(const float* q, const std::vector<Cand>& eps, uint32_t ef, uint32_t layer,
                           std::vector<uint32_t>& seen, uint32_t& epoch, bool lock) {
        if (++epoch == 0) {
            std::fill(seen.begin(), seen.end(), 0u);
            epoch = 1;
        }
        std::priority_queue<Cand, std::vector<Cand>, std::greater<Cand>> cand;  // min-heap
        std::priority_queue<Cand> res;                                          // max-heap
        for (const Cand& e : eps) {
            if (seen[e.id] == epoch) continue;
            seen[e.id] = epoch;
            cand.push(e);
            res.push(e);
            if (res.size() > ef) res.pop();
        }
        std::vector<uint32_t> nb, todo;
        std::vector<float> dv4;
        while (!cand.empty()) {
            const Cand c = cand.top();
            if (res.size() >= ef && c.d > res.top().d) break;
            cand.pop();
            uint32_t* cnt;
            {
                uint32_t* l = links(c.id, layer, cnt);
                if (lock) {
                    std::lock_guard<std::mutex> g(locks[c.id]);
                    nb.assign(l, l + *cnt);
                } else {
                    nb.assign(l, l + *cnt);
                }
            }
            // unseen neighbours in list order, their distances four at a time
            todo.clear();
            for (uint32_t v : nb) {
                if (seen[v] == epoch) continue;
                seen[v] = epoch;
                todo.push_back(v);
            }
            dv4.resize(todo.size() + 3);
            size_t j = 0;
            for (; j + 4 <= todo.size(); j += 4) {
                const float* r4[4];
                for (int t = 0; t < 4; ++t) r4[t] = rows + (uint64_t)todo[j + t] * d;
                dist4(q, r4, &dv4[j]);
            }
            for (; j < todo.size(); ++j) dv4[j] = dist(q, todo[j]);
            for (size_t t = 0; t < todo.size(); ++t) {
                const uint32_t v = todo[t];
                const float dv = dv4[t];
                if (res.size() < ef || dv < res.top().d) {
                    cand.push({dv, v});
                    res.push({dv, v});
                    if (res.size() > ef) res.pop();
                }
            }
        }
        std::vector<Cand> out(res.size());
        for (size_t i = out.size(); i-- > 0;) {
            out[i] = res.top();
            res.pop();
        }
        return out;
    }

    // heuristic neighbour selection (keep_pruned = true, extend_candidates = false)
    std::vector<Cand> select(const std::vector<Cand>& asc, uint32_t m) {
        std::vector<Cand> keep, pruned;
        for (const Cand& c : asc) {
            if (keep.size() >= m) break;
            bool good = true;
            const float* x = rows + (uint64_t)c.id * d;
            size_t j = 0;
            for (; good && j + 4 <= keep.size(); j += 4) {  // same test, four distances at a time
                const float* r4[4];
                float d4[4];
                for (int t = 0; t < 4; ++t) r4[t] = rows + (uint64_t)keep[j + t].id * d;
                dist4(x, r4, d4);
                for (int t = 0; t < 4; ++t) good = good && !(d4[t] < c.d);
            }
            for (; good && j < keep.size(); ++j)
                if (dist_rows(x, rows + (uint64_t)keep[j].id * d) < c.d) good = false;
            (good ? keep : pruned).push_back(c);
        }
        for (size_t i = 0; i < pruned.size() && keep.size() < m; ++i) keep.push_back(pruned[i]);
        return keep;
    }

    void connect(uint32_t a, uint32_t b, float dab, uint32_t layer) {  // add b to a's sorted list
        std::lock_guard<std::mutex> g(locks[a]);
        uint32_t* cnt;
        float* ds;
        uint32_t* l = links(a, layer, cnt, &ds);
        for (uint32_t i = 0; i < *cnt; ++i)
            if (l[i] == b) return;
        uint32_t pos = *cnt;
        while (pos > 0 && ds[pos - 1] > dab) --pos;
        if (pos >= cap(layer)) return;  // full and farther than every link
        const uint32_t last = std::min(*cnt, cap(layer) - 1);
        for (uint32_t i = last; i > pos; --i) {
            l[i] = l[i - 1];
            ds[i] = ds[i - 1];
        }
        l[pos] = b;
        ds[pos] = dab;
        *cnt = std::min(*cnt + 1, cap(layer));
    }

    void insert(uint32_t p, std::vector<uint32_t>& seen, uint32_t& epoch) {
        const float* q = rows + (uint64_t)p * d;
        std::vector<Cand> ep{{dist(q, entry), entry}};
        for (uint32_t layer = top; layer > level[p]; --layer) ep = {beam(q, ep, 1, layer, seen, epoch, true)[0]};
        for (int layer = (int)std::min<uint32_t>(level[p], top); layer >= 0; --layer) {
            std::vector<Cand> w = beam(q, ep, ef_c, (uint32_t)layer, seen, epoch, true);
            std::vector<Cand> wn;
            for (const Cand& c : w)
                if (c.id != p) wn.push_back(c);
            const std::vector<Cand> nb = select(wn, cap((uint32_t)layer));
            {
                std::lock_guard<std::mutex> g(locks[p]);
                uint32_t* cnt;
                float* ds;
                uint32_t* l = links(p, (uint32_t)layer, cnt, &ds);
                std::vector<Cand> srt = nb;  // keep_pruned refills may be out of order
                std::sort(srt.begin(), srt.end());
                *cnt = (uint32_t)srt.size();
                for (size_t i = 0; i < srt.size(); ++i) {
                    l[i] = srt[i].id;
                    ds[i] = srt[i].d;
                }
            }
            for (const Cand& v : nb) connect(v.id, p, v.d, (uint32_t)layer);
            ep = w;
        }
    }
};

}  // namespace

extern "C" {

void* hnsw_build2(const float* rows, uint64_t n, uint32_t d, uint32_t M, uint32_t ef_construction, uint64_t seed,
                  int threads, int fast);
// Build over caller-owned rows (must outlive the handle).  threads<=0 -> all cores.
void* hnsw_build(const float* rows, uint64_t n, uint32_t d, uint32_t M, uint32_t ef_construction, uint64_t seed,
                 int threads) {
    return hnsw_build2(rows, n, d, M, ef_construction, seed, threads, 0);
}
// fast = 1: build with l2_fast (see above)
void hnsw_set_fast(void* p, int fast) {
    if (p) ((Hnsw*)p)->fast = fast != 0;
}
void* hnsw_build2(const float* rows, uint64_t n, uint32_t d, uint32_t M, uint32_t ef_construction, uint64_t seed,
                  int threads, int fast) {
    if (!rows || n == 0 || d == 0 || n > 0xFFFFFFFFull) return nullptr;
    Hnsw* h = new Hnsw;
    h->fast = fast != 0;
    h->rows = rows;
    h->n = n;
    h->d = d;
    h->M = M ? M : 32;
    h->ef_c = ef_construction ? ef_construction : 100;
    // layer sizes (geometric by ml = 1/ln M), counts of points at layer >= l
    const float ml = 1.0f / std::log((float)h->M);
    std::vector<uint64_t> at_least{n};
    for (uint64_t num = n;;) {
        const uint64_t next = (uint64_t)((float)num * ml);
        if (next < h->M) break;
        at_least.push_back(next);
        num = next;
    }
    h->top = (uint32_t)at_least.size() - 1;
    h->order.resize(n);
    for (uint64_t i = 0; i < n; ++i) h->order[i] = (uint32_t)i;
    uint64_t s = seed;
    for (uint64_t i = n - 1; i > 0; --i) std::swap(h->order[i], h->order[splitmix(s) % (i + 1)]);
    h->level.assign(n, 0);
    for (uint64_t r = 0; r < n; ++r) {
        uint32_t lv = 0;
        while (lv + 1 < at_least.size() && r < at_least[lv + 1]) ++lv;
        h->level[h->order[r]] = (uint8_t)lv;
    }
    h->entry = h->order[0];
    h->l0.assign(n * 2 * h->M, 0);
    h->l0d.assign(n * 2 * h->M, 0.0f);
    h->l0n.assign(n, 0);
    h->up.resize(h->top);
    h->upd.resize(h->top);
    h->upn.resize(h->top);
    h->upslot.assign(n, ~0u);
    const uint64_t nup = at_least.size() > 1 ? at_least[1] : 0;  // points on layer >= 1
    for (uint64_t r = 0; r < nup; ++r) h->upslot[h->order[r]] = (uint32_t)r;
    for (uint32_t l = 1; l <= h->top; ++l) {
        h->up[l - 1].assign(nup * h->M, 0);
        h->upd[l - 1].assign(nup * h->M, 0.0f);
        h->upn[l - 1].assign(nup, 0);
    }
    h->locks = std::vector<std::mutex>(n);
    const int T = threads > 0 ? threads : (int)std::max(1u, std::thread::hardware_concurrency());
    // layer by layer from the top, each layer's points in parallel (as the
    // crate does: points of one layer are inserted concurrently once every
    // higher layer is complete); rank 0 is the entry point
    std::atomic<uint64_t> done{0};
    for (int L = (int)h->top; L >= 0; --L) {
        const uint64_t lo = std::max<uint64_t>(L + 1 < (int)at_least.size() ? at_least[L + 1] : 0, 1);
        const uint64_t hi = at_least[L];
        if (lo >= hi) continue;
        std::atomic<uint64_t> next{lo};
        std::vector<std::thread> pool;
        const int TL = (int)std::min<uint64_t>((uint64_t)T, hi - lo);
        for (int t = 0; t < TL; ++t)
            pool.emplace_back([&] {
                std::vector<uint32_t> seen(n, 0);
                uint32_t epoch = 0;
                for (;;) {
                    const uint64_t r = next.fetch_add(1);
                    if (r >= hi) break;
                    h->insert(h->order[r], seen, epoch);
                    // progress for long builds (a silent multi-minute run looks hung to the GPU-box runner)
                    const uint64_t c = done.fetch_add(1) + 1;
                    if (n >= 200000 && c % 50000 == 0)
                        fprintf(stderr, "[hnsw] inserted %llu / %llu\n", (unsigned long long)c, (unsigned long long)n);
                }
            });
        for (auto& th : pool) th.join();
    }
    return h;
}

void hnsw_free(void* p) { delete (Hnsw*)p; }

// B queries, k results each (ascending L2), ef_search beam; threads<=0 -> all cores.
// out_n[b] = number of results (min(k, ef, n)).
int hnsw_search(void* p, const float* q, uint64_t B, uint32_t k, uint32_t ef_search, int threads, uint64_t* out_ids,
                float* out_dist, uint32_t* out_n) {
    Hnsw* h = (Hnsw*)p;
    if (!h || !q) return 1;
    const uint32_t ef = std::max(ef_search ? ef_search : 100u, 1u);
    const int T = threads > 0 ? threads : (int)std::max(1u, std::thread::hardware_concurrency());
    std::atomic<uint64_t> next{0};
    auto work = [&] {
        std::vector<uint32_t> seen(h->n, 0);
        uint32_t epoch = 0;
        for (;;) {
            const uint64_t b = next.fetch_add(1);
            if (b >= B) break;
            const float* x = q + b * h->d;
            std::vector<Cand> ep{{h->dist(x, h->entry), h->entry}};
            for (uint32_t layer = h->top; layer > 0; --layer) ep = {h->beam(x, ep, 1, layer, seen, epoch, false)[0]};
            const std::vector<Cand> res = h->beam(x, ep, ef, 0, seen, epoch, false);
            const uint32_t m = (uint32_t)std::min<size_t>(k, res.size());
            for (uint32_t i = 0; i < m; ++i) {
                out_ids[b * k + i] = res[i].id;
                out_dist[b * k + i] = res[i].d;
            }
            out_n[b] = m;
        }
    };
    if (T == 1) {
        work();
    } else {
        std::vector<std::thread> pool;
        for (int t = 0; t < T; ++t) pool.emplace_back(work);
        for (auto& th : pool) th.join();
    }
    return 0;
}

}  // extern "C"
