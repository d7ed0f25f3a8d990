// coalesce_bench — concurrent batch-1 searches through the C ABI only
// (include/gvdb.h): T threads each run single-query searches, either one
// gvdb_index_search(B = 1) per query (the reference's concurrent readers, each
// running its own HnswVectorIndex::search, src/lib.rs:238 + index.rs:212-231)
// or gvdb_coalescer_search (concurrent queries share batched searches).
// Prints one JSON line per (mode, threads) point: QPS, p50 / p99 latency, mean
// batch size, and whether every coalesced answer equals the serial one.
//
//   coalesce_bench N D R K SECONDS THREADS...   (corpus: N x D i.i.d. normal,
//   unit rows, seed 0x6772617065; 4096 i.i.d. queries)
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#include "../../include/gvdb.h"

namespace {
struct Rng {  // splitmix64 -> Box-Muller
    uint64_t s;
    uint64_t next() {
        uint64_t z = (s += 0x9e3779b97f4a7c15ull);
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
        return z ^ (z >> 31);
    }
    double u() { return ((next() >> 11) + 0.5) * (1.0 / 9007199254740992.0); }
    float normal() { return (float)(sqrt(-2.0 * log(u())) * cos(6.283185307179586 * u())); }
};
void fill_unit_rows(float* x, uint64_t n, uint32_t d, uint64_t seed) {
    const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> ts;
    for (unsigned t = 0; t < nt; ++t)
        ts.emplace_back([=] {
            for (uint64_t i = t; i < n; i += nt) {
                Rng r{seed * 0x100000001b3ull + i};
                double ss = 0;
                float* row = x + i * d;
                for (uint32_t j = 0; j < d; ++j) {
                    row[j] = r.normal();
                    ss += (double)row[j] * row[j];
                }
                const float inv = (float)(1.0 / sqrt(ss));
                for (uint32_t j = 0; j < d; ++j) row[j] *= inv;
            }
        });
    for (auto& t : ts) t.join();
}
#define CHECK(x)                                                                          \
    do {                                                                                  \
        gvdb_status st_ = (x);                                                            \
        if (st_ != GVDB_OK) {                                                             \
            fprintf(stderr, "%s:%d %s -> %d: %s\n", __FILE__, __LINE__, #x, (int)st_,     \
                    gvdb_last_error());                                                   \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)
double pct(std::vector<double>& v, double p) {
    if (v.empty()) return 0;
    std::sort(v.begin(), v.end());
    return v[std::min(v.size() - 1, (size_t)(p * (v.size() - 1) + 0.5))];
}
}  // namespace

int main(int argc, char** argv) {
    if (argc < 7) {
        fprintf(stderr, "usage: %s N D R K SECONDS THREADS...\n", argv[0]);
        return 2;
    }
    const uint64_t N = strtoull(argv[1], 0, 10);
    const uint32_t D = (uint32_t)atoi(argv[2]);
    const uint64_t R = strtoull(argv[3], 0, 10), K = strtoull(argv[4], 0, 10);
    const double secs = atof(argv[5]);
    std::vector<int> thr;
    for (int i = 6; i < argc; ++i) thr.push_back(atoi(argv[i]));

    gvdb_params p{};
    p.dimension = D;
    p.capacity_hint = N;
    gvdb_index* ix = nullptr;
    CHECK(gvdb_index_create(&p, &ix));
    const uint64_t chunk = 1ull << 20;
    std::vector<float> buf(chunk * D);
    std::vector<uint64_t> ids(chunk);
    auto t0 = std::chrono::steady_clock::now();
    for (uint64_t c0 = 0; c0 < N; c0 += chunk) {
        const uint64_t n = std::min(chunk, N - c0);
        fill_unit_rows(buf.data(), n, D, 0x6772617065ull + c0);
        for (uint64_t i = 0; i < n; ++i) ids[i] = c0 + i;
        CHECK(gvdb_index_add(ix, buf.data(), n, D, ids.data()));
    }
    fprintf(stderr, "[coalesce] corpus %llu x %u: %.1f s\n", (unsigned long long)N, D,
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    const uint64_t NQ = 4096;
    std::vector<float> Q(NQ * D);
    fill_unit_rows(Q.data(), NQ, D, 0x6772617066ull);
    gvdb_search_params sp{};
    sp.mode = GVDB_SEARCH_BQ_RERANK;
    sp.metric = GVDB_METRIC_COSINE;
    sp.rescore_count = R;
    sp.rescore_ratio = 0.1f;
    // serial reference answers (one B = 1 search per query) for the first 512 queries
    const uint64_t NC = 512;
    std::vector<uint64_t> ref_i(NC * K);
    std::vector<float> ref_s(NC * K);
    std::vector<uint32_t> ref_n(NC);
    for (uint64_t i = 0; i < NC; ++i)
        CHECK(gvdb_index_search(ix, Q.data() + i * D, 1, D, K, &sp, ref_i.data() + i * K, ref_s.data() + i * K,
                                ref_n.data() + i));

    for (int mode = 0; mode < 2; ++mode) {  // 0: gvdb_index_search B = 1 per caller; 1: coalescer
        for (int T : thr) {
            gvdb_coalescer* co = nullptr;
            if (mode == 1) CHECK(gvdb_coalescer_create(ix, D, K, &sp, 256, 1, &co));
            std::atomic<uint64_t> next{0};
            std::atomic<bool> stop{false};
            std::atomic<uint64_t> mismatches{0}, checked{0};
            std::vector<std::vector<double>> lat(T);
            std::vector<std::thread> ts;
            const auto start = std::chrono::steady_clock::now();
            for (int t = 0; t < T; ++t)
                ts.emplace_back([&, t] {
                    std::vector<uint64_t> oi(K);
                    std::vector<float> os(K);
                    uint32_t on = 0;
                    while (!stop.load(std::memory_order_relaxed)) {
                        const uint64_t qi = next.fetch_add(1) % NQ;
                        const auto a = std::chrono::steady_clock::now();
                        if (mode == 0)
                            CHECK(gvdb_index_search(ix, Q.data() + qi * D, 1, D, K, &sp, oi.data(), os.data(), &on));
                        else
                            CHECK(gvdb_coalescer_search(co, Q.data() + qi * D, oi.data(), os.data(), &on));
                        lat[t].push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a)
                                             .count());
                        if (qi < NC) {
                            checked += 1;
                            if (on != ref_n[qi] || memcmp(oi.data(), ref_i.data() + qi * K, K * 8) ||
                                memcmp(os.data(), ref_s.data() + qi * K, K * 4))
                                mismatches += 1;
                        }
                    }
                });
            std::this_thread::sleep_for(std::chrono::duration<double>(secs));
            stop = true;
            for (auto& x : ts) x.join();
            const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - start).count();
            std::vector<double> all;
            for (auto& v : lat) all.insert(all.end(), v.begin(), v.end());
            uint64_t batches = 0, queries = 0, largest = 0;
            if (co) {
                CHECK(gvdb_coalescer_stats(co, &batches, &queries, &largest));
                gvdb_coalescer_destroy(co);
            }
            const double nq = (double)all.size();
            printf("{\"mode\": \"%s\", \"threads\": %d, \"queries\": %.0f, \"qps\": %.1f, \"p50_us\": %.1f, "
                   "\"p99_us\": %.1f, \"mean_batch\": %.2f, \"largest_batch\": %llu, \"checked\": %llu, "
                   "\"mismatches\": %llu}\n",
                   mode == 0 ? "search_b1" : "coalescer", T, nq, nq / el, pct(all, 0.5), pct(all, 0.99),
                   batches ? (double)queries / batches : 1.0, (unsigned long long)largest,
                   (unsigned long long)checked.load(), (unsigned long long)mismatches.load());
            fflush(stdout);
        }
    }
    gvdb_index_destroy(ix);
    return 0;
}
