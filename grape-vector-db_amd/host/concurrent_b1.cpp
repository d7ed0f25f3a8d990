// concurrent_b1 — measurement driver (bench.py's CPU-HNSW pairing leg): T host
// threads each run single-query searches through the C ABI alone
// (gvdb_index_search with B = 1, exactly as the Rust binding's
// VectorIndex::search does for the reference's concurrent readers of
// Arc<RwLock<dyn VectorIndex>>, src/lib.rs:238 + index.rs:212-231), for a
// fixed wall time over a query set; the library coalesces concurrent B = 1
// calls itself.  Reports QPS, p50 / p99 latency, and each query's result
// (the first time it ran) so the caller scores recall.  Not part of
// libgvdb; built as build/libgvdb_drive.so.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#include "../../include/gvdb.h"

extern "C" int gvdb_drive_concurrent_b1(const gvdb_index* ix, const float* queries, uint64_t nq, uint32_t dim,
                                        uint64_t k, const gvdb_search_params* sp, uint32_t threads, double seconds,
                                        uint64_t* out_ids, double* out_stats) {
    if (!ix || !queries || nq == 0 || k == 0 || threads == 0 || !out_ids || !out_stats) return -1;
    std::vector<uint8_t> seen(nq, 0);
    std::atomic<uint64_t> next{0};
    std::atomic<bool> stop{false};
    std::atomic<int> err{0};
    std::vector<std::vector<double>> lat(threads);
    std::vector<std::thread> ts;
    const auto start = std::chrono::steady_clock::now();
    for (uint32_t t = 0; t < threads; ++t)
        ts.emplace_back([&, t] {
            std::vector<uint64_t> oi(k);
            std::vector<float> os(k);
            uint32_t on = 0;
            lat[t].reserve(1 << 16);
            while (!stop.load(std::memory_order_relaxed)) {
                const uint64_t i = next.fetch_add(1);
                const uint64_t qi = i % nq;
                const auto a = std::chrono::steady_clock::now();
                if (gvdb_index_search(ix, queries + qi * dim, 1, dim, k, sp, oi.data(), os.data(), &on) != GVDB_OK) {
                    err = 1;
                    return;
                }
                lat[t].push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
                if (i < nq) memcpy(out_ids + qi * k, oi.data(), k * 8);  // the first pass over the set (indices unique)
            }
        });
    // at least one full pass over the query set, then the time budget
    while (next.load() < nq + threads && !err.load()) std::this_thread::sleep_for(std::chrono::milliseconds(1));
    const double el0 = std::chrono::duration<double>(std::chrono::steady_clock::now() - start).count();
    if (el0 < seconds) std::this_thread::sleep_for(std::chrono::duration<double>(seconds - el0));
    stop = true;
    for (auto& x : ts) x.join();
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - start).count();
    if (err.load()) return -2;
    std::vector<double> all;
    for (auto& v : lat) all.insert(all.end(), v.begin(), v.end());
    std::sort(all.begin(), all.end());
    auto pct = [&](double p) { return all.empty() ? 0.0 : all[std::min(all.size() - 1, (size_t)(p * (all.size() - 1) + 0.5))]; };
    out_stats[0] = (double)all.size() / el;
    out_stats[1] = pct(0.5);
    out_stats[2] = pct(0.99);
    out_stats[3] = (double)all.size();
    out_stats[4] = el;
    return 0;
}
