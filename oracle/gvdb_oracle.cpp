// ============================================================================
// gvdb_oracle.cpp — CPU ORACLE (TEST INFRASTRUCTURE ONLY)
//
// A sequential C++ restatement of grape-vector-db's ANN hot path
// (reference snapshot 2025-08-24, Rust).  It exists to CHECK the HIP product
// path; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
// may load it.  Nothing in grape-vector-db_amd/ links or calls it.
//
// Parity status: the reference is Rust and no Rust toolchain exists in this
// image, so it cannot be compiled or run here (toolchain ABSENT, not a denied
// action).  This restatement is pinned by the reference's own known-answer
// tests (quantization.rs:361-386, query.rs:428-483, hybrid.rs:991-1025,
// sparse.rs:383-420) re-expressed in tests/golden/kat.json, plus the
// published algorithms of the third-party crates the path calls:
//   * bitvec 1.0.1   (Cargo.lock:326)  BitVec<u8, Msb0>: bit i -> byte i/8,
//                    bit position 7 - i%8; dead bits of the last byte are 0.
//   * hamming 0.1.3  (Cargo.lock:1204) distance(&[u8],&[u8]) = popcount(a^b),
//                    asserting equal lengths.
//   * instant-distance 0.6.1 (Cargo.lock:1609) — HNSW, restated separately
//                    (oracle/hnsw_oracle.cpp), parity by recall only.
//
// Floating-point rules (Rust defaults): no FMA contraction, no reassociation
// (build with -ffp-contract=off -fno-fast-math), strict left-to-right f32
// sums.  `impl Sum for f32` folds from -0.0 on current stable Rust (the
// reference CI uses dtolnay/rust-toolchain@stable), so sums start at -0.0f.
// Sorting: Rust's slice::sort_by is a STABLE sort: equal keys keep their
// input order.  `x as usize` on f32 saturates (NaN -> 0).
// ============================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <numeric>
#include <vector>
#include <unordered_map>
#include <string>
#include <chrono>

#ifdef _OPENMP
#include <omp.h>
#endif

extern "C" {

// Status codes shared with include/gvdb.h (kept numerically identical).
enum {
    ORC_OK = 0,
    ORC_ERR_INDEX_NOT_BUILT = 1,
    ORC_ERR_DIMENSION_MISMATCH = 2,
    ORC_ERR_INVALID_VECTOR_DIMENSION = 3,
    ORC_ERR_QUANTIZATION = 4,
    ORC_ERR_INDEX = 5,
    ORC_ERR_INVALID_ARGUMENT = 6,
};

// Rust `f32 as usize` (saturating, NaN -> 0).
static uint64_t rust_f32_as_usize(float v) {
    if (!(v == v)) return 0;
    if (v <= 0.0f) return 0;
    if (v >= 18446744073709551615.0f) return UINT64_MAX;
    return (uint64_t)v;
}

uint64_t orc_rust_f32_as_usize(float v) { return rust_f32_as_usize(v); }

// ---------------------------------------------------------------------------
// BinaryQuantizer::quantize  (quantization.rs:86-122; cache path 89-109 and
// direct path 111-121 compute identical bits).  bit_i = (x_i > threshold),
// pushed into BitVec<u8, Msb0>: byte i/8, bit (7 - i%8).  NaN > t is false.
// out: n rows of ceil(D/8) bytes.
// ---------------------------------------------------------------------------
void orc_bq_quantize(const float* x, uint64_t n, uint32_t D, float threshold, uint8_t* out) {
    const uint64_t nb = (D + 7u) / 8u;
    for (uint64_t r = 0; r < n; ++r) {
        const float* row = x + r * D;
        uint8_t* o = out + r * nb;
        std::memset(o, 0, nb);
        for (uint32_t i = 0; i < D; ++i)
            if (row[i] > threshold) o[i >> 3] |= (uint8_t)(0x80u >> (i & 7u));
    }
}

// hamming 0.1.3 `distance` (called at quantization.rs:139): popcount(a XOR b)
// over the byte slices.
uint64_t orc_hamming(const uint8_t* a, const uint8_t* b, uint64_t nbytes) {
    uint64_t d = 0;
    for (uint64_t i = 0; i < nbytes; ++i) d += (uint64_t)__builtin_popcount((unsigned)(a[i] ^ b[i]));
    return d;
}

// BinaryQuantizer::similarity (quantization.rs:144-148):
//   1.0 - (distance as f32 / dimension as f32), all f32.
float orc_similarity(uint64_t distance, uint32_t dimension) {
    float dist = (float)distance;
    float maxd = (float)dimension;
    return 1.0f - (dist / maxd);
}

// Sequential f32 sums, Rust iterator semantics (`zip` truncates).
static float dot_seq(const float* a, const float* b, uint64_t len) {
    float s = -0.0f;
    for (uint64_t i = 0; i < len; ++i) {
        float p = a[i] * b[i];
        s = s + p;
    }
    return s;
}
static float sumsq_seq(const float* a, uint64_t len) {
    float s = -0.0f;
    for (uint64_t i = 0; i < len; ++i) {
        float p = a[i] * a[i];
        s = s + p;
    }
    return s;
}

// BinaryQuantizer::cosine_similarity_manual (quantization.rs:206-216) —
// also storage.rs:851-865 minus its length check.  0.0 if a norm is 0.
float orc_cosine_manual(const float* a, uint64_t la, const float* b, uint64_t lb) {
    float dot = dot_seq(a, b, std::min(la, lb));
    float na = std::sqrt(sumsq_seq(a, la));
    float nb = std::sqrt(sumsq_seq(b, lb));
    if (na == 0.0f || nb == 0.0f) return 0.0f;
    return dot / (na * nb);
}

// storage.rs:851-865 `cosine_similarity`: 0.0 on length mismatch.
float orc_storage_cosine(const float* a, uint64_t la, const float* b, uint64_t lb) {
    if (la != lb) return 0.0f;
    return orc_cosine_manual(a, la, b, lb);
}

// index.rs:686-700 `cosine_distance`: +inf on length mismatch or zero norm.
float orc_cosine_distance(const float* a, uint64_t la, const float* b, uint64_t lb) {
    if (la != lb) return std::numeric_limits<float>::infinity();
    float dot = dot_seq(a, b, la);
    float na = std::sqrt(sumsq_seq(a, la));
    float nb = std::sqrt(sumsq_seq(b, lb));
    if (na == 0.0f || nb == 0.0f) return std::numeric_limits<float>::infinity();
    return 1.0f - (dot / (na * nb));
}

// index.rs:69-78 `VectorPoint::distance`: sqrt(sum((x-y).powi(2))), with
// powi(2) lowered to x*x; zip truncation.
float orc_l2_distance(const float* a, uint64_t la, const float* b, uint64_t lb) {
    uint64_t len = std::min(la, lb);
    float s = -0.0f;
    for (uint64_t i = 0; i < len; ++i) {
        float d = a[i] - b[i];
        float p = d * d;
        s = s + p;
    }
    return std::sqrt(s);
}

// ---------------------------------------------------------------------------
// BinaryQuantizer::multi_stage_search (quantization.rs:151-193).
//
//   q_bits        : ceil(qdim/8) Msb0 bytes of the binary query
//   c_bits        : N rows of ceil(cdim/8) Msb0 bytes (BinaryVector data)
//   q, qlen       : original f32 query
//   cands         : N rows of clen f32 (original candidates)
//   rescore_ratio : BinaryQuantizationConfig.rescore_ratio (default 0.1)
// Outputs (capacity >= min(R, N)): (idx, cosine) sorted like the reference.
// Optional stage-1 outputs (capacity N) receive the full stable-sorted
// binary list (idx, similarity) when non-null.
//
// Semantics restated:
//  * stage 1: similarity(query, cand).unwrap_or(0.0): a dimension mismatch
//    scores 0.0 (quantization.rs:168).  Stable sort by score descending (175).
//    A NaN score (dimension 0) makes partial_cmp().unwrap() panic when the
//    sort compares it: reported as ORC_ERR_QUANTIZATION.
//  * R = (N as f32 * ratio) as usize, then min(R, N) (178-179).
//  * stage 2: cosine_similarity_manual(original_query, cand[idx]) (181-187),
//    stable sort by cosine descending (190), NaN -> panic -> error.
//  * output length is min(R, N): NOT truncated to any k.
// ---------------------------------------------------------------------------
static int multi_stage_one(const uint8_t* q_bits, uint32_t qdim, const uint8_t* c_bits, uint32_t cdim,
                           uint64_t N, const float* q, uint64_t qlen, const float* cands, uint64_t clen,
                           float rescore_ratio, uint64_t* out_idx, float* out_score, uint64_t* out_n,
                           uint64_t* s1_idx, float* s1_score) {
    const uint64_t nbytes = (cdim + 7u) / 8u;
    std::vector<std::pair<uint64_t, float>> s1(N);
    for (uint64_t i = 0; i < N; ++i) {
        float score;
        if (qdim != cdim) {
            score = 0.0f;  // hamming_distance Err(InvalidVectorDimension) -> unwrap_or(0.0)
        } else {
            uint64_t d = orc_hamming(q_bits, c_bits + i * nbytes, nbytes);
            score = orc_similarity(d, cdim);
        }
        s1[i] = {i, score};
    }
    if (N >= 2) {
        for (uint64_t i = 0; i < N; ++i)
            if (s1[i].second != s1[i].second) return ORC_ERR_QUANTIZATION;
    }
    std::stable_sort(s1.begin(), s1.end(),
                     [](const std::pair<uint64_t, float>& a, const std::pair<uint64_t, float>& b) {
                         return a.second > b.second;
                     });
    if (s1_idx) {
        for (uint64_t i = 0; i < N; ++i) {
            s1_idx[i] = s1[i].first;
            if (s1_score) s1_score[i] = s1[i].second;
        }
    }
    uint64_t R = rust_f32_as_usize((float)N * rescore_ratio);
    R = std::min(R, N);
    std::vector<std::pair<uint64_t, float>> s2(R);
    for (uint64_t r = 0; r < R; ++r) {
        uint64_t idx = s1[r].first;
        s2[r] = {idx, orc_cosine_manual(q, qlen, cands + idx * clen, clen)};
    }
    if (R >= 2) {
        for (uint64_t r = 0; r < R; ++r)
            if (s2[r].second != s2[r].second) return ORC_ERR_QUANTIZATION;
    }
    std::stable_sort(s2.begin(), s2.end(),
                     [](const std::pair<uint64_t, float>& a, const std::pair<uint64_t, float>& b) {
                         return a.second > b.second;
                     });
    for (uint64_t r = 0; r < R; ++r) {
        out_idx[r] = s2[r].first;
        out_score[r] = s2[r].second;
    }
    *out_n = R;
    return ORC_OK;
}

int orc_multi_stage_search(const uint8_t* q_bits, uint32_t qdim, const uint8_t* c_bits, uint32_t cdim,
                           uint64_t N, const float* q, uint64_t qlen, const float* cands, uint64_t clen,
                           float rescore_ratio, uint64_t* out_idx, float* out_score, uint64_t* out_n,
                           uint64_t* s1_idx, float* s1_score) {
    return multi_stage_one(q_bits, qdim, c_bits, cdim, N, q, qlen, cands, clen, rescore_ratio, out_idx,
                           out_score, out_n, s1_idx, s1_score);
}

// Batched form used as the CPU baseline: B independent queries, one per
// thread (mirrors rayon over queries in parallel_search.rs:130-134 and the
// concurrent RwLock readers of lib.rs:470).  Per-query output stride = R_cap.
int orc_multi_stage_search_batch(const uint8_t* q_bits, uint32_t dim, const uint8_t* c_bits, uint64_t N,
                                 const float* q, const float* cands, uint64_t B, float rescore_ratio,
                                 uint64_t R_cap, uint64_t* out_idx, float* out_score, uint64_t* out_n,
                                 int threads) {
    const uint64_t nbytes = (dim + 7u) / 8u;
    int status = ORC_OK;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int64_t b = 0; b < (int64_t)B; ++b) {
        uint64_t R = std::min(rust_f32_as_usize((float)N * rescore_ratio), N);
        if (R > R_cap) {
            status = ORC_ERR_INVALID_ARGUMENT;
            continue;
        }
        int st = multi_stage_one(q_bits + b * nbytes, dim, c_bits, dim, N, q + b * dim, dim, cands, dim,
                                 rescore_ratio, out_idx + b * R_cap, out_score + b * R_cap, out_n + b, nullptr,
                                 nullptr);
        if (st != ORC_OK) status = st;
    }
    return status;
}

// Batched multi-stage search with an explicit rescore depth R (instead of
// the ratio): stage 1 exact top-R (d asc, idx asc), stage 2 cosine (or L2 /
// cosine distance: kind 0/1/2) stable-sorted (descending for cosine).
void orc_multi_stage_search_batch_r(const uint8_t* q_bits, uint32_t dim, const uint8_t* c_bits, uint64_t N,
                                    const float* q, const float* cands, uint64_t B, uint64_t R, int kind,
                                    uint64_t* out_idx, float* out_score, int threads) {
    const uint64_t nbytes = (dim + 7u) / 8u;
    const uint64_t r = std::min(R, N);
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int64_t b = 0; b < (int64_t)B; ++b) {
        std::vector<std::pair<uint32_t, uint64_t>> v(N);
        for (uint64_t i = 0; i < N; ++i)
            v[i] = {(uint32_t)orc_hamming(q_bits + b * nbytes, c_bits + i * nbytes, nbytes), i};
        std::partial_sort(v.begin(), v.begin() + r, v.end());
        std::vector<std::pair<uint64_t, float>> s2(r);
        for (uint64_t i = 0; i < r; ++i) {
            const float* x = cands + v[i].second * dim;
            const float* qq = q + b * dim;
            float s = kind == 0   ? orc_cosine_manual(qq, dim, x, dim)
                      : kind == 1 ? orc_l2_distance(qq, dim, x, dim)
                                  : orc_cosine_distance(qq, dim, x, dim);
            s2[i] = {v[i].second, s};
        }
        if (kind == 0)
            std::stable_sort(s2.begin(), s2.end(), [](const std::pair<uint64_t, float>& a,
                                                      const std::pair<uint64_t, float>& c) { return a.second > c.second; });
        else
            std::stable_sort(s2.begin(), s2.end(), [](const std::pair<uint64_t, float>& a,
                                                      const std::pair<uint64_t, float>& c) { return a.second < c.second; });
        for (uint64_t i = 0; i < r; ++i) {
            out_idx[b * R + i] = s2[i].first;
            out_score[b * R + i] = s2[i].second;
        }
    }
}

// Stage-1 only, batched: exact top-R (idx ascending on ties) by Hamming
// distance — the (idx, distance) list the GPU stage-1 must reproduce.
void orc_bq_topr_batch(const uint8_t* q_bits, const uint8_t* c_bits, uint64_t N, uint32_t dim, uint64_t B,
                       uint64_t R, uint64_t* out_idx, uint32_t* out_dist, int threads) {
    const uint64_t nbytes = (dim + 7u) / 8u;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int64_t b = 0; b < (int64_t)B; ++b) {
        std::vector<std::pair<uint32_t, uint64_t>> v(N);
        for (uint64_t i = 0; i < N; ++i)
            v[i] = {(uint32_t)orc_hamming(q_bits + b * nbytes, c_bits + i * nbytes, nbytes), i};
        uint64_t r = std::min(R, N);
        std::partial_sort(v.begin(), v.begin() + r, v.end());  // (d asc, idx asc) == stable desc by similarity
        for (uint64_t i = 0; i < r; ++i) {
            out_idx[b * R + i] = v[i].second;
            out_dist[b * R + i] = v[i].first;
        }
    }
}

// ---------------------------------------------------------------------------
// BasicVectorStore::vector_search (storage.rs:296-339): every record in
// iteration order, similarity = cosine_similarity (851-865), drop if
// similarity < threshold (313-317), stable sort descending with NaN ==
// Equal (331-335), truncate(limit) (336).  Record order = row order here.
// ---------------------------------------------------------------------------
void orc_storage_vector_search(const float* q, uint64_t qlen, const float* rows, uint64_t N, uint64_t D,
                               uint64_t limit, int has_threshold, float threshold, uint64_t* out_idx,
                               float* out_score, uint64_t* out_n) {
    std::vector<std::pair<uint64_t, float>> res;
    res.reserve(N);
    for (uint64_t i = 0; i < N; ++i) {
        float s = orc_storage_cosine(q, qlen, rows + i * D, D);
        if (has_threshold && s < threshold) continue;
        res.push_back({i, s});
    }
    std::stable_sort(res.begin(), res.end(),
                     [](const std::pair<uint64_t, float>& a, const std::pair<uint64_t, float>& b) {
                         return a.second > b.second;
                     });
    uint64_t n = std::min<uint64_t>(limit, res.size());
    for (uint64_t i = 0; i < n; ++i) {
        out_idx[i] = res[i].first;
        out_score[i] = res[i].second;
    }
    *out_n = n;
}

// FaissVectorIndex::search, Flat (index.rs:620-640): cosine_distance over
// every live row, stable sort ASCENDING (NaN == Equal), truncate(k).
void orc_flat_cosine_distance_search(const float* q, uint64_t qlen, const float* rows, uint64_t N, uint64_t D,
                                     uint64_t k, uint64_t* out_idx, float* out_score, uint64_t* out_n) {
    std::vector<std::pair<uint64_t, float>> res(N);
    for (uint64_t i = 0; i < N; ++i) res[i] = {i, orc_cosine_distance(q, qlen, rows + i * D, D)};
    std::stable_sort(res.begin(), res.end(),
                     [](const std::pair<uint64_t, float>& a, const std::pair<uint64_t, float>& b) {
                         return a.second < b.second;
                     });
    uint64_t n = std::min<uint64_t>(k, N);
    for (uint64_t i = 0; i < n; ++i) {
        out_idx[i] = res[i].first;
        out_score[i] = res[i].second;
    }
    *out_n = n;
}

// Exact top-k by cosine similarity, batched (ground truth for recall@k):
// same ordering as orc_storage_vector_search without a threshold.
void orc_exact_topk_cosine_batch(const float* q, const float* rows, uint64_t N, uint64_t D, uint64_t B,
                                 uint64_t k, uint64_t* out_idx, float* out_score, int threads) {
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int64_t b = 0; b < (int64_t)B; ++b) {
        uint64_t n;
        std::vector<uint64_t> idx(k);
        std::vector<float> sc(k);
        orc_storage_vector_search(q + b * D, D, rows, N, D, k, 0, 0.0f, idx.data(), sc.data(), &n);
        for (uint64_t i = 0; i < n; ++i) {
            out_idx[b * k + i] = idx[i];
            out_score[b * k + i] = sc[i];
        }
    }
}

// B independent FaissVectorIndex::search calls (index.rs:620-640), one query
// per thread: the checker for batched GPU flat searches with metric 2.
void orc_flat_cosine_distance_batch(const float* q, const float* rows, uint64_t N, uint64_t D, uint64_t B,
                                    uint64_t k, uint64_t* out_idx, float* out_score, uint64_t* out_n, int threads) {
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int64_t b = 0; b < (int64_t)B; ++b)
        orc_flat_cosine_distance_search(q + b * D, D, rows, N, D, k, out_idx + b * k, out_score + b * k, out_n + b);
}

// The "ref-faithful" cost of HnswVectorIndex::search's id remap (index.rs:219-228,
// BASELINE.md §2): for each of the k hits, the reference walks id_to_index
// (HashMap<String, usize>) and format!s "vec_{index}" for every entry until it
// equals the hit's value -- O(N k) string formatting per query.  Restated with a
// heap-allocated string per format! (a Rust String always allocates); the map holds
// N ids "doc_{i}" -> i, hits are k rows drawn per query.  Returns the mean wall
// seconds of the remap per query (nq queries, one per thread).
double orc_ref_id_remap_seconds(uint64_t N, uint64_t k, uint64_t nq, int threads) {
    std::unordered_map<std::string, uint64_t> id_to_index;
    id_to_index.reserve(N);
    for (uint64_t i = 0; i < N; ++i) id_to_index.emplace("doc_" + std::to_string(i), i);
    std::vector<double> secs(nq, 0.0);
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int64_t qi = 0; qi < (int64_t)nq; ++qi) {
        uint64_t st = 0x6772617065ull + (uint64_t)qi * 0x9e3779b97f4a7c15ull;
        std::vector<std::string> hits;
        for (uint64_t j = 0; j < k; ++j) {
            st = st * 6364136223846793005ull + 1442695040888963407ull;
            hits.push_back("vec_" + std::to_string((st >> 17) % N));
        }
        const auto t0 = std::chrono::steady_clock::now();
        std::vector<std::string> found;
        for (const std::string& value : hits) {
            for (const auto& e : id_to_index) {
                std::string f;
                f.reserve(32);  // past the SSO buffer: one heap allocation, as format! makes
                f += "vec_";
                f += std::to_string(e.second);
                if (f == value) {
                    found.push_back(e.first);
                    break;
                }
            }
        }
        secs[qi] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (found.size() != k) secs[qi] = -1.0;
    }
    double sum = 0.0;
    for (double v : secs) {
        if (v < 0) return -1.0;
        sum += v;
    }
    return nq ? sum / (double)nq : 0.0;
}

// ShardManager::search_vectors merge (distributed/shard.rs:776-784): concat
// the per-shard lists in shard order, stable sort by score DESCENDING
// (NaN == Equal), truncate(limit).
void orc_shard_merge(const uint64_t* ids, const float* scores, const uint64_t* counts, uint64_t n_shards,
                     uint64_t stride, uint64_t limit, uint64_t* out_ids, float* out_scores, uint64_t* out_n) {
    std::vector<std::pair<uint64_t, float>> all;
    for (uint64_t s = 0; s < n_shards; ++s)
        for (uint64_t i = 0; i < counts[s]; ++i) all.push_back({ids[s * stride + i], scores[s * stride + i]});
    std::stable_sort(all.begin(), all.end(),
                     [](const std::pair<uint64_t, float>& a, const std::pair<uint64_t, float>& b) {
                         return a.second > b.second;
                     });
    uint64_t n = std::min<uint64_t>(limit, all.size());
    for (uint64_t i = 0; i < n; ++i) {
        out_ids[i] = all[i].first;
        out_scores[i] = all[i].second;
    }
    *out_n = n;
}

// Host form of the exact sharded merge (gvdb_bq_shard_merge): per query the
// union of shard lists sorted by (distance asc, gid asc), first R, then stable
// by cosine descending, first k.  Layout [(g*B + q)*stride + i].
void orc_bq_shard_merge(const uint64_t* gids, const uint32_t* dist, const float* cosv, const uint64_t* counts,
                        uint64_t G, uint64_t B, uint64_t stride, uint64_t R, uint64_t k, uint64_t* out_ids,
                        float* out_scores, uint64_t* out_n) {
    struct E {
        uint32_t d;
        uint64_t gid;
        float c;
    };
    for (uint64_t q = 0; q < B; ++q) {
        std::vector<E> all;
        for (uint64_t g = 0; g < G; ++g)
            for (uint64_t i = 0; i < std::min(counts[g * B + q], stride); ++i) {
                const uint64_t at = (g * B + q) * stride + i;
                all.push_back({dist[at], gids[at], cosv[at]});
            }
        std::stable_sort(all.begin(), all.end(),
                         [](const E& a, const E& b) { return a.d != b.d ? a.d < b.d : a.gid < b.gid; });
        if (all.size() > R) all.resize(R);
        std::stable_sort(all.begin(), all.end(), [](const E& a, const E& b) { return a.c > b.c; });
        const uint64_t take = std::min<uint64_t>(k, all.size());
        for (uint64_t i = 0; i < take; ++i) {
            out_ids[q * k + i] = all[i].gid;
            out_scores[q * k + i] = all[i].c;
        }
        out_n[q] = take;
    }
}

// Row norms with the reference's sequential order (used by tests to check
// the device norm precompute bit for bit).
void orc_row_norms(const float* rows, uint64_t N, uint64_t D, float* out) {
    for (uint64_t i = 0; i < N; ++i) out[i] = std::sqrt(sumsq_seq(rows + i * D, D));
}

}  // extern "C"
