// gvdb_capi.hip — the C ABI (include/gvdb.h) over the gfx950 kernels.
//
// Owns: the index object (HBM-resident rows / codes / norms / ids for one
// shard), the per-call workspace pool (reentrant searches), the BQ search
// orchestration (stage 1 fast path + exact slow path, stage 2, final sort)
// and the error contract (thread-local last error, VectorDbError codes).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/gvdb.h"
#include "gvdb_internal.h"

using namespace gvdb;

// ============================================================================
// errors
// ============================================================================
namespace {
thread_local std::string t_err = "";
thread_local uint64_t t_dim_expected = 0, t_dim_actual = 0;

gvdb_status fail(gvdb_status s, const std::string& msg) {
    t_err = msg;
    return s;
}
gvdb_status dev_fail(hipError_t e, const char* where) {
    if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation)
        return fail(GVDB_ERR_OUT_OF_MEMORY, std::string(where) + ": " + hipGetErrorString(e));
    return fail(GVDB_ERR_DEVICE, std::string(where) + ": " + hipGetErrorString(e));
}
gvdb_status dim_mismatch(uint64_t expected, uint64_t actual) {
    t_dim_expected = expected;
    t_dim_actual = actual;
    char b[128];
    snprintf(b, sizeof b, "Dimension mismatch: expected %llu, actual %llu", (unsigned long long)expected,
             (unsigned long long)actual);
    return fail(GVDB_ERR_DIMENSION_MISMATCH, b);
}

#define HIP_TRY(expr, where)                          \
    do {                                              \
        hipError_t e_ = (expr);                       \
        if (e_ != hipSuccess) return dev_fail(e_, where); \
    } while (0)

// GVDB_DEBUG_SYNC=1: synchronize and check after each launch of the flat
// MFMA path (fault attribution while developing; off in production)
#define DBG_SYNC(s, where)                                                     \
    do {                                                                       \
        static const bool on_ = getenv("GVDB_DEBUG_SYNC") != nullptr;          \
        if (on_) HIP_TRY(hipStreamSynchronize(s), where);                      \
    } while (0)

// Rust `f32 as usize` (saturating; NaN -> 0).
uint64_t rust_f32_as_usize(float v) {
    if (!(v == v) || v <= 0.0f) return 0;
    if (v >= 18446744073709551615.0f) return UINT64_MAX;
    return (uint64_t)v;
}

// ============================================================================
// Kernel timing (HIP events around the launches, read after the batch's
// stream sync; enabled by gvdb_timing_enable, used by bench.py)
// ============================================================================
bool getenv_flag(const char* name) {
    const char* v = getenv(name);
    return v && *v && strcmp(v, "0") != 0;
}
// flat searches whose bf16-MFMA candidate pass could not be certified (exact rescan)
std::atomic<uint64_t>& flat_fallbacks() {
    static std::atomic<uint64_t> n{0};
    return n;
}
// flat searches whose i8-MFMA candidate pass could not be certified (bf16 retry)
std::atomic<uint64_t>& flat_fallbacks_i8() {
    static std::atomic<uint64_t> n{0};
    return n;
}
// certified default-depth searches: [0] certified batches, [1] batches sent to bq_search
std::atomic<uint64_t>& deep_cert_count(int which) {
    static std::atomic<uint64_t> c[2];
    return c[which & 1];
}

enum { kTimSampleHist = 0, kTimScan = 1, kTimSelect = 2, kTimRerank = 3, kTimFinal = 4, kTimFlatEmit = 5, kTimFlat = 6,
       kTimFlatEmitI8 = 7, kTimFlatI8 = 8, kTimN = 9 };
struct EvSet;
struct Timing {
    std::mutex mu;
    bool on = false;
    double ms[kTimN] = {0};
    uint64_t n[kTimN] = {0};
    std::vector<EvSet*> pending, free_sets;  // BQ search events awaiting collection / reusable
};
Timing& timing() {
    static Timing t;
    return t;
}
struct EvSet {
    hipEvent_t e[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    bool ok = false;
    void create() {
        ok = true;
        for (auto& x : e)
            if (hipEventCreate(&x) != hipSuccess) ok = false;
    }
    ~EvSet() {
        for (auto& x : e)
            if (x) (void)hipEventDestroy(x);
    }
};

// ============================================================================
// device buffers
// ============================================================================
struct DBuf {
    void* p = nullptr;
    size_t n = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= n) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        size_t want = bytes + bytes / 4 + 256;
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) n = want;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    template <class T>
    T* as() const {
        return (T*)p;
    }
};

struct Workspace {
    int device = 0;
    hipStream_t stream = nullptr;
    DBuf q, qnorm, qcodes, zero, thr, buf, s1_rows, s1_dist, scores, out_ids, out_scores, out_n, slow, sort_tmp, flags,
        rows, norms, codes, misc, fx_qb, fx_smp, fx_cand, fx_scores, fx_probe, flt_rows, flt_ids, flt_codes, s1_mx,
        deep, seg;
    uint32_t* h_flags = nullptr;  // pinned [4]: any_fail / nan
    EvSet ev;                     // timing events (created on first timed call)
    // Searches return without a host sync: the workspace goes back to the pool
    // while its kernels may still run on the caller's stream.  `done` marks the
    // end of that work; the next user on another stream waits for it on the
    // device (hipStreamWaitEvent), never on the host.
    hipEvent_t done = nullptr;
    hipStream_t last = nullptr;
    bool pending = false;
    // batch-1 fast path state (self-cleaning: zero between calls); b1_sig
    // = the layout it was zeroed for, 0 = must be zeroed
    DBuf b1;
    uint64_t b1_sig = 0;
    ~Workspace() {
        if (done) (void)hipEventDestroy(done);
        for (DBuf* b : {&q, &qnorm, &qcodes, &zero, &thr, &buf, &s1_rows, &s1_dist, &scores, &out_ids, &out_scores,
                        &out_n, &slow, &sort_tmp, &flags, &rows, &norms, &codes, &misc, &fx_qb, &fx_smp, &fx_probe, &fx_cand,
                        &fx_scores, &flt_rows, &flt_ids, &flt_codes, &s1_mx, &deep, &seg, &b1})
            b->release();
        if (h_flags) (void)hipHostFree(h_flags);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

struct WsPool {
    std::mutex mu;
    std::vector<std::unique_ptr<Workspace>> free;
    Workspace* acquire(int device) {
        {
            // LIFO: a call that nests a second workspace (deep_cert_search's flat pass)
            // releases the inner one first, so the next call gets the same pair in the
            // same roles (their buffers stay sized for one role each)
            std::lock_guard<std::mutex> g(mu);
            for (size_t i = free.size(); i-- > 0;) {
                if (free[i]->device == device) {
                    Workspace* w = free[i].release();
                    free.erase(free.begin() + i);
                    return w;
                }
            }
        }
        auto* w = new Workspace();
        w->device = device;
        if (hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking) != hipSuccess ||
            hipHostMalloc((void**)&w->h_flags, 16, hipHostMallocDefault) != hipSuccess) {
            delete w;
            return nullptr;
        }
        return w;
    }
    void release(Workspace* w) {
        std::lock_guard<std::mutex> g(mu);
        free.emplace_back(w);
    }
};

WsPool& global_pool() {
    static WsPool p;
    return p;
}

struct WsGuard {
    Workspace* w;
    hipStream_t s = nullptr;
    bool begun = false;
    explicit WsGuard(int dev) : w(global_pool().acquire(dev)) {}
    // order this call's work on stream st after the workspace's previous user
    void begin(hipStream_t st) {
        s = st;
        begun = true;
        if (w->pending && w->last != st) (void)hipStreamWaitEvent(st, w->done, 0);
    }
    ~WsGuard() {
        if (!w) return;
        if (begun) {
            if (!w->done) (void)hipEventCreateWithFlags(&w->done, hipEventDisableTiming);
            w->pending = w->done && hipEventRecord(w->done, s) == hipSuccess;
            w->last = s;
        }
        global_pool().release(w);
    }
};

// ============================================================================
// BQ search on one shard view (stage 1 + stage 2 + final ordering)
// ============================================================================
struct ShardView {
    const float* rows;      // [N][clen]
    uint64_t clen;
    const float* norms;     // [N]
    const uint4* codes;     // [W4][cap]
    uint64_t cap;
    uint32_t N;
    uint32_t D;             // candidate dimension (bits)
    const uint64_t* ids;    // row -> id or nullptr
    uint64_t row_offset;
};

constexpr uint32_t kExactN = 262144;  // below this the "sample" is the whole shard
constexpr uint64_t kFlatScoreBytes = 1ull << 30;  // dense score block cap of the exact flat scan
// ... and of its device-gated form (the _device FLAT search's last tier, enqueued behind every
// batch and skipped on the device when the candidate tier certified): a skipped launch still
// costs its dispatch (~7 us with the gap), so fewer, larger query groups -- 4 GiB: 107 queries
// per group at 10M rows, 8 launches per batch of 256 instead of 22 (round 6)
constexpr uint64_t kFlatScoreBytesGated = 4ull << 30;

// Stage-1 sampling plan: S rows in 4096-row chunks spread over the shard.
// sample_div: the sample is ~N/sample_div rows (32; 64 for large batches,
// where the VALU sample pass would otherwise cost ~10% of the MFMA scan).
void plan_sampling(uint32_t N, uint32_t R, uint32_t sample_div, uint32_t& chunks, uint32_t& stride, uint32_t& target,
                   uint32_t& bufcap) {
    if (N <= kExactN) {
        chunks = (N + 4095u) / 4096u;
        stride = 4096u;
        target = R;  // exact threshold: count(d <= T) >= R guaranteed
        bufcap = std::min<uint64_t>(N, 8ull * R + 2048ull);
        return;
    }
    // GVDB_SAMPLE_FLOOR: minimum sample rows (timing experiments).  Default kExactN / 4
    // (64K): at the 8-GPU shard (1.25M rows) the fastest in round 3 (per-rank step
    // 0.300 -> 0.282 ms).  For R <= 1000, kExactN / 8: with round 5's fused FP4 sample
    // pass and cheaper emits 32K is faster (config-3 per rank 0.1525 -> 0.1491 ms mean,
    // 1M x 768 batch 256 0.161 -> 0.158 ms; twice each on one box,
    // profiles/r05/c3/c3floor_r05.log).  Deeper R keeps 64K: its target-th sampled
    // distance sits in a sparser histogram at 32K, so the dense form's 16-row group
    // minima loosen the threshold more often (test_sample_histogram_mfma_thresholds_equal_valu)
    static const uint64_t floor_env = [] {
        const char* e = getenv("GVDB_SAMPLE_FLOOR");
        const long long v = e ? atoll(e) : 0;
        return v >= 4096 ? (uint64_t)v : 0ull;
    }();
    const uint64_t floor_rows = floor_env ? floor_env : (uint64_t)(R <= 1000u ? kExactN / 8 : kExactN / 4);
    uint64_t S = std::max<uint64_t>(floor_rows, N / sample_div);
    chunks = (uint32_t)(S / 4096u);
    stride = N / chunks;  // >= 4096: chunks never overlap
    S = (uint64_t)chunks * 4096u;
    const double m = (double)R * (double)S / (double)N;  // expected sample hits of the top-R set
    target = (uint32_t)std::ceil(m + 4.0 * std::sqrt(m) + 4.0);
    const double expect_full = (double)target * (double)N / (double)S;
    bufcap = (uint32_t)std::min<double>((double)N, 8.0 * expect_full + 2048.0);
}

// Stage-1 workspace: ONE memset zeroes flags | counts | fail | hist, which
// sit contiguously in ws.zero (flags[0] = any stage-1 failure, flags[1] = NaN).
// fast: launch_stage1_fast will run (its first kernel may zero the state)
gvdb_status prepare_stage1(Workspace& ws, Stage1Args& s1, uint32_t B, uint32_t D, uint32_t R, uint32_t N,
                           hipStream_t s, bool fast, bool lists = true) {
    // GVDB_SCAN=valu forces the popcount scan for every batch size; default:
    // FP4 MFMA for large batches.  (The round-1/2 A/B scans -- i8 MFMA, uniform
    // FP4 waves, LDS-shared tiles, mx3 -- were removed from the tree after
    // commit 8c12da2; DESIGN.md §4 keeps their measurements.)
    const char* scan = getenv("GVDB_SCAN");
    s1.use_mfma = (scan && strcmp(scan, "valu") == 0) ? 0 : 1;
    s1.force_rescan = getenv_flag("GVDB_FORCE_RESCAN") ? 1 : 0;  // tests of the device-side fallback
    // GVDB_SAMPLE_DIV: sample ~N/div rows for large batches (timing experiments; default 64)
    static const uint32_t big_div = [] {
        const char* e = getenv("GVDB_SAMPLE_DIV");
        const int v = e ? atoi(e) : 0;
        return v >= 8 && v <= 4096 ? (uint32_t)v : 64u;
    }();
    plan_sampling(N, R, (s1.use_mfma && B >= kMfmaMinB) ? big_div : 32u, s1.sample_chunks, s1.sample_stride,
                  s1.target, s1.bufcap);
    if (R > kSelectLdsCap) {
        // k_select_big: R candidates or more per query -- twice the expected
        // emission (one Hamming bin of ties can add a few % of N), not 8x
        const uint64_t S = (uint64_t)s1.sample_chunks * 4096u;
        const double expect = N <= kExactN ? (double)N : (double)s1.target * (double)N / (double)S;
        s1.bufcap = (uint32_t)std::min<double>((double)N, 2.0 * expect + 4096.0);
        s1.big_select = 1;
    }
    s1.B = B;
    s1.D = D;
    s1.N = N;
    s1.R = R;
    const size_t extra = stage1_plan(s1);
    const size_t nb = (size_t)D + 1u;
    // the dense sample needs no histogram: only flags | counts | fail are zeroed
    const size_t words =
        4 + 2 * (size_t)B + (s1.sample_mode == kSampleDense || s1.sample_mode == kSampleWide ? 0 : (size_t)B * nb);
    HIP_TRY(ws.zero.ensure(words * 4 + 16), "alloc stage-1 state");
    if (extra) {
        HIP_TRY(ws.s1_mx.ensure(extra), "alloc stage-1 MFMA operands");
        char* p = ws.s1_mx.as<char>();
        if (s1.mfma_scan) {
            const size_t ng = (B + 255u) / 256u;
            s1.qfrag = (uint4*)p;
            p += ng * 8u * 2u * code_w4(D) * 64u * 16u;
            s1.qpc = (uint32_t*)p;
            p += ng * 256u * 4u;
        }
        if (s1.sample_mode == kSampleDense || s1.sample_mode == kSampleWide)
            s1.smp = (uint16_t*)(((uintptr_t)p + 255) & ~(uintptr_t)255);
        if (s1.dense_sel && !s1.dense_keep) s1.dense = (uint16_t*)(((uintptr_t)p + 255) & ~(uintptr_t)255);
    }
    HIP_TRY(ws.thr.ensure((size_t)B * 4), "alloc thr");
    if (s1.dense_sel) s1.bufcap = 1;  // no candidate buffer: every distance goes to the dense block
    HIP_TRY(ws.buf.ensure((size_t)B * s1.bufcap * 8), "alloc candidate buffer");
    if (lists) {  // else the caller points s1_rows / s1_dist at its own buffers
        HIP_TRY(ws.s1_rows.ensure((size_t)B * R * 4), "alloc s1_rows");
        HIP_TRY(ws.s1_dist.ensure((size_t)B * R * 4), "alloc s1_dist");
    }
    uint32_t* z = ws.zero.as<uint32_t>();
    if (fast && s1.mfma_scan && s1.sample_mode == kSampleDense) {  // k_qfrag, the first stage-1 kernel, zeroes them
        s1.zero = z;
        s1.nzero = (uint32_t)words;
    } else {
        HIP_TRY(hipMemsetAsync(ws.zero.p, 0, ((words * 4 + 15) / 16) * 16, s), "memset stage-1 state");
    }
    s1.any_fail = z;
    s1.counts = z + 4;
    s1.fail = z + 4 + B;
    s1.hist = z + 4 + 2 * (size_t)B;
    s1.thr = ws.thr.as<uint32_t>();
    s1.buf = ws.buf.as<uint64_t>();
    s1.s1_rows = lists ? ws.s1_rows.as<uint32_t>() : nullptr;
    s1.s1_dist = lists ? ws.s1_dist.as<uint32_t>() : nullptr;
    return GVDB_OK;
}

struct BqSearchArgs {
    ShardView v;
    const float* d_q;       // [B][qlen]
    uint64_t qlen;
    uint32_t B;
    const uint32_t* d_qwords;  // optional pre-packed query codes [B][4*W4] (else packed from d_q)
    float thr;              // packing threshold
    bool dims_match;        // binary query dim == candidate dim
    uint32_t R;
    uint32_t kout;
    int kind;
    int descending;
    uint64_t* d_out_ids;
    float* d_out_scores;
    uint32_t* d_out_n;
    uint32_t* d_out_dist;   // candidates mode: stage-1 order, no final sort
    uint64_t out_stride;    // candidates mode: output row stride (0 = R)
    const uint32_t* row_map;  // filtered search: v's codes are the compacted allowed rows; subset row -> index row
    const uint32_t* gate;     // device-side fallback (deep_cert_search): runs iff *gate != 0 (large-R dense path)
};

// Stage-1 + stage-2 timing without a host round trip: events are recorded
// on the search stream and their elapsed times are collected lazily (at
// gvdb_timing_read / reset, or when too many are pending).
EvSet* timing_events() {
    std::lock_guard<std::mutex> g(timing().mu);
    auto& fr = timing().free_sets;
    if (!fr.empty()) {
        EvSet* e = fr.back();
        fr.pop_back();
        return e;
    }
    auto* e = new EvSet();
    e->create();
    if (!e->ok) {
        delete e;
        return nullptr;
    }
    return e;
}
void timing_drain_locked(size_t n) {
    auto& pend = timing().pending;
    n = std::min(n, pend.size());
    for (size_t i = 0; i < n; ++i) {
        EvSet* e = pend[i];
        if (hipEventSynchronize(e->e[5]) == hipSuccess) {
            float t[4] = {0, 0, 0, 0};
            (void)hipEventElapsedTime(&t[0], e->e[0], e->e[1]);
            (void)hipEventElapsedTime(&t[1], e->e[1], e->e[2]);
            (void)hipEventElapsedTime(&t[2], e->e[2], e->e[3]);
            (void)hipEventElapsedTime(&t[3], e->e[3], e->e[5]);
            for (int k = 0; k < 4; ++k) {
                timing().ms[k] += t[k];
                timing().n[k] += 1;
            }
        }
        timing().free_sets.push_back(e);
    }
    pend.erase(pend.begin(), pend.begin() + n);
}
void timing_submit(EvSet* e) {
    std::lock_guard<std::mutex> g(timing().mu);
    timing().pending.push_back(e);
    if (timing().pending.size() > 512) timing_drain_locked(256);
}

// tests: the stage-1 thresholds of the last batch searched with GVDB_DEBUG_THR=1
uint32_t*& debug_thr() {
    static uint32_t* p = nullptr;
    return p;
}
uint32_t& debug_thr_cap() {
    static uint32_t n = 0;
    return n;
}
// ... and whether any query of that batch took the device-side all-rows rescan
uint32_t*& debug_fail() {
    static uint32_t* p = nullptr;
    return p;
}
static hipError_t debug_keep_thr(const uint32_t* thr, uint32_t B, hipStream_t s, const uint32_t* any_fail = nullptr) {
    if (!getenv_flag("GVDB_DEBUG_THR")) return hipSuccess;
    if (any_fail) {
        if (!debug_fail()) {
            hipError_t e = hipMalloc((void**)&debug_fail(), 4);
            if (e != hipSuccess) return e;
        }
        hipError_t e = hipMemcpyAsync(debug_fail(), any_fail, 4, hipMemcpyDeviceToDevice, s);
        if (e != hipSuccess) return e;
    }
    uint32_t*& dt = debug_thr();
    if (debug_thr_cap() < B) {
        if (dt) (void)hipFree(dt);
        hipError_t e = hipMalloc((void**)&dt, (size_t)B * 4);
        if (e != hipSuccess) return e;
        debug_thr_cap() = B;
    }
    return hipMemcpyAsync(dt, thr, (size_t)B * 4, hipMemcpyDeviceToDevice, s);
}
unsigned long long*& debug_b1_clk() {
    static unsigned long long* p = nullptr;
    return p;
}

// GVDB_B1=0 disables the batch-1 fast path (A/B timing; the general path is exact too)
bool b1_enabled() {
    static const bool on = [] {
        const char* e = getenv("GVDB_B1");
        return !(e && strcmp(e, "0") == 0);
    }();
    return on;
}

// Batch-1 fast path (launch_b1_search): sample + threshold, scan, and a tail
// kernel that selects, re-scores and sorts -- three launches, no memset (the
// state is left zeroed by the previous call), no host sync.
gvdb_status bq_search_b1(const BqSearchArgs& a, Workspace& ws, hipStream_t s) {
    const ShardView& v = a.v;
    const uint32_t R = a.R, D = v.D;
    B1Args b{};
    uint32_t chunks, stride, target, bufcap;
    if (v.N <= kExactN) {
        chunks = (v.N + kB1ChunkRows - 1) / kB1ChunkRows;
        stride = kB1ChunkRows;
        target = R;  // the "sample" is the whole shard: exact threshold
        bufcap = std::min<uint64_t>(v.N, 8ull * R + 2048ull);
    } else {
        // GVDB_B1_SAMPLE_DIV: sample ~N/div rows (timing knob; default 32)
        static const uint32_t div = [] {
            const char* e = getenv("GVDB_B1_SAMPLE_DIV");
            const int d = e ? atoi(e) : 0;
            return d >= 4 && d <= 4096 ? (uint32_t)d : 32u;
        }();
        const uint64_t S = std::max<uint64_t>(kExactN / 4, v.N / div);
        chunks = (uint32_t)(S / kB1ChunkRows);
        stride = v.N / chunks;  // >= kB1ChunkRows: chunks never overlap
        const double Sr = (double)chunks * kB1ChunkRows;
        const double m = (double)R * Sr / (double)v.N;
        target = (uint32_t)std::ceil(m + 4.0 * std::sqrt(m) + 4.0);
        const double expect_full = (double)target * (double)v.N / Sr;
        bufcap = (uint32_t)std::min<double>((double)v.N, std::max(8.0 * expect_full + 2048.0, 16384.0));
    }
    bufcap = std::min<uint32_t>(bufcap, kB1MaxBufcap);
    const size_t hw = ((size_t)D + 64) & ~(size_t)63;  // hist words (D+1, padded)
    const size_t off_ctl = hw, off_qw = off_ctl + 16, off_rsc = off_qw + 32;
    const size_t off_top = (off_rsc + R + 1) & ~(size_t)1;  // u64-aligned
    const size_t off_sc = off_top + 2 * (size_t)R;
    const size_t off_buf = (off_sc + bufcap + 1) & ~(size_t)1;
    const size_t bytes = off_buf * 4 + (size_t)bufcap * 8;
    const uint64_t sig = ((uint64_t)D << 44) ^ ((uint64_t)R << 24) ^ (uint64_t)bufcap ^ 0x5a5a000000000000ull;
    if (ws.b1.n < bytes || ws.b1_sig != sig) {
        HIP_TRY(ws.b1.ensure(bytes), "alloc batch-1 state");
        HIP_TRY(hipMemsetAsync(ws.b1.p, 0, bytes, s), "zero batch-1 state");
        ws.b1_sig = sig;
    }
    uint32_t* w = ws.b1.as<uint32_t>();
    b.codes = v.codes;
    b.cap = v.cap;
    b.N = v.N;
    b.D = D;
    b.R = R;
    b.kout = a.kout;
    b.q = a.d_q;
    b.qlen = a.qlen;
    b.thr = a.thr;
    b.rows = v.rows;
    b.clen = v.clen;
    b.norms = v.norms;
    b.ids = v.ids;
    b.row_offset = v.row_offset;
    b.kind = a.kind;
    b.descending = a.descending;
    b.force_rescan = getenv_flag("GVDB_FORCE_RESCAN") ? 1 : 0;
    b.sample_chunks = chunks;
    b.sample_stride = stride;
    b.target = target;
    b.bufcap = bufcap;
    b.hist = w;
    b.counts = w + off_ctl;
    b.ticket = w + off_ctl + 4;
    b.rescans = w + off_ctl + 8;
    b.qwords = w + off_qw;
    b.scores = (float*)(w + off_sc);
    b.rscores = (float*)(w + off_rsc);
    b.topr = (uint64_t*)(w + off_top);
    b.buf = (uint64_t*)(w + off_buf);
    b.out_ids = a.d_out_ids;
    b.out_scores = a.d_out_scores;
    b.out_n = a.d_out_n;
    // GVDB_B1_CLK=1: phase clocks of the tail kernel (timing study; gvdb_debug_b1_clock)
    static unsigned long long* clk = nullptr;
    if (getenv_flag("GVDB_B1_CLK") && !clk) (void)hipMalloc((void**)&clk, 16 * 8);
    b.clk = getenv_flag("GVDB_B1_CLK") ? clk : nullptr;
    debug_b1_clk() = b.clk;
    bool timed = false;
    {
        std::lock_guard<std::mutex> g(timing().mu);
        timed = timing().on;
    }
    EvSet* ev = timed ? timing_events() : nullptr;
    b.ev = ev ? ev->e : nullptr;
    hipError_t e = launch_b1_search(b, s);
    if (e != hipSuccess) {
        ws.b1_sig = 0;  // state unknown: zero it again next time
        if (ev) {
            std::lock_guard<std::mutex> lk(timing().mu);
            timing().free_sets.push_back(ev);
        }
        return dev_fail(e, "batch-1 search");
    }
    if (ev) {
        HIP_TRY(hipEventRecord(ev->e[5], s), "event");
        timing_submit(ev);
    }
    return GVDB_OK;
}

// BQ multi-stage search on one shard view, enqueued on stream s with NO host
// synchronisation: stage 1 (certified fast path whose rare fallbacks run on
// the device, k_select), stage 2 (exact rerank), final ordering.  A query whose
// top-R holds a NaN score gets out_n = GVDB_N_POISONED (the reference panics).
gvdb_status bq_search(const BqSearchArgs& a, Workspace& ws, hipStream_t s) {
    const ShardView& v = a.v;
    const uint32_t B = a.B, R = a.R;
    if (B == 0) return GVDB_OK;
    // the batched large-R path (gvdb_bigr.hip): unordered exact top-R + k_topk_big
    const bool big = R > kSelectLdsCap && a.dims_match && v.D > 0 && v.D < 4096 && R <= kBigRMax && a.kout <= 1024 &&
                     !a.d_out_dist && !getenv_flag("GVDB_BIGR_OFF");
    // a gated search (the device-side fallback of deep_cert_search) exists only on the large-R
    // path: only its launches honour the gate
    if (a.gate && (!big || a.row_map))
        return fail(GVDB_ERR_INVALID_ARGUMENT, "gated search: the large-R path only");
    if (R == 0) {
        if (a.d_out_n) HIP_TRY(hipMemsetAsync(a.d_out_n, 0, (size_t)B * 4, s), "memset out_n");
        return GVDB_OK;
    }
    const uint32_t W4 = code_w4(v.D);
    if (B == 1 && a.dims_match && v.D > 0 && v.D <= kB1MaxD && !a.d_qwords && !a.d_out_dist && R <= kSortLdsCap &&
        a.qlen == v.clen && v.clen == v.D && !a.row_map && b1_enabled())
        return bq_search_b1(a, ws, s);
    HIP_TRY(ws.qnorm.ensure((size_t)B * 4), "alloc qnorm");
    HIP_TRY(ws.qcodes.ensure((size_t)B * W4 * 16), "alloc qcodes");
    HIP_TRY(ws.scores.ensure((size_t)B * R * 4), "alloc scores");
    Stage1Args s1{};
    gvdb_status pst =
        prepare_stage1(ws, s1, B, v.D, R, v.N, s, a.dims_match && v.D > 0 && (R <= kSelectLdsCap || big));
    if (pst != GVDB_OK) return pst;
    uint32_t* d_flags = s1.any_fail;  // [0] any stage-1 rescan, [1] NaN seen, [2] per-query NaN scratch

    bool timed = false;
    {
        std::lock_guard<std::mutex> g(timing().mu);
        timed = timing().on;
    }
    EvSet* ev = nullptr;
    struct EvBack {  // an EvSet not submitted (error return) goes back to the pool
        EvSet*& e;
        ~EvBack() {
            if (!e) return;
            std::lock_guard<std::mutex> lk(timing().mu);
            timing().free_sets.push_back(e);
        }
    } ev_back{ev};
    if (!a.dims_match || v.D == 0) {
        HIP_TRY(launch_iota_rows(ws.s1_rows.as<uint32_t>(), B, R, s), "iota");
    } else {
        if (a.d_qwords) {
            HIP_TRY(hipMemcpyAsync(ws.qcodes.p, a.d_qwords, (size_t)B * W4 * 16, hipMemcpyDeviceToDevice, s), "qcopy");
        } else if (s1.mfma_scan && (R <= kSelectLdsCap || big) && a.qlen == v.D) {
            s1.qf32 = a.d_q;  // k_qprep packs the queries with the operand build (one launch)
            s1.qthr = a.thr;
        } else {
            HIP_TRY(launch_pack(a.d_q, B, v.D, a.thr, ws.qcodes.p, kPackWordsAoS, 0, 0, s), "pack queries");
        }
        if (R <= kSelectLdsCap) {
            if (timed) ev = timing_events();
            s1.codes = v.codes;
            s1.cap = v.cap;
            s1.N = v.N;
            s1.D = v.D;
            s1.qcodes = ws.qcodes.as<uint4>();
            s1.B = B;
            s1.R = R;
            s1.ev = ev ? ev->e : nullptr;
            HIP_TRY(launch_stage1_fast(s1, s), "stage1");
            HIP_TRY(debug_keep_thr(s1.thr, B, s, s1.any_fail), "copy thresholds");
        } else if (big) {
            // R beyond the LDS select (the reference's default ratio 0.1): the
            // batched stage 1 with k_select_big (exact top-R membership)
            if (timed && !a.gate) ev = timing_events();
            s1.gate = a.gate;
            s1.codes = v.codes;
            s1.cap = v.cap;
            s1.N = v.N;
            s1.D = v.D;
            s1.qcodes = ws.qcodes.as<uint4>();
            s1.B = B;
            s1.R = R;
            s1.ev = ev ? ev->e : nullptr;
            HIP_TRY(launch_stage1_fast(s1, s), "stage1 (large R)");
            HIP_TRY(debug_keep_thr(s1.thr, B, s, s1.any_fail), "copy thresholds");
        } else {
            // R beyond the LDS select: every query on the exact all-rows path
            HIP_TRY(ws.slow.ensure(stage1_slow_bytes(v.N)), "alloc slow path");
            for (uint32_t q = 0; q < B; ++q)
                HIP_TRY(launch_stage1_slow(v.codes, v.cap, v.N, v.D, ws.qcodes.as<uint4>() + (uint64_t)q * W4, R,
                                           ws.s1_rows.as<uint32_t>() + (uint64_t)q * R,
                                           ws.s1_dist.as<uint32_t>() + (uint64_t)q * R, ws.slow.p, ws.slow.n, s),
                        "stage1 slow");
        }
    }

    if (a.row_map)  // stage-1 rows are subset rows: back to index rows (order kept: the subset ascends)
        HIP_TRY(launch_map_rows(ws.s1_rows.as<uint32_t>(), (uint64_t)B * R, a.row_map, s), "map filtered rows");
    RerankArgs rr{};
    rr.rows = v.rows;
    rr.clen = v.clen;
    rr.norms = v.norms;
    rr.q = a.d_q;
    rr.qlen = a.qlen;
    rr.s1_rows = ws.s1_rows.as<uint32_t>();
    rr.B = B;
    rr.R = R;
    rr.kind = a.kind;
    rr.scores = ws.scores.as<float>();
    rr.gate = a.gate;
    HIP_TRY(launch_rerank(rr, s), "rerank");
    if (a.d_out_dist) {
        const uint64_t ostr = a.out_stride ? a.out_stride : R;
        HIP_TRY(launch_emit_candidates(rr.s1_rows, ws.s1_dist.as<uint32_t>(), rr.scores, B, R, v.ids, a.d_out_ids,
                                       a.d_out_dist, a.d_out_scores, s, ostr),
                "emit candidates");
    } else {
        FinalArgs fa{};
        fa.scores = rr.scores;
        fa.s1_rows = rr.s1_rows;
        fa.B = B;
        fa.R = R;
        fa.kout = a.kout;
        fa.descending = a.descending;
        fa.ids = v.ids;
        fa.row_offset = v.row_offset;
        fa.out_ids = a.d_out_ids;
        fa.out_scores = a.d_out_scores;
        fa.out_n = a.d_out_n;
        fa.nan_flag = d_flags + 1;
        fa.gate = a.gate;
        if (big) {
            HIP_TRY(launch_topk_big(fa, ws.s1_dist.as<uint32_t>(), s), "final top-k (large R)");
        } else if (R <= kSortLdsCap) {
            HIP_TRY(launch_final_sort(fa, s), "final sort");
        } else {
            HIP_TRY(ws.sort_tmp.ensure(final_sort_global_bytes(R)), "alloc sort tmp");
            HIP_TRY(launch_final_sort_global(fa, ws.sort_tmp.p, ws.sort_tmp.n, s), "final sort (global)");
        }
    }
    if (ev) {
        HIP_TRY(hipEventRecord(ev->e[5], s), "event");
        timing_submit(ev);
        ev = nullptr;
    }
    return GVDB_OK;
}

// Host-buffer entry points synchronise anyway: map a poisoned query (NaN
// score, GVDB_N_POISONED) to the reference's failure.
gvdb_status check_poisoned(const uint32_t* h_n, uint64_t B) {
    for (uint64_t q = 0; q < B; ++q)
        if (h_n[q] == GVDB_N_POISONED)
            return fail(GVDB_ERR_QUANTIZATION, "NaN score: the reference's partial_cmp().unwrap() sort would panic");
    return GVDB_OK;
}

}  // namespace

// ============================================================================
// tier outcomes of the host-sync-free searches
// ============================================================================
// The _device entry points decide their fallback tiers on the device (gated
// launches, gvdb_device.h gate_closed).  What the host keeps from a tier's
// outcome -- the adaptive i8 skip and the diagnostics counters -- arrives
// through a pinned word copied behind the search on its stream and read once
// the search's event has completed (tier_poll, at the next search): never
// waited for (the diagnostics getters wait, a destroyed index's records are
// dropped).  One process-wide log.
// kTierDeepFlatI8: the i8 flat pass inside the async certified default depth (its failure
// drives the index's i8 skip and backoff like a FLAT-mode i8 batch; counters untouched)
enum TierKind : int { kTierFlatI8 = 0, kTierFlatBf16 = 1, kTierDeepCert = 2, kTierDeepFlatI8 = 3 };
struct FlagLog {
    static constexpr uint32_t kSlots = 256;
    std::mutex mu;
    uint32_t* h = nullptr;  // pinned [kSlots]
    struct Rec {
        hipEvent_t ev;
        uint32_t slot;
        int kind;
        const gvdb_index* ix;  // the adaptive i8 skip's owner (nullptr once destroyed)
    };
    std::vector<Rec> pend;  // oldest first
    std::vector<hipEvent_t> spare;
    uint32_t next = 0;
    ~FlagLog() {
        for (auto& r : pend) (void)hipEventDestroy(r.ev);
        for (auto e : spare) (void)hipEventDestroy(e);
        if (h) (void)hipHostFree(h);
    }
};

// ============================================================================
// index object
// ============================================================================
struct gvdb_index {
    int device = 0;
    uint32_t dim = 0;  // 0 = not fixed yet
    float thr = 0.0f;
    uint64_t n = 0, cap = 0;
    float* rows = nullptr;
    uint4* codes = nullptr;
    float* norms = nullptr;
    uint64_t* ids = nullptr;
    std::vector<uint64_t> h_ids;                      // row -> id (kOrphan for shadowed rows)
    std::unordered_map<uint64_t, uint64_t> id_row;    // live id -> row
    hipStream_t stream = nullptr;                     // mutations
    uint64_t capacity_hint = 0;
    // bf16 k-chunk-major mirror of the rows for the MFMA flat search, built
    // lazily by the first flat search after a mutation (version counter)
    uint64_t version = 0;
    mutable std::mutex rowsb_mu;
    mutable uint16_t* rowsb = nullptr;
    mutable uint64_t rowsb_cap = 0, rowsb_version = ~0ull;
    mutable bool rows_have_nan = false;
    // int8 mirror (k-chunk-major, [KC_i8][cap][128]) + per-row s_x/|x|
    // (rowsq_aux[0, cap)) and relative quantisation error (rowsq_aux[cap, 2cap))
    mutable int8_t* rowsq = nullptr;
    mutable float* rowsq_aux = nullptr;
    mutable uint64_t rowsq_cap = 0, rowsq_version = ~0ull;
    mutable bool rows_nonfinite = false;
    // adaptive flat tiers: batches left that skip the i8 tier after it failed
    mutable std::atomic<uint32_t> i8_skip{0};
    // batches skipped after the next i8 failure: doubles per failure (16 .. 4096), back to 16
    // after an i8 batch certifies -- data whose i8 candidate sets overflow (e.g. i.i.d. rows at
    // D = 3072, where the spread of cosines is below the int8 margin) stop paying the i8 pass
    // plus the exact scan every 17th async batch, whose outcome the host learns late
    mutable std::atomic<uint32_t> i8_backoff{16};
    // concurrent batch-1 host-buffer searches (the reference's many readers of
    // Arc<RwLock<dyn VectorIndex>>, lib.rs:238) share batched searches: see b1_coalesced
    mutable std::mutex b1_mu;
    mutable std::condition_variable b1_cv;
    mutable std::vector<struct B1Req*> b1_pend;  // arrival order
    mutable bool b1_exec = false;
    void i8_failed() const {
        const uint32_t b = i8_backoff.load();
        i8_skip.store(b);
        i8_backoff.store(std::min<uint32_t>(b * 2u, 4096u));
    }
    // searches return before their kernels finish: each records an event on
    // its stream after its last read of this index; a mutation waits for those
    // events only (not for the whole device)
    mutable std::mutex use_mu;
    // per stream that searched this index: an event re-recorded at each search's end
    // (stream order: the latest record covers the earlier ones on that stream)
    mutable std::vector<std::pair<hipStream_t, hipEvent_t>> use_ev;

    uint32_t w4() const { return code_w4(dim); }
    size_t device_bytes() const {
        return cap * ((size_t)dim * 4 + (size_t)w4() * 16 + 4 + 8);
    }
    void free_all() {
        for (void* p : {(void*)rows, (void*)codes, (void*)norms, (void*)ids, (void*)rowsb, (void*)rowsq,
                        (void*)rowsq_aux})
            if (p) (void)hipFree(p);
        rowsb = nullptr;
        rowsb_cap = 0;
        rowsq = nullptr;
        rowsq_aux = nullptr;
        rowsq_cap = 0;
        ++version;
        rows = nullptr;
        codes = nullptr;
        norms = nullptr;
        ids = nullptr;
        n = cap = 0;
    }
};

namespace {

gvdb_status set_device(int dev) {
    hipError_t e = hipSetDevice(dev);
    if (e != hipSuccess) return dev_fail(e, "hipSetDevice");
    return GVDB_OK;
}

// Mutations take the caller's exclusive lock, but searches return before
// their kernels finish: wait for the searches still reading this index (their
// end events, index_track_use) before rows / codes / ids change under them.
gvdb_status quiesce(const gvdb_index* ix) {
    gvdb_status st = set_device(ix->device);
    if (st != GVDB_OK) return st;
    std::lock_guard<std::mutex> g(ix->use_mu);
    hipError_t e = hipSuccess;
    for (auto& p : ix->use_ev) {
        const hipError_t e2 = hipEventSynchronize(p.second);
        if (e == hipSuccess) e = e2;
    }
    if (e == hipSuccess) e = hipStreamSynchronize(ix->stream);
    if (e != hipSuccess) return dev_fail(e, "drain in-flight searches");
    return GVDB_OK;
}

// Record the end of this call's reads of ix on stream s (see quiesce): one
// event per stream, re-recorded -- O(1) per search (the earlier form queried
// every in-flight search's event on each call, ~10 us of host time per call
// once a few dozen searches were queued).
void track_use(const gvdb_index* ix, hipStream_t s) {
    std::lock_guard<std::mutex> g(ix->use_mu);
    for (auto& p : ix->use_ev)
        if (p.first == s) {
            if (hipEventRecord(p.second, s) != hipSuccess) (void)hipStreamSynchronize(s);
            return;
        }
    if (ix->use_ev.size() >= 16)  // many streams: take over the entry of one whose last search finished
        for (auto& p : ix->use_ev)
            if (hipEventQuery(p.second) == hipSuccess) {
                p.first = s;
                if (hipEventRecord(p.second, s) != hipSuccess) (void)hipStreamSynchronize(s);
                return;
            }
    hipEvent_t ev = nullptr;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
        (void)hipStreamSynchronize(s);  // no event: make this call synchronous instead
        return;
    }
    if (hipEventRecord(ev, s) == hipSuccess) {
        ix->use_ev.push_back({s, ev});
    } else {
        (void)hipEventDestroy(ev);
        (void)hipStreamSynchronize(s);
    }
}
struct UseGuard {  // records the use when the entry point returns (any path)
    const gvdb_index* ix;
    hipStream_t s;
    ~UseGuard() { track_use(ix, s); }
};

// Grow HBM storage to hold `need` rows (copies the live rows; planes are
// re-strided because the SoA plane stride is the capacity).
gvdb_status ensure_capacity(gvdb_index* ix, uint64_t need) {
    if (need <= ix->cap) return GVDB_OK;
    uint64_t ncap = std::max<uint64_t>({need, ix->cap * 2, ix->capacity_hint, 1024});
    const uint32_t D = ix->dim, W4 = ix->w4();
    float* nrows = nullptr;
    uint4* ncodes = nullptr;
    float* nnorms = nullptr;
    uint64_t* nids = nullptr;
    hipError_t e = hipMalloc((void**)&nrows, ncap * D * 4);
    if (e == hipSuccess) e = hipMalloc((void**)&ncodes, ncap * W4 * 16);
    if (e == hipSuccess) e = hipMalloc((void**)&nnorms, ncap * 4);
    if (e == hipSuccess) e = hipMalloc((void**)&nids, ncap * 8);
    if (e != hipSuccess) {
        for (void* p : {(void*)nrows, (void*)ncodes, (void*)nnorms, (void*)nids})
            if (p) (void)hipFree(p);
        return dev_fail(e, "grow index");
    }
    if (ix->n) {
        HIP_TRY(hipMemcpyAsync(nrows, ix->rows, ix->n * D * 4, hipMemcpyDeviceToDevice, ix->stream), "grow rows");
        for (uint32_t w = 0; w < W4; ++w)
            HIP_TRY(hipMemcpyAsync(ncodes + w * ncap, ix->codes + w * ix->cap, ix->n * 16, hipMemcpyDeviceToDevice,
                                   ix->stream),
                    "grow codes");
        HIP_TRY(hipMemcpyAsync(nnorms, ix->norms, ix->n * 4, hipMemcpyDeviceToDevice, ix->stream), "grow norms");
        HIP_TRY(hipMemcpyAsync(nids, ix->ids, ix->n * 8, hipMemcpyDeviceToDevice, ix->stream), "grow ids");
        HIP_TRY(hipStreamSynchronize(ix->stream), "grow sync");
    }
    uint64_t n = ix->n;
    ix->free_all();
    ix->rows = nrows;
    ix->codes = ncodes;
    ix->norms = nnorms;
    ix->ids = nids;
    ix->cap = ncap;
    ix->n = n;
    return GVDB_OK;
}

// Host bookkeeping for appended ids (HashMap insert semantics, index.rs:175-176:
// a re-added id shadows its old row, which stays in the corpus but can no
// longer be returned).  Returns the rows whose id must become kOrphan on device.
std::vector<uint64_t> register_ids(gvdb_index* ix, const uint64_t* h_new_ids, uint64_t n) {
    std::vector<uint64_t> orphaned;
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t row = ix->n + i;
        const uint64_t id = h_new_ids[i];
        auto it = ix->id_row.find(id);
        if (it != ix->id_row.end()) {
            ix->h_ids[it->second] = kOrphan;
            orphaned.push_back(it->second);
            it->second = row;
        } else {
            ix->id_row.emplace(id, row);
        }
        ix->h_ids.push_back(id);
    }
    return orphaned;
}

gvdb_status finish_add(gvdb_index* ix, uint64_t n, const std::vector<uint64_t>& orphaned) {
    const uint64_t r0 = ix->n;
    ++ix->version;
    HIP_TRY(launch_pack(ix->rows + r0 * ix->dim, n, ix->dim, ix->thr, ix->codes, kPackSoA, ix->cap, r0, ix->stream),
            "pack rows");
    HIP_TRY(launch_row_norms(ix->rows + r0 * ix->dim, n, ix->dim, ix->norms + r0, ix->stream), "row norms");
    // rows shadowed inside this batch live at >= r0: fix them after the id upload
    static const uint64_t orphan = kOrphan;
    for (uint64_t row : orphaned)
        HIP_TRY(hipMemcpyAsync(ix->ids + row, &orphan, 8, hipMemcpyHostToDevice, ix->stream), "orphan id");
    HIP_TRY(hipStreamSynchronize(ix->stream), "add sync");
    ix->n += n;
    return GVDB_OK;
}

gvdb_status check_add_dim(gvdb_index* ix, uint32_t dim) {
    if (dim == 0) return fail(GVDB_ERR_INVALID_VECTOR_DIMENSION, "vector dimension 0");
    if (ix->dim == 0) {
        ix->dim = dim;  // dimension fixed by the first vector (index.rs:169-171)
    } else if (dim != ix->dim) {
        return dim_mismatch(ix->dim, dim);
    }
    return GVDB_OK;
}

uint32_t effective_R(const gvdb_index* ix, const gvdb_search_params* sp, uint64_t k) {
    uint64_t R = sp->rescore_count ? sp->rescore_count : rust_f32_as_usize((float)ix->n * sp->rescore_ratio);
    R = std::max<uint64_t>(R, k);  // search(k) returns k hits like HnswMap::search().take(k)
    R = std::min<uint64_t>(R, ix->n);
    return (uint32_t)R;
}

FlagLog& tier_log() {
    static FlagLog* L = new FlagLog();  // never destroyed: records may outlive static destructors
    return *L;
}
void tier_apply(const FlagLog::Rec& r, uint32_t failed) {
    if (r.kind == kTierFlatI8) {
        if (!failed) {
            if (r.ix) r.ix->i8_backoff.store(16);
            return;
        }
        flat_fallbacks_i8().fetch_add(1);
        flat_fallbacks().fetch_add(1);  // the async form's next tier is the exact scan
        const char* fk = getenv("GVDB_FLAT");
        if (r.ix && !(fk && strcmp(fk, "i8") == 0)) r.ix->i8_failed();
    } else if (r.kind == kTierFlatBf16) {
        if (failed) flat_fallbacks().fetch_add(1);
    } else if (r.kind == kTierDeepFlatI8) {
        const char* fk = getenv("GVDB_FLAT");
        if (!r.ix || (fk && strcmp(fk, "i8") == 0)) return;
        if (failed)
            r.ix->i8_failed();
        else
            r.ix->i8_backoff.store(16);
    } else {
        deep_cert_count(failed ? 1 : 0).fetch_add(1);
    }
}
// the completed outcomes, oldest first (wait = true: every pending one)
void tier_poll(bool wait = false) {
    FlagLog& L = tier_log();
    std::lock_guard<std::mutex> g(L.mu);
    size_t done = 0;
    for (; done < L.pend.size(); ++done) {
        const FlagLog::Rec& r = L.pend[done];
        if (wait ? hipEventSynchronize(r.ev) != hipSuccess : hipEventQuery(r.ev) != hipSuccess) break;
        tier_apply(r, L.h[r.slot]);
        L.spare.push_back(r.ev);
    }
    L.pend.erase(L.pend.begin(), L.pend.begin() + done);
}
// an index being destroyed: its pending records keep their counters, lose their owner
void tier_forget(const gvdb_index* ix) {
    FlagLog& L = tier_log();
    std::lock_guard<std::mutex> g(L.mu);
    for (auto& r : L.pend)
        if (r.ix == ix) r.ix = nullptr;
}
// copy the tier's device outcome word (non-zero = not certified) behind the search
gvdb_status tier_record(const gvdb_index* ix, const uint32_t* d_word, int kind, hipStream_t s) {
    tier_poll();
    FlagLog& L = tier_log();
    std::lock_guard<std::mutex> g(L.mu);
    if (!L.h) HIP_TRY(hipHostMalloc((void**)&L.h, FlagLog::kSlots * 4, hipHostMallocDefault), "alloc tier log");
    if (L.pend.size() >= FlagLog::kSlots) {
        // a full log: the oldest record's slot is the one the new record takes (slots are
        // handed out in order), so its copy must have landed before the slot is reused --
        // wait for it and apply it rather than dropping it
        const FlagLog::Rec& r = L.pend.front();
        if (hipEventSynchronize(r.ev) == hipSuccess) tier_apply(r, L.h[r.slot]);
        L.spare.push_back(r.ev);
        L.pend.erase(L.pend.begin());
    }
    hipEvent_t ev = nullptr;
    if (!L.spare.empty()) {
        ev = L.spare.back();
        L.spare.pop_back();
    } else {
        HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "tier event");
    }
    const uint32_t slot = L.next++ % FlagLog::kSlots;
    hipError_t e = hipMemcpyAsync(L.h + slot, d_word, 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipEventRecord(ev, s);
    if (e != hipSuccess) {
        L.spare.push_back(ev);
        return dev_fail(e, "tier record");
    }
    L.pend.push_back({ev, slot, kind, ix});
    return GVDB_OK;
}

}  // namespace

// ============================================================================
// C ABI
// ============================================================================
extern "C" {

uint32_t gvdb_abi_version(void) { return GVDB_ABI_VERSION; }

const char* gvdb_last_error(void) { return t_err.c_str(); }

const char* gvdb_status_string(gvdb_status s) {
    switch (s) {
        case GVDB_OK: return "ok";
        case GVDB_ERR_INDEX_NOT_BUILT: return "IndexNotBuilt";
        case GVDB_ERR_DIMENSION_MISMATCH: return "DimensionMismatch";
        case GVDB_ERR_INVALID_VECTOR_DIMENSION: return "InvalidVectorDimension";
        case GVDB_ERR_QUANTIZATION: return "QuantizationError";
        case GVDB_ERR_INDEX: return "IndexError";
        case GVDB_ERR_INVALID_ARGUMENT: return "InvalidArgument";
        case GVDB_ERR_DEVICE: return "DeviceError";
        case GVDB_ERR_OUT_OF_MEMORY: return "OutOfMemory";
        case GVDB_ERR_STORAGE: return "Storage";
    }
    return "unknown";
}

void gvdb_last_dimension_mismatch(uint64_t* expected, uint64_t* actual) {
    if (expected) *expected = t_dim_expected;
    if (actual) *actual = t_dim_actual;
}

int32_t gvdb_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

gvdb_status gvdb_index_create(const gvdb_params* params, gvdb_index** out) {
    if (!out) return fail(GVDB_ERR_INVALID_ARGUMENT, "out is null");
    *out = nullptr;
    gvdb_params p{};
    if (params) p = *params;
    gvdb_status st = set_device(p.device);
    if (st != GVDB_OK) return st;
    auto* ix = new gvdb_index();
    ix->device = p.device;
    ix->dim = p.dimension;
    ix->thr = p.bq_threshold;
    ix->capacity_hint = p.capacity_hint;
    if (hipStreamCreateWithFlags(&ix->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ix;
        return fail(GVDB_ERR_DEVICE, "hipStreamCreate failed");
    }
    *out = ix;
    return GVDB_OK;
}

void gvdb_index_destroy(gvdb_index* ix) {
    if (!ix) return;
    (void)quiesce(ix);
    tier_forget(ix);
    for (auto& p : ix->use_ev) (void)hipEventDestroy(p.second);
    ix->free_all();
    (void)hipStreamDestroy(ix->stream);
    delete ix;
}

gvdb_status gvdb_index_add(gvdb_index* ix, const float* rows, uint64_t n, uint32_t dim, const uint64_t* ids) {
    if (!ix || (n && (!rows || !ids))) return fail(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    if (n == 0) return GVDB_OK;
    gvdb_status st = quiesce(ix);
    if (st != GVDB_OK) return st;
    if ((st = check_add_dim(ix, dim)) != GVDB_OK) return st;
    if ((st = ensure_capacity(ix, ix->n + n)) != GVDB_OK) return st;
    HIP_TRY(hipMemcpyAsync(ix->rows + ix->n * dim, rows, n * dim * 4, hipMemcpyHostToDevice, ix->stream), "upload rows");
    HIP_TRY(hipMemcpyAsync(ix->ids + ix->n, ids, n * 8, hipMemcpyHostToDevice, ix->stream), "upload ids");
    std::vector<uint64_t> orphaned = register_ids(ix, ids, n);
    return finish_add(ix, n, orphaned);
}

gvdb_status gvdb_index_add_device(gvdb_index* ix, const float* d_rows, uint64_t n, uint32_t dim, const uint64_t* d_ids,
                                  void* stream) {
    if (!ix || (n && (!d_rows || !d_ids))) return fail(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    if (n == 0) return GVDB_OK;
    gvdb_status st = quiesce(ix);
    if (st != GVDB_OK) return st;
    // the rows / ids were produced on the caller's stream; the copies run on the index's own
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream), "sync the producing stream");
    if ((st = check_add_dim(ix, dim)) != GVDB_OK) return st;
    if ((st = ensure_capacity(ix, ix->n + n)) != GVDB_OK) return st;
    HIP_TRY(hipMemcpyAsync(ix->rows + ix->n * dim, d_rows, n * dim * 4, hipMemcpyDeviceToDevice, ix->stream),
            "copy rows");
    HIP_TRY(hipMemcpyAsync(ix->ids + ix->n, d_ids, n * 8, hipMemcpyDeviceToDevice, ix->stream), "copy ids");
    std::vector<uint64_t> h(n);
    HIP_TRY(hipMemcpyAsync(h.data(), d_ids, n * 8, hipMemcpyDeviceToHost, ix->stream), "ids to host");
    HIP_TRY(hipStreamSynchronize(ix->stream), "sync");
    std::vector<uint64_t> orphaned = register_ids(ix, h.data(), n);
    return finish_add(ix, n, orphaned);
}

gvdb_status gvdb_index_build(gvdb_index* ix) {
    if (!ix) return fail(GVDB_ERR_INVALID_ARGUMENT, "null index");
    return GVDB_OK;  // codes and norms are maintained on every add
}

gvdb_status gvdb_index_optimize(gvdb_index* ix) { return gvdb_index_build(ix); }

// Lazily (re)build the bf16 mirror of the rows for the MFMA flat search.
static gvdb_status ensure_rowsb(const gvdb_index* ix, Workspace& ws, hipStream_t s) {
    std::lock_guard<std::mutex> g(ix->rowsb_mu);
    if (ix->rowsb && ix->rowsb_version == ix->version) return GVDB_OK;
    const uint32_t KC = fx_kc(ix->dim);
    if (!ix->rowsb || ix->rowsb_cap != ix->cap) {
        if (ix->rowsb) (void)hipFree(ix->rowsb);
        ix->rowsb = nullptr;
        HIP_TRY(hipMalloc((void**)&ix->rowsb, fx_mirror_bytes(ix->cap, KC)), "alloc bf16 rows");
        ix->rowsb_cap = ix->cap;
    }
    HIP_TRY(ws.flags.ensure(16), "alloc flags");
    uint32_t* d_nan = ws.flags.as<uint32_t>() + 3;
    HIP_TRY(hipMemsetAsync(d_nan, 0, 4, s), "memset nan flag");
    HIP_TRY(launch_rows_to_bf16(ix->rows, ix->n, ix->dim, ix->rowsb, ix->cap, d_nan, s), "rows to bf16");
        DBG_SYNC(s, "dbg: rows to bf16");
    HIP_TRY(hipMemcpyAsync(ws.h_flags + 3, d_nan, 4, hipMemcpyDeviceToHost, s), "nan flag");
    HIP_TRY(hipStreamSynchronize(s), "sync bf16 rows");
    ix->rows_have_nan = ws.h_flags[3] != 0;
    ix->rowsb_version = ix->version;
    return GVDB_OK;
}

// Lazily (re)build the int8 mirror of the rows for the i8-MFMA flat search.
static gvdb_status ensure_rowsq(const gvdb_index* ix, Workspace& ws, hipStream_t s) {
    std::lock_guard<std::mutex> g(ix->rowsb_mu);
    if (ix->rowsq && ix->rowsq_version == ix->version) return GVDB_OK;
    const uint32_t KC = fx_kc_i8(ix->dim);
    if (!ix->rowsq || ix->rowsq_cap != ix->cap) {
        if (ix->rowsq) (void)hipFree(ix->rowsq);
        if (ix->rowsq_aux) (void)hipFree(ix->rowsq_aux);
        ix->rowsq = nullptr;
        ix->rowsq_aux = nullptr;
        HIP_TRY(hipMalloc((void**)&ix->rowsq, fx_mirror_bytes(ix->cap, KC)), "alloc i8 rows");
        HIP_TRY(hipMalloc((void**)&ix->rowsq_aux, (size_t)ix->cap * 8), "alloc i8 row scales");
        ix->rowsq_cap = ix->cap;
    }
    HIP_TRY(ws.flags.ensure(16), "alloc flags");
    uint32_t* d_bad = ws.flags.as<uint32_t>() + 3;
    HIP_TRY(hipMemsetAsync(d_bad, 0, 4, s), "memset flag");
    HIP_TRY(launch_rows_to_i8(ix->rows, ix->norms, ix->n, ix->dim, ix->rowsq, ix->cap, ix->rowsq_aux,
                              ix->rowsq_aux + ix->cap, d_bad, s),
            "rows to i8");
    DBG_SYNC(s, "dbg: rows to i8");
    HIP_TRY(hipMemcpyAsync(ws.h_flags + 3, d_bad, 4, hipMemcpyDeviceToHost, s), "flag");
    HIP_TRY(hipStreamSynchronize(s), "sync i8 rows");
    ix->rows_nonfinite = ws.h_flags[3] != 0;
    ix->rowsq_version = ix->version;
    return GVDB_OK;
}

// K4 on MFMA: certified candidate pass + exact rerank (gvdb_flat.hip).  Sets
// *certified = false when any query's list could not be proven exact (the
// caller then runs the exact full scan); results are then meaningless.
// host-buffer searches: slots past a query's count read as id 0 / score 0, not
// whatever an earlier search left in the device output buffers
static void zero_past_counts(uint64_t* ids, float* scores, const uint32_t* n, uint64_t B, uint64_t k) {
    for (uint64_t q = 0; q < B; ++q) {
        const uint64_t nq = n[q] <= k ? n[q] : k;  // GVDB_N_POISONED: the whole row stays as written
        if (n[q] != GVDB_N_POISONED && nq < k) {
            memset(ids + q * k + nq, 0, (k - nq) * 8);
            memset(scores + q * k + nq, 0, (k - nq) * 4);
        }
    }
}

// fail_out != nullptr: the host-sync-free form -- nothing is read back; *fail_out
// points at the device word that is non-zero when the batch is NOT certified (the
// gate of the caller's device-side fallback), and *certified stays false.
static gvdb_status flat_mx_search(const gvdb_index* ix, const float* d_q, uint32_t B, uint32_t dim, uint32_t k, int kind,
                           int descending, uint64_t* d_ids, float* d_scores, uint32_t* d_n, Workspace& ws,
                           hipStream_t s, bool i8, bool* certified, bool rows_out = false,
                           uint32_t** fail_out = nullptr) {
    *certified = false;
    gvdb_status st = i8 ? ensure_rowsq(ix, ws, s) : ensure_rowsb(ix, ws, s);
    if (st != GVDB_OK) return st;
    HIP_TRY(ws.zero.ensure((kFxQ + 4) * 4), "alloc counts");
    uint32_t* fail = ws.zero.as<uint32_t>();
    if (fail_out) *fail_out = fail;
    // a tier that cannot run at all is a failed tier (async form: its gate word says so)
    auto uncertified = [&]() -> gvdb_status {
        if (fail_out) HIP_TRY(hipMemsetD32Async(fail, 1u, 1, s), "mark tier failed");
        return GVDB_OK;
    };
    // the exact scan reproduces the reference's NaN behaviour
    if (i8 ? ix->rows_nonfinite : ix->rows_have_nan) return uncertified();
    const uint32_t N = (uint32_t)ix->n, KC = i8 ? fx_kc_i8(dim) : fx_kc(dim);
    const uint32_t ntiles = (N + kFxRows - 1) / kFxRows;
    static const uint32_t every_env = [] {  // GVDB_FLAT_EVERY: sample-pass tile stride (A/B timing)
        const char* e = getenv("GVDB_FLAT_EVERY");
        const int v = e ? atoi(e) : 0;
        return v > 0 ? (uint32_t)v : 0u;
    }();
    // (a 4x denser sample for K2 >= 24 lists paid off while k_flat_i8q flushed one global atomic per
    // nomination: 0.656 -> 0.568 ms per batch at the 1.25M-row shard; with the aggregated flush the
    // strides 64 / 32 / 16 measure 0.446 / 0.448 / 0.457 ms there, so the default stride stays)
    const uint32_t every = every_env ? every_env : kFxSampleEvery;
    const uint32_t sampled = (ntiles + every - 1) / every;
    const uint32_t S = sampled * kFxRows;

    // mk: the sample rank whose score (minus eps) bounds the threshold.  The
    // sample holds ~Poisson(lambda = k*S/N) of the true top-k rows; mk is the
    // smallest rank with P(X >= mk) <= 1e-6, so T + eps stays below the k-th
    // score unless the sample over-represents the top k that much.
    const double lambda = (double)k * (double)S / (double)N;
    uint32_t mk = 1;
    {
        double p = std::exp(-lambda), cdf = p;  // P(X = 0), P(X <= 0)
        while (mk < 16 && 1.0 - cdf > 1e-6) {
            p *= lambda / (double)mk;
            cdf += p;
            ++mk;
        }
    }
    if (mk > S) return uncertified();
    const uint32_t cc = kFxCandCap;
    HIP_TRY(ws.qnorm.ensure(kFxQ * 4), "alloc qnorm");
    HIP_TRY(ws.fx_qb.ensure((size_t)KC * kFxQ * 128 + kFxQ * 12), "alloc converted queries");
    HIP_TRY(ws.fx_smp.ensure((size_t)kFxQ * S * 4), "alloc sample scores");
    HIP_TRY(ws.fx_probe.ensure((size_t)kFxQ * 34 * 4 + (size_t)kFxQ * kFxProbeParts * 16 * 8), "alloc probes");
    uint32_t* probes = ws.fx_probe.as<uint32_t>();
    float* pscores = (float*)(probes + kFxQ * 16);
    uint32_t* pcount = probes + kFxQ * 32;
    uint64_t* ppart = (uint64_t*)(probes + kFxQ * 34);  // partial top-16 lists of the probe selection
    HIP_TRY(ws.fx_cand.ensure((size_t)kFxQ * cc * 8), "alloc candidates");  // rows, then their approx scores
    HIP_TRY(ws.fx_scores.ensure((size_t)kFxQ * cc * 4), "alloc candidate scores");
    HIP_TRY(ws.thr.ensure(kFxQ * 4), "alloc thresholds");
    char* qx = ws.fx_qb.as<char>();
    float* qinv = (float*)(qx + (size_t)KC * kFxQ * 128);
    float* qa = qinv + kFxQ;
    float* qd = qa + kFxQ;
    uint32_t* counts = fail + 4;
    bool timed;
    {
        std::lock_guard<std::mutex> g(timing().mu);
        timed = timing().on;
    }
    if (timed && !ws.ev.ok) ws.ev.create();
    timed = timed && ws.ev.ok;
    HIP_TRY(hipMemsetAsync(fail, 0, 16, s), "memset fail");
    // GVDB_FLAT_PRUNE=0: rerank every nominated candidate (A/B timing)
    static const bool prune = [] {
        const char* e = getenv("GVDB_FLAT_PRUNE");
        return !(e && e[0] == '0');
    }();
    for (uint32_t g0 = 0; g0 < B; g0 += kFxQ) {
        if (timed) HIP_TRY(hipEventRecord(ws.ev.e[0], s), "event");
        const uint32_t Bg = std::min<uint32_t>(kFxQ, B - g0);
        const float* q = d_q + (size_t)g0 * dim;
        HIP_TRY(hipMemsetAsync(counts, 0, kFxQ * 4, s), "memset counts");
        HIP_TRY(launch_row_norms(q, Bg, dim, ws.qnorm.as<float>(), s), "qnorm");
        if (i8)
            HIP_TRY(launch_queries_to_i8(q, Bg, dim, ws.qnorm.as<float>(), (int8_t*)qx, qinv, qa, qd, s),
                    "queries to i8");
        else
            HIP_TRY(launch_queries_to_bf16(q, Bg, dim, ws.qnorm.as<float>(), (uint16_t*)qx, qinv, qd, s),
                    "queries to bf16");
        DBG_SYNC(s, "dbg: queries converted");
        FlatMxArgs a{};
        a.i8 = i8 ? 1 : 0;
        a.rowsx = i8 ? (const void*)ix->rowsq : (const void*)ix->rowsb;
        a.cap = ix->cap;
        a.N = N;
        a.KC = KC;
        a.qx = qx;
        a.qinv = qinv;
        a.rnorm = ix->norms;
        a.rscale = ix->rowsq_aux;
        a.rrho = ix->rowsq_aux ? ix->rowsq_aux + ix->cap : nullptr;
        a.qa = qa;
        a.qd = qd;
        a.B = Bg;
        a.every = every;
        a.smp = ws.fx_smp.as<float>();
        a.S = S;
        a.thr = ws.thr.as<float>();
        a.counts = counts;
        a.cand = ws.fx_cand.as<uint32_t>();
        a.cscore = prune ? (float*)(a.cand + (size_t)kFxQ * cc) : nullptr;
        a.candcap = cc;
        a.overflow = fail;
        HIP_TRY(launch_flat_mx_sample(a, s), "flat sample pass");
        DBG_SYNC(s, "dbg: flat sample pass");
        // tau from exactly re-scored probes (the 16 best sampled rows per query)
        HIP_TRY(launch_flat_probes(a.smp, Bg, S, every, N, ix->n != ix->id_row.size() ? ix->ids : nullptr, probes,
                                   pcount, ppart, s), "flat probes");
        {
            RerankArgs pr{};
            pr.rows = ix->rows;
            pr.clen = dim;
            pr.norms = ix->norms;
            pr.q = q;
            pr.qlen = dim;
            pr.s1_rows = probes;
            pr.B = Bg;
            pr.R = 16;
            pr.kind = kind;
            pr.scores = pscores;
            pr.counts = pcount;
            HIP_TRY(launch_rerank(pr, s), "flat probe rerank");
        }
        HIP_TRY(launch_flat_tau(pscores, pcount, Bg, mk, kind == kScoreCosineDistance, qd,
                                ws.thr.as<float>(), s),
                "flat thresholds");
        DBG_SYNC(s, "dbg: flat thresholds");
        if (timed) HIP_TRY(hipEventRecord(ws.ev.e[1], s), "event");
        HIP_TRY(launch_flat_mx_emit(a, s), "flat candidate pass");
        if (timed) HIP_TRY(hipEventRecord(ws.ev.e[2], s), "event");
        DBG_SYNC(s, "dbg: flat candidate pass");
#ifdef GVDB_FLAT_STATS
        auto cstats = [&](const char* what) {  // variant builds: candidate counts per query (mean / max)
            std::vector<uint32_t> h(Bg);
            (void)hipMemcpyAsync(h.data(), counts, Bg * 4, hipMemcpyDeviceToHost, s);
            (void)hipStreamSynchronize(s);
            uint64_t sum = 0, mx = 0;
            for (uint32_t c : h) {
                sum += c;
                mx = std::max<uint64_t>(mx, c);
            }
            fprintf(stderr, "[flatstats] N=%u B=%u k=%u S=%u mk=%u %s: mean %.1f max %llu\n", N, Bg, k, S, mk, what,
                    (double)sum / Bg, (unsigned long long)mx);
        };
        cstats("nominated");
#endif
        if (prune)
            HIP_TRY(launch_flat_prune(counts, a.cand, a.cscore, cc, Bg, k, i8 ? qa : nullptr, qd, i8 ? a.rrho : nullptr,
                                      ix->ids, s),
                    "flat prune");
#ifdef GVDB_FLAT_STATS
        cstats("after prune");
#endif
        RerankArgs rr{};
        rr.rows = ix->rows;
        rr.clen = dim;
        rr.norms = ix->norms;
        rr.q = q;
        rr.qlen = dim;
        rr.s1_rows = a.cand;
        rr.B = Bg;
        rr.R = cc;
        rr.kind = kind;
        rr.scores = ws.fx_scores.as<float>();
        rr.counts = counts;
        HIP_TRY(launch_rerank(rr, s), "flat rerank");
        DBG_SYNC(s, "dbg: flat rerank");
        HIP_TRY(launch_flat_final(counts, a.cand, cc, rr.scores, ws.thr.as<float>(), qd, Bg, k, descending,
                                  rows_out ? nullptr : ix->ids,
                                  d_ids + (size_t)g0 * k, d_scores + (size_t)g0 * k, d_n ? d_n + g0 : nullptr, fail, s),
                "flat final");
        DBG_SYNC(s, "dbg: flat final");
        if (timed) {  // timing mode only: per-group sync to read the events
            HIP_TRY(hipEventRecord(ws.ev.e[3], s), "event");
            HIP_TRY(hipEventSynchronize(ws.ev.e[3]), "event sync");
            float te = 0, tt = 0;
            (void)hipEventElapsedTime(&te, ws.ev.e[1], ws.ev.e[2]);
            (void)hipEventElapsedTime(&tt, ws.ev.e[0], ws.ev.e[3]);
            std::lock_guard<std::mutex> g(timing().mu);
            const int se = i8 ? kTimFlatEmitI8 : kTimFlatEmit, sg = i8 ? kTimFlatI8 : kTimFlat;
            timing().ms[se] += te;
            timing().n[se] += 1;
            timing().ms[sg] += tt;
            timing().n[sg] += 1;
        }
    }
    if (fail_out) return GVDB_OK;
    HIP_TRY(hipMemcpyAsync(ws.h_flags, fail, 4, hipMemcpyDeviceToHost, s), "fail flag");
    HIP_TRY(hipStreamSynchronize(s), "sync");
    *certified = ws.h_flags[0] == 0;
    return GVDB_OK;
}

// Certified search at the reference's DEFAULT rescore depth (R = 0.1 N,
// quantization.rs:27,178) without the rerank of B x R rows (3 KiB each: 256 ms
// per batch-256 step at 10M rows): the exact cosine top-kDeepK2 of the whole
// shard (flat_mx_search, rows instead of ids) is filtered by the stage-1
// membership rule -- the dense FP4 scan and k_select_dense's (T, cut), no member
// lists -- and k_deep_certify keeps the first min(k, R) members in the
// reference's (cosine desc, Hamming, row) order when the list certifies them
// (gvdb_bigr.hip).  Any query it cannot certify (members below the list's last
// score, a flat tier that cannot certify, non-finite rows) sends the whole batch
// to bq_search.  Shards with orphan rows (the reference truncates before
// dropping them) and metrics other than cosine take bq_search directly
// (*eligible = false).
// sync = true (host-buffer entry points): the flat tiers and the certificate are
//   read back on the host; *done tells the caller whether bq_search must run.
// sync = false (the _device entry points): nothing is read back -- the flat pass
//   runs one tier, k_deep_certify folds that tier's failure word into its own,
//   and the B x R rerank (bq_search) is enqueued behind it GATED by that word, so
//   it runs on the device only for a batch that did not certify (*done = true:
//   the caller has nothing left to do).
static gvdb_status deep_cert_search(const gvdb_index* ix, const float* d_q, uint32_t B, uint32_t dim, uint32_t k,
                                    uint32_t R, int kind, uint64_t* d_ids, float* d_scores, uint32_t* d_n,
                                    Workspace& ws, hipStream_t s, bool* done, bool sync) {
    *done = false;
    const uint32_t N = (uint32_t)ix->n, W4 = code_w4(dim);
    const char* env = getenv("GVDB_DEEP_CERT");
    if ((env && env[0] == '0') || kind != kScoreCosine || k == 0 || k > 32 || B == 0 || N < kFxMinN ||
        R <= kSelectLdsCap || R > N || R > kBigRMax || dim == 0 || dim >= 4096 || !mfma_scan_supported(W4) ||
        (uint64_t)R * 64u < N || ix->n != ix->id_row.size() || (!sync && getenv_flag("GVDB_BIGR_OFF")))
        return GVDB_OK;  // (async: the gated fallback below needs bq_search's large-R path)
    Stage1Args s1{};
    gvdb_status pst = prepare_stage1(ws, s1, B, dim, R, N, s, true, false);
    if (pst != GVDB_OK) return pst;
    if (!s1.dense_sel || !s1.mfma_scan) return GVDB_OK;
    // list length: 32 entries certify k <= 16 on all but adversarial data at half the exact
    // rerank of 64 (the i8 pass nominates by the K2-th score)
    const uint32_t K2 = k <= 16u ? 32u : kDeepK2;
    HIP_TRY(ws.qcodes.ensure((size_t)B * W4 * 16), "alloc qcodes");
    HIP_TRY(ws.deep.ensure((size_t)B * K2 * 12 + (size_t)B * 28 + 32), "alloc certified-depth lists");
    if (!sync) {  // the gated fallback's buffers, sized before anything is enqueued (no reallocation under it)
        HIP_TRY(ws.s1_rows.ensure((size_t)B * R * 4), "alloc s1_rows");
        HIP_TRY(ws.s1_dist.ensure((size_t)B * R * 4), "alloc s1_dist");
        HIP_TRY(ws.scores.ensure((size_t)B * R * 4), "alloc scores");
        HIP_TRY(ws.qnorm.ensure((size_t)B * 4), "alloc qnorm");
    }
    char* p = ws.deep.as<char>();
    uint64_t* frow = (uint64_t*)p;
    float* fsc = (float*)(p + (size_t)B * K2 * 8);
    uint32_t* tcut = (uint32_t*)(p + (size_t)B * K2 * 12);
    uint32_t* fn = tcut + 4ull * B;
    uint32_t* dfail = fn + B;  // [4]: the certify word, the flat tier's word (async), 2 spare
    // the byte form of the dense rule (GVDB_DENSE8=0: the f16 form): its windows after the words
    {
        const char* e8 = getenv("GVDB_DENSE8");
        s1.dense8 = !(e8 && e8[0] == '0');
    }
    s1.qwin = dfail + 4;  // [2][B]
    s1.qf32 = d_q;  // k_qprep packs the query codes (the certify pass reads them)
    s1.qthr = ix->thr;
    s1.codes = ix->codes;
    s1.cap = ix->cap;
    s1.qcodes = ws.qcodes.as<uint4>();
    s1.ev = nullptr;
    s1.tcut = tcut;
    {  // the rule in parallel over row segments (k_dense_seg_hist + k_dense_rule)
        dense_segments(N, kDenseSegs, &s1.seg_n, &s1.seg_len);
        const size_t gq = std::min<uint32_t>(B, 256u);  // one 256-query group at a time
        HIP_TRY(ws.seg.ensure(gq * s1.seg_n * (dim + 1u) * 4 * ((B + 255u) / 256u)), "alloc segment histograms");
        s1.seg_hist = ws.seg.as<uint32_t>();
    }
    // the flat pass runs on a second workspace's stream, concurrently with stage 1 (they share
    // nothing until the certify pass): ordered after the caller's queries, joined before certify
    struct Ev {
        hipEvent_t e = nullptr;
        ~Ev() {
            if (e) (void)hipEventDestroy(e);
        }
    } e_in, e_flat;
    WsGuard g2(ix->device);
    Workspace* ws2 = &ws;
    hipStream_t s2 = s;
    if (g2.w && hipEventCreateWithFlags(&e_in.e, hipEventDisableTiming) == hipSuccess &&
        hipEventCreateWithFlags(&e_flat.e, hipEventDisableTiming) == hipSuccess) {
        ws2 = g2.w;
        s2 = g2.w->stream;
        g2.begin(s2);
        HIP_TRY(hipEventRecord(e_in.e, s), "event");
        HIP_TRY(hipStreamWaitEvent(s2, e_in.e, 0), "stream wait");
    }
    UseGuard ug2{ix, s2};
    bool timed = false;
    {
        std::lock_guard<std::mutex> g(timing().mu);
        timed = timing().on;
    }
    EvSet* tev = timed ? timing_events() : nullptr;  // timing mode: the dense scan in the scan slot
    s1.ev = tev ? tev->e : nullptr;
    HIP_TRY(launch_stage1_fast(s1, s), "certified depth: stage 1");
    if (tev) {
        HIP_TRY(hipEventRecord(tev->e[5], s), "event");
        timing_submit(tev);
    }
    bool cert = false, i8_tier = false;
    uint32_t* flat_fail = nullptr;
    gvdb_status st;
    if (sync) {
        st = flat_mx_search(ix, d_q, B, dim, K2, kind, 1, frow, fsc, fn, *ws2, s2, true, &cert, true);
        if (st != GVDB_OK) return st;
        if (!cert) {
            st = flat_mx_search(ix, d_q, B, dim, K2, kind, 1, frow, fsc, fn, *ws2, s2, false, &cert, true);
            if (st != GVDB_OK) return st;
        }
    } else {  // one tier (i8, or bf16 while the index skips i8), its failure word read on the device
        i8_tier = ix->i8_skip.load() == 0;
        st = flat_mx_search(ix, d_q, B, dim, K2, kind, 1, frow, fsc, fn, *ws2, s2, i8_tier, &cert, true, &flat_fail);
        if (st != GVDB_OK) return st;
    }
    uint32_t* ffail = dfail + 1;  // the flat tier's failure word, copied into THIS call's workspace
    if (!sync) {
        // ws2 returns to the pool when this call returns and its next user may clear its words before
        // the certify pass (on s) has read them: copy the word out on s2, ahead of the join event
        HIP_TRY(hipMemcpyAsync(ffail, flat_fail, 4, hipMemcpyDeviceToDevice, s2), "flat failure word");
    }
    if (s2 != s) {
        HIP_TRY(hipEventRecord(e_flat.e, s2), "event");
        HIP_TRY(hipStreamWaitEvent(s, e_flat.e, 0), "stream wait");
    }
    if (sync && !cert) {
        deep_cert_count(1).fetch_add(1);
        return GVDB_OK;
    }
    HIP_TRY(hipMemsetAsync(dfail, 0, 4, s), "memset certify flag");
    HIP_TRY(launch_deep_certify(frow, fsc, fn, K2, tcut, ix->codes, ix->cap, W4, ws.qcodes.as<uint4>(), B, k, R,
                                ix->ids, d_ids, d_scores, d_n, dfail, s, nullptr, nullptr, nullptr, nullptr, nullptr,
                                0, sync ? nullptr : ffail),
            "certified depth: certify");
    if (sync) {
        HIP_TRY(hipMemcpyAsync(ws.h_flags, dfail, 4, hipMemcpyDeviceToHost, s), "certify flag");
        HIP_TRY(hipStreamSynchronize(s), "sync");
        cert = ws.h_flags[0] == 0;
        deep_cert_count(cert ? 0 : 1).fetch_add(1);
        *done = cert;
        return GVDB_OK;
    }
    // the B x R rerank, run by the device only if the certify pass failed
    BqSearchArgs a{};
    a.v = ShardView{ix->rows, dim, ix->norms, ix->codes, ix->cap, N, dim, ix->ids, 0};
    a.d_q = d_q;
    a.qlen = dim;
    a.B = B;
    a.thr = ix->thr;
    a.dims_match = true;
    a.R = R;
    a.kout = k;
    a.kind = kind;
    a.descending = 1;
    a.d_out_ids = d_ids;
    a.d_out_scores = d_scores;
    a.d_out_n = d_n;
    a.gate = dfail;
    st = bq_search(a, ws, s);
    if (st != GVDB_OK) return st;
    if ((st = tier_record(ix, dfail, kTierDeepCert, s)) != GVDB_OK) return st;
    if (i8_tier && (st = tier_record(ix, ffail, kTierDeepFlatI8, s)) != GVDB_OK) return st;
    *done = true;
    return GVDB_OK;
}

// FLAT mode's exact tier: the exact scan + one-launch top-k, in query groups whose
// dense score block stays within kFlatScoreBytes (1 GiB: 26 queries per group at
// 10M rows) instead of one B x N block (10 GB at B = 256).  gate: the device-side
// fallback form (runs only if *gate != 0; k <= 1024).
static gvdb_status flat_exact(const gvdb_index* ix, const float* d_q, uint64_t B, uint32_t dim, uint64_t k, int kind,
                              int descending, uint64_t* d_ids, float* d_scores, uint32_t* d_n, Workspace& ws,
                              hipStream_t s, const uint32_t* gate) {
    const uint64_t per_q = std::max<uint64_t>(ix->n * 4, 1);
    const uint64_t cap_bytes = gate ? kFlatScoreBytesGated : kFlatScoreBytes;
    const uint64_t G = std::max<uint64_t>(1, std::min<uint64_t>(B, cap_bytes / per_q));
    HIP_TRY(ws.qnorm.ensure(B * 4), "alloc qnorm");
    HIP_TRY(ws.scores.ensure(G * per_q), "alloc flat scores");
    HIP_TRY(ws.flags.ensure(16), "alloc flags");
    HIP_TRY(hipMemsetAsync(ws.flags.p, 0, 16, s), "memset flags");
    HIP_TRY(launch_row_norms(d_q, B, dim, ws.qnorm.as<float>(), s, gate), "qnorm");
    if (!gate) HIP_TRY(ws.sort_tmp.ensure(flat_select_bytes((uint32_t)ix->n)), "alloc sort tmp");
    for (uint64_t g0 = 0; g0 < B; g0 += G) {
        const uint32_t bg = (uint32_t)std::min<uint64_t>(G, B - g0);
        HIP_TRY(launch_flat_scores(d_q + g0 * dim, bg, ws.qnorm.as<float>() + g0, ix->rows, (uint32_t)ix->n, dim,
                                   ix->norms, kind, nullptr, ws.scores.as<float>(), s, gate),
                "flat scores");
        HIP_TRY(launch_flat_select(ws.scores.as<float>(), bg, (uint32_t)ix->n, (uint32_t)k, descending, 0, 0.0f, ix->ids,
                                   d_ids + g0 * k, d_scores + g0 * k, d_n ? d_n + g0 : nullptr, ws.sort_tmp.p,
                                   ws.sort_tmp.n, ws.flags.as<uint32_t>() + 1, s, gate),
                "flat select");
    }
    return GVDB_OK;
}

// sync: the host-buffer entry points (they synchronise anyway) decide the flat
// tiers and the certified default depth on the host; the _device entry points
// (sync = false) return after enqueueing: every fallback tier is enqueued behind
// the tier it backs up and gated on the device by that tier's failure word.
static gvdb_status index_search_impl(const gvdb_index* ix, const float* d_q, uint64_t B, uint32_t dim, uint64_t k,
                                     const gvdb_search_params* sp_in, uint64_t* d_ids, float* d_scores, uint32_t* d_n,
                                     Workspace& ws, hipStream_t s, bool sync) {
    gvdb_search_params sp{};
    sp.mode = GVDB_SEARCH_BQ_RERANK;
    sp.metric = GVDB_METRIC_COSINE;
    sp.rescore_ratio = 0.1f;
    if (sp_in) sp = *sp_in;
    const int kind = sp.metric == GVDB_METRIC_L2 ? kScoreL2
                     : sp.metric == GVDB_METRIC_COSINE_DISTANCE ? kScoreCosineDistance
                                                                 : kScoreCosine;
    const int descending = kind == kScoreCosine;
    tier_poll();  // earlier async searches' tier outcomes (adaptive i8 skip)
    if (sp.mode == GVDB_SEARCH_FLAT && kind != kScoreL2 && ix->n >= kFxMinN && k >= 1 && k <= 256 &&
        !getenv_flag("GVDB_FLAT_EXACT_ONLY")) {
        // Tiers: i8 candidates first (half the bytes of bf16, twice the MFMA
        // rate, a ~4x wider certified margin: ~2K candidates per query at
        // 10M x 768 i.i.d.), then bf16 (2^-8 margin), then the exact scan; a
        // batch a tier cannot certify is retried on the next one.  Default:
        // adaptive -- after an i8 batch fails to certify, this index skips the
        // i8 tier for its next 16 batches (bounding the wasted pass on data
        // whose i8 candidate sets overflow).  GVDB_FLAT=i8 / bf16 forces the
        // first tier.  The async form runs the first tier, then the exact scan
        // gated by its failure word (no bf16 retry: that tier's mirror is built
        // only once a synchronous search or the skip asks for it).
        const char* fk = getenv("GVDB_FLAT");
        const bool force_i8 = fk && strcmp(fk, "i8") == 0;
        const bool force_bf16 = fk && strcmp(fk, "bf16") == 0;
        bool try_i8 = force_i8;
        if (!force_i8 && !force_bf16) {
            uint32_t skip = ix->i8_skip.load();
            while (skip > 0 && !ix->i8_skip.compare_exchange_weak(skip, skip - 1)) {
            }
            try_i8 = skip == 0;
        }
        bool certified = false;
        if (!sync) {
            uint32_t* fail = nullptr;
            gvdb_status st = flat_mx_search(ix, d_q, (uint32_t)B, dim, (uint32_t)k, kind, descending, d_ids, d_scores,
                                            d_n, ws, s, try_i8, &certified, false, &fail);
            if (st != GVDB_OK) return st;
            if ((st = flat_exact(ix, d_q, B, dim, k, kind, descending, d_ids, d_scores, d_n, ws, s, fail)) != GVDB_OK)
                return st;
            return tier_record(ix, fail, try_i8 ? kTierFlatI8 : kTierFlatBf16, s);
        }
        if (try_i8) {
            gvdb_status st = flat_mx_search(ix, d_q, (uint32_t)B, dim, (uint32_t)k, kind, descending, d_ids, d_scores,
                                            d_n, ws, s, true, &certified);
            if (st != GVDB_OK) return st;
            if (certified) {
                ix->i8_backoff.store(16);
                return st;
            }
            flat_fallbacks_i8().fetch_add(1);
            if (!force_i8) ix->i8_failed();
        }
        gvdb_status st = flat_mx_search(ix, d_q, (uint32_t)B, dim, (uint32_t)k, kind, descending, d_ids, d_scores,
                                        d_n, ws, s, false, &certified);
        if (st != GVDB_OK || certified) return st;
        flat_fallbacks().fetch_add(1);
    }
    if (sp.mode == GVDB_SEARCH_FLAT)
        return flat_exact(ix, d_q, B, dim, k, kind, descending, d_ids, d_scores, d_n, ws, s, nullptr);
    const uint32_t R = effective_R(ix, &sp, k);
    if (sp.mode == GVDB_SEARCH_BQ_RERANK) {  // the reference's default depth: certified, no B x R rerank
        bool done = false;
        gvdb_status st = deep_cert_search(ix, d_q, (uint32_t)B, dim, (uint32_t)k, R, kind, d_ids, d_scores, d_n, ws, s,
                                          &done, sync);
        if (st != GVDB_OK || done) return st;
    }
    BqSearchArgs a{};
    a.v = ShardView{ix->rows, dim, ix->norms, ix->codes, ix->cap, (uint32_t)ix->n, dim, ix->ids, 0};
    a.d_q = d_q;
    a.qlen = dim;
    a.B = (uint32_t)B;
    a.thr = ix->thr;
    a.dims_match = true;
    a.R = R;
    a.kout = (uint32_t)k;
    a.kind = kind;
    a.descending = descending;
    a.d_out_ids = d_ids;
    a.d_out_scores = d_scores;
    a.d_out_n = d_n;
    return bq_search(a, ws, s);
}

static gvdb_status check_search(const gvdb_index* ix, uint32_t dim, uint64_t B, uint64_t k) {
    if (!ix) return fail(GVDB_ERR_INVALID_ARGUMENT, "null index");
    if (ix->n == 0) return fail(GVDB_ERR_INDEX_NOT_BUILT, "Index not built");
    if (dim != ix->dim) return dim_mismatch(ix->dim, dim);
    if (ix->n > 0xFFFFFFFFull) return fail(GVDB_ERR_INDEX, "shard exceeds 2^32 rows");
    if (B > 0xFFFFFFFFull || k > 0xFFFFFFFFull) return fail(GVDB_ERR_INVALID_ARGUMENT, "batch or k too large");
    return GVDB_OK;
}

// one host-buffer search of B queries (arguments already checked)
static gvdb_status index_search_host(const gvdb_index* ix, const float* queries, uint64_t B, uint32_t dim,
                                     uint64_t k, const gvdb_search_params* sp, uint64_t* out_ids, float* out_scores,
                                     uint32_t* out_n) {
    gvdb_status st = set_device(ix->device);
    if (st != GVDB_OK) return st;
    WsGuard g(ix->device);
    if (!g.w) return fail(GVDB_ERR_DEVICE, "workspace");
    Workspace& ws = *g.w;
    hipStream_t s = ws.stream;
    g.begin(s);
    const uint64_t kk = k ? k : 1;
    HIP_TRY(ws.q.ensure(B * dim * 4), "alloc queries");
    HIP_TRY(ws.out_ids.ensure(B * kk * 8), "alloc out");
    HIP_TRY(ws.out_scores.ensure(B * kk * 4), "alloc out");
    HIP_TRY(ws.out_n.ensure(B * 4), "alloc out");
    HIP_TRY(hipMemcpyAsync(ws.q.p, queries, B * dim * 4, hipMemcpyHostToDevice, s), "upload queries");
    if (k == 0) {
        memset(out_n, 0, B * 4);
        return GVDB_OK;
    }
    st = index_search_impl(ix, ws.q.as<float>(), B, dim, k, sp, ws.out_ids.as<uint64_t>(), ws.out_scores.as<float>(),
                           ws.out_n.as<uint32_t>(), ws, s, true);
    if (st != GVDB_OK) return st;
    HIP_TRY(hipMemcpyAsync(out_ids, ws.out_ids.p, B * k * 8, hipMemcpyDeviceToHost, s), "download ids");
    HIP_TRY(hipMemcpyAsync(out_scores, ws.out_scores.p, B * k * 4, hipMemcpyDeviceToHost, s), "download scores");
    HIP_TRY(hipMemcpyAsync(out_n, ws.out_n.p, B * 4, hipMemcpyDeviceToHost, s), "download n");
    HIP_TRY(hipStreamSynchronize(s), "sync");
    zero_past_counts(out_ids, out_scores, out_n, B, k);
    return check_poisoned(out_n, B);
}

// Built-in coalescing of concurrent batch-1 host-buffer searches.  The reference
// serves single-query searches from many concurrent readers of
// Arc<RwLock<dyn VectorIndex>> (lib.rs:238), each running
// HnswVectorIndex::search(q, k) (index.rs:212-231).  On the GPU a batch-1 search
// reads the whole code array once (k_b1_scan, HBM-bound), and independent batch-1
// searches from many threads each take a pooled workspace with its own stream --
// 64 callers put 64 streams on the 4 hardware queues (2.1K QPS, p99 92 ms in round 5).
// So a B = 1 call joins the index's pending list; whenever no coalesced batch is
// executing, the first waiting caller takes the oldest pending request and every
// later one with the same (k, params) (up to kB1MaxBatch) and runs them as ONE
// index_search_host, then hands each caller its own results.  No timer: a lone
// caller leads its own batch of one at once; batches grow with the load.  Every
// search mode is exact, so a query's answer does not depend on its batch
// (tests/test_gpu_concurrent.py, test_gpu_coalesce.py).  GVDB_B1_COALESCE=0 turns
// it off (every call runs alone).
struct B1Req {
    const float* q;
    uint64_t k;
    bool has_sp;
    gvdb_search_params sp;
    uint64_t* ids;
    float* scores;
    uint32_t* n;
    gvdb_status st = GVDB_OK;
    std::string err;
    bool taken = false, done = false;
    bool same_batch(const B1Req& o) const {
        return k == o.k && has_sp == o.has_sp &&
               (!has_sp || (sp.mode == o.sp.mode && sp.metric == o.sp.metric &&
                            sp.rescore_count == o.sp.rescore_count && sp.rescore_ratio == o.sp.rescore_ratio &&
                            sp.reserved == o.sp.reserved));
    }
};
constexpr size_t kB1MaxBatch = 256;
std::atomic<uint64_t> g_b1_batches{0}, g_b1_queries{0}, g_b1_max{0};  // gvdb_debug_b1_coalesce

static void b1_run_batch(const gvdb_index* ix, uint32_t dim, const std::vector<B1Req*>& reqs) {
    const size_t B = reqs.size();
    const uint64_t k = reqs[0]->k;
    std::vector<float> q(B * (size_t)dim);
    for (size_t i = 0; i < B; ++i) memcpy(q.data() + i * dim, reqs[i]->q, (size_t)dim * 4);
    std::vector<uint64_t> ids(B * k);
    std::vector<float> sc(B * k);
    std::vector<uint32_t> n(B);
    const gvdb_status st = index_search_host(ix, q.data(), B, dim, k, reqs[0]->has_sp ? &reqs[0]->sp : nullptr,
                                             ids.data(), sc.data(), n.data());
    const std::string err = st == GVDB_OK ? std::string() : t_err;
    // a NaN score fails only the queries it poisoned: index_search_host downloads every
    // query's results and counts before it reports GVDB_ERR_QUANTIZATION
    const bool per_query = st == GVDB_ERR_QUANTIZATION;
    for (size_t i = 0; i < B; ++i) {
        B1Req* r = reqs[i];
        const bool poisoned = n[i] == GVDB_N_POISONED;
        const bool ok = st == GVDB_OK || (per_query && !poisoned);
        r->st = ok ? GVDB_OK : st;
        r->err = ok ? std::string() : err;
        if (ok || (per_query && poisoned)) {  // a poisoned query's slots as the serial call leaves them
            memcpy(r->ids, ids.data() + i * k, k * 8);
            memcpy(r->scores, sc.data() + i * k, k * 4);
            *r->n = n[i];
        }
    }
}

static gvdb_status b1_coalesced(const gvdb_index* ix, const float* query, uint32_t dim, uint64_t k,
                                const gvdb_search_params* sp, uint64_t* out_ids, float* out_scores, uint32_t* out_n) {
    B1Req r;
    r.q = query;
    r.k = k;
    r.has_sp = sp != nullptr;
    if (sp) r.sp = *sp;
    r.ids = out_ids;
    r.scores = out_scores;
    r.n = out_n;
    std::unique_lock<std::mutex> lk(ix->b1_mu);
    ix->b1_pend.push_back(&r);
    while (!r.done) {
        if (!r.taken && !ix->b1_exec) {
            // lead the next batch: the oldest pending request and the later ones it can share a search with
            std::vector<B1Req*> mine;
            std::vector<B1Req*> rest;
            for (B1Req* x : ix->b1_pend)
                (mine.size() < kB1MaxBatch && x->same_batch(*ix->b1_pend.front()) ? mine : rest).push_back(x);
            ix->b1_pend.swap(rest);
            for (B1Req* x : mine) x->taken = true;
            g_b1_batches.fetch_add(1);
            g_b1_queries.fetch_add(mine.size());
            for (uint64_t m = g_b1_max.load(); m < mine.size() && !g_b1_max.compare_exchange_weak(m, mine.size());) {
            }
            ix->b1_exec = true;
            lk.unlock();
            b1_run_batch(ix, dim, mine);
            lk.lock();
            ix->b1_exec = false;
            for (B1Req* x : mine) x->done = true;
            ix->b1_cv.notify_all();
        } else {
            ix->b1_cv.wait(lk);
        }
    }
    lk.unlock();
    if (r.st != GVDB_OK) return fail(r.st, r.err);
    return GVDB_OK;
}

gvdb_status gvdb_index_search(const gvdb_index* ix, const float* queries, uint64_t B, uint32_t dim, uint64_t k,
                              const gvdb_search_params* sp, uint64_t* out_ids, float* out_scores, uint32_t* out_n) {
    gvdb_status st = check_search(ix, dim, B, k);
    if (st != GVDB_OK) return st;
    if (B == 0) return GVDB_OK;
    if (!queries || !out_n || (k && (!out_ids || !out_scores))) return fail(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    static const bool coalesce = [] {
        const char* e = getenv("GVDB_B1_COALESCE");
        return !(e && e[0] == '0');
    }();
    if (B == 1 && k > 0 && coalesce) return b1_coalesced(ix, queries, dim, k, sp, out_ids, out_scores, out_n);
    return index_search_host(ix, queries, B, dim, k, sp, out_ids, out_scores, out_n);
}

// Filtered search (§8(f) rank 4): the pre-mask of FilterEngine::execute_filter
// (filtering.rs:374) applied to the vector search.  The allowed ids map to
// live rows on the host (unknown ids are ignored, repeats count once), sorted
// ascending so ties keep the index's row order.  Then, by sp->mode:
//   BQ (the reference's multi_stage_search, quantization.rs:151-193, over the
//   subset): the allowed rows' code planes are compacted (one gather of
//   M x 16 W4 bytes), the unchanged stage-1 kernels run over them with R from
//   the subset size, the candidates map back to index rows, and the exact
//   rerank + final sort read the resident rows -- memory O(M) codes, no
//   per-row test in the unfiltered hot kernels;
//   FLAT: the exact scan of the allowed rows, in query groups whose score
//   block stays within kFlatScoreBytes.
gvdb_status gvdb_index_search_filtered(const gvdb_index* ix, const float* queries, uint64_t B, uint32_t dim, uint64_t k,
                                       const gvdb_search_params* sp_in, const uint64_t* allowed, uint64_t n_allowed,
                                       uint64_t* out_ids, float* out_scores, uint32_t* out_n) {
    gvdb_status st = check_search(ix, dim, B, k);
    if (st != GVDB_OK) return st;
    if (B == 0) return GVDB_OK;
    if (!queries || !out_n || (k && (!out_ids || !out_scores)) || (n_allowed && !allowed))
        return fail(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    std::vector<uint32_t> rows;
    rows.reserve((size_t)std::min<uint64_t>(n_allowed, ix->n));
    for (uint64_t i = 0; i < n_allowed; ++i) {
        auto it = ix->id_row.find(allowed[i]);
        if (it != ix->id_row.end()) rows.push_back((uint32_t)it->second);
    }
    std::sort(rows.begin(), rows.end());
    rows.erase(std::unique(rows.begin(), rows.end()), rows.end());
    const uint64_t M = rows.size();
    if (k == 0 || M == 0) {
        memset(out_n, 0, B * 4);
        return GVDB_OK;
    }
    // sp == NULL: the exact scan of the allowed rows (BQ with the default ratio
    // would keep only R = 0.1 M candidates of a small allowed set)
    gvdb_search_params sp{};
    sp.metric = GVDB_METRIC_COSINE;
    sp.mode = GVDB_SEARCH_FLAT;
    sp.rescore_ratio = 0.1f;
    if (sp_in) sp = *sp_in;
    const int kind = sp.metric == GVDB_METRIC_L2 ? kScoreL2
                     : sp.metric == GVDB_METRIC_COSINE_DISTANCE ? kScoreCosineDistance
                                                                 : kScoreCosine;
    const int descending = kind == kScoreCosine;
    if ((st = set_device(ix->device)) != GVDB_OK) return st;
    WsGuard g(ix->device);
    if (!g.w) return fail(GVDB_ERR_DEVICE, "workspace");
    Workspace& ws = *g.w;
    hipStream_t s = ws.stream;
    g.begin(s);
    HIP_TRY(hipStreamSynchronize(ix->stream), "sync mutations");
    HIP_TRY(ws.q.ensure(B * dim * 4), "alloc queries");
    HIP_TRY(ws.flt_rows.ensure(M * 4), "alloc filter rows");
    HIP_TRY(ws.out_ids.ensure(B * k * 8), "alloc out");
    HIP_TRY(ws.out_scores.ensure(B * k * 4), "alloc out");
    HIP_TRY(ws.out_n.ensure(B * 4), "alloc out");
    HIP_TRY(hipMemcpyAsync(ws.q.p, queries, B * dim * 4, hipMemcpyHostToDevice, s), "upload queries");
    HIP_TRY(hipMemcpyAsync(ws.flt_rows.p, rows.data(), M * 4, hipMemcpyHostToDevice, s), "upload filter rows");
    if (sp.mode == GVDB_SEARCH_FLAT) {
        std::vector<uint64_t> sub_ids(M);
        for (uint64_t j = 0; j < M; ++j) sub_ids[j] = ix->h_ids[rows[j]];
        const uint64_t per_q = M * 4;
        const uint64_t G = std::max<uint64_t>(1, std::min<uint64_t>(B, kFlatScoreBytes / per_q));
        HIP_TRY(ws.qnorm.ensure(B * 4), "alloc qnorm");
        HIP_TRY(ws.flt_ids.ensure(M * 8), "alloc filter ids");
        HIP_TRY(ws.scores.ensure(G * per_q), "alloc filtered scores");
        HIP_TRY(ws.flags.ensure(16), "alloc flags");
        HIP_TRY(ws.sort_tmp.ensure(flat_select_bytes((uint32_t)M)), "alloc sort tmp");
        HIP_TRY(hipMemsetAsync(ws.flags.p, 0, 16, s), "memset flags");
        HIP_TRY(hipMemcpyAsync(ws.flt_ids.p, sub_ids.data(), M * 8, hipMemcpyHostToDevice, s), "upload filter ids");
        HIP_TRY(launch_row_norms(ws.q.as<float>(), B, dim, ws.qnorm.as<float>(), s), "qnorm");
        for (uint64_t g0 = 0; g0 < B; g0 += G) {
            const uint32_t bg = (uint32_t)std::min<uint64_t>(G, B - g0);
            HIP_TRY(launch_flat_scores(ws.q.as<float>() + g0 * dim, bg, ws.qnorm.as<float>() + g0, ix->rows,
                                       (uint32_t)M, dim, ix->norms, kind, ws.flt_rows.as<uint32_t>(),
                                       ws.scores.as<float>(), s),
                    "filtered scores");
            HIP_TRY(launch_flat_select(ws.scores.as<float>(), bg, (uint32_t)M, (uint32_t)k, descending, 0, 0.0f,
                                       ws.flt_ids.as<uint64_t>(), ws.out_ids.as<uint64_t>() + g0 * k,
                                       ws.out_scores.as<float>() + g0 * k, ws.out_n.as<uint32_t>() + g0,
                                       ws.sort_tmp.p, ws.sort_tmp.n, ws.flags.as<uint32_t>() + 1, s),
                    "filtered select");
        }
    } else {
        HIP_TRY(ws.flt_codes.ensure(M * code_w4(dim) * 16), "alloc filter codes");
        HIP_TRY(launch_gather_code_rows(ix->codes, ix->cap, ws.flt_rows.as<uint32_t>(), (uint32_t)M, dim,
                                        ws.flt_codes.as<uint4>(), s),
                "gather filter codes");
        uint64_t R = sp.rescore_count ? sp.rescore_count : rust_f32_as_usize((float)M * sp.rescore_ratio);
        R = std::min<uint64_t>(std::max<uint64_t>(R, k), M);
        BqSearchArgs a{};
        a.v = ShardView{ix->rows, dim, ix->norms, ws.flt_codes.as<uint4>(), M, (uint32_t)M, dim, ix->ids, 0};
        a.d_q = ws.q.as<float>();
        a.qlen = dim;
        a.B = (uint32_t)B;
        a.thr = ix->thr;
        a.dims_match = true;
        a.R = (uint32_t)R;
        a.kout = (uint32_t)k;
        a.kind = kind;
        a.descending = descending;
        a.d_out_ids = ws.out_ids.as<uint64_t>();
        a.d_out_scores = ws.out_scores.as<float>();
        a.d_out_n = ws.out_n.as<uint32_t>();
        a.row_map = ws.flt_rows.as<uint32_t>();
        if ((st = bq_search(a, ws, s)) != GVDB_OK) return st;
    }
    HIP_TRY(hipMemcpyAsync(out_ids, ws.out_ids.p, B * k * 8, hipMemcpyDeviceToHost, s), "download ids");
    HIP_TRY(hipMemcpyAsync(out_scores, ws.out_scores.p, B * k * 4, hipMemcpyDeviceToHost, s), "download scores");
    HIP_TRY(hipMemcpyAsync(out_n, ws.out_n.p, B * 4, hipMemcpyDeviceToHost, s), "download n");
    HIP_TRY(hipStreamSynchronize(s), "sync");
    zero_past_counts(out_ids, out_scores, out_n, B, k);
    return check_poisoned(out_n, B);
}

gvdb_status gvdb_index_search_device(const gvdb_index* ix, const float* d_queries, uint64_t B, uint32_t dim, uint64_t k,
                                     const gvdb_search_params* sp, uint64_t* d_out_ids, float* d_out_scores,
                                     uint32_t* d_out_n, void* stream) {
    gvdb_status st = check_search(ix, dim, B, k);
    if (st != GVDB_OK) return st;
    if (B == 0 || k == 0) return GVDB_OK;
    if (!d_queries || !d_out_ids || !d_out_scores) return fail(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    if ((st = set_device(ix->device)) != GVDB_OK) return st;
    WsGuard g(ix->device);
    if (!g.w) return fail(GVDB_ERR_DEVICE, "workspace");
    hipStream_t s = (hipStream_t)stream;  // NULL = the legacy default stream (orders with the caller's work)
    g.begin(s);
    UseGuard ug{ix, s};
    return index_search_impl(ix, d_queries, B, dim, k, sp, d_out_ids, d_out_scores, d_out_n, *g.w, s, false);
}

gvdb_status gvdb_index_bq_topr_device(const gvdb_index* ix, const float* d_queries, uint64_t B, uint32_t dim, uint64_t R,
                                      uint64_t* d_out_rows, uint32_t* d_out_dist, void* stream) {
    gvdb_status st = check_search(ix, dim, B, R);
    if (st != GVDB_OK) return st;
    if (B == 0 || R == 0) return GVDB_OK;
    if (R > ix->n) return fail(GVDB_ERR_INVALID_ARGUMENT, "R exceeds the number of rows");
    if (!d_queries || !d_out_rows || !d_out_dist) return fail(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    if ((st = set_device(ix->device)) != GVDB_OK) return st;
    WsGuard g(ix->device);
    if (!g.w) return fail(GVDB_ERR_DEVICE, "workspace");
    Workspace& ws = *g.w;
    hipStream_t s = (hipStream_t)stream;  // NULL = the legacy default stream
    g.begin(s);
    UseGuard ug{ix, s};
    const uint32_t W4 = code_w4(dim);
    const uint32_t RR = (uint32_t)R;
    HIP_TRY(ws.qcodes.ensure(B * W4 * 16), "alloc");
    Stage1Args s1{};
    st = prepare_stage1(ws, s1, (uint32_t)B, dim, RR, (uint32_t)ix->n, s, RR <= kSelectLdsCap);
    if (st != GVDB_OK) return st;
    HIP_TRY(launch_pack(d_queries, B, dim, ix->thr, ws.qcodes.p, kPackWordsAoS, 0, 0, s), "pack queries");
    if (RR <= kSelectLdsCap) {
        s1.codes = ix->codes;
        s1.cap = ix->cap;
        s1.N = (uint32_t)ix->n;
        s1.D = dim;
        s1.qcodes = ws.qcodes.as<uint4>();
        s1.B = (uint32_t)B;
        s1.R = RR;
        HIP_TRY(launch_stage1_fast(s1, s), "stage1");
        HIP_TRY(debug_keep_thr(s1.thr, (uint32_t)B, s, s1.any_fail), "copy thresholds");
    } else {
        HIP_TRY(ws.slow.ensure(stage1_slow_bytes((uint32_t)ix->n)), "alloc slow");
        for (uint64_t q = 0; q < B; ++q)
            HIP_TRY(launch_stage1_slow(ix->codes, ix->cap, (uint32_t)ix->n, dim, ws.qcodes.as<uint4>() + q * W4, RR,
                                       ws.s1_rows.as<uint32_t>() + q * R, ws.s1_dist.as<uint32_t>() + q * R, ws.slow.p,
                                       ws.slow.n, s),
                    "stage1 slow");
    }
    HIP_TRY(launch_widen(ws.s1_rows.as<uint32_t>(), d_out_rows, B * R, s), "widen rows");
    HIP_TRY(hipMemcpyAsync(d_out_dist, ws.s1_dist.p, B * R * 4, hipMemcpyDeviceToDevice, s), "dist");
    return GVDB_OK;
}

gvdb_status gvdb_index_remove(gvdb_index* ix, uint64_t id, int32_t* removed) {
    if (!ix) return fail(GVDB_ERR_INVALID_ARGUMENT, "null index");
    if (removed) *removed = 0;
    auto it = ix->id_row.find(id);
    if (it == ix->id_row.end()) return GVDB_OK;  // Ok(false) (index.rs:282-284)
    gvdb_status st = quiesce(ix);
    if (st != GVDB_OK) return st;
    const uint64_t gone = it->second;
    ix->id_row.erase(it);
    // Keep rows that still map to an id, in order (index.rs:248-258: orphans
    // have no id and vanish too).
    std::vector<uint64_t> map;
    map.reserve(ix->n);
    for (uint64_t r = 0; r < ix->n; ++r)
        if (r != gone && ix->h_ids[r] != kOrphan) map.push_back(r);
    const uint64_t m = map.size();
    if (m == 0) {  // all vectors deleted: index unbuilt (index.rs:271-274)
        (void)hipStreamSynchronize(ix->stream);
        uint32_t dim = ix->dim;
        ix->free_all();
        ix->dim = dim;
        ix->h_ids.clear();
        ix->id_row.clear();
        if (removed) *removed = 1;
        return GVDB_OK;
    }
    const uint64_t cap = std::max<uint64_t>(m, 1024);
    const uint32_t D = ix->dim, W4 = ix->w4();
    float *nrows = nullptr, *nnorms = nullptr;
    uint4* ncodes = nullptr;
    uint64_t *nids = nullptr, *dmap = nullptr;
    hipError_t e = hipMalloc((void**)&nrows, cap * D * 4);
    if (e == hipSuccess) e = hipMalloc((void**)&ncodes, cap * W4 * 16);
    if (e == hipSuccess) e = hipMalloc((void**)&nnorms, cap * 4);
    if (e == hipSuccess) e = hipMalloc((void**)&nids, cap * 8);
    if (e == hipSuccess) e = hipMalloc((void**)&dmap, m * 8);
    if (e != hipSuccess) {
        for (void* p : {(void*)nrows, (void*)ncodes, (void*)nnorms, (void*)nids, (void*)dmap})
            if (p) (void)hipFree(p);
        return dev_fail(e, "remove: allocation");
    }
    HIP_TRY(hipMemcpyAsync(dmap, map.data(), m * 8, hipMemcpyHostToDevice, ix->stream), "remove map");
    // codes: plane stride changes from old cap to new cap
    HIP_TRY(launch_gather(ix->rows, nrows, ix->codes, ncodes, ix->norms, nnorms, ix->ids, nids, dmap, m, cap, D,
                          ix->stream),
            "remove gather");
    HIP_TRY(hipStreamSynchronize(ix->stream), "remove sync");
    (void)hipFree(dmap);
    std::vector<uint64_t> nh(m);
    for (uint64_t i = 0; i < m; ++i) nh[i] = ix->h_ids[map[i]];
    ix->free_all();
    ix->rows = nrows;
    ix->codes = ncodes;
    ix->norms = nnorms;
    ix->ids = nids;
    ix->cap = cap;
    ix->n = m;
    ix->h_ids.swap(nh);
    ix->id_row.clear();
    for (uint64_t r = 0; r < m; ++r) ix->id_row.emplace(ix->h_ids[r], r);
    if (removed) *removed = 1;
    return GVDB_OK;
}

uint64_t gvdb_index_len(const gvdb_index* ix) { return ix ? ix->id_row.size() : 0; }

int32_t gvdb_index_is_empty(const gvdb_index* ix) { return gvdb_index_len(ix) == 0; }

void gvdb_index_clear(gvdb_index* ix) {
    if (!ix) return;
    (void)quiesce(ix);
    ix->free_all();
    ix->dim = 0;  // dimension = None (index.rs:304-309)
    ix->h_ids.clear();
    ix->id_row.clear();
}

gvdb_status gvdb_index_get_stats(const gvdb_index* ix, gvdb_index_stats* out) {
    if (!ix || !out) return fail(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    out->vector_count = gvdb_index_len(ix);
    out->dimension = ix->dim;
    out->memory_usage = ix->n * (uint64_t)ix->dim * 4;  // vectors.len() * dim * 4 (index.rs:318-320)
    out->device_bytes = ix->device_bytes();
    return GVDB_OK;
}

const float* gvdb_index_device_rows(const gvdb_index* ix) { return ix ? ix->rows : nullptr; }

gvdb_status gvdb_index_export(const gvdb_index* ix, float* rows, uint64_t* ids, uint64_t cap, uint64_t* n_out) {
    if (!ix || !n_out) return fail(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    uint64_t live = 0;
    for (uint64_t r = 0; r < ix->n; ++r) live += ix->h_ids[r] != kOrphan;
    *n_out = live;
    if (live == 0) return GVDB_OK;
    if (cap < live) return fail(GVDB_ERR_INVALID_ARGUMENT, "export capacity below the live row count");
    if (!rows || !ids) return fail(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    HIP_TRY(hipSetDevice(ix->device), "set device");
    HIP_TRY(hipStreamSynchronize(ix->stream), "sync mutations");
    const size_t rb = (size_t)ix->dim * 4;
    // copy runs of live rows straight into place
    uint64_t out = 0, r = 0;
    while (r < ix->n) {
        if (ix->h_ids[r] == kOrphan) {
            ++r;
            continue;
        }
        uint64_t e = r;
        while (e < ix->n && ix->h_ids[e] != kOrphan) ids[out + (e - r)] = ix->h_ids[e], ++e;
        HIP_TRY(hipMemcpy(rows + out * ix->dim, ix->rows + r * ix->dim, (e - r) * rb, hipMemcpyDeviceToHost),
                "export rows");
        out += e - r;
        r = e;
    }
    return GVDB_OK;
}

// ---- kernel timing -------------------------------------------------------------------
void gvdb_timing_enable(int32_t on) {
    std::lock_guard<std::mutex> g(timing().mu);
    timing().on = on != 0;
}

void gvdb_timing_reset(void) {
    std::lock_guard<std::mutex> g(timing().mu);
    timing_drain_locked(timing().pending.size());
    for (int i = 0; i < kTimN; ++i) {
        timing().ms[i] = 0;
        timing().n[i] = 0;
    }
}

gvdb_status gvdb_timing_read(uint32_t which, double* total_ms, uint64_t* launches) {
    if (which >= (uint32_t)kTimN || !total_ms || !launches) return fail(GVDB_ERR_INVALID_ARGUMENT, "bad timing slot");
    std::lock_guard<std::mutex> g(timing().mu);
    timing_drain_locked(timing().pending.size());
    *total_ms = timing().ms[which];
    *launches = timing().n[which];
    return GVDB_OK;
}

// ---- BinaryQuantizer ---------------------------------------------------------------
gvdb_status gvdb_bq_quantize_device(const float* d_rows, uint64_t n, uint32_t D, float threshold, uint8_t* d_out,
                                    void* stream) {
    if (n == 0) return GVDB_OK;
    if (!d_rows || !d_out) return fail(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    HIP_TRY(launch_pack(d_rows, n, D, threshold, d_out, kPackBytesAoS, 0, 0, (hipStream_t)stream), "pack");
    return GVDB_OK;
}

gvdb_status gvdb_bq_quantize(const float* rows, uint64_t n, uint32_t D, float threshold, uint8_t* out) {
    if (n == 0 || D == 0) return GVDB_OK;
    if (!rows || !out) return fail(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    WsGuard g(0);
    if (!g.w) return fail(GVDB_ERR_DEVICE, "workspace");
    Workspace& ws = *g.w;
    g.begin(ws.stream);
    const size_t nb = (D + 7u) / 8u;
    HIP_TRY(ws.rows.ensure(n * D * 4), "alloc");
    HIP_TRY(ws.misc.ensure(n * nb), "alloc");
    HIP_TRY(hipMemcpyAsync(ws.rows.p, rows, n * D * 4, hipMemcpyHostToDevice, ws.stream), "upload");
    HIP_TRY(launch_pack(ws.rows.as<float>(), n, D, threshold, ws.misc.p, kPackBytesAoS, 0, 0, ws.stream), "pack");
    HIP_TRY(hipMemcpyAsync(out, ws.misc.p, n * nb, hipMemcpyDeviceToHost, ws.stream), "download");
    HIP_TRY(hipStreamSynchronize(ws.stream), "sync");
    return GVDB_OK;
}

gvdb_status gvdb_bq_hamming(const uint8_t* a, const uint8_t* b, uint64_t n, uint32_t D, uint32_t* out) {
    if (n == 0) return GVDB_OK;
    if (!a || !b || !out) return fail(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    WsGuard g(0);
    if (!g.w) return fail(GVDB_ERR_DEVICE, "workspace");
    Workspace& ws = *g.w;
    g.begin(ws.stream);
    const size_t nb = (D + 7u) / 8u;
    HIP_TRY(ws.misc.ensure(2 * n * nb + n * 4 + 512), "alloc");
    uint8_t* da = ws.misc.as<uint8_t>();
    uint8_t* db = da + n * nb;
    uint32_t* dout = (uint32_t*)(((uintptr_t)(db + n * nb) + 255) & ~(uintptr_t)255);
    HIP_TRY(hipMemcpyAsync(da, a, n * nb, hipMemcpyHostToDevice, ws.stream), "upload");
    HIP_TRY(hipMemcpyAsync(db, b, n * nb, hipMemcpyHostToDevice, ws.stream), "upload");
    HIP_TRY(launch_hamming_pairs(da, db, n, D, dout, ws.stream), "hamming");
    HIP_TRY(hipMemcpyAsync(out, dout, n * 4, hipMemcpyDeviceToHost, ws.stream), "download");
    HIP_TRY(hipStreamSynchronize(ws.stream), "sync");
    return GVDB_OK;
}

gvdb_status gvdb_bq_multi_stage_search(const uint8_t* q_bits, uint32_t qdim, const uint8_t* c_bits, uint32_t cdim,
                                       uint64_t N, const float* q, uint64_t qlen, const float* cands, uint64_t clen,
                                       float rescore_ratio, uint64_t* out_idx, float* out_cos, uint64_t* out_n) {
    if (!out_n) return fail(GVDB_ERR_INVALID_ARGUMENT, "out_n is null");
    *out_n = 0;
    if (N > 0xFFFFFFFFull) return fail(GVDB_ERR_INVALID_ARGUMENT, "more than 2^32 candidates");
    // len check (quantization.rs:158-162) is structural here: one N for both.
    const bool dims_match = qdim == cdim;
    if (dims_match && cdim == 0 && N >= 2)
        return fail(GVDB_ERR_QUANTIZATION, "dimension 0: similarity is NaN and the reference sort panics");
    uint64_t R = std::min<uint64_t>(rust_f32_as_usize((float)N * rescore_ratio), N);
    if (R == 0 || N == 0) return GVDB_OK;
    if (!q_bits || !c_bits || !q || !cands || !out_idx || !out_cos)
        return fail(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    WsGuard g(0);
    if (!g.w) return fail(GVDB_ERR_DEVICE, "workspace");
    Workspace& ws = *g.w;
    hipStream_t s = ws.stream;
    g.begin(s);
    const uint32_t W4 = code_w4(cdim);
    const size_t nb = (cdim + 7u) / 8u;
    // upload: candidate rows + norms, codes (SoA from Msb0 bytes), query
    HIP_TRY(ws.rows.ensure(std::max<size_t>(N * clen * 4, 4)), "alloc rows");
    HIP_TRY(ws.norms.ensure(N * 4), "alloc norms");
    HIP_TRY(ws.codes.ensure(N * W4 * 16 + N * nb + 16), "alloc codes");
    HIP_TRY(ws.q.ensure(std::max<size_t>(qlen * 4, 4)), "alloc q");
    HIP_TRY(ws.out_ids.ensure(R * 8), "alloc out");
    HIP_TRY(ws.out_scores.ensure(R * 4), "alloc out");
    HIP_TRY(ws.misc.ensure(W4 * 16 + nb + 16), "alloc qbits");
    if (clen) HIP_TRY(hipMemcpyAsync(ws.rows.p, cands, N * clen * 4, hipMemcpyHostToDevice, s), "upload cands");
    if (qlen) HIP_TRY(hipMemcpyAsync(ws.q.p, q, qlen * 4, hipMemcpyHostToDevice, s), "upload q");
    HIP_TRY(launch_row_norms(ws.rows.as<float>(), N, (uint32_t)clen, ws.norms.as<float>(), s), "norms");
    uint32_t* d_qwords = nullptr;
    if (dims_match && cdim) {
        uint8_t* cbytes = ws.codes.as<uint8_t>() + N * W4 * 16;
        HIP_TRY(hipMemcpyAsync(cbytes, c_bits, N * nb, hipMemcpyHostToDevice, s), "upload codes");
        HIP_TRY(launch_bytes_to_soa(cbytes, N, cdim, ws.codes.as<uint4>(), N, 0, s), "codes to SoA");
        uint8_t* qb = ws.misc.as<uint8_t>() + W4 * 16;
        HIP_TRY(hipMemcpyAsync(qb, q_bits, nb, hipMemcpyHostToDevice, s), "upload qbits");
        HIP_TRY(launch_bytes_to_words(qb, 1, cdim, ws.misc.as<uint32_t>(), s), "qbits to words");
        d_qwords = ws.misc.as<uint32_t>();
    }
    BqSearchArgs a{};
    a.v = ShardView{ws.rows.as<float>(), clen, ws.norms.as<float>(), ws.codes.as<uint4>(), N, (uint32_t)N, cdim,
                    nullptr, 0};
    a.d_q = ws.q.as<float>();
    a.qlen = qlen;
    a.B = 1;
    a.d_qwords = d_qwords;
    a.dims_match = dims_match && cdim;
    a.R = (uint32_t)R;
    a.kout = (uint32_t)R;
    a.kind = kScoreCosine;
    a.descending = 1;
    a.d_out_ids = ws.out_ids.as<uint64_t>();
    a.d_out_scores = ws.out_scores.as<float>();
    HIP_TRY(ws.out_n.ensure(4), "alloc out");
    a.d_out_n = ws.out_n.as<uint32_t>();
    gvdb_status st = bq_search(a, ws, s);
    if (st != GVDB_OK) return st;
    uint32_t got = 0;
    HIP_TRY(hipMemcpyAsync(out_idx, ws.out_ids.p, R * 8, hipMemcpyDeviceToHost, s), "download idx");
    HIP_TRY(hipMemcpyAsync(out_cos, ws.out_scores.p, R * 4, hipMemcpyDeviceToHost, s), "download cos");
    HIP_TRY(hipMemcpyAsync(ws.h_flags, ws.out_n.p, 4, hipMemcpyDeviceToHost, s), "download n");
    HIP_TRY(hipStreamSynchronize(s), "sync");
    got = ws.h_flags[0];
    if ((st = check_poisoned(&got, 1)) != GVDB_OK) return st;
    *out_n = R;
    return GVDB_OK;
}

// ---- flat scan -----------------------------------------------------------------
gvdb_status gvdb_flat_search(const float* queries, uint64_t B, const float* rows, uint64_t N, uint32_t D, uint64_t limit,
                             uint32_t metric, int32_t has_threshold, float threshold, uint64_t* out_idx,
                             float* out_scores, uint32_t* out_n) {
    if (B == 0) return GVDB_OK;
    if (!queries || !out_n || (N && !rows) || (limit && (!out_idx || !out_scores)))
        return fail(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    if (N > 0xFFFFFFFFull) return fail(GVDB_ERR_INVALID_ARGUMENT, "more than 2^32 rows");
    if (N == 0 || limit == 0) {
        memset(out_n, 0, B * 4);
        return GVDB_OK;
    }
    WsGuard g(0);
    if (!g.w) return fail(GVDB_ERR_DEVICE, "workspace");
    Workspace& ws = *g.w;
    hipStream_t s = ws.stream;
    g.begin(s);
    const int kind = metric == GVDB_METRIC_L2 ? kScoreL2
                     : metric == GVDB_METRIC_COSINE_DISTANCE ? kScoreCosineDistance
                                                             : kScoreCosine;
    HIP_TRY(ws.rows.ensure(N * D * 4 + 4), "alloc rows");
    HIP_TRY(ws.norms.ensure(N * 4), "alloc norms");
    HIP_TRY(ws.q.ensure(B * D * 4 + 4), "alloc q");
    HIP_TRY(ws.qnorm.ensure(B * 4), "alloc qnorm");
    HIP_TRY(ws.scores.ensure(B * N * 4), "alloc scores");
    HIP_TRY(ws.out_ids.ensure(B * limit * 8), "alloc out");
    HIP_TRY(ws.out_scores.ensure(B * limit * 4), "alloc out");
    HIP_TRY(ws.out_n.ensure(B * 4), "alloc out");
    HIP_TRY(ws.flags.ensure(16), "alloc flags");
    HIP_TRY(ws.sort_tmp.ensure(flat_select_bytes((uint32_t)N)), "alloc sort");
    HIP_TRY(hipMemsetAsync(ws.flags.p, 0, 16, s), "memset");
    if (D) HIP_TRY(hipMemcpyAsync(ws.rows.p, rows, N * D * 4, hipMemcpyHostToDevice, s), "upload rows");
    if (D) HIP_TRY(hipMemcpyAsync(ws.q.p, queries, B * D * 4, hipMemcpyHostToDevice, s), "upload q");
    HIP_TRY(launch_row_norms(ws.rows.as<float>(), N, D, ws.norms.as<float>(), s), "norms");
    HIP_TRY(launch_row_norms(ws.q.as<float>(), B, D, ws.qnorm.as<float>(), s), "qnorm");
    HIP_TRY(launch_flat_scores(ws.q.as<float>(), (uint32_t)B, ws.qnorm.as<float>(), ws.rows.as<float>(), (uint32_t)N, D,
                               ws.norms.as<float>(), kind, nullptr, ws.scores.as<float>(), s),
            "flat scores");
    HIP_TRY(launch_flat_select(ws.scores.as<float>(), (uint32_t)B, (uint32_t)N, (uint32_t)limit, kind == kScoreCosine,
                               has_threshold && kind == kScoreCosine, threshold, nullptr, ws.out_ids.as<uint64_t>(),
                               ws.out_scores.as<float>(), ws.out_n.as<uint32_t>(), ws.sort_tmp.p, ws.sort_tmp.n,
                               ws.flags.as<uint32_t>() + 1, s),
            "flat select");
    HIP_TRY(hipMemcpyAsync(out_idx, ws.out_ids.p, B * limit * 8, hipMemcpyDeviceToHost, s), "download");
    HIP_TRY(hipMemcpyAsync(out_scores, ws.out_scores.p, B * limit * 4, hipMemcpyDeviceToHost, s), "download");
    HIP_TRY(hipMemcpyAsync(out_n, ws.out_n.p, B * 4, hipMemcpyDeviceToHost, s), "download");
    HIP_TRY(hipStreamSynchronize(s), "sync");
    return GVDB_OK;
}

gvdb_status gvdb_index_bq_candidates_device(const gvdb_index* ix, const float* d_queries, uint64_t B, uint32_t dim,
                                            uint64_t R, uint64_t* d_out_ids, uint32_t* d_out_dist,
                                            float* d_out_scores, void* stream) {
    gvdb_status st = check_search(ix, dim, B, R);
    if (st != GVDB_OK) return st;
    if (B == 0 || R == 0) return GVDB_OK;
    if (R > ix->n) return fail(GVDB_ERR_INVALID_ARGUMENT, "R exceeds the number of rows");
    if (!d_queries || !d_out_ids || !d_out_dist || !d_out_scores) return fail(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    if ((st = set_device(ix->device)) != GVDB_OK) return st;
    WsGuard g(ix->device);
    if (!g.w) return fail(GVDB_ERR_DEVICE, "workspace");
    hipStream_t s = (hipStream_t)stream;  // NULL = the legacy default stream (orders with the caller's work)
    g.begin(s);
    UseGuard ug{ix, s};
    BqSearchArgs a{};
    a.v = ShardView{ix->rows, dim, ix->norms, ix->codes, ix->cap, (uint32_t)ix->n, dim, ix->ids, 0};
    a.d_q = d_queries;
    a.qlen = dim;
    a.B = (uint32_t)B;
    a.thr = ix->thr;
    a.dims_match = true;
    a.R = (uint32_t)R;
    a.kout = (uint32_t)R;
    a.kind = kScoreCosine;
    a.descending = 1;
    a.d_out_ids = d_out_ids;
    a.d_out_scores = d_out_scores;
    a.d_out_dist = d_out_dist;
    return bq_search(a, *g.w, s);
}

gvdb_status gvdb_bq_shard_merge_device(const uint64_t* d_gids, const uint32_t* d_dist, const float* d_cos,
                                       const uint32_t* d_counts, uint64_t G, uint64_t B, uint64_t stride, uint64_t R,
                                       uint64_t k, uint64_t* d_out_ids, float* d_out_scores, uint32_t* d_out_n,
                                       void* stream) {
    if (B == 0) return GVDB_OK;
    if (G * stride > kSortLdsCap) return fail(GVDB_ERR_INVALID_ARGUMENT, "G*stride exceeds 4096");
    if (!d_gids || !d_dist || !d_cos || !d_counts || !d_out_ids || !d_out_scores)
        return fail(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    WsGuard g(0);
    if (!g.w) return fail(GVDB_ERR_DEVICE, "workspace");
    hipStream_t s = (hipStream_t)stream;  // NULL = the legacy default stream (orders with the caller's work)
    g.begin(s);
    HIP_TRY(g.w->flags.ensure(16), "alloc flags");
    HIP_TRY(hipMemsetAsync(g.w->flags.p, 0, 16, s), "memset flags");
    HIP_TRY(launch_bq_shard_merge(d_gids, d_dist, d_cos, d_counts, (uint32_t)G, (uint32_t)B, (uint32_t)stride,
                                  (uint32_t)R, (uint32_t)k, d_out_ids, d_out_scores, d_out_n,
                                  g.w->flags.as<uint32_t>() + 1, s),
            "shard merge");
    HIP_TRY(hipMemcpyAsync(g.w->h_flags, g.w->flags.p, 8, hipMemcpyDeviceToHost, s), "flags");
    HIP_TRY(hipStreamSynchronize(s), "sync");
    if (g.w->h_flags[1]) return fail(GVDB_ERR_QUANTIZATION, "NaN score in merge");
    return GVDB_OK;
}

gvdb_status gvdb_bq_shard_merge_packed_device(const uint32_t* d_gathered, const uint32_t* d_counts, uint64_t G,
                                              uint64_t B, uint64_t R, uint64_t k, uint64_t* d_out_ids,
                                              float* d_out_scores, uint32_t* d_out_n, void* stream) {
    if (B == 0) return GVDB_OK;
    if (G * R > kSortLdsCap) return fail(GVDB_ERR_INVALID_ARGUMENT, "G*R exceeds 4096");
    if (!d_gathered || !d_counts || !d_out_ids || !d_out_scores) return fail(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    if (reinterpret_cast<uintptr_t>(d_gathered) % 8u) return fail(GVDB_ERR_INVALID_ARGUMENT, "gathered buffer not 8-byte aligned");
    WsGuard g(0);
    if (!g.w) return fail(GVDB_ERR_DEVICE, "workspace");
    hipStream_t s = (hipStream_t)stream;
    g.begin(s);
    const uint64_t BR = B * R;  // rank block: ids (2*BR words) | dist (BR) | cos (BR)
    HIP_TRY(g.w->flags.ensure(16), "alloc flags");
    HIP_TRY(hipMemsetAsync(g.w->flags.p, 0, 16, s), "memset flags");
    HIP_TRY(launch_bq_shard_merge(reinterpret_cast<const uint64_t*>(d_gathered), d_gathered + 2 * BR,
                                  reinterpret_cast<const float*>(d_gathered + 3 * BR), d_counts, (uint32_t)G,
                                  (uint32_t)B, (uint32_t)R, (uint32_t)R, (uint32_t)k, d_out_ids, d_out_scores, d_out_n,
                                  g.w->flags.as<uint32_t>() + 1, s, 2 * BR, 4 * BR),
            "packed shard merge");
    HIP_TRY(hipMemcpyAsync(g.w->h_flags, g.w->flags.p, 8, hipMemcpyDeviceToHost, s), "flags");
    HIP_TRY(hipStreamSynchronize(s), "sync");
    if (g.w->h_flags[1]) return fail(GVDB_ERR_QUANTIZATION, "NaN score in merge");
    return GVDB_OK;
}

gvdb_status gvdb_bq_shard_merge(const uint64_t* gids, const uint32_t* dist, const float* cosv, const uint32_t* counts,
                                uint64_t G, uint64_t B, uint64_t stride, uint64_t R, uint64_t k, uint64_t* out_ids,
                                float* out_scores, uint32_t* out_n) {
    // Host form of the same merge (used where the gathered lists are on the host).
    if (B == 0) return GVDB_OK;
    if (!gids || !dist || !cosv || !counts || !out_n || (k && (!out_ids || !out_scores)))
        return fail(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    struct E {
        uint32_t d;
        uint64_t gid;
        float c;
    };
    std::vector<E> all;
    for (uint64_t q = 0; q < B; ++q) {
        all.clear();
        for (uint64_t g = 0; g < G; ++g) {
            const uint64_t c = std::min<uint64_t>(counts[g * B + q], stride);
            for (uint64_t i = 0; i < c; ++i) {
                const uint64_t at = (g * B + q) * stride + i;
                all.push_back({dist[at], gids[at], cosv[at]});
            }
        }
        std::stable_sort(all.begin(), all.end(),
                         [](const E& a, const E& b) { return a.d != b.d ? a.d < b.d : a.gid < b.gid; });
        const uint64_t r = std::min<uint64_t>(R, all.size());
        all.resize(r);
        for (const E& e : all)
            if (e.c != e.c && r >= 2) return fail(GVDB_ERR_QUANTIZATION, "NaN score in merge");
        std::stable_sort(all.begin(), all.end(), [](const E& a, const E& b) { return a.c > b.c; });
        const uint64_t take = std::min<uint64_t>(k, r);
        for (uint64_t i = 0; i < take; ++i) {
            out_ids[q * k + i] = all[i].gid;
            out_scores[q * k + i] = all[i].c;
        }
        out_n[q] = (uint32_t)take;
    }
    return GVDB_OK;
}

// ---- shard merge -----------------------------------------------------------------
gvdb_status gvdb_topk_merge(const uint64_t* ids, const float* scores, const uint32_t* counts, uint64_t n_shards,
                            uint64_t B, uint64_t stride, uint64_t limit, int32_t descending, uint64_t* out_ids,
                            float* out_scores, uint32_t* out_n) {
    // Host merge: the reference's merge is host-side too (shard.rs:776-784).
    if (B == 0) return GVDB_OK;
    if (!ids || !scores || !counts || !out_n || (limit && (!out_ids || !out_scores)))
        return fail(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    std::vector<std::pair<float, uint64_t>> all;
    for (uint64_t q = 0; q < B; ++q) {
        all.clear();
        for (uint64_t s = 0; s < n_shards; ++s) {
            const uint64_t c = std::min<uint64_t>(counts[s * B + q], stride);
            for (uint64_t i = 0; i < c; ++i) {
                const uint64_t at = (s * B + q) * stride + i;
                all.push_back({scores[at], ids[at]});
            }
        }
        auto cmp = [descending](const std::pair<float, uint64_t>& a, const std::pair<float, uint64_t>& b) {
            return descending ? a.first > b.first : a.first < b.first;  // NaN compares as Equal
        };
        std::stable_sort(all.begin(), all.end(), cmp);
        const uint64_t n = std::min<uint64_t>(limit, all.size());
        for (uint64_t i = 0; i < n; ++i) {
            out_ids[q * limit + i] = all[i].second;
            out_scores[q * limit + i] = all[i].first;
        }
        out_n[q] = (uint32_t)n;
    }
    return GVDB_OK;
}

gvdb_status gvdb_topk_merge_device(const uint64_t* d_ids, const float* d_scores, const uint32_t* d_counts,
                                   uint64_t n_shards, uint64_t B, uint64_t stride, uint64_t limit, int32_t descending,
                                   uint64_t* d_out_ids, float* d_out_scores, uint32_t* d_out_n, void* stream) {
    if (B == 0) return GVDB_OK;
    if (n_shards * stride > kSortLdsCap) return fail(GVDB_ERR_INVALID_ARGUMENT, "n_shards*stride exceeds 4096");
    if (!d_ids || !d_scores || !d_counts || !d_out_n || (limit && (!d_out_ids || !d_out_scores)))
        return fail(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    hipStream_t s = (hipStream_t)stream;
    HIP_TRY(launch_topk_merge(d_ids, d_scores, d_counts, (uint32_t)n_shards, (uint32_t)B, (uint32_t)stride,
                              (uint32_t)limit, descending, d_out_ids, d_out_scores, d_out_n, s),
            "merge");
    return GVDB_OK;
}

// (diagnostics: they wait for the tier outcomes of the async searches still in flight)
uint64_t gvdb_flat_fallback_count(void) {
    tier_poll(true);
    return flat_fallbacks().load();
}
uint64_t gvdb_flat_i8_fallback_count(void) {
    tier_poll(true);
    return flat_fallbacks_i8().load();
}

}  // extern "C"


// Shared error reporting for the other translation units (gvdb_sparse.hip).
gvdb_status gvdb::report_status(gvdb_status s, const std::string& msg) { return fail(s, msg); }

int gvdb::index_device(const gvdb_index* ix) { return ix->device; }

// timing study: the last k_b1_tail phase clocks (GVDB_B1_CLK=1), 16 words
// tests only (not part of include/gvdb.h): thresholds T[0..B) of the last GVDB_DEBUG_THR=1 batch
extern "C" int gvdb_debug_stage1_thresholds(uint32_t* out, uint32_t B) {
    if (!debug_thr() || B > debug_thr_cap()) return -1;
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    return (int)hipMemcpy(out, debug_thr(), (size_t)B * 4, hipMemcpyDeviceToHost);
}
// tests only: 1 if a query of the last GVDB_DEBUG_THR=1 batch took the all-rows rescan
extern "C" int gvdb_debug_b1_coalesce(uint64_t* out) {  // [0] batches, [1] queries, [2] largest batch
    out[0] = g_b1_batches.load();
    out[1] = g_b1_queries.load();
    out[2] = g_b1_max.load();
    return 0;
}
extern "C" int gvdb_debug_deep_cert(uint64_t* out) {  // [0] certified batches, [1] sent to the rerank path
    if (!out) return 1;
    tier_poll(true);
    out[0] = deep_cert_count(0).load();
    out[1] = deep_cert_count(1).load();
    return 0;
}

extern "C" int gvdb_debug_stage1_rescanned(uint32_t* out) {
    if (!debug_fail()) return -1;
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    return (int)hipMemcpy(out, debug_fail(), 4, hipMemcpyDeviceToHost);
}
extern "C" int gvdb_debug_b1_clock(unsigned long long* out) {
    if (!debug_b1_clk()) return -1;
    return (int)hipMemcpy(out, debug_b1_clk(), 16 * 8, hipMemcpyDeviceToHost);
}

// Sharded-search building blocks (gvdb_shard.hip / gvdb_comm.hip).
void gvdb::index_track_use(const gvdb_index* ix, hipStream_t s) { track_use(ix, s); }

gvdb::ShardInfo gvdb::index_shard_info(const gvdb_index* ix) {
    ShardInfo si{};
    si.rows = ix->rows;
    si.norms = ix->norms;
    si.ids = ix->ids;
    si.n = ix->n;
    si.dim = ix->dim;
    si.device = ix->device;
    return si;
}

// This shard's exact stage-1 top-min(R, rows) by (Hamming asc, row asc) as
// sorted keys (d << 32 | row) into keys[q*R + i] (the exchange-1 block of the
// two-exchange sharded search).  An empty shard writes nothing (the caller
// sends count 0).  R <= kSelectLdsCap.
gvdb_status gvdb::shard_stage1_keys(const gvdb_index* ix, const float* d_q, uint64_t B, uint32_t dim, uint64_t R,
                                    uint64_t* keys, hipStream_t s) {
    if (!ix) return fail(GVDB_ERR_INVALID_ARGUMENT, "null index");
    if (ix->n == 0 || B == 0 || R == 0) return GVDB_OK;
    if (dim != ix->dim) return dim_mismatch(ix->dim, dim);
    if (ix->n > 0xFFFFFFFFull) return fail(GVDB_ERR_INDEX, "shard exceeds 2^32 rows");
    const uint32_t Rl = (uint32_t)std::min<uint64_t>(R, ix->n);
    if (Rl > kSelectLdsCap) return fail(GVDB_ERR_INVALID_ARGUMENT, "sharded search: R exceeds 8192");
    gvdb_status st = set_device(ix->device);
    if (st != GVDB_OK) return st;
    WsGuard g(ix->device);
    if (!g.w) return fail(GVDB_ERR_DEVICE, "workspace");
    Workspace& ws = *g.w;
    g.begin(s);
    UseGuard ug{ix, s};
    const uint32_t W4 = code_w4(dim);
    HIP_TRY(ws.qcodes.ensure(B * W4 * 16), "alloc qcodes");
    Stage1Args s1{};
    st = prepare_stage1(ws, s1, (uint32_t)B, dim, Rl, (uint32_t)ix->n, s, true);
    if (st != GVDB_OK) return st;
    if (s1.mfma_scan) {
        s1.qf32 = d_q;  // packed by k_qprep
        s1.qthr = ix->thr;
    } else {
        HIP_TRY(launch_pack(d_q, B, dim, ix->thr, ws.qcodes.p, kPackWordsAoS, 0, 0, s), "pack queries");
    }
    bool timed = false;
    {
        std::lock_guard<std::mutex> lk(timing().mu);
        timed = timing().on;
    }
    EvSet* ev = timed ? timing_events() : nullptr;
    s1.codes = ix->codes;
    s1.cap = ix->cap;
    s1.qcodes = ws.qcodes.as<uint4>();
    s1.keys_out = keys;
    s1.keys_stride = (uint32_t)R;  // the block's row stride is the global R (this shard may hold fewer rows)
    s1.ev = ev ? ev->e : nullptr;
    hipError_t e = launch_stage1_fast(s1, s);
    if (e == hipSuccess && ev) {
        // stage-2 slot of the timing: zero here (the sharded rerank is timed by the caller)
        (void)hipEventRecord(ev->e[5], s);
        timing_submit(ev);
    } else if (ev) {
        std::lock_guard<std::mutex> lk(timing().mu);
        timing().free_sets.push_back(ev);
    }
    if (e != hipSuccess) return dev_fail(e, "sharded stage 1");
    return GVDB_OK;
}

// Deep sharded search (R > kSelectLdsCap): this shard's exact stage-1
// top-min(R, rows) MEMBERSHIP (rows + Hamming, unordered: k_select_big; a
// shard of at most kSelectLdsCap rows: k_select's sorted list) into
// m_rows / m_dist [B][Rl], then its per-query Hamming histogram and count into
// the deep exchange-1 block (gvdb_shard.hip).  Nothing for an empty shard.
gvdb_status gvdb::shard_stage1_members(const gvdb_index* ix, const float* d_q, uint64_t B, uint32_t dim, uint64_t R,
                                       uint32_t* m_rows, uint32_t* m_dist, uint32_t* block1, hipStream_t s) {
    if (!ix) return fail(GVDB_ERR_INVALID_ARGUMENT, "null index");
    if (ix->n == 0 || B == 0 || R == 0) return GVDB_OK;
    if (dim != ix->dim) return dim_mismatch(ix->dim, dim);
    if (ix->n > 0xFFFFFFFFull) return fail(GVDB_ERR_INDEX, "shard exceeds 2^32 rows");
    if (dim >= 4096 || R > kBigRMax) return fail(GVDB_ERR_INVALID_ARGUMENT, "deep sharded search: dim < 4096, R <= 2^20");
    const uint32_t Rl = (uint32_t)std::min<uint64_t>(R, ix->n);
    gvdb_status st = set_device(ix->device);
    if (st != GVDB_OK) return st;
    WsGuard g(ix->device);
    if (!g.w) return fail(GVDB_ERR_DEVICE, "workspace");
    Workspace& ws = *g.w;
    g.begin(s);
    UseGuard ug{ix, s};
    const uint32_t W4 = code_w4(dim);
    HIP_TRY(ws.qcodes.ensure(B * W4 * 16), "alloc qcodes");
    ShardDenseLayout lay;
    const ShardDenseLayout* dl = shard_dense_layout(ix, B, R, dim, m_rows, &lay) ? &lay : nullptr;
    Stage1Args s1{};
    s1.dense_keep = dl ? 1 : 0;  // (before the plan: no workspace dense block)
    st = prepare_stage1(ws, s1, (uint32_t)B, dim, Rl, (uint32_t)ix->n, s, true, false);
    if (st != GVDB_OK) return st;
    if (dl && !s1.dense_sel) return fail(GVDB_ERR_DEVICE, "deep sharded stage 1: dense layout without a dense scan");
    if (s1.mfma_scan) {
        s1.qf32 = d_q;  // packed by k_qprep
        s1.qthr = ix->thr;
    } else {
        HIP_TRY(launch_pack(d_q, B, dim, ix->thr, ws.qcodes.p, kPackWordsAoS, 0, 0, s), "pack queries");
    }
    s1.codes = ix->codes;
    s1.cap = ix->cap;
    s1.qcodes = ws.qcodes.as<uint4>();
    s1.s1_rows = m_rows;
    s1.s1_dist = m_dist;
    if (s1.dense_sel) {  // k_select_dense writes the members' histogram itself (it holds the full one)
        s1.mhist = block1;
        s1.mcount = block1 + (uint64_t)B * (dim + 1u);
    }
    if (dl) {  // the dense block, the rule, |q| and the segment histograms stay in the scratch
        s1.dense = dl->dense;
        s1.dense_keep = 1;
        s1.tcut = dl->rule;
        s1.pc_out = dl->qpc;
        s1.seg_hist = dl->seg;
        s1.seg_n = dl->S;
        s1.seg_len = dl->L;
        s1.s1_rows = nullptr;
        s1.s1_dist = nullptr;
    }
    HIP_TRY(launch_stage1_fast(s1, s), "deep sharded stage 1");
    if (!s1.dense_sel)
        HIP_TRY(launch_shard_member_hist(m_dist, (uint32_t)B, Rl, dim + 1u, block1, s),
                "deep sharded stage 1 histogram");
    return GVDB_OK;
}

// stage1_plan's dense_sel decision for (D, R, N) under the current GVDB_SCAN / GVDB_DENSE_SEL
static bool plan_dense_sel(uint32_t D, uint32_t R, uint32_t N) {
    const char* scan = getenv("GVDB_SCAN");
    if (scan && strcmp(scan, "valu") == 0) return false;
    const char* ds = getenv("GVDB_DENSE_SEL");
    if (ds && strcmp(ds, "0") == 0) return false;
    return R > kSelectLdsCap && mfma_scan_supported(code_w4(D)) && (uint64_t)R * 64u >= N;
}

bool gvdb::shard_dense_layout(const gvdb_index* ix, uint64_t B, uint64_t R, uint32_t dim, void* scratch,
                              ShardDenseLayout* dl) {
    const char* env = getenv("GVDB_DEEP_DENSE");  // =0: the member-list form (A/B, tests)
    if (env && env[0] == '0') return false;
    if (!ix || !scratch || !dl || ix->n == 0 || ix->n > 0xFFFFFFFFull || B == 0 || dim != ix->dim || dim == 0 ||
        dim >= 4096 || R > kBigRMax)
        return false;
    const uint32_t n = (uint32_t)ix->n, Rl = (uint32_t)std::min<uint64_t>(R, n);
    if (!plan_dense_sel(dim, Rl, n)) return false;
    const uint64_t np = ((uint64_t)n + 31u) & ~31ull, H = dim + 1ull;
    if (2 * np > 8 * R || R < 12 + H) return false;  // the row within m_rows | m_dist; one segment at least
    uint32_t S = 0, L = 0;
    dense_segments(n, (uint32_t)std::min<uint64_t>(kDenseSegs, (R - 12) / H), &S, &L);
    if ((uint64_t)S * H + 12 > R) return false;
    uint32_t* base = (uint32_t*)scratch;
    uint32_t* m_cos = base + 4 * B * R;
    dl->S = S;
    dl->L = L;
    dl->np = (uint32_t)np;
    dl->n = n;
    dl->dense = (uint16_t*)base;
    dl->rule = m_cos + 4 * B;
    dl->qpc = m_cos + 8 * B;
    dl->seg = m_cos + 12 * B;
    return true;
}

// The certified deep phase 2 (gvdb_shard.hip, R > 8192): this rank's exact cosine
// top-K2 over its shard (flat_mx_search, rows), filtered by the rule of its owned
// rows that k_shard_deep_own wrote (tcut), gives its local top-min(k, own) entries
// whenever the list certifies them (k_deep_certify) -- instead of reranking
// ~R / G owned rows per query.  No host sync: the flat tier's failure word is
// folded into the certificate's, *dfail (a device word that must outlive the call:
// the caller's scratch), which gates the caller's rerank fallback on the device.
// Shards with orphan rows, k > 32 or fewer than kFxMinN rows are not eligible
// (*enqueued = false: the caller reranks ungated).
bool gvdb::shard_certified_eligible(const gvdb_index* ix, uint32_t dim, uint64_t k) {
    const char* env = getenv("GVDB_DEEP_CERT");
    return !(env && env[0] == '0') && ix && k >= 1 && k <= 32 && ix->n >= kFxMinN && ix->n <= 0xFFFFFFFFull &&
           ix->n == ix->id_row.size() && dim == ix->dim && dim > 0;
}

// The deep sharded form's exact cosine list, computed EARLY: enqueued by the
// stage-1 call on a second pooled stream, concurrently with the dense stage 1 --
// it reads nothing stage 1 writes -- into the caller's scratch (`list`: rows u64
// [B][K2] | scores f32 [B][K2] | counts u32 [B] | tier failure word), then joined
// by phase 2 through an event kept per scratch list.  K2 = 32 (phase 2's k is not
// known yet; k <= 16 certifies on it like the single-index search).
namespace {
constexpr uint32_t kEarlyK2 = 32;
struct EarlyFlat {
    std::mutex mu;
    std::unordered_map<const void*, hipEvent_t> ev;  // scratch list -> the list's completion
};
EarlyFlat& early_flat() {
    static EarlyFlat* e = new EarlyFlat();  // never destroyed: events may outlive static destructors
    return *e;
}
}  // namespace

size_t gvdb::shard_early_list_bytes(uint64_t B) { return (size_t)B * kEarlyK2 * 12 + (size_t)B * 4 + 16; }

gvdb_status gvdb::shard_deep_flat_early(const gvdb_index* ix, const float* d_q, uint64_t B, uint32_t dim, void* list,
                                        hipStream_t s) {
    {  // a list an earlier search left here unjoined is stale from now on
        std::lock_guard<std::mutex> lk(early_flat().mu);
        auto it = early_flat().ev.find(list);
        if (it != early_flat().ev.end()) {
            (void)hipEventDestroy(it->second);
            early_flat().ev.erase(it);
        }
    }
    // GVDB_DEEP_EARLY=1: enqueue the list early (A/B).  Off by default: with the dense stage 1
    // down to ~0.13 ms the second stream's event traffic costs more than the overlap gains
    // (10M, 8 shards, batch 64: 0.788 ms per rank with it, 0.720 without; stage-1 host
    // enqueue 81 vs 34 us per call)
    const char* env = getenv("GVDB_DEEP_EARLY");
    if (!(env && env[0] == '1') || !shard_certified_eligible(ix, dim, 1) || B == 0 || B > 0xFFFFFFFFull) return GVDB_OK;
    gvdb_status st = set_device(ix->device);
    if (st != GVDB_OK) return st;
    tier_poll();
    WsGuard g(ix->device);
    if (!g.w) return fail(GVDB_ERR_DEVICE, "workspace");
    Workspace& ws = *g.w;
    hipStream_t s2 = ws.stream;
    hipEvent_t e_in = nullptr, e_done = nullptr;
    HIP_TRY(hipEventCreateWithFlags(&e_in, hipEventDisableTiming), "event");
    HIP_TRY(hipEventCreateWithFlags(&e_done, hipEventDisableTiming), "event");
    struct EvDel {
        hipEvent_t& e;
        ~EvDel() {
            if (e) (void)hipEventDestroy(e);
        }
    } del_in{e_in}, del_done{e_done};
    HIP_TRY(hipEventRecord(e_in, s), "event");  // after the caller's queries
    g.begin(s2);
    HIP_TRY(hipStreamWaitEvent(s2, e_in, 0), "stream wait");
    UseGuard ug{ix, s2};
    char* p = (char*)list;
    uint64_t* frow = (uint64_t*)p;
    float* fsc = (float*)(p + (size_t)B * kEarlyK2 * 8);
    uint32_t* fn = (uint32_t*)(p + (size_t)B * kEarlyK2 * 12);
    uint32_t* lfail = fn + B;
    bool cert = false;
    uint32_t* flat_fail = nullptr;
    const bool i8 = ix->i8_skip.load() == 0;
    st = flat_mx_search(ix, d_q, (uint32_t)B, dim, kEarlyK2, kScoreCosine, 1, frow, fsc, fn, ws, s2, i8, &cert, true,
                        &flat_fail);
    if (st != GVDB_OK) return st;
    // the tier's failure word into the list (the pooled workspace may serve another call next)
    HIP_TRY(hipMemcpyAsync(lfail, flat_fail, 4, hipMemcpyDeviceToDevice, s2), "list failure word");
    HIP_TRY(hipEventRecord(e_done, s2), "event");
    std::lock_guard<std::mutex> lk(early_flat().mu);
    early_flat().ev[list] = e_done;
    e_done = nullptr;  // owned by the map now
    return GVDB_OK;
}

gvdb_status gvdb::shard_certified_phase2(const gvdb_index* ix, const float* d_q, uint64_t B, uint32_t dim, uint64_t k,
                                         const uint32_t* tcut, const uint32_t* own_cnt, const uint32_t* reff,
                                         const uint32_t* m_rows, const uint32_t* m_dist, uint32_t Rl,
                                         uint32_t* block2, uint32_t* dfail, void* early_list, hipStream_t s,
                                         bool* enqueued, const ShardDenseLayout* dl) {
    *enqueued = false;
    if (!shard_certified_eligible(ix, dim, k) || B == 0 || B > 0xFFFFFFFFull) return GVDB_OK;
    gvdb_status st = set_device(ix->device);
    if (st != GVDB_OK) return st;
    // the early list of this scratch (shard_deep_flat_early), if the stage-1 call made one
    hipEvent_t early = nullptr;
    if (early_list) {
        std::lock_guard<std::mutex> lk(early_flat().mu);
        auto it = early_flat().ev.find(early_list);
        if (it != early_flat().ev.end()) {
            early = it->second;
            early_flat().ev.erase(it);
        }
    }
    struct EvDel {
        hipEvent_t& e;
        ~EvDel() {
            if (e) (void)hipEventDestroy(e);
        }
    } del_early{early};
    WsGuard g(ix->device);
    if (!g.w) return fail(GVDB_ERR_DEVICE, "workspace");
    Workspace& ws = *g.w;
    g.begin(s);
    UseGuard ug{ix, s};
    tier_poll();
    const uint32_t W4 = code_w4(dim);
    uint32_t K2 = k <= 16 ? 32u : kDeepK2;
    HIP_TRY(ws.qcodes.ensure(B * W4 * 16), "alloc qcodes");
    HIP_TRY(launch_pack(d_q, B, dim, ix->thr, ws.qcodes.p, kPackWordsAoS, 0, 0, s), "pack queries");
    const uint64_t* frow;
    const float* fsc;
    const uint32_t* fn;
    const uint32_t* flat_fail = nullptr;
    if (early) {  // joined here: the list ran beside stage 1 and the exchange
        K2 = kEarlyK2;
        HIP_TRY(hipStreamWaitEvent(s, early, 0), "stream wait");
        const char* p = (const char*)early_list;
        frow = (const uint64_t*)p;
        fsc = (const float*)(p + (size_t)B * K2 * 8);
        fn = (const uint32_t*)(p + (size_t)B * K2 * 12);
        flat_fail = fn + B;
    } else {
        HIP_TRY(ws.deep.ensure((size_t)B * K2 * 12 + (size_t)B * 4 + 16), "alloc certified lists");
        char* p = ws.deep.as<char>();
        bool cert = false;
        uint32_t* ff = nullptr;
        const bool i8 = ix->i8_skip.load() == 0;
        st = flat_mx_search(ix, d_q, (uint32_t)B, dim, K2, kScoreCosine, 1, (uint64_t*)p, (float*)(p + (size_t)B * K2 * 8),
                            (uint32_t*)(p + (size_t)B * K2 * 12), ws, s, i8, &cert, true, &ff);
        if (st != GVDB_OK) return st;
        frow = (const uint64_t*)p;
        fsc = (const float*)(p + (size_t)B * K2 * 8);
        fn = (const uint32_t*)(p + (size_t)B * K2 * 12);
        flat_fail = ff;
    }
    HIP_TRY(hipMemsetAsync(dfail, 0, 4, s), "memset certify flag");
    HIP_TRY(launch_deep_certify(frow, fsc, fn, K2, tcut, ix->codes, ix->cap, W4, ws.qcodes.as<uint4>(), (uint32_t)B,
                                (uint32_t)k, 0u, ix->ids, nullptr, nullptr, nullptr, dfail, s, own_cnt, block2, reff,
                                dl ? nullptr : m_rows, dl ? nullptr : m_dist, Rl, flat_fail, dl ? dl->seg : nullptr,
                                dl ? dl->S : 0u, dl ? dl->L : 0u, dim + 1u, dl ? dl->dense : nullptr, dl ? dl->np : 0u),
            "certified deep phase 2");
    if ((st = tier_record(ix, dfail, kTierDeepCert, s)) != GVDB_OK) return st;
    *enqueued = true;
    return GVDB_OK;
}
