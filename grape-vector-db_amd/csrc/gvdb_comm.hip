// gvdb_comm.hip — RCCL communicator + exact sharded search (include/gvdb.h).
//
// Replaces ShardManager::search_vectors (src/distributed/shard.rs:760-786:
// fan out to every shard, concat, sort by score, truncate) inside one node:
// one process per GPU, each holding a contiguous row range of the corpus.
// gvdb_index_search_sharded_device composes the two-exchange protocol of
// gvdb_shard.hip with two ncclAllGather calls on the caller's stream:
//
//   BQ:    local stage-1 keys -> AllGather -> global top-R merge + rerank of
//          the owned rows + local top-k -> AllGather -> final merge
//   FLAT:  local exact top-k -> AllGather -> merge
//
// Results are bit-identical to one search over the concatenated corpus.  RCCL
// is dlopen'ed on first use so that a host that never shards does not need it
// (and a process that already loaded librccl.so.1, e.g. PyTorch, shares that
// copy).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>

#include "../../include/gvdb.h"
#include "gvdb_internal.h"

using namespace gvdb;

namespace {

struct Rccl {
    bool ok = false;
    std::string why;
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    const char* (*get_error_string)(ncclResult_t) = nullptr;
};

const Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            const char* e = dlerror();
            r.why = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
            return;
        }
        r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
        r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(h, "ncclCommInitRank");
        r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
        r.all_gather = (decltype(r.all_gather))dlsym(h, "ncclAllGather");
        r.get_error_string = (decltype(r.get_error_string))dlsym(h, "ncclGetErrorString");
        r.ok = r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.all_gather && r.get_error_string;
        if (!r.ok) r.why = "librccl.so.1 lacks a required symbol";
    });
    return r;
}

gvdb_status rccl_fail(ncclResult_t e, const char* where) {
    const char* m = rccl().get_error_string ? rccl().get_error_string(e) : "?";
    return report_status(GVDB_ERR_DEVICE, std::string(where) + ": " + m);
}

}  // namespace

struct gvdb_comm {
    ncclComm_t comm = nullptr;
    int32_t world = 1, rank = 0, device = 0;
    std::mutex mu;                // one search at a time per communicator
    void* buf = nullptr;          // exchange blocks + scratch (see search_sharded)
    size_t buf_bytes = 0;
    // the buffer is reused by the next call, possibly on another stream: the
    // next call's stream waits for `done` (recorded after the final merge)
    hipEvent_t done = nullptr;
    hipStream_t last = nullptr;
    bool pending = false;
};

extern "C" {

gvdb_status gvdb_comm_get_unique_id(uint8_t id[GVDB_COMM_ID_BYTES]) {
    if (!id) return report_status(GVDB_ERR_INVALID_ARGUMENT, "null id");
    const Rccl& r = rccl();
    if (!r.ok) return report_status(GVDB_ERR_DEVICE, r.why);
    ncclUniqueId u;
    ncclResult_t e = r.get_unique_id(&u);
    if (e != ncclSuccess) return rccl_fail(e, "ncclGetUniqueId");
    static_assert(sizeof(ncclUniqueId) == GVDB_COMM_ID_BYTES, "ncclUniqueId size");
    memcpy(id, &u, GVDB_COMM_ID_BYTES);
    return GVDB_OK;
}

gvdb_status gvdb_comm_create(const uint8_t id[GVDB_COMM_ID_BYTES], int32_t world, int32_t rank, int32_t device,
                             gvdb_comm** out) {
    if (!id || !out) return report_status(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    *out = nullptr;
    if (world < 1 || rank < 0 || rank >= world) return report_status(GVDB_ERR_INVALID_ARGUMENT, "bad world/rank");
    const Rccl& r = rccl();
    if (!r.ok) return report_status(GVDB_ERR_DEVICE, r.why);
    hipError_t he = hipSetDevice(device);
    if (he != hipSuccess) return report_status(GVDB_ERR_DEVICE, std::string("hipSetDevice: ") + hipGetErrorString(he));
    ncclUniqueId u;
    memcpy(&u, id, GVDB_COMM_ID_BYTES);
    auto* c = new gvdb_comm();
    c->world = world;
    c->rank = rank;
    c->device = device;
    ncclResult_t e = r.comm_init_rank(&c->comm, world, u, rank);
    if (e != ncclSuccess) {
        delete c;
        return rccl_fail(e, "ncclCommInitRank");
    }
    *out = c;
    return GVDB_OK;
}

void gvdb_comm_destroy(gvdb_comm* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    // only this communicator's last call has to finish (not every stream of the device)
    if (c->pending) (void)hipEventSynchronize(c->done);
    if (c->comm) (void)rccl().comm_destroy(c->comm);
    if (c->buf) (void)hipFreeAsync(c->buf, nullptr);
    if (c->done) (void)hipEventDestroy(c->done);
    delete c;
}

gvdb_status gvdb_comm_info(const gvdb_comm* c, int32_t* world, int32_t* rank) {
    if (!c) return report_status(GVDB_ERR_INVALID_ARGUMENT, "null comm");
    if (world) *world = c->world;
    if (rank) *rank = c->rank;
    return GVDB_OK;
}

gvdb_status gvdb_index_search_sharded_device(const gvdb_index* shard, gvdb_comm* c, const float* d_q, uint64_t B,
                                             uint32_t dim, uint64_t k, const gvdb_search_params* sp,
                                             uint64_t* d_out_ids, float* d_out_scores, uint32_t* d_out_n,
                                             void* stream) {
    // argument checks that are the same on every rank come first: a rank that
    // returns here returns on every rank, so no collective is left waiting
    if (!shard || !c || !sp) return report_status(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    if (B == 0 || k == 0) return GVDB_OK;
    if (!d_q || !d_out_ids || !d_out_scores) return report_status(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    const bool flat = sp->mode == GVDB_SEARCH_FLAT;
    if (!flat && (sp->mode != GVDB_SEARCH_BQ_RERANK || sp->metric != GVDB_METRIC_COSINE))
        return report_status(GVDB_ERR_INVALID_ARGUMENT, "sharded search: BQ + cosine rerank, or FLAT");
    if (!flat && sp->rescore_count == 0)
        return report_status(GVDB_ERR_INVALID_ARGUMENT, "sharded search needs rescore_count (global R)");
    if (index_device(shard) != c->device)
        return report_status(GVDB_ERR_INVALID_ARGUMENT, "shard and communicator on different devices");
    const uint64_t G = (uint64_t)c->world;
    const uint64_t R = flat ? k : std::max<uint64_t>(sp->rescore_count, k);
    if (G * k > kSelectLdsCap || B > 0xFFFFFFFFull || dim > 8192)
        return report_status(GVDB_ERR_INVALID_ARGUMENT, "sharded search: world * k <= 8192, dim <= 8192");
    // R > 8192 (the reference's default ratio at scale): the deep protocol
    // (histogram exchange, gvdb_shard.hip) -- R <= 2^20, dim < 4096, k <= 1024
    if (!flat && shard_deep(R) && (R > kBigRMax || dim == 0 || dim >= 4096 || k > 1024))
        return report_status(GVDB_ERR_INVALID_ARGUMENT, "sharded search, R > 8192: R <= 2^20, 0 < dim < 4096, k <= 1024");
    std::lock_guard<std::mutex> g(c->mu);
    hipError_t he = hipSetDevice(c->device);
    if (he != hipSuccess) return report_status(GVDB_ERR_DEVICE, std::string("hipSetDevice: ") + hipGetErrorString(he));
    hipStream_t s = (hipStream_t)stream;
    // the next call (possibly on another stream) and gvdb_comm_destroy wait for
    // everything enqueued here: `done` is recorded on EVERY return path below
    struct DoneGuard {
        gvdb_comm* c;
        hipStream_t s;
        ~DoneGuard() {
            if (!c->done) (void)hipEventCreateWithFlags(&c->done, hipEventDisableTiming);
            c->pending = c->done && hipEventRecord(c->done, s) == hipSuccess;
            c->last = s;
        }
    } done_guard{c, s};
    uint64_t w1 = 0, w2 = 0, scratch = 0;
    gvdb_shard_sizes(B, R, k, dim, &w1, &w2, &scratch);
    const uint64_t wf = shard_words_flat(B, k);
    // layout: send1 | recv1 [G] | send2 | recv2 [G] | scratch   (FLAT: sendF | recvF [G])
    const size_t need = flat ? wf * 4 * (G + 1) : ((w1 + w2) * (G + 1)) * 4 + scratch;
    if (c->pending && c->last != s) (void)hipStreamWaitEvent(s, c->done, 0);
    if (need > c->buf_bytes) {
        // stream-ordered: s already waits for the previous call (same stream, or
        // the event above), so the old blocks are released after their last use
        // without a device-wide synchronisation (co-tenant streams keep running)
        if (c->buf) (void)hipFreeAsync(c->buf, s);
        c->buf = nullptr;
        c->buf_bytes = 0;
        he = hipMallocAsync(&c->buf, need, s);
        if (he != hipSuccess)
            return report_status(he == hipErrorOutOfMemory ? GVDB_ERR_OUT_OF_MEMORY : GVDB_ERR_DEVICE,
                                 std::string("sharded search buffers: ") + hipGetErrorString(he));
        c->buf_bytes = need;
    }
    auto all_gather = [&](const uint32_t* send, uint32_t* recv, uint64_t words) -> gvdb_status {
        if (G == 1) return GVDB_OK;
        ncclResult_t e = rccl().all_gather(send, recv, words, ncclUint32, c->comm, s);
        return e == ncclSuccess ? GVDB_OK : rccl_fail(e, "ncclAllGather");
    };
    gvdb_status local = GVDB_OK, st = GVDB_OK;
    uint32_t* base = (uint32_t*)c->buf;
    if (flat) {
        uint32_t* send = base;
        uint32_t* recv = G > 1 ? base + wf : send;
        const uint64_t BK = B * k;
        // the rank's exact top-k (certified MFMA tiers / exact scan, storage.rs:296-339)
        local = gvdb_index_search_device(shard, d_q, B, dim, k, sp, reinterpret_cast<uint64_t*>(send),
                                         reinterpret_cast<float*>(send + 2 * BK), send + 3 * BK, stream);
        if (local == GVDB_ERR_INDEX_NOT_BUILT) local = GVDB_OK;  // an empty shard contributes nothing
        const bool ok = local == GVDB_OK && gvdb_index_len(shard) > 0;
        if (!ok) (void)hipMemsetD32Async(send + 3 * BK, 0, B, s);
        (void)hipMemsetD32Async(send + 3 * BK + B, local == GVDB_OK ? 0 : 1, 1, s);
        st = all_gather(send, recv, wf);
        if (st == GVDB_OK)
            st = gvdb_shard_flat_final_device(recv, G, B, k, sp->metric, d_out_ids, d_out_scores, d_out_n, stream);
    } else {
        uint32_t* send1 = base;
        uint32_t* recv1 = G > 1 ? send1 + w1 : send1;
        uint32_t* send2 = base + w1 * (G + 1);
        uint32_t* recv2 = G > 1 ? send2 + w2 : send2;
        void* scr = base + (w1 + w2) * (G + 1);
        // 1. local stage 1 (an empty or failing shard still joins with no entries)
        local = gvdb_shard_stage1_device(shard, d_q, B, dim, R, send1, scr, stream);
        std::string local_err = local != GVDB_OK ? std::string(gvdb_last_error()) : std::string();
        if ((st = all_gather(send1, recv1, w1)) != GVDB_OK) return st;
        // 2. global top-R, rerank of the owned rows, local top-k.  A rank whose
        // phase 2 fails still joins exchange 2 (no entries, the merge poisoned),
        // so its peers are never left waiting in the collective
        const gvdb_status rr =
            gvdb_shard_rerank_device(shard, d_q, B, dim, R, k, recv1, G, (uint64_t)c->rank, scr, send2, stream);
        if (rr != GVDB_OK) {
            if (local == GVDB_OK) {
                local = rr;
                local_err = gvdb_last_error();
            }
            (void)hipMemsetD32Async(send2 + 4 * B * k, 0, 2 * B, s);  // meta: no entries
        }
        if (local != GVDB_OK) (void)hipMemsetD32Async(send2 + 4 * B * k + 2 * B, 1, 1, s);  // poison the merge
        st = all_gather(send2, recv2, w2);
        // 3. the merged top-k on every rank
        if (st == GVDB_OK) st = gvdb_shard_final_device(recv2, G, B, k, d_out_ids, d_out_scores, d_out_n, stream);
        if (st == GVDB_OK && local != GVDB_OK) report_status(local, local_err);
    }
    return st != GVDB_OK ? st : local;
}

}  // extern "C"
