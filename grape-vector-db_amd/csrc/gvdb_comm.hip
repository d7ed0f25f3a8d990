// gvdb_comm.hip — RCCL communicator + exact sharded search (include/gvdb.h).
//
// Replaces ShardManager::search_vectors (src/distributed/shard.rs:760-786:
// fan out to every shard, concat, sort by score, truncate) inside one node:
// one process per GPU, each holding a contiguous row range of the corpus
// whose ids are global row numbers.  One exchange per batch:
//
//   rank g:  stage-1 local top-R + exact cosines (gvdb::shard_candidates)
//            written straight into its send block
//              [ids u64 B*R | dist u32 B*R | cos f32 B*R | counts u32 B | pad]
//   all:     ncclAllGather of the blocks on the caller's stream (xGMI)
//   all:     k_bq_shard_merge over the gathered blocks in place
//
// The union of the local top-R lists holds the global top-R by
// (Hamming, id), so the merge reproduces multi_stage_search over the whole
// corpus bit for bit.  RCCL is dlopen'ed on first use so that a host that
// never shards does not need it (and a process that already loaded
// librccl.so.1, e.g. PyTorch, shares that copy).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

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
    uint32_t* buf = nullptr;      // [send block][world recv blocks]
    size_t buf_words = 0;
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
    (void)hipDeviceSynchronize();
    if (c->comm) (void)rccl().comm_destroy(c->comm);
    if (c->buf) (void)hipFree(c->buf);
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
    if (!shard || !c || !sp) return report_status(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    if (B == 0 || k == 0) return GVDB_OK;
    if (!d_q || !d_out_ids || !d_out_scores) return report_status(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    if (sp->mode != GVDB_SEARCH_BQ_RERANK || sp->metric != GVDB_METRIC_COSINE)
        return report_status(GVDB_ERR_INVALID_ARGUMENT, "sharded search: BQ + cosine rerank only");
    if (sp->rescore_count == 0)
        return report_status(GVDB_ERR_INVALID_ARGUMENT, "sharded search needs rescore_count (global R)");
    if (index_device(shard) != c->device)
        return report_status(GVDB_ERR_INVALID_ARGUMENT, "shard and communicator on different devices");
    const uint64_t R = sp->rescore_count > k ? sp->rescore_count : k;
    if ((uint64_t)c->world * R > kSortLdsCap || B > 0xFFFFFFFFull)
        return report_status(GVDB_ERR_INVALID_ARGUMENT, "world * R exceeds the 4096-entry merge");
    std::lock_guard<std::mutex> g(c->mu);
    hipError_t he = hipSetDevice(c->device);
    if (he != hipSuccess) return report_status(GVDB_ERR_DEVICE, std::string("hipSetDevice: ") + hipGetErrorString(he));
    hipStream_t s = (hipStream_t)stream;
    const uint64_t BR = B * R;
    const uint64_t blk = (4 * BR + B + 1) & ~1ull;  // words per rank block, even (u64 ids stay aligned)
    const size_t need = blk * (size_t)(c->world + 1);
    if (need > c->buf_words) {
        if (c->buf) {
            (void)hipStreamSynchronize(s);
            (void)hipFree(c->buf);
        }
        c->buf = nullptr;
        c->buf_words = 0;
        he = hipMalloc((void**)&c->buf, need * 4);
        if (he != hipSuccess)
            return report_status(he == hipErrorOutOfMemory ? GVDB_ERR_OUT_OF_MEMORY : GVDB_ERR_DEVICE,
                                 std::string("sharded search buffers: ") + hipGetErrorString(he));
        c->buf_words = need;
    }
    uint32_t* send = c->buf;
    uint32_t* recv = c->world > 1 ? c->buf + blk : send;
    gvdb_status st = shard_candidates(shard, d_q, B, dim, R, R, reinterpret_cast<uint64_t*>(send), send + 2 * BR,
                                      reinterpret_cast<float*>(send + 3 * BR), send + 4 * BR, s);
    if (st != GVDB_OK) return st;
    if (c->world > 1) {
        ncclResult_t e = rccl().all_gather(send, recv, blk, ncclUint32, c->comm, s);
        if (e != ncclSuccess) return rccl_fail(e, "ncclAllGather");
    }
    he = launch_bq_shard_merge(reinterpret_cast<const uint64_t*>(recv), recv + 2 * BR,
                               reinterpret_cast<const float*>(recv + 3 * BR), recv + 4 * BR, (uint32_t)c->world,
                               (uint32_t)B, (uint32_t)R, (uint32_t)R, (uint32_t)k, d_out_ids, d_out_scores, d_out_n,
                               nullptr, s, blk / 2, blk, blk, 1);
    if (he != hipSuccess) return report_status(GVDB_ERR_DEVICE, std::string("shard merge: ") + hipGetErrorString(he));
    return GVDB_OK;
}

}  // extern "C"
