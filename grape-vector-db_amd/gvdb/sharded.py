"""Exact sharded search over torch.distributed.

Replaces ``ShardManager::search_vectors`` (src/distributed/shard.rs:760-786:
scatter to shards, concat, sort, truncate) inside one node.  Each rank owns a
contiguous row range whose ids are global row numbers (ranks in corpus order).

:class:`TwoExchangeSearch` is the production protocol (the same one
``gvdb_index_search_sharded_device`` runs with RCCL inside libgvdb, see
``csrc/gvdb_shard.hip``) driven over ANY torch.distributed transport:

1. every rank: its exact local stage-1 top-R as (Hamming << 32 | row) keys;
   for R > 8192 (the reference's default ratio at scale, the "deep" form) the
   per-query Hamming histogram of that local top-R instead;
2. all-gather of those blocks (B*R*8 bytes per rank; deep: B*(dim+1)*4);
3. every rank: the global top-R by (Hamming, corpus row), the exact cosine of
   the rows IT owns among them (~R/G per query), its local top-k;
4. all-gather of the local top-k (B*k*16 bytes per rank);
5. every rank: the merged top-k = the first k of the stable cosine sort of the
   global top-R, bit-identical to one multi_stage_search over the corpus.

A rank whose phase fails still joins both all-gathers (no entries, an error
word that poisons every query of the merge) and raises only afterwards, so no
peer is left waiting in a collective.  On a GPU the phases are the device
forms; on a CPU transport (gloo) the local stage 1 and the cosines come from
callables and the merges run as host forms.

:class:`ShardedBQSearch` is the earlier ONE-exchange variant (every rank
reranks its whole local top-R and ships (id, Hamming, cosine) triplets, B*R*16
bytes per rank), kept as a lower-level form; :class:`RcclShardedSearch` wraps
the in-library RCCL composition.
"""
from __future__ import annotations

from typing import Callable, List, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import check
from ._ffi import lib

# candidates_fn(queries, R_local) -> (gids int64 [B,R_local], dist int32 [B,R_local], cos f32 [B,R_local])
CandidatesFn = Callable[[torch.Tensor, int], Tuple[torch.Tensor, torch.Tensor, torch.Tensor]]


def _status_error(rc: int) -> Exception:
    try:
        check(rc)
    except Exception as e:  # noqa: BLE001 -- the mapped VectorDbError
        return e
    return RuntimeError(f"gvdb status {rc}")


def shard_bounds(n: int, world: int) -> List[int]:
    return [n * g // world for g in range(world + 1)]


class TwoExchangeSearch:
    """Two-exchange exact sharded search for B queries, global depth R, k results.

    device mode (``index`` given): the rank's shard is a GpuVectorIndex whose
    rows are the rank's contiguous range of the corpus (ranks in corpus order);
    the phases run on the GPU and the all-gathers move device tensors.
    host mode (``stage1_fn`` / ``cosine_fn`` given, CPU tensors): stage1_fn(q, R)
    -> (local rows int [B, Rl], Hamming int [B, Rl]) sorted by (d, row) with
    Rl = min(R, shard rows); cosine_fn(q_index, local_rows) -> f32 cosines;
    ``id_offset`` turns local rows into the ids reported (global row numbers).
    ``dim`` (the vectors' dimension) sizes the deep form's histograms and is
    required when R > 8192.
    """

    DEEP_R = 8192  # R above this: the deep form (histogram exchange)

    def __init__(self, B: int, R: int, k: int, device: torch.device, group=None, index=None, stage1_fn=None,
                 cosine_fn=None, id_offset: int = 0, dim: int = 0):
        import ctypes as C

        self.B, self.R, self.k, self.dim = B, R, k, dim
        self.deep = R > self.DEEP_R
        if self.deep and dim <= 0:
            raise ValueError("TwoExchangeSearch: R > 8192 (deep form) needs dim")
        self.dev, self.group = device, group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.index, self.stage1_fn, self.cosine_fn, self.id_offset = index, stage1_fn, cosine_fn, id_offset
        w1, w2, scr = C.c_uint64(), C.c_uint64(), C.c_uint64()
        lib().gvdb_shard_sizes(B, R, k, dim, C.byref(w1), C.byref(w2), C.byref(scr))
        self.w1, self.w2 = w1.value, w2.value
        self.send1 = torch.zeros(self.w1, dtype=torch.int32, device=device)
        self.recv1 = torch.zeros((self.world, self.w1), dtype=torch.int32, device=device)
        self.send2 = torch.zeros(self.w2, dtype=torch.int32, device=device)
        self.recv2 = torch.zeros((self.world, self.w2), dtype=torch.int32, device=device)
        self.scratch = torch.zeros(scr.value, dtype=torch.uint8, device=device) if index is not None else None
        self.out_ids = torch.zeros((B, k), dtype=torch.int64, device=device)
        self.out_scores = torch.zeros((B, k), dtype=torch.float32, device=device)
        self.out_n = torch.zeros(B, dtype=torch.int32, device=device)

    def _gather(self, send, recv):
        if self.world == 1:
            recv[0].copy_(send)
        elif send.is_cuda:
            dist.all_gather_into_tensor(recv, send, group=self.group)
        else:
            parts = list(recv.unbind(0))
            dist.all_gather(parts, send, group=self.group)

    # exchange-2 block: [B*k entries of 4 words | meta: count[B] | reff[B] | err]
    def _meta2(self):
        return 4 * self.B * self.k

    def search(self, q: torch.Tensor):
        """Both all-gathers run on every rank whatever happens locally; a local
        failure poisons the merge (every query GVDB_N_POISONED on every rank)
        and is raised on the failing rank after the second exchange."""
        B, R, k = self.B, self.R, self.k
        L = lib()
        err = None  # the first local failure (raised after both exchanges)
        m2 = self._meta2()
        if self.index is not None:
            st = torch.cuda.current_stream(q.device).cuda_stream or None
            D = q.shape[1]
            # a failing stage 1 writes zero counts + its err word itself (the C ABI contract)
            rc = L.gvdb_shard_stage1_device(self.index._h, q.data_ptr(), B, D, R, self.send1.data_ptr(),
                                            self.scratch.data_ptr(), st)
            if rc != 0:
                err = _status_error(rc)
            self._gather(self.send1, self.recv1)
            rc = L.gvdb_shard_rerank_device(self.index._h, q.data_ptr(), B, D, R, k, self.recv1.data_ptr(), self.world,
                                            self.rank, self.scratch.data_ptr(), self.send2.data_ptr(), st)
            if rc != 0:
                err = err or _status_error(rc)
                self.send2[m2:m2 + 2 * B].zero_()  # no entries from this rank
            if err is not None:
                self.send2[m2 + 2 * B] = 1  # poison the merge
            self._gather(self.send2, self.recv2)
            check(L.gvdb_shard_final_device(self.recv2.data_ptr(), self.world, B, k, self.out_ids.data_ptr(),
                                            self.out_scores.data_ptr(), self.out_n.data_ptr(), st))
            if err is not None:
                raise err
            return self.out_ids, self.out_scores, self.out_n
        # host transport: the same blocks, host merges
        s1 = self.send1.numpy().view(np.uint32)
        s1[:] = 0
        H = self.dim + 1
        cnt_at = B * H if self.deep else 2 * B * R  # word of counts[0]
        m_rows = np.zeros((B, R), np.uint32)
        m_dist = np.zeros((B, R), np.uint32)
        try:
            rows, dd = self.stage1_fn(q, R)
            rows, dd = np.asarray(rows, np.uint64), np.asarray(dd, np.uint64)
            rl = rows.shape[1]
            if self.deep:  # this rank's top-R membership stays local; its histogram goes out
                m_rows[:, :rl] = rows
                m_dist[:, :rl] = dd
                hist = s1[:B * H].reshape(B, H)
                for i in range(B):
                    hist[i] = np.bincount(dd[i].astype(np.int64), minlength=H)[:H]
            else:
                keys = s1[:2 * B * R].view(np.uint64).reshape(B, R)
                keys[:, :rl] = (dd << np.uint64(32)) | rows
            s1[cnt_at:cnt_at + B] = rl
        except Exception as e:  # noqa: BLE001 -- re-raised after the exchanges
            err = e
            s1[:] = 0
            s1[cnt_at + B] = 1
        self._gather(self.send1, self.recv1)
        g1 = np.ascontiguousarray(self.recv1.numpy().view(np.uint32))
        own_rows = np.zeros((B, R), np.uint32)
        own_pos = np.zeros((B, R), np.uint32)  # deep: the Hamming distances (the merge's order key)
        own_cnt = np.zeros(B, np.uint32)
        reff = np.zeros(B, np.uint32)
        scores = np.zeros((B, R), np.float32)
        ids = np.zeros((B, R), np.uint64)
        s2 = self.send2.numpy().view(np.uint32)
        s2[:] = 0
        try:
            if self.deep:
                check(L.gvdb_shard_deep_own_host(g1.ctypes.data, self.world, self.rank, B, R, self.dim,
                                                 m_rows.ctypes.data, m_dist.ctypes.data, own_rows.ctypes.data,
                                                 own_pos.ctypes.data, own_cnt.ctypes.data, reff.ctypes.data))
            else:
                check(L.gvdb_shard_merge_host(g1.ctypes.data, self.world, self.rank, B, R, own_rows.ctypes.data,
                                              own_pos.ctypes.data, own_cnt.ctypes.data, reff.ctypes.data))
            if err is None:
                for i in range(B):
                    c = int(own_cnt[i])
                    if c:
                        scores[i, :c] = self.cosine_fn(i, own_rows[i, :c])
                        ids[i, :c] = own_rows[i, :c].astype(np.uint64) + np.uint64(self.id_offset)
            else:
                own_cnt[:] = 0
            check(L.gvdb_shard_local_topk_host(scores.ctypes.data, own_pos.ctypes.data, ids.ctypes.data,
                                               own_cnt.ctypes.data, reff.ctypes.data, B, R, k, int(err is not None),
                                               s2.ctypes.data))
        except Exception as e:  # noqa: BLE001
            err = err or e
            s2[:] = 0
            s2[m2 + 2 * B] = 1
        self._gather(self.send2, self.recv2)
        g2 = np.ascontiguousarray(self.recv2.numpy().view(np.uint32))
        oi = np.zeros((B, k), np.uint64)
        osc = np.zeros((B, k), np.float32)
        on = np.zeros(B, np.uint32)
        check(L.gvdb_shard_final_host(g2.ctypes.data, self.world, B, k, oi.ctypes.data, osc.ctypes.data,
                                      on.ctypes.data))
        if err is not None:
            raise err
        return torch.from_numpy(oi.view(np.int64)), torch.from_numpy(osc), torch.from_numpy(on.view(np.int32))


class ShardedBQSearch:
    """TEST-ONLY legacy one-exchange form (each rank's top-R with its exact
    cosines, one all-gather of B*R*16 B, gvdb_bq_shard_merge_packed_device):
    kept as a second, independent orchestration the tests compare the
    two-exchange protocol against.  Production sharding is
    gvdb_index_search_sharded_device / RcclShardedSearch / TwoExchangeSearch."""

    def __init__(self, candidates_fn: CandidatesFn, shard_rows: Sequence[int], B: int, R: int, k: int,
                 device: torch.device, group=None):
        self.cand = candidates_fn
        self.world = len(shard_rows)
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.B, self.R, self.k = B, R, k
        self.dev = device
        self.group = group
        self.on_gpu = device.type == "cuda"
        self.r_local = [min(R, n) for n in shard_rows]
        self.pack = torch.zeros((B, R, 4), dtype=torch.int32, device=device)
        self.gathered = torch.zeros((self.world, B, R, 4), dtype=torch.int32, device=device)
        self.counts = torch.tensor([[r] * B for r in self.r_local], dtype=torch.int32, device=device)
        self.out_ids = torch.zeros((B, k), dtype=torch.int64, device=device)
        self.out_scores = torch.zeros((B, k), dtype=torch.float32, device=device)
        self.out_n = torch.zeros(B, dtype=torch.int32, device=device)
        # packed fast path (GPU, every shard holds >= R rows): the local
        # candidates are written straight into this rank's send block
        # [ids u64 B*R | dist u32 B*R | cos f32 B*R], the all-gather moves the
        # blocks and the merge reads them in place (no packing copies)
        self.into = getattr(candidates_fn, "into", None)
        self.packed = self.on_gpu and self.into is not None and all(r == R for r in self.r_local)
        if self.packed:
            self.send = torch.zeros(4 * B * R, dtype=torch.int32, device=device)
            self.recv = torch.zeros((self.world, 4 * B * R), dtype=torch.int32, device=device)

    def _search_packed(self, q: torch.Tensor):
        B, R, k = self.B, self.R, self.k
        p = self.send.data_ptr()
        self.into(q, R, p, p + 8 * B * R, p + 12 * B * R)
        if self.world > 1:
            dist.all_gather_into_tensor(self.recv, self.send, group=self.group)
            src = self.recv
        else:
            src = self.send
        stream = torch.cuda.current_stream(self.dev).cuda_stream or None
        check(lib().gvdb_bq_shard_merge_packed_device(src.data_ptr(), self.counts.data_ptr(), self.world, B, R, k,
                                                      self.out_ids.data_ptr(), self.out_scores.data_ptr(),
                                                      self.out_n.data_ptr(), stream))
        return self.out_ids, self.out_scores, self.out_n

    def search(self, q: torch.Tensor):
        if self.packed:
            return self._search_packed(q)
        B, R, k = self.B, self.R, self.k
        rl = self.r_local[self.rank]
        gids, d, c = self.cand(q, rl)
        self.pack[:, :rl, 0:2] = gids[:, :rl].contiguous().view(torch.int32).view(B, rl, 2)
        self.pack[:, :rl, 2] = d[:, :rl]
        self.pack[:, :rl, 3] = c[:, :rl].contiguous().view(torch.int32)
        if self.world > 1:
            if self.on_gpu:
                dist.all_gather_into_tensor(self.gathered, self.pack, group=self.group)
            else:
                parts = list(self.gathered.unbind(0))
                dist.all_gather(parts, self.pack, group=self.group)
                self.gathered = torch.stack(parts)
        else:
            self.gathered[0].copy_(self.pack)
        g_ids = self.gathered[..., 0:2].contiguous().view(torch.int64).view(self.world, B, R)
        g_d = self.gathered[..., 2].contiguous()
        g_c = self.gathered[..., 3].contiguous().view(torch.float32)
        L = lib()
        if self.on_gpu:
            stream = torch.cuda.current_stream(self.dev).cuda_stream or None
            check(L.gvdb_bq_shard_merge_device(g_ids.data_ptr(), g_d.data_ptr(), g_c.data_ptr(),
                                               self.counts.data_ptr(), self.world, B, R, R, k,
                                               self.out_ids.data_ptr(), self.out_scores.data_ptr(),
                                               self.out_n.data_ptr(), stream))
        else:
            check(L.gvdb_bq_shard_merge(g_ids.data_ptr(), g_d.data_ptr(), g_c.data_ptr(), self.counts.data_ptr(),
                                        self.world, B, R, R, k, self.out_ids.data_ptr(),
                                        self.out_scores.data_ptr(), self.out_n.data_ptr()))
        return self.out_ids, self.out_scores, self.out_n


def gpu_candidates_fn(index) -> CandidatesFn:
    """Local candidates from a GpuVectorIndex whose ids are global row numbers."""
    bufs = {}

    def fn(q: torch.Tensor, r: int):
        B = q.shape[0]
        key = (B, r)
        if key not in bufs:
            bufs[key] = (torch.zeros((B, r), dtype=torch.int64, device=q.device),
                         torch.zeros((B, r), dtype=torch.int32, device=q.device),
                         torch.zeros((B, r), dtype=torch.float32, device=q.device))
        ids, d, c = bufs[key]
        into(q, r, ids.data_ptr(), d.data_ptr(), c.data_ptr())
        return ids, d, c

    def into(q: torch.Tensor, r: int, ids_ptr: int, dist_ptr: int, cos_ptr: int):
        stream = torch.cuda.current_stream(q.device).cuda_stream or None
        check(lib().gvdb_index_bq_candidates_device(index._h, q.data_ptr(), q.shape[0], q.shape[1], r, ids_ptr,
                                                     dist_ptr, cos_ptr, stream))

    fn.into = into
    return fn


class RcclShardedSearch:
    """The two-exchange search with the collectives inside libgvdb
    (``gvdb_index_search_sharded_device``: two ncclAllGather calls on the
    caller's stream), all behind the C ABI, so a host without torch (the Rust
    FFI of INTEGRATION.md) shards the same way.  ``params`` may select FLAT
    (the ranks' exact top-k merged).  torch.distributed is used here only to
    hand rank 0's RCCL unique id to the other ranks."""

    def __init__(self, index, R: int, k: int, group=None, params=None):
        import ctypes as C

        self.index, self.R, self.k = index, R, k
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        L = lib()
        uid = (C.c_uint8 * 128)()
        if self.rank == 0:
            check(L.gvdb_comm_get_unique_id(uid))
        if self.world > 1:
            box = [bytes(uid)]
            dist.broadcast_object_list(box, src=0, group=group)
            C.memmove(uid, box[0], 128)
        h = C.c_void_p()
        check(L.gvdb_comm_create(uid, self.world, self.rank, index.device, C.byref(h)))
        self._h = h
        from . import SearchParams

        self.sp = (params or SearchParams(rescore_count=R)).to_c()

    def search_into(self, q: torch.Tensor, out_ids: torch.Tensor, out_scores: torch.Tensor, out_n=None) -> None:
        import ctypes as C

        stream = torch.cuda.current_stream(q.device).cuda_stream or None
        check(lib().gvdb_index_search_sharded_device(self.index._h, self._h, q.data_ptr(), q.shape[0], q.shape[1],
                                                     self.k, C.byref(self.sp), out_ids.data_ptr(),
                                                     out_scores.data_ptr(),
                                                     out_n.data_ptr() if out_n is not None else None, stream))

    def close(self) -> None:
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib().gvdb_comm_destroy(h)
            self._h = None

    def __del__(self):
        self.close()
