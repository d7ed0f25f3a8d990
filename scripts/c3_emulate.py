#!/usr/bin/env python3
"""Config 3 (10M x 768, BQ top-100 + exact rerank, k = 10, batch 256) split
into the 8 contiguous shards of the 8-GPU layout, emulated on ONE MI355X with
the two-exchange protocol's phase ABI (the same calls
gvdb_index_search_sharded_device makes around its two ncclAllGather):

  rank g: gvdb_shard_stage1_device  -> its exchange-1 block, written where the
          all-gather would deliver it
  rank g: gvdb_shard_rerank_device  -> global top-R, exact cosine of the rows it
          owns, local top-k -> its exchange-2 block
  every rank: gvdb_shard_final_device -> merged top-k

Per-rank step time = the three phases of one rank run back to back on the GPU
(each rank timed separately; the max over ranks is the 8-GPU step minus the two
collectives, whose payloads are printed).  Checks: merged results bit-identical
to ONE 10M x 768 index on the same GPU (ids, cosine bits, counts), and to the
CPU oracle's multi_stage_search over the whole corpus on a query sample.
Prints one JSON line.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "grape-vector-db_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

import bench  # noqa: E402  (the bench's corpus / query generators)
import gvdb  # noqa: E402


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--R", type=int, default=100)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--oracle-queries", type=int, default=32)
    ap.add_argument("--no-single", action="store_true", help="skip the single-index comparison")
    ap.add_argument("--p2clk", action="store_true", help="print phase-2 phase clocks (timing study)")
    a = ap.parse_args()
    N, D, G, B, R, k = a.n, a.dim, a.shards, a.batch, a.R, a.k
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    L = gvdb.lib()
    q = bench.gen_queries(B, D, dev)
    bounds = [N * s // G for s in range(G + 1)]
    nq_or = min(a.oracle_queries, B)
    host_rows = np.empty((N, D), np.float32) if nq_or else None
    host_codes = np.empty((N, (D + 7) // 8), np.uint8) if nq_or else None
    code_buf = torch.empty((bench.CHUNK, (D + 7) // 8), dtype=torch.uint8, device=dev) if nq_or else None

    t0 = time.time()
    shards = [gvdb.GpuVectorIndex(dimension=D, capacity_hint=bounds[s + 1] - bounds[s]) for s in range(G)]
    single = None if a.no_single else gvdb.GpuVectorIndex(dimension=D, capacity_hint=N)
    for c in range((N + bench.CHUNK - 1) // bench.CHUNK):
        c0, c1 = c * bench.CHUNK, min(N, (c + 1) * bench.CHUNK)
        x = bench.gen_chunk(c, c1 - c0, D, dev)  # the bench's own corpus
        for s in range(G):
            lo, hi = max(c0, bounds[s]), min(c1, bounds[s + 1])
            if lo < hi:
                shards[s].add_device(x[lo - c0:hi - c0].contiguous(), torch.arange(lo, hi, dtype=torch.int64, device=dev))
        if single is not None:
            single.add_device(x, torch.arange(c0, c1, dtype=torch.int64, device=dev))
        if nq_or:
            host_rows[c0:c1] = x.cpu().numpy()
            L.gvdb_bq_quantize_device(x.data_ptr(), c1 - c0, D, 0.0, code_buf.data_ptr(), None)
            torch.cuda.synchronize()
            host_codes[c0:c1] = code_buf[:c1 - c0].cpu().numpy()
        del x
    torch.cuda.synchronize()
    log(f"[c3] corpus + {G} shards{' + single index' if single is not None else ''}: {time.time() - t0:.0f}s")

    w1, w2, scr = C.c_uint64(), C.c_uint64(), C.c_uint64()
    L.gvdb_shard_sizes(B, R, k, D, C.byref(w1), C.byref(w2), C.byref(scr))
    g1 = torch.zeros((G, w1.value), dtype=torch.int32, device=dev)
    g2 = torch.zeros((G, w2.value), dtype=torch.int32, device=dev)
    deep = R > 8192  # the deep form keeps each rank's stage-1 membership in its scratch until phase 2
    scratch = torch.zeros((G if deep else 1, scr.value), dtype=torch.uint8, device=dev)
    oi = torch.zeros((B, k), dtype=torch.int64, device=dev)
    osc = torch.zeros((B, k), dtype=torch.float32, device=dev)
    on = torch.zeros(B, dtype=torch.int32, device=dev)

    def p1(r):
        gvdb.check(L.gvdb_shard_stage1_device(shards[r]._h, q.data_ptr(), B, D, R, g1[r].data_ptr(),
                                              scratch[r if deep else 0].data_ptr(), None))

    def p2(r):
        gvdb.check(L.gvdb_shard_rerank_device(shards[r]._h, q.data_ptr(), B, D, R, k, g1.data_ptr(), G, r,
                                              scratch[r if deep else 0].data_ptr(), g2[r].data_ptr(), None))

    def p3():
        gvdb.check(L.gvdb_shard_final_device(g2.data_ptr(), G, B, k, oi.data_ptr(), osc.data_ptr(), on.data_ptr(),
                                             None))

    for r in range(G):
        p1(r)
    for r in range(G):
        p2(r)
    p3()
    torch.cuda.synchronize()
    A_i, A_s, A_n = oi.cpu().numpy().view(np.uint64).copy(), osc.cpu().numpy().copy(), on.cpu().numpy().copy()

    def timed(fn, steps):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / steps

    # steady state before any rank is timed (the first-timed rank otherwise carries
    # the clock ramp of the idle GPU)
    for _ in range(10):
        for r in range(G):
            p1(r)
            p2(r)
            p3()
    torch.cuda.synchronize()
    per_rank = []
    for r in range(G):
        step = timed(lambda: (p1(r), p2(r), p3()), a.steps)
        t1 = timed(lambda: p1(r), a.steps)
        t2 = timed(lambda: p2(r), a.steps)
        per_rank.append({"rank": r, "rows": bounds[r + 1] - bounds[r], "step_ms": 1e3 * step,
                         "stage1_ms": 1e3 * t1, "merge_rerank_topk_ms": 1e3 * t2})
    t3 = timed(p3, a.steps)
    # host enqueue cost per phase call (no sync inside the loop; the GPU queue absorbs it)
    host_us = {}
    for nm, fn in (("stage1", lambda: p1(0)), ("rerank", lambda: p2(0)), ("final", p3)):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.steps):
            fn()
        host_us[nm] = 1e6 * (time.perf_counter() - t) / a.steps
        torch.cuda.synchronize()
    log(f"[c3] host enqueue per call (us): {host_us}")
    if a.p2clk:  # phase clocks of one rank's phase 2 (GVDB_P2_CLK timing study)
        os.environ["GVDB_P2_CLK"] = "1"
        p2(0)
        torch.cuda.synchronize()
        del os.environ["GVDB_P2_CLK"]
        ck = (C.c_double * 4)()
        if L.gvdb_debug_shard_clock(ck) == 0:
            log("[c3] phase-2 clocks (us from block start, mean over blocks): round A %.2f, ranking %.2f, "
                "folds %.2f, end %.2f" % tuple(v / 100.0 for v in ck))
    # all-gather surrogate: what each rank RECEIVES per exchange (G blocks) moved as
    # one device copy -- a floor for ncclAllGather's data movement, not its latency
    # (RCCL over 8-GPU xGMI adds its own small-message latency, unmeasurable here)
    src1 = torch.zeros_like(g1)
    src2 = torch.zeros_like(g2)
    ag1 = timed(lambda: g1.copy_(src1), a.steps)
    ag2 = timed(lambda: g2.copy_(src2), a.steps)
    worst = max(p["step_ms"] for p in per_rank)
    log(f"[c3] per-rank step (no collectives): max {worst:.4f} ms, "
        f"mean {np.mean([p['step_ms'] for p in per_rank]):.4f} ms; final merge {1e3 * t3:.4f} ms")
    cfg = "configs[3]" if D == 3072 else "configs[2]"
    line = {"workload": f"BASELINE {cfg} corpus ({N / 1e6:g}M x {D}) in {G} contiguous shards on one GPU, "
                        f"two-exchange{' (deep form)' if deep else ''} BQ top-{R} + exact cosine rerank, k={k}, "
                        f"batch {B}",
            "per_rank": per_rank, "final_merge_ms": 1e3 * t3, "per_rank_step_max_ms": worst,
            "emulated_qps": B / (worst * 1e-3),
            "emulated_qps_with_surrogates": B / ((worst + 1e3 * (ag1 + ag2)) * 1e-3),
            "exchange_bytes_per_rank": {"all_gather_1": 4 * w1.value, "all_gather_2": 4 * w2.value},
            "allgather_surrogate_ms": {"all_gather_1": 1e3 * ag1, "all_gather_2": 1e3 * ag2,
                                       "what": f"one device copy of the G x block bytes a rank receives "
                                               f"({4 * G * w1.value} + {4 * G * w2.value} B)"},
            "per_rank_step_plus_surrogates_ms": worst + 1e3 * (ag1 + ag2),
            "host_enqueue_us_per_call": host_us,
            "note": "per-rank step = stage 1 + merge/rerank/top-k + final merge of one rank, back to back on the "
                    "GPU (host launch overhead included); the 8-GPU step adds the two ncclAllGather calls"}
    if single is not None:
        sp = gvdb.SearchParams(rescore_count=R)
        si = torch.zeros((B, k), dtype=torch.int64, device=dev)
        ss = torch.zeros((B, k), dtype=torch.float32, device=dev)
        sn = torch.zeros(B, dtype=torch.int32, device=dev)
        t_single = timed(lambda: single.search_device(q, k, si, ss, sn, sp), a.steps)
        S_i, S_s, S_n = si.cpu().numpy().view(np.uint64), ss.cpu().numpy(), sn.cpu().numpy()
        same = bool((A_i == S_i).all() and A_s.tobytes() == S_s.tobytes() and (A_n == S_n).all())
        line.update({"single_index_step_ms": 1e3 * t_single, "single_gpu_qps": B / t_single,
                     "sharded_equals_single_index": same,
                     "emulated_speedup_vs_single_gpu": t_single / (worst * 1e-3)})
        log(f"[c3] single {N / 1e6:g}M index step {1e3 * t_single:.4f} ms; sharded == single: {same}; "
            f"speedup {t_single / (worst * 1e-3):.2f}x")
        del single
    if nq_or:
        import oracle  # checker only

        qn = q.cpu().numpy()
        threads = max(1, min(16, len(os.sched_getaffinity(0))))
        t = time.perf_counter()
        ri, rs = oracle.multi_stage_search_batch_r(oracle.quantize(qn[:nq_or]), host_codes, qn[:nq_or], host_rows, R,
                                                   threads=threads)
        line["oracle_parity"] = {"queries": nq_or, "ids_equal": bool((ri[:, :k] == A_i[:nq_or]).all()),
                                 "cosine_bit_exact": rs[:, :k].tobytes() == A_s[:nq_or].tobytes(),
                                 "oracle_s": time.perf_counter() - t, "threads": threads}
        log(f"[c3] oracle parity: {line['oracle_parity']}")
    print(json.dumps(line), flush=True)
    ok = line.get("sharded_equals_single_index", True) and (
        not nq_or or (line["oracle_parity"]["ids_equal"] and line["oracle_parity"]["cosine_bit_exact"]))
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
