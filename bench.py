#!/usr/bin/env python3
"""bench.py — QPS @ recall@10 of the MI355X BQ search path (BASELINE.json metric).

Workload (BASELINE.json configs[2], the metric's own config; it fits one GPU):
10M x 768 f32 corpus, i.i.d. N(0,1) rows L2-normalised (so cosine and L2
ground truths coincide), BQ Hamming prefilter -> top-R=100 -> exact cosine
rerank -> top-10, batch of 256 queries per step.  Batch-1 latency/QPS is
reported beside it.  A "step" = one search call over one 256-query batch
with the corpus already resident in HBM.

N GPUs (torchrun, one process per GPU): the corpus is sharded by contiguous
row ranges (the same 10M rows in total: strong scaling); every step runs the
two-exchange protocol inside libgvdb (gvdb_index_search_sharded_device): local
stage-1 keys -> ncclAllGather -> global top-R, rerank of the rows each rank
owns, local top-k -> ncclAllGather -> merged top-k, bit-identical to the
single-GPU result.  The exact flat search (recall 1.0) is reported beside it
through the same communicator.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "grape-vector-db_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

import gvdb  # noqa: E402

METRIC = "QPS @ recall@10, 10M×768 f32 (BQ on), batch-1 and batch-256, 1/2/4/8 GPU"
SEED = 0x6772617065  # "grape"
CHUNK = 1 << 20      # rows per generated chunk (global chunking: shard-independent data)
PEAK_HBM_GBS = 8000.0            # MI355X_MICROARCH.md: HBM3E 8 TB/s
PEAK_VALU_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12  # 256 CU x 4 SIMD x 32 lanes x 2.4 GHz int32 ops
PEAK_I8_TOPS = 5000.0  # dense i8 MFMA = 2x the 2.5 PF dense bf16 peak (MI355X_MICROARCH.md, Matrix cores)
PEAK_FP4_TFLOPS = 10000.0  # dense MX-FP4 MFMA = 4x dense bf16 (MI355X_MICROARCH.md: ~10 PF dense)


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def gen_chunk(c, n_rows, dim, device):
    g = torch.Generator(device=device)
    g.manual_seed(SEED + 1000 + c)
    x = torch.randn((n_rows, dim), generator=g, device=device, dtype=torch.float32)
    x /= torch.linalg.vector_norm(x, dim=1, keepdim=True)
    return x


def gen_queries(B, dim, device, seed_off=1):
    g = torch.Generator(device=device)
    g.manual_seed(SEED + seed_off)
    q = torch.randn((B, dim), generator=g, device=device, dtype=torch.float32)
    q /= torch.linalg.vector_norm(q, dim=1, keepdim=True)
    return q


def recall_at(found: np.ndarray, truth: np.ndarray) -> float:
    k = truth.shape[1]
    hits = 0
    for f, t in zip(found, truth):
        hits += len(set(int(v) for v in f[:k]) & set(int(v) for v in t))
    return hits / truth.size


def timing_slot(L, which):
    import ctypes as C

    ms, n = C.c_double(), C.c_uint64()
    L.gvdb_timing_read(which, C.byref(ms), C.byref(n))
    return ms.value, n.value


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=50)  # ~45 ms: the clocks settle (3 warm steps: scan +6 %)
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--R", type=int, default=100)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--b1-queries", type=int, default=200)
    ap.add_argument("--no-timing-events", dest="timing_events", action="store_false",
                    help="A/B probe only: no HIP events inside the timed loop (the roofline then has no live time)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget per CPU-baseline leg")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ref-faithful", dest="ref_faithful", action="store_false",
                    help="skip the ref-faithful id-remap side number of the CPU baseline")
    ap.add_argument("--hnsw-rows", type=int, default=1_000_000,
                    help="corpus prefix for the CPU-HNSW leg and its matched-N GPU points (0 = skip)")
    ap.add_argument("--no-points", dest="points", action="store_false", help="skip the QPS/recall operating points")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    comm_info = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=dev)
        assert dist.get_world_size() == world == args.gpus, (dist.get_world_size(), world, args.gpus)
        comm_info = {"world_size": dist.get_world_size(), "torch_backend": dist.get_backend(),
                     "merge_collective": "two ncclAllGather inside libgvdb (gvdb_index_search_sharded_device: "
                                         "stage-1 keys B*R*8 B, then local top-k B*k*16 B per rank)"}
        log(f"[bench] world={dist.get_world_size()} backend={dist.get_backend()} rank={rank} device={local_rank}")
    elif args.gpus != 1:
        raise SystemExit(f"--gpus {args.gpus} needs torch.distributed.run with {args.gpus} processes (WORLD_SIZE=1)")
    L = gvdb.lib()

    N, D, B, R, k = args.n, args.dim, args.batch, args.R, args.k
    lo, hi = N * rank // world, N * (rank + 1) // world
    n_local = hi - lo
    want_cpu = (not args.no_cpu_baseline) and world == 1 and rank == 0

    # ---------------- data: generate on device, build the shard index, ground truth
    t0 = time.time()
    q = gen_queries(B, D, dev)
    ix = gvdb.GpuVectorIndex(dimension=D, device=local_rank, capacity_hint=n_local)
    gt_val = torch.full((B, k), -2.0, device=dev)
    gt_idx = torch.zeros((B, k), dtype=torch.int64, device=dev)
    host_rows = np.empty((N, D), np.float32) if want_cpu else None
    host_codes = np.empty((N, (D + 7) // 8), np.uint8) if want_cpu else None
    code_buf = torch.empty((CHUNK, (D + 7) // 8), dtype=torch.uint8, device=dev) if want_cpu else None
    # planted queries (SURVEY §8(d) "Q-planted"): q = x_j + 0.1 n with |n| ~ 1 (the
    # rows are unit vectors), normalised, for B random rows j of the first chunk,
    # so every query has a true near neighbour (cos(q, x_j) ~ 0.995)
    planted = world == 1 and args.points
    if planted:
        pj = torch.from_numpy(np.sort(np.random.default_rng(SEED + 5).choice(min(N, CHUNK), B, replace=False)))
        pv = torch.full((B, k), -2.0, device=dev)
        pi = torch.zeros((B, k), dtype=torch.int64, device=dev)
        qp = None
    for c in range(lo // CHUNK, (hi - 1) // CHUNK + 1):
        c_lo, c_hi = c * CHUNK, min((c + 1) * CHUNK, N)
        x = gen_chunk(c, c_hi - c_lo, D, dev)
        a, b = max(lo, c_lo) - c_lo, min(hi, c_hi) - c_lo
        xs = x[a:b].contiguous()
        ids = torch.arange(c_lo + a, c_lo + b, dtype=torch.int64, device=dev)
        ix.add_device(xs, ids)
        s = q @ xs.T  # f32 exact top-k ground truth (cosine == dot for unit rows)
        v, i = torch.topk(torch.cat([gt_val, s], 1), k, dim=1)
        gt_idx = torch.gather(torch.cat([gt_idx, ids.expand(B, -1)], 1), 1, i)
        gt_val = v
        if planted:
            if qp is None:
                gq = torch.Generator(device=dev).manual_seed(SEED + 6)
                qp = xs[pj.to(dev)] + (0.1 / D ** 0.5) * torch.randn((B, D), generator=gq, device=dev)
                qp /= torch.linalg.vector_norm(qp, dim=1, keepdim=True)
            sp_ = qp @ xs.T
            v, i = torch.topk(torch.cat([pv, sp_], 1), k, dim=1)
            pi = torch.gather(torch.cat([pi, ids.expand(B, -1)], 1), 1, i)
            pv = v
            del sp_
        if want_cpu:
            host_rows[c_lo + a:c_lo + b] = xs.cpu().numpy()
            L.gvdb_bq_quantize_device(xs.data_ptr(), xs.shape[0], D, 0.0, code_buf.data_ptr(), None)
            torch.cuda.synchronize()
            host_codes[c_lo + a:c_lo + b] = code_buf[: xs.shape[0]].cpu().numpy()
        del x, xs, s
    torch.cuda.synchronize()
    if world > 1:
        import torch.distributed as dist

        allv = [torch.empty_like(gt_val) for _ in range(world)]
        alli = [torch.empty_like(gt_idx) for _ in range(world)]
        dist.all_gather(allv, gt_val)
        dist.all_gather(alli, gt_idx)
        v, i = torch.topk(torch.cat(allv, 1), k, dim=1)
        gt_idx = torch.gather(torch.cat(alli, 1), 1, i)
    truth = gt_idx.cpu().numpy()
    log(f"[bench] data+index+ground truth: {time.time() - t0:.1f}s  (shard rows {n_local})")

    sp = gvdb.SearchParams(rescore_count=R)
    out_ids = torch.zeros((B, k), dtype=torch.int64, device=dev)
    out_sc = torch.zeros((B, k), dtype=torch.float32, device=dev)
    out_n = torch.zeros(B, dtype=torch.int32, device=dev)

    if world == 1:
        def step():
            ix.search_device(q, k, out_ids, out_sc, out_n, sp)
    else:
        # the product path: local candidates -> ncclAllGather -> merge, all in libgvdb
        from gvdb.sharded import RcclShardedSearch

        sharded = RcclShardedSearch(ix, R, k)

        def step():
            sharded.search_into(q, out_ids, out_sc, out_n)

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            import torch.distributed as dist

            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    barrier()
    L.gvdb_timing_reset()
    L.gvdb_timing_enable(1 if args.timing_events else 0)
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    t_local = time.perf_counter() - t_start
    barrier()
    L.gvdb_timing_enable(0)
    t_max = t_local
    if world > 1:
        import torch.distributed as dist

        tt = torch.tensor([t_local], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_max = float(tt.item())
    if not args.timing_events:  # A/B probe: the per-kernel averages from an instrumented pass after the timed loop
        L.gvdb_timing_reset()
        L.gvdb_timing_enable(1)
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        L.gvdb_timing_enable(0)
    scan_ms, scan_n = timing_slot(L, 1)
    s1_ms = sum(timing_slot(L, i)[0] for i in (0, 1, 2))
    s2_ms, _ = timing_slot(L, 3)
    found = out_ids.cpu().numpy()
    rec = recall_at(found, truth)
    qps = B * args.steps / t_max

    # ---------------- batch-1 (single GPU only)
    b1 = None
    if world == 1 and args.b1_queries > 0:
        q1 = [q[i:i + 1].contiguous() for i in range(B)]
        o1i = torch.zeros((1, k), dtype=torch.int64, device=dev)
        o1s = torch.zeros((1, k), dtype=torch.float32, device=dev)
        # results (for recall and the batch comparison) and the scan's HIP-event
        # average come from an untimed pass; the timed pass is the searches alone
        # (no per-query result copies, no event records)
        res1 = []
        L.gvdb_timing_reset()
        L.gvdb_timing_enable(1)
        for i in range(min(B, args.b1_queries)):
            ix.search_device(q1[i], k, o1i, o1s, None, sp)
            res1.append(o1i.clone())
        torch.cuda.synchronize()
        L.gvdb_timing_enable(0)
        b1_scan_ms, b1_scan_n = timing_slot(L, 1)
        tb = time.perf_counter()
        for i in range(args.b1_queries):
            ix.search_device(q1[i % B], k, o1i, o1s, None, sp)
        torch.cuda.synchronize()
        tb = time.perf_counter() - tb
        f1 = torch.cat(res1).cpu().numpy()
        b1_scan_avg = b1_scan_ms / max(b1_scan_n, 1)
        code_bytes = n_local * gvdb_code_w4(D) * 16
        b1 = {
            "qps": args.b1_queries / tb,
            "ms_per_query": 1e3 * tb / args.b1_queries,
            "recall_at_10": recall_at(f1, truth[: len(f1)]),
            "same_results_as_batch": bool((f1 == found[: len(f1)]).all()),
            "roofline": {
                "kernel": "k_b1_scan (stage-1 BQ Hamming filter, batch 1: v_xor + v_bcnt, non-temporal code loads)",
                "bound": "hbm",
                "achieved": code_bytes / (b1_scan_avg * 1e-3) / 1e9,
                "peak": PEAK_HBM_GBS,
                "unit": "GB/s",
                "frac": code_bytes / (b1_scan_avg * 1e-3) / 1e9 / PEAK_HBM_GBS,
                "traffic": pmc_traffic("gvdb::k_b1_scan<", n_local, D),
                "avg_launch_ms": b1_scan_avg,
                "algorithmic_bytes_per_launch": code_bytes,
                "source": "avg_launch_ms: HIP events around each k_b1_scan launch on its stream; traffic: "
                          "rocprofv3 --pmc FETCH_SIZE x 2 (gfx950 streaming correction), " + PMC_FILE,
            },
        }

    # ---------------- QPS/recall operating points (single GPU): deeper BQ rescore
    # and the exact flat search (GVDB_SEARCH_FLAT, K4), same queries, same corpus
    points = None
    if world == 1 and args.points:
        points = []
        op_steps = max(2, args.steps // 4)

        def run_point(name, params, queries=None, gt=None, label="iid"):
            qq = q if queries is None else queries
            oi = torch.zeros((B, k), dtype=torch.int64, device=dev)
            osc = torch.zeros((B, k), dtype=torch.float32, device=dev)
            ix.search_device(qq, k, oi, osc, None, params)
            torch.cuda.synchronize()
            f0 = L.gvdb_flat_fallback_count()
            tp = time.perf_counter()
            for _ in range(op_steps):
                ix.search_device(qq, k, oi, osc, None, params)
            torch.cuda.synchronize()
            tp = time.perf_counter() - tp
            found, tr = oi.cpu().numpy(), truth if gt is None else gt
            points.append({"search": name, "queries": label, "qps": B * op_steps / tp,
                           "ms_per_step": 1e3 * tp / op_steps,
                           "recall_at_10": recall_at(found, tr),
                           "recall_at_1": float(np.mean(found[:, 0] == tr[:, 0])), "steps": op_steps,
                           **({"flat_fallbacks": int(L.gvdb_flat_fallback_count() - f0)} if params.mode == 1 else {})})

        points.append({"search": f"bq R={R}", "queries": "iid", "qps": qps, "ms_per_step": 1e3 * t_max / args.steps,
                       "recall_at_10": rec, "recall_at_1": float(np.mean(found[:, 0] == truth[:, 0])),
                       "steps": args.steps})
        for r in (1000, 4000):
            run_point(f"bq R={r}", gvdb.SearchParams(rescore_count=r))
        # the reference's DEFAULT depth, R = (N as f32 * 0.1) as usize (quantization.rs:27,178), answered by
        # the certified search (exact cosine top-32 filtered by the stage-1 membership rule)
        c0 = deep_cert_counts(L)
        run_point("bq R=0.1 N (reference default rescore_ratio, certified)", gvdb.SearchParams(rescore_ratio=0.1))
        c1 = deep_cert_counts(L)
        points[-1]["certified_batches"], points[-1]["rerank_batches"] = c1[0] - c0[0], c1[1] - c0[1]
        points[-1]["rooflines"] = deep_rooflines(L, ix, q, k, n_local, D)
        run_point("exact flat (i8/bf16-MFMA certified candidates + exact f32 rerank)", gvdb.SearchParams(mode=1))
        points[-1]["emit_roofline"] = flat_emit_roofline(L, ix, q, k, n_local, D)
        if planted:
            ptruth = pi.cpu().numpy()
            for r in (R, 1000):
                run_point(f"bq R={r}", gvdb.SearchParams(rescore_count=r), qp, ptruth, "planted (x_j + 0.1 n, |n| = 1)")
            run_point("exact flat (i8/bf16-MFMA certified candidates + exact f32 rerank)", gvdb.SearchParams(mode=1),
                      qp, ptruth, "planted (x_j + 0.1 n, |n| = 1)")

    # ---------------- N GPUs: the exact flat operating point (recall 1.0) through the
    # same communicator path (each rank's exact top-k, one ncclAllGather, merge)
    if world > 1 and args.points:
        import torch.distributed as dist
        from gvdb.sharded import RcclShardedSearch

        points = [{"search": f"bq R={R} (two-exchange)", "queries": "iid", "qps": qps,
                   "ms_per_step": 1e3 * t_max / args.steps, "recall_at_10": rec, "steps": args.steps}]
        shf = RcclShardedSearch(ix, R, k, params=gvdb.SearchParams(mode=1))
        fi = torch.zeros((B, k), dtype=torch.int64, device=dev)
        fs = torch.zeros((B, k), dtype=torch.float32, device=dev)
        shf.search_into(q, fi, fs, None)
        op_steps = max(2, args.steps // 4)
        barrier()
        tp = time.perf_counter()
        for _ in range(op_steps):
            shf.search_into(q, fi, fs, None)
        torch.cuda.synchronize()
        tp = time.perf_counter() - tp
        tt = torch.tensor([tp], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        tp = float(tt.item())
        points.append({"search": "exact flat (sharded: each rank's certified exact top-k, ncclAllGather, merge)",
                       "queries": "iid", "qps": B * op_steps / tp, "ms_per_step": 1e3 * tp / op_steps,
                       "recall_at_10": recall_at(fi.cpu().numpy(), truth), "steps": op_steps})
        shf.close()

    # ---------------- roofline of the dominant kernel (stage-1 scan at batch B)
    scan_avg = scan_ms / max(scan_n, 1)
    words = 4 * gvdb_code_w4(D)          # 32-bit code words per row (padded)
    variant = os.environ.get("GVDB_SCAN", "fp4")
    w4 = gvdb_code_w4(D)
    wide = w4 in MX4_QT and variant == "fp4"  # k_scan_mx4: ceil(B / 32QT) launches per batch
    mfma = B >= 96 and (w4 in (2, 3, 4, 6) and variant != "valu" or wide)
    scan_launches = -(-B // (32 * MX4_QT[w4])) if (mfma and wide) else 1
    if mfma:
        bpad = ((B + 31) // 32) * 32
        ops = float(n_local) * bpad * words * 32 * 2  # MACs x 2: one +/-1 product per code bit
        if wide:
            peak, kname = PEAK_FP4_TFLOPS, (f"k_scan_mx4 (+/-1 e2m1 dot, v_mfma_scale_f32_32x32x64_f8f6f4, rows in "
                                            f"VGPRs, {32 * MX4_QT[w4]} queries per launch, {scan_launches} launches "
                                            f"per batch; achieved over the batch's launches)")
        else:
            peak, kname = PEAK_FP4_TFLOPS, ("k_scan_mx7 ({0,1} x {+-1} e2m1 dot, rows as the A operand so a "
                                            "lane's 16 dots share one threshold, v_mfma_scale_f32_32x32x64_f8f6f4, "
                                            "rows in VGPRs, sub-tile boundary pipelined into the next sub-tile's "
                                            "first k-step)")
        roof = {
            "kernel": "stage-1 BQ Hamming filter: " + kname,
            "bound": "mfma",
            "achieved": ops / (scan_avg * 1e-3) / 1e12,
            "peak": peak,
            "unit": "TFLOP/s (MAC = 2 ops)",
        }
    else:
        ops = float(n_local) * B * words * 2  # v_xor_b32 + v_bcnt_u32_b32 per 32-bit word per pair
        peak = PEAK_VALU_TOPS
        roof = {
            "kernel": "k_scan (stage-1 BQ Hamming, xor+popcount on VALU)",
            "bound": "valu",
            "achieved": ops / (scan_avg * 1e-3) / 1e12,
            "peak": peak,
            "unit": "Tops/s (int32 lane-ops)",
        }
    roof.update({
        "frac": roof["achieved"] / peak,
        "traffic": pmc_traffic("gvdb::k_scan_mx7<6, false" if variant == "fp4" else "gvdb::k_scan<", n_local, D) if mfma else None,
        "avg_launch_ms": scan_avg,
        "algorithmic_ops_per_launch": ops,
        "hbm_bytes_per_launch": n_local * w4 * 16 * scan_launches,
        "source": f"avg_launch_ms: HIP events around each scan launch of the {args.steps} timed steps, on the "
                  f"search stream; the rocprofv3 kernel trace of this command gives the same launches' average "
                  f"(scripts/roofline_from_trace.py); traffic: rocprofv3 --pmc FETCH_SIZE x 2, {PMC_FILE}",
        "note": "batch-256 stage 1 is compute-bound (96 B of codes per row read once per batch); "
                "the HBM-bound batch-1 scan is in batch1.roofline",
    })

    # ---------------- CPU baseline (oracle = reference algorithm restated), bounded sample
    cpu = None
    parity = None
    if want_cpu:
        import oracle

        threads = cpu_share()
        qn = q.cpu().numpy()
        qbits = oracle.quantize(qn)
        ratio = np.float32(R) / np.float32(N)
        if oracle.rust_f32_as_usize(np.float32(N) * ratio) != R:
            ratio = np.nextafter(ratio, np.float32(1))
        # one query first to size the sample to the time budget
        t1 = time.perf_counter()
        oi, oc, on = oracle.multi_stage_search_batch(qbits[:1], host_codes, qn[:1], host_rows, float(ratio), R, 1)
        t_one = time.perf_counter() - t1
        nq = int(max(threads, min(B, (args.cpu_seconds / max(t_one, 1e-3)) * threads)))
        nq = max(threads, (nq // threads) * threads)
        t1 = time.perf_counter()
        oi, oc, on = oracle.multi_stage_search_batch(qbits[:nq], host_codes, qn[:nq], host_rows, float(ratio), R,
                                                     threads)
        t_cpu = time.perf_counter() - t1
        cpu = {
            "value": nq / t_cpu,
            "unit": "queries/s",
            "cores": threads,
            "kind": "port",
            "sample": f"{nq} of the {B} benchmark queries, full {N}x{D} corpus, "
                      f"BinaryQuantizer::multi_stage_search restated (stable sort of all N, R={R}), "
                      f"one query per thread",
            "single_thread_s_per_query": t_one,
        }
        # ref-faithful side number: HnswVectorIndex::search's O(N k) id remap
        # alone (index.rs:219-228), one query per thread -- an upper bound on the reference's
        # own search QPS at this N, before any graph traversal
        if args.ref_faithful:
            t1 = time.perf_counter()
            remap_s = oracle.ref_id_remap_seconds(N, k, threads, threads)
            cpu["ref_faithful"] = {
                "hnsw_search_id_remap_s_per_query": remap_s,
                "qps_upper_bound": threads / remap_s if remap_s > 0 else None,
                "cores": threads,
                "sample": f"{threads} queries x {k} hits, id_to_index of {N} entries (index.rs:219-228 restated: "
                          f"a heap-allocated format!(\"vec_{{}}\") per entry until the hit's value matches)",
                "wall_s_incl_map_build": time.perf_counter() - t1,
            }
        # full-scale parity on the CPU sample: GPU top-k == oracle top-k (ids + bit-exact cosine)
        gpu_sc = out_sc.cpu().numpy()
        ok_ids = bool((oi[:, :k] == found[:nq].astype(np.uint64)).all())
        ok_sc = oc[:, :k].tobytes() == gpu_sc[:nq].tobytes()
        parity = {"queries": nq, "ids_equal": ok_ids, "cosine_bit_exact": ok_sc}
        del host_codes

    # ---------------- CPU-HNSW leg at matched N: HnswVectorIndex's graph search
    # (instant-distance 0.6.1 restated, oracle/hnsw_oracle.cpp) on the first
    # --hnsw-rows rows of the same corpus, same box, same run (the full 10M-row CPU
    # build took 2.5 h on the 8-thread build container --
    # profiles/r03/equal_recall_10000000x768.json -- so the in-run leg is bounded
    # to 1M rows: ~215 s of build on the box's 16 cores), and the GPU on THE SAME
    # rows: a BQ rescore sweep and the exact flat search at batch 256 AND at batch 1
    # (one query per call, the reference's HnswVectorIndex::search contract), all
    # scored against the exact top-10 of that prefix.  gpu_vs_cpu_hnsw pairs every
    # ef_search point with the fastest GPU point of recall >= its recall - 0.02, at
    # each batch size.
    cpu_hnsw = None
    matched = None
    if want_cpu and args.hnsw_rows > 0:
        import oracle

        threads = cpu_share()
        ns = min(args.hnsw_rows, N)
        xs = np.ascontiguousarray(host_rows[:ns])
        qn = q.cpu().numpy()
        # exact top-k of the prefix on the GPU (f32; a CPU argsort of B x 1M scores took ~15 s)
        xt = torch.from_numpy(xs).to(dev)
        sub_truth = torch.topk(q @ xt.T, k, dim=1).indices.cpu().numpy()
        # planted queries (x_j + 0.1 n) whose row j lies in the prefix: their own truth
        use_planted = planted
        if use_planted:
            keep = torch.nonzero(pj < ns).flatten()
            qps_ = qp[keep.to(dev)].contiguous()
            use_planted = qps_.shape[0] > 0
        if use_planted:
            qpn = qps_.cpu().numpy()
            sub_ptruth = torch.topk(qps_ @ xt.T, k, dim=1).indices.cpu().numpy()
        log(f"[bench] CPU-HNSW leg: building M=32 ef_construction=100 on {ns} rows ({threads} threads)")
        tb = time.perf_counter()
        h = oracle.Hnsw(xs, threads=threads)
        tb = time.perf_counter() - tb

        def hnsw_point(ef, qq, tr, label):
            h.search(qq[:threads], k=k, ef_search=ef, threads=threads)
            th = time.perf_counter()
            hid, _, _ = h.search(qq, k=k, ef_search=ef, threads=threads)
            th = time.perf_counter() - th
            hid = hid.astype(np.int64)
            return {"ef_search": ef, "queries": label, "n_queries": len(qq), "qps": len(qq) / th,
                    "recall_at_10": recall_at(hid, tr), "recall_at_1": float(np.mean(hid[:, 0] == tr[:, 0]))}

        hpts = [hnsw_point(ef, qn, sub_truth, "iid") for ef in (64, 100, 200, 400)]
        # the high-ef end of the curve (recall@10 >= 0.9 needs ef ~ 16-32K at 1M i.i.d. unit rows,
        # profiles/r06/hnsw_recall_curve_*.json): 2 queries per thread, so it stays bounded
        nh = min(B, 2 * threads)
        hpts += [hnsw_point(ef, qn[:nh], sub_truth[:nh], "iid") for ef in (4000, 16000, 32000)]
        hpl = []
        if use_planted:
            hpl = [hnsw_point(ef, qpn, sub_ptruth, "planted") for ef in (64, 100, 200, 400)]
        t1 = time.perf_counter()
        h.search(qn[:16], k=k, ef_search=100, threads=1)
        t1 = (time.perf_counter() - t1) / 16
        ref = next(p for p in hpts if p["ef_search"] == 100)
        cpu_hnsw = {
            "value": ref["qps"], "unit": "queries/s", "cores": threads, "kind": "port",
            "recall_at_10": ref["recall_at_10"], "rows": ns, "build_s": tb,
            "single_thread_ms_per_query": 1e3 * t1, "points": hpts, "points_planted": hpl,
            "sample": f"HNSW M=32 ef_construction=100 (instant-distance 0.6.1 defaults, restated; value at "
                      f"ef_search=100) built on the first {ns} rows of the corpus; the {B} benchmark queries (ef >= "
                      f"4000: the first {nh}), one query per thread; recall vs the exact top-{k} of those {ns} rows",
        }
        del h
        # the GPU on the same prefix
        sub_ix = gvdb.GpuVectorIndex(dimension=D, capacity_hint=ns)
        sub_ix.add_device(xt, torch.arange(ns, dtype=torch.int64, device=dev))
        del xt
        osi = torch.zeros((B, k), dtype=torch.int64, device=dev)
        oss = torch.zeros((B, k), dtype=torch.float32, device=dev)
        searches = [(f"bq R={r}", gvdb.SearchParams(rescore_count=r)) for r in (10, 30, 100, 300, 1000, 3000)] + \
            [("bq R=0.1 N (reference default, certified)", gvdb.SearchParams(rescore_ratio=0.1)),
             ("exact flat", gvdb.SearchParams(mode=1))]

        def gpu_point(name, prm, qq, tr, label):
            nq = qq.shape[0]
            oi_ = osi if nq == B else torch.zeros((nq, k), dtype=torch.int64, device=dev)
            os_ = oss if nq == B else torch.zeros((nq, k), dtype=torch.float32, device=dev)
            sub_ix.search_device(qq, k, oi_, os_, None, prm)
            torch.cuda.synchronize()
            reps = 5
            tp = time.perf_counter()
            for _ in range(reps):
                sub_ix.search_device(qq, k, oi_, os_, None, prm)
            torch.cuda.synchronize()
            tp = time.perf_counter() - tp
            f = oi_.cpu().numpy()
            return {"search": name, "queries": label, "qps": nq * reps / tp, "batch": nq,
                    "recall_at_10": recall_at(f, tr), "recall_at_1": float(np.mean(f[:, 0] == tr[:, 0]))}

        gpts = [gpu_point(nm, prm, q, sub_truth, "iid") for nm, prm in searches]
        gpl = [gpu_point(nm, prm, qps_, sub_ptruth, "planted") for nm, prm in searches[:3] + searches[-1:]] \
            if use_planted else []
        # batch 1: one query per call over the benchmark queries (host sync per call excluded:
        # calls queue back to back on the stream, as a serving loop would)
        g1pts = []
        o1i = torch.zeros((1, k), dtype=torch.int64, device=dev)
        o1s = torch.zeros((1, k), dtype=torch.float32, device=dev)
        found = np.zeros((B, k), np.int64)
        for name, prm in [(f"bq R={r}", gvdb.SearchParams(rescore_count=r)) for r in (10, 100, 1000)] + \
                [("exact flat", gvdb.SearchParams(mode=1))]:
            for i in range(4):
                sub_ix.search_device(q[i:i + 1], k, o1i, o1s, None, prm)
            torch.cuda.synchronize()
            tp = time.perf_counter()
            for i in range(B):
                sub_ix.search_device(q[i:i + 1], k, o1i, o1s, None, prm)
            torch.cuda.synchronize()
            tp = time.perf_counter() - tp
            for i in range(B):  # the answers (recall), untimed
                sub_ix.search_device(q[i:i + 1], k, o1i, o1s, None, prm)
                found[i] = o1i[0].cpu().numpy()
            g1pts.append({"search": name, "queries": "iid", "qps": B / tp, "batch": 1,
                          "recall_at_10": recall_at(found, sub_truth),
                          "recall_at_1": float(np.mean(found[:, 0] == sub_truth[:, 0]))})
        # 64 concurrent single-query callers (the reference's readers of Arc<RwLock<dyn VectorIndex>>,
        # lib.rs:238), each calling gvdb_index_search(B = 1) from its own host thread through the
        # C ABI (grape-vector-db_amd/host/concurrent_b1.cpp); the library coalesces them
        gcpts = concurrent_b1_points(sub_ix, D, k, qn, sub_truth, qpn if use_planted else None,
                                     sub_ptruth if use_planted else None,
                                     [(f"bq R={r}", gvdb.SearchParams(rescore_count=r)) for r in (100, 1000)] +
                                     [("exact flat", gvdb.SearchParams(mode=1))], threads=64)
        del sub_ix
        torch.cuda.empty_cache()

        def pair_up(hp_list, points, key="recall_at_10"):
            out = []
            for hp in hp_list:
                ok = [g for g in points if g[key] >= hp[key] - 0.02]
                if ok:
                    best = max(ok, key=lambda g: g["qps"])
                    out.append({"hnsw_ef_search": hp["ef_search"], "hnsw_qps": hp["qps"], "hnsw_" + key: hp[key],
                                "gpu_search": best["search"], "gpu_qps": best["qps"], "gpu_" + key: best[key],
                                "speedup": best["qps"] / hp["qps"],
                                "degenerate": hp[key] < 0.5})
            return out

        iid_c = [g for g in gcpts if g["queries"] == "iid"]
        pl_c = [g for g in gcpts if g["queries"] == "planted"]
        pairs = {"batch256": pair_up(hpts, gpts), "batch1": pair_up(hpts, g1pts),
                 "concurrent64_batch1": pair_up(hpts, iid_c)}
        if use_planted:
            pairs["planted_recall_at_1_batch256"] = pair_up(hpl, gpl, "recall_at_1")
            pairs["planted_recall_at_1_concurrent64_batch1"] = pair_up(hpl, pl_c, "recall_at_1")
        # the north-star reading: HNSW's fastest point at recall@10 >= 0.9 against each GPU serving form
        hi = [p for p in hpts if p["recall_at_10"] >= 0.9]
        headline = None
        if hi:
            hb = max(hi, key=lambda p: p["qps"])
            headline = {"hnsw": hb}
            for tag, pts in (("batch256", gpts), ("batch1", g1pts), ("concurrent64_batch1", iid_c)):
                ok = [g for g in pts if g["recall_at_10"] >= hb["recall_at_10"] - 0.02]
                if ok:
                    best = max(ok, key=lambda g: g["qps"])
                    headline[tag] = {"gpu_search": best["search"], "gpu_qps": best["qps"],
                                     "gpu_recall_at_10": best["recall_at_10"], "speedup": best["qps"] / hb["qps"]}
        matched = {"rows": ns, "gpu_points": gpts, "gpu_points_planted": gpl, "gpu_points_batch1": g1pts,
                   "gpu_points_concurrent64": gcpts, "pairs": pairs, "equal_recall_at_least_0_9": headline,
                   "note": "same box, same run: matched N (the same prefix rows, ids = prefix rows) and matched recall "
                           "(GPU >= HNSW - 0.02). 'degenerate': the HNSW point is below 0.5 recall (i.i.d. unit rows "
                           "at 1M: graph search needs ef ~ 16-32K for recall@10 >= 0.9, "
                           "profiles/r06/hnsw_recall_curve_*.json). GPU forms: batch 256; batch 1 (one query per "
                           "call, back to back); 64 concurrent host threads each calling gvdb_index_search(B = 1) "
                           "(library-coalesced). The 10M-row CPU-HNSW table (profiles/r03/"
                           "equal_recall_10000000x768.json) was built in the 8-thread build container."}
        del xs

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": qps,
            "unit": "queries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * t_max / args.steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u32",
            "data": f"synthetic: i.i.d. N(0,1) f32 rows and queries, L2-normalised, torch Philox seed {SEED}"
                    + ("; operating_points also on planted queries x_j + 0.1 n, |n| = 1 (SURVEY 8(d))" if planted else ""),
            "config": {
                "workload": f"{N / 1e6:g}Mx{D} f32 corpus, BQ Hamming prefilter top-{R} + exact cosine rerank, "
                            f"k={k}, batch-{B} ({config_label(N, D)})",
                "n": N, "dim": D, "batch": B, "rescore_R": R, "k": k,
                "parallelism": f"corpus-shard x{world}" + (" + RCCL all-gather merge" if world > 1 else ""),
            },
            "recall_at_10": rec,
            "distributed": comm_info,
            "stage_ms_per_step": {"stage1": s1_ms / max(scan_n, 1), "scan": scan_avg, "stage2": s2_ms / max(scan_n, 1)},
            "roofline": roof,
            "batch1": b1,
            "cpu_baseline": cpu,
            "full_scale_parity": parity,
            "operating_points": points,
            "cpu_hnsw": cpu_hnsw,
        }
        if matched:
            line["gpu_vs_cpu_hnsw"] = matched
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist

        torch.cuda.synchronize()
        sharded.close()
        dist.destroy_process_group()


PMC_FILE = "profiles/r06/pmc_bench_10M.json"
PMC_FLAT_FILE = PMC_FILE  # the same passes cover k_flat_i8q (bench.py operating points, 10M x 768, B = 256)


def pmc_traffic(kernel_prefix, n_local, D, pmc_file=None):
    """HBM read bytes per launch of `kernel_prefix` from the committed PMC pass of
    this round (PMC_FILE: rocprofv3 --pmc FETCH_SIZE over bench.py's own command,
    x2 gfx950 streaming correction), only when collected at this workload's
    shard size."""
    if n_local != 10_000_000 or D != 768:
        return None
    for rel in ((pmc_file or PMC_FILE).split("/")[1:],):
        path = os.path.join(ROOT, "profiles", *rel)
        if not os.path.exists(path):
            continue
        with open(path) as f:
            kern = json.load(f)["kernels"]
        for name, d in kern.items():
            if name.startswith(kernel_prefix) and "hbm_read_bytes_per_launch" in d:
                return d["hbm_read_bytes_per_launch"]
    return None


def concurrent_b1_points(ix, D, k, qn, truth, qpn, ptruth, searches, threads=64, seconds=2.0):
    """QPS / latency / recall of `threads` host threads each calling gvdb_index_search(B = 1)
    concurrently on `ix` (build/libgvdb_drive.so, host/concurrent_b1.cpp: the C ABI only)."""
    import ctypes

    path = os.path.join(ROOT, "grape-vector-db_amd", "build", "libgvdb_drive.so")
    if not os.path.exists(path):  # built by __graft_entry__.build() (make); never fail the bench line over it
        log(f"[bench] {path} missing: no concurrent batch-1 points")
        return []
    drv = ctypes.CDLL(path)
    drv.gvdb_drive_concurrent_b1.restype = ctypes.c_int
    drv.gvdb_drive_concurrent_b1.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                             ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_double,
                                             ctypes.c_void_p, ctypes.c_void_p]
    out = []
    sets = [("iid", qn, truth)] + ([("planted", qpn, ptruth)] if qpn is not None else [])
    for label, qq, tr in sets:
        qq = np.ascontiguousarray(qq, np.float32)
        for name, prm in searches:
            if label == "planted" and name != "bq R=100":
                continue
            ids = np.zeros((len(qq), k), np.uint64)
            st = np.zeros(8, np.float64)
            c = prm.to_c()
            rc = drv.gvdb_drive_concurrent_b1(ix._h.value, qq.ctypes.data, len(qq), D, k, ctypes.addressof(c), threads,
                                              seconds, ids.ctypes.data, st.ctypes.data)
            if rc != 0:
                raise RuntimeError(f"concurrent batch-1 driver failed ({rc})")
            f = ids.astype(np.int64)
            out.append({"search": name, "queries": label, "callers": threads, "batch": 1, "qps": float(st[0]),
                        "p50_us": float(st[1]), "p99_us": float(st[2]), "recall_at_10": recall_at(f, tr),
                        "recall_at_1": float(np.mean(f[:, 0] == tr[:, 0]))})
    return out


def deep_cert_counts(L):
    """(certified, reranked) batch counters of the certified default-depth search."""
    import ctypes

    L.gvdb_debug_deep_cert.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
    out = (ctypes.c_uint64 * 2)()
    L.gvdb_debug_deep_cert(out)
    return int(out[0]), int(out[1])


def deep_rooflines(L, ix, q, k, n_local, D):
    """The reference default depth's two big kernels (certified search): the
    dense FP4 stage-1 scan (k_scan_mx7<DENSE>: every Hamming dot of the 256-slot query
    tile written as f16 -- HBM-bound on its writes) and the flat pass's i8 candidate
    kernel (k_flat_i8q, HBM-bound on the i8 mirror).  HIP events around each launch
    (gvdb_timing slots 1 and 7) over 3 searches."""
    B = q.shape[0]
    oi = torch.zeros((B, k), dtype=torch.int64, device=q.device)
    osc = torch.zeros((B, k), dtype=torch.float32, device=q.device)
    prm = gvdb.SearchParams(rescore_ratio=0.1)
    ix.search_device(q, k, oi, osc, None, prm)
    torch.cuda.synchronize()
    L.gvdb_timing_reset()
    L.gvdb_timing_enable(1)
    for _ in range(3):
        ix.search_device(q, k, oi, osc, None, prm)
    torch.cuda.synchronize()
    L.gvdb_timing_enable(0)
    sm, sn = timing_slot(L, 1)
    em, en = timing_slot(L, 7)
    L.gvdb_timing_reset()
    out = {}
    w4 = gvdb_code_w4(D)
    if sn:
        ms = sm / sn
        groups = -(-B // 256)
        byte_form = os.environ.get("GVDB_DENSE8", "1") != "0"  # round 6: one byte per pair
        if byte_form:
            wr = B * n_local  # the byte block: clamp(d - base, 0, 255) per (query, row)
        else:
            wr = 256 * groups * (-(-n_local // 32) * 32) * 2  # the f16 dot block
        rd = n_local * w4 * 16 * groups + wr  # the codes, and the block again by the rule's segment histograms
        ops = float(n_local) * 256 * groups * w4 * 128 * 2
        out["dense_scan"] = {
            "kernel": ("dense stage 1, byte form: k_dense_base (per-query window) + k_scan_mx7<DENSE, D8> (every "
                       "FP4-MFMA Hamming distance stored as one byte around the window) + the rule over that block "
                       "(k_dense_seg_hist8, k_dense_rule8)") if byte_form else
                      "dense stage 1: k_scan_mx7<DENSE> (every FP4-MFMA Hamming dot of the 256-slot tile stored as "
                      "f16) + the membership rule over that block (k_dense_seg_hist, k_dense_rule)",
            "bound": "hbm", "achieved": (rd + wr) / (ms * 1e-3) / 1e9, "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": (rd + wr) / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS, "traffic": None, "avg_launch_ms": ms,
            "algorithmic_bytes_per_launch": rd + wr, "reads": rd, "writes": wr,
            "mfma_frac": ops / (ms * 1e-3) / 1e12 / PEAK_FP4_TFLOPS,
            "source": "avg_launch_ms: HIP events around the dense scan + rule launches (gvdb_timing slot 1), "
                      "3 searches"}
    if en:
        ms = em / en
        algo = n_local * ((D + 127) // 128) * 128
        out["flat_pass"] = {
            "kernel": "k_flat_i8q (the certified list's i8 MFMA candidate pass over the int8 mirror)",
            "bound": "hbm", "achieved": algo / (ms * 1e-3) / 1e9, "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": algo / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS, "traffic": None, "avg_launch_ms": ms,
            "algorithmic_bytes_per_launch": algo,
            "source": "avg_launch_ms: HIP events around each emit launch (gvdb_timing slot 7), 3 searches"}
    return out or None


def flat_emit_roofline(L, ix, q, k, n_local, D):
    """The exact flat search's dominant kernel, its i8 candidate pass (k_flat_i8q at
    D = 768): HIP-event time per launch (gvdb_timing slot 7, 3 searches) against the
    algorithmic bytes of one launch (the N x ceil(D/128)*128 B int8 mirror, read
    once) -> HBM roofline fraction; traffic from the committed PMC pass."""
    B = q.shape[0]
    oi = torch.zeros((B, k), dtype=torch.int64, device=q.device)
    osc = torch.zeros((B, k), dtype=torch.float32, device=q.device)
    L.gvdb_timing_reset()
    L.gvdb_timing_enable(1)
    for _ in range(3):
        ix.search_device(q, k, oi, osc, None, gvdb.SearchParams(mode=1))
    torch.cuda.synchronize()
    L.gvdb_timing_enable(0)
    em, en = timing_slot(L, 7)
    L.gvdb_timing_reset()
    if en == 0:
        return None  # the bf16 tier or the exact scan answered
    ms = em / en
    algo = n_local * ((D + 127) // 128) * 128
    achieved = algo / (ms * 1e-3) / 1e9
    return {"kernel": "k_flat_i8q (exact flat, i8 MFMA candidate pass, query fragments in VGPRs, rows DMA'd to LDS)"
                      if D > 640 and D <= 768 else "k_flat_mx (exact flat, i8 candidate pass)",
            "bound": "hbm", "achieved": achieved, "peak": 8000.0, "unit": "GB/s", "frac": achieved / 8000.0,
            "traffic": pmc_traffic("gvdb::k_flat_i8q<", n_local, D, PMC_FLAT_FILE), "avg_launch_ms": ms,
            "algorithmic_bytes_per_launch": algo,
            "source": "avg_launch_ms: HIP events around each emit launch (gvdb_timing slot 7) over 3 searches; "
                      "traffic: rocprofv3 --pmc FETCH_SIZE x 2, " + PMC_FLAT_FILE}


def cpu_share():
    """Host cores this process may use: the job's CPU share (OMP_NUM_THREADS,
    16 per GPU on the GPU box, where nproc reports the whole machine), else
    the affinity mask."""
    omp = os.environ.get("OMP_NUM_THREADS", "")
    aff = len(os.sched_getaffinity(0))
    return max(1, min(aff, int(omp))) if omp.isdigit() and int(omp) > 0 else aff


def config_label(n, d):
    """Which BASELINE.json config a bench shape is (other shapes are labelled as such)."""
    if (n, d) == (10_000_000, 768):
        return "BASELINE configs[2]"
    if (n, d) == (1_000_000, 768):
        return "BASELINE configs[1]"
    if (n, d) == (10_000_000, 3072):
        return "BASELINE configs[3] corpus"
    if (n, d) == (1_250_000, 3072):
        return "one GPU's shard of BASELINE configs[3] (10M x 3072 over 8 GPUs)"
    return "not a BASELINE config"


# query tiles of 32 per k_scan_mx4 launch (LDS-bound), by code planes W4 (gvdb_kernels.hip dispatch)
MX4_QT = {8: 4, 12: 4, 16: 3, 24: 2, 32: 1}


def gvdb_code_w4(D):
    words = (((D + 7) // 8) + 3) // 4
    raw = (words + 3) // 4
    for w in (1, 2, 3, 4, 6, 8, 12, 16, 24, 32):
        if raw <= w:
            return w
    return raw


if __name__ == "__main__":
    main()
