#!/usr/bin/env python3
"""BASELINE.json configs[4]: hybrid dense + sparse search with RRF
(src/hybrid.rs:286-356), 5M x 768 dense corpus + BM25 over a synthetic
Zipf(1.1) vocabulary of 50k terms (~40 tokens per document), batch 64.

A step = one batch of 64 hybrid queries: dense search top 2*limit
(HnswVectorIndex::search semantics: L2, here the GPU BQ prefilter + exact
rerank, R = 100), BM25 top 2*limit (SparseIndex::search_bm25 on the GPU),
RRF of the two lists top `limit` (GPU) -- with the corpus and the forward
index resident in HBM.  Prints one JSON line.

CPU baseline: the BM25 leg only (the reference's dense leg is an HNSW whose
5M-row build is out of reach), restated as the oracle's posting-list walk
(oracle/bm25_oracle.cpp), one query per thread on a bounded sample of the
same queries; its results are also compared with the GPU's (bit-exact).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "grape-vector-db_amd")]
import torch  # noqa: E402

import gvdb  # noqa: E402
from gvdb import sparse as gsp  # noqa: E402

SEED = 0x6772617065


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def zipf_corpus(n, vocab, tokens, a, seed, chunk=250_000):
    """CSR of n documents: `tokens` Zipf(a) draws each -> distinct terms
    (ascending) with relative frequency tf = count / tokens, dl = sum tf."""
    r = np.random.default_rng(seed)
    p = 1.0 / np.arange(1, vocab + 1, dtype=np.float64) ** a
    cdf = np.cumsum(p / p.sum())
    ptrs, terms, tfs, dls = [np.zeros(1, np.uint64)], [], [], []
    base = 0
    for c0 in range(0, n, chunk):
        m = min(chunk, n - c0)
        tok = np.searchsorted(cdf, r.random((m, tokens))).astype(np.uint32)
        tok = np.minimum(tok, vocab - 1)
        tok.sort(axis=1)
        new = np.ones_like(tok, dtype=bool)
        new[:, 1:] = tok[:, 1:] != tok[:, :-1]
        idx = np.flatnonzero(new.ravel())
        run = np.diff(np.append(idx, m * tokens)).astype(np.float32)
        tf = (run / np.float32(tokens)).astype(np.float32)
        cnt = new.sum(axis=1)
        p0 = np.concatenate([[0], np.cumsum(cnt)]).astype(np.uint64)
        dl = np.add.reduceat(tf.astype(np.float64), p0[:-1].astype(np.int64)).astype(np.float32)
        terms.append(tok.ravel()[idx])
        tfs.append(tf)
        dls.append(dl)
        ptrs.append(p0[1:] + base)
        base += int(p0[-1])
    return np.concatenate(ptrs), np.concatenate(terms), np.concatenate(tfs), np.concatenate(dls)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=5_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--limit", type=int, default=10)
    ap.add_argument("--vocab", type=int, default=50_000)
    ap.add_argument("--tokens", type=int, default=40)
    ap.add_argument("--qterms", type=int, default=8)
    ap.add_argument("--zipf", type=float, default=1.1)
    ap.add_argument("--R", type=int, default=100)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    N, D, B, L = args.n, args.dim, args.batch, args.limit
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    t0 = time.time()
    # dense corpus (L2-normalised N(0,1) rows) straight into HBM
    ix = gvdb.GpuVectorIndex(dimension=D, capacity_hint=N)
    for c0 in range(0, N, 1 << 20):
        m = min(1 << 20, N - c0)
        g = torch.Generator(device=dev).manual_seed(SEED + 7000 + c0)
        x = torch.randn((m, D), generator=g, device=dev)
        x /= torch.linalg.vector_norm(x, dim=1, keepdim=True)
        ix.add_device(x, torch.arange(c0, c0 + m, dtype=torch.int64, device=dev))
        del x
    torch.cuda.synchronize()
    log(f"[hybrid] dense corpus {N}x{D}: {time.time() - t0:.1f}s")
    t1 = time.time()
    dptr, dterms, dtfs, ddls = zipf_corpus(N, args.vocab, args.tokens, args.zipf, SEED + 1)
    log(f"[hybrid] sparse corpus: {dterms.size} postings, {time.time() - t1:.1f}s")
    t1 = time.time()
    sp = gsp.SparseIndex()
    sp.add_documents_u64(np.arange(N, dtype=np.uint64), dptr, dterms, dtfs, ddls)
    log(f"[hybrid] BM25 index add: {time.time() - t1:.1f}s")

    # queries
    g = torch.Generator(device=dev).manual_seed(SEED + 11)
    qd = torch.randn((B, D), generator=g, device=dev)
    qd /= torch.linalg.vector_norm(qd, dim=1, keepdim=True)
    qptr, qterms, qtfs, _ = zipf_corpus(B, args.vocab, args.qterms, args.zipf, SEED + 12)
    want = 2 * L
    params = gvdb.SearchParams(metric=gvdb._ffi.GVDB_METRIC_L2, rescore_count=args.R)
    d_ids = torch.zeros((B, want), dtype=torch.int64, device=dev)
    d_sc = torch.zeros((B, want), dtype=torch.float32, device=dev)
    d_n = torch.zeros(B, dtype=torch.int32, device=dev)
    Lb = gvdb.lib()
    f_ids = np.zeros((B, L), np.uint64)
    f_sc = np.zeros((B, L), np.float32)
    f_n = np.zeros(B, np.uint32)
    tm = {"dense": 0.0, "bm25": 0.0, "rrf": 0.0}

    def step(timed):
        ta = time.perf_counter()
        ix.search_device(qd, want, d_ids, d_sc, d_n, params)
        torch.cuda.synchronize()
        tb = time.perf_counter()
        s_ids, s_sc, s_n = sp.search_bm25_csr(qptr, qterms, qtfs, want)
        tc = time.perf_counter()
        di = d_ids.cpu().numpy().astype(np.uint64)
        ds = d_sc.cpu().numpy()
        dn = d_n.cpu().numpy().astype(np.uint32)
        s_ids = np.ascontiguousarray(s_ids)
        s_sc = np.ascontiguousarray(s_sc)
        gvdb.check(Lb.gvdb_rrf_fuse(di.ctypes.data, ds.ctypes.data, dn.ctypes.data, want, s_ids.ctypes.data,
                                    s_sc.ctypes.data, s_n.ctypes.data, want, None, None, None, 0, B, 60.0, L,
                                    f_ids.ctypes.data, f_sc.ctypes.data, None, f_n.ctypes.data))
        td = time.perf_counter()
        if timed:
            tm["dense"] += tb - ta
            tm["bm25"] += tc - tb
            tm["rrf"] += td - tc
        return s_ids, s_sc, s_n

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.steps):
        s_ids, s_sc, s_n = step(True)
    torch.cuda.synchronize()
    t = time.perf_counter() - t
    nnz = int(dterms.size)
    bm25_ms = 1e3 * tm["bm25"] / args.steps
    line = {
        "metric": "hybrid QPS (dense top-2k + BM25 top-2k + RRF top-k), BASELINE configs[4]",
        "value": B * args.steps / t, "unit": "queries/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": 1e3 * t / args.steps, "higher_is_better": True, "dtype": "f32",
        "data": f"synthetic: dense i.i.d. N(0,1) L2-normalised; sparse Zipf({args.zipf}) over {args.vocab} terms, "
                f"{args.tokens} tokens/doc, {args.qterms}-token queries",
        "config": {"workload": f"{N}x{D} dense (BQ R={args.R} + exact L2 rerank) + BM25 ({nnz} postings), RRF k=60, "
                               f"limit {L}, batch {B}", "n": N, "dim": D, "batch": B, "limit": L,
                   "postings": nnz},
        "stage_ms_per_step": {k: 1e3 * v / args.steps for k, v in tm.items()},
        "bm25_forward_index_GBps": nnz * 12 / (bm25_ms * 1e-3) / 1e9,
        "bm25_dense_fallbacks": sp.get_stats().dense_fallbacks,
    }
    if not args.no_cpu_baseline:
        import oracle

        threads = max(1, min(16, len(os.sched_getaffinity(0))))
        t1 = time.time()
        o = oracle.Bm25()
        o.add_documents_csr(np.arange(N, dtype=np.uint64), dptr, dterms, dtfs, ddls)
        build_s = time.time() - t1
        t1 = time.perf_counter()
        oi, osc, on = o.search_batch(qptr[:2], qterms, qtfs, want, threads=1)
        t_one = (time.perf_counter() - t1) / 1
        nq = int(max(threads, min(B, (args.cpu_seconds / max(t_one, 1e-3)) * threads)))
        nq = min(B, max(threads, (nq // threads) * threads))
        t1 = time.perf_counter()
        oi, osc, on = o.search_batch(qptr[: nq + 1], qterms, qtfs, want, threads=threads)
        t_cpu = time.perf_counter() - t1
        ok_ids = all(list(oi[q, : on[q]]) == list(s_ids[q, : s_n[q]]) for q in range(nq))
        ok_sc = all(osc[q, : on[q]].tobytes() == s_sc[q, : s_n[q]].tobytes() for q in range(nq))
        line["cpu_baseline"] = {"value": nq / t_cpu, "unit": "BM25 queries/s", "cores": threads, "kind": "port",
                                "sample": f"BM25 leg only: {nq} of the {B} queries over the full {N}-document "
                                          f"index (posting-list walk, sparse.rs:151-198 restated; build {build_s:.0f}s)",
                                "gpu_bm25_qps": B / (bm25_ms * 1e-3)}
        line["bm25_parity"] = {"queries": nq, "ids_equal": bool(ok_ids), "scores_bit_exact": bool(ok_sc)}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
