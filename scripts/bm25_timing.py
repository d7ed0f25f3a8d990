#!/usr/bin/env python3
"""BM25 leg of configs[4] alone: the 5M-document Zipf(1.1) corpus of
scripts/bench_hybrid.py, 64-query batches of 2*limit, timed per call; with
--check, the first batch is compared with the oracle (bit-exact)."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "grape-vector-db_amd"), os.path.join(ROOT, "scripts")]
from bench_hybrid import SEED, zipf_corpus  # noqa: E402

from gvdb import sparse as gsp  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=5_000_000)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--limit", type=int, default=10)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--check", action="store_true")
    a = ap.parse_args()
    t0 = time.time()
    dptr, dterms, dtfs, ddls = zipf_corpus(a.n, 50_000, 40, 1.1, SEED + 1)
    sp = gsp.SparseIndex()
    sp.add_documents_u64(np.arange(a.n, dtype=np.uint64), dptr, dterms, dtfs, ddls)
    qptr, qterms, qtfs, _ = zipf_corpus(a.batch, 50_000, 8, 1.1, SEED + 12)
    print(f"[bm25] corpus {dterms.size} postings in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    want = 2 * a.limit
    t = time.perf_counter()
    ids, sc, n = sp.search_bm25_csr(qptr, qterms, qtfs, want)
    first = time.perf_counter() - t
    ts = []
    for _ in range(a.steps):
        t = time.perf_counter()
        ids, sc, n = sp.search_bm25_csr(qptr, qterms, qtfs, want)
        ts.append(time.perf_counter() - t)
    line = {"n": a.n, "postings": int(dterms.size), "batch": a.batch, "limit": want,
            "first_call_ms": 1e3 * first, "ms_per_batch": 1e3 * float(np.median(ts)), "min_ms": 1e3 * min(ts)}
    if a.check:
        import oracle

        o = oracle.Bm25()
        o.add_documents_csr(np.arange(a.n, dtype=np.uint64), dptr, dterms, dtfs, ddls)
        nq = min(16, a.batch)
        oi, osc, on = o.search_batch(qptr[: nq + 1], qterms, qtfs, want, threads=16)
        line["parity"] = all(list(oi[q, : on[q]]) == list(ids[q, : n[q]]) and
                             osc[q, : on[q]].tobytes() == sc[q, : n[q]].tobytes() for q in range(nq))
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
