"""Timing of the exact flat search (GVDB_SEARCH_FLAT, bf16-MFMA candidates +
exact rerank) on the GPU box: N x D corpus, batches of B queries.
Prints ms per batch, QPS and the certification fallback count."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "grape-vector-db_amd")]
import torch  # noqa: E402

import gvdb  # noqa: E402

N = int(os.environ.get("N", 10_000_000))
D = int(os.environ.get("D", 768))
K = int(os.environ.get("K", 10))
dev = torch.device("cuda", 0)
ix = gvdb.GpuVectorIndex(dimension=D, capacity_hint=N)
g = torch.Generator(device=dev).manual_seed(7)
for c0 in range(0, N, 1 << 20):
    n = min(1 << 20, N - c0)
    x = torch.randn((n, D), generator=g, device=dev)
    ix.add_device(x, torch.arange(c0, c0 + n, dtype=torch.int64, device=dev))
L = gvdb.lib()
p = gvdb.SearchParams(mode=1, metric=0)
for B in [int(b) for b in os.environ.get("BS", "256,64,1").split(",")]:
    q = torch.randn((B, D), generator=g, device=dev)
    oi = torch.zeros((B, K), dtype=torch.int64, device=dev)
    osc = torch.zeros((B, K), device=dev)
    for _ in range(2):
        ix.search_device(q, K, oi, osc, None, p)
    torch.cuda.synchronize()
    f0 = L.gvdb_flat_fallback_count()
    f8 = L.gvdb_flat_i8_fallback_count()
    reps = int(os.environ.get("FLAT_REPS", 10 if B > 1 else 20))
    t = time.perf_counter()
    for _ in range(reps):
        ix.search_device(q, K, oi, osc, None, p)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) * 1e3 / reps
    L.gvdb_timing_reset()
    L.gvdb_timing_enable(1)
    for _ in range(3):
        ix.search_device(q, K, oi, osc, None, p)
    L.gvdb_timing_enable(0)
    import ctypes as C
    em, en, tm, tn = C.c_double(), C.c_uint64(), C.c_double(), C.c_uint64()
    # slots 7/8 = the i8 tier, 5/6 = bf16: report the tier that ran
    L.gvdb_timing_read(7, C.byref(em), C.byref(en))
    L.gvdb_timing_read(8, C.byref(tm), C.byref(tn))
    i8 = en.value > 0
    if not i8:
        L.gvdb_timing_read(5, C.byref(em), C.byref(en))
        L.gvdb_timing_read(6, C.byref(tm), C.byref(tn))
    e_ms = em.value / max(en.value, 1)
    kpad = (D + 127) // 128 * 128 if i8 else (D + 63) // 64 * 64
    tf = 2.0 * N * kpad * 256 / (e_ms * 1e-3) / 1e12 if e_ms > 0 else 0.0  # 0: the small-N path ran
    gbs = N * kpad * (1 if i8 else 2) / (e_ms * 1e-3) / 1e9 if e_ms > 0 else 0.0
    print(f"        k_flat_mx emit {e_ms:.3f} ms ({tf:.0f} TOP/s incl. padding slots, {gbs:.0f} GB/s rows), "
          f"group total {tm.value / max(tn.value, 1):.3f} ms", flush=True)
    print(f"B={B:4d}  {ms:8.3f} ms/batch  {B / ms * 1e3:10.0f} QPS  fallbacks {L.gvdb_flat_fallback_count() - f0}"
          f"  i8->bf16 retries {L.gvdb_flat_i8_fallback_count() - f8}  [{'i8' if i8 else 'bf16'} tier timed]",
          flush=True)
