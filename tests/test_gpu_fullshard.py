"""GPU parity at the sizes the bench and config 3 time, against the CPU oracle.

The bench step (BASELINE configs[2]) and the config-3 rank run the stage-1
path that only exists above 262,144 rows: a SAMPLED Hamming threshold (the
fused FP4 sample pass, k_sample_prep), the k_scan_mx7 FP4-MFMA scan for
B >= 96, then select, the exact rerank (k_rerank_dma) and the final stable
sort.  The smaller oracle tests (test_gpu_parity.py) cover the whole-shard
"sample"; these run the sampled path at the config-3 shard (1.25M x 768) and
config 2 (1M x 768), batch 256, R = 100, k = 10, through ``search_device``
(the entry point bench.py times), and compare ids and cosine bits with
oracle.multi_stage_search_batch_r (quantization.rs:151-193 restated).

Ties at the sampled threshold: rows [N - T, N) are copies of rows [0, T),
so every distance that occurs among the first T rows occurs twice (equal
Hamming AND equal cosine: the (d asc, row asc) stage-1 order and the stable
cosine sort decide between the twins).  A block of 300 copies of row 5 with
query 0 = row 5 puts 300 rows at distance 0 for R = 100 (the cut inside one
tie run), and query 1 = row 9 plants a single exact hit.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def corpus(N, D, seed, twins=100_000, block=300):
    r = np.random.default_rng(seed)
    x = r.standard_normal((N, D), dtype=np.float32)
    x[N - twins:] = x[:twins]
    x[1000:1000 + block] = x[5]
    q = r.standard_normal((256, D), dtype=np.float32)
    q[0] = x[5]
    q[1] = x[9]
    q[2] = x[N - 1]  # a twin: rows twins-1 and N-1 tie at distance 0
    return x, q


@pytest.mark.parametrize("N", [1_250_000, 1_000_000])
def test_sampled_path_b256_matches_oracle(gvdb_mod, oracle_mod, N):
    import ctypes as C
    import os

    import torch

    g = gvdb_mod
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    D, B, R, k = 768, 256, 100, 10
    x, Q = corpus(N, D, seed=N // 1000)
    dev = torch.device("cuda", 0)
    ix = g.GpuVectorIndex(dimension=D, capacity_hint=N)
    for c0 in range(0, N, 1 << 19):
        n = min(1 << 19, N - c0)
        ix.add_device(torch.from_numpy(x[c0:c0 + n]).to(dev), torch.arange(c0, c0 + n, device=dev))
    q = torch.from_numpy(Q).to(dev)
    oi = torch.zeros((B, k), dtype=torch.int64, device=dev)
    osc = torch.zeros((B, k), dtype=torch.float32, device=dev)
    on = torch.zeros(B, dtype=torch.int32, device=dev)
    L = g.lib()
    L.gvdb_debug_stage1_thresholds.argtypes = [C.POINTER(C.c_uint32), C.c_uint32]
    os.environ["GVDB_DEBUG_THR"] = "1"
    try:
        ix.search_device(q, k, oi, osc, on, g.SearchParams(rescore_count=R))
        torch.cuda.synchronize()
        thr = (C.c_uint32 * B)()
        assert L.gvdb_debug_stage1_thresholds(thr, B) == 0
    finally:
        os.environ.pop("GVDB_DEBUG_THR", None)
    # the sampled estimate is a real one (not the no-pruning fallback)
    assert max(thr) < D
    # stage-1 rows + Hamming distances against the oracle's exact top-R
    rows = torch.zeros((B, R), dtype=torch.int64, device=dev)
    dist = torch.zeros((B, R), dtype=torch.int32, device=dev)
    ix.bq_topr_device(q, R, rows, dist)
    torch.cuda.synchronize()
    qb, xb = oracle_mod.quantize(Q), oracle_mod.quantize(x)
    ri, rd = oracle_mod.bq_topr_batch(qb, xb, D, R, threads=16)
    assert (dist.cpu().numpy().astype(np.uint32) == rd).all()
    assert (rows.cpu().numpy().astype(np.uint64) == ri).all()
    # the whole search: ids equal, cosine bits equal
    mi, ms = oracle_mod.multi_stage_search_batch_r(qb, xb, Q, x, R, threads=16)
    gi = oi.cpu().numpy().astype(np.uint64)
    gs = osc.cpu().numpy()
    assert (on.cpu().numpy() == k).all()
    assert (gi == mi[:, :k]).all()
    assert gs.tobytes() == np.ascontiguousarray(ms[:, :k]).tobytes()
    # the planted rows (the tie block's first copies and the exact hits) are found
    assert gi[0, 0] == 5 and gi[1, 0] == 9 and gi[2, 0] == 100_000 - 1
