"""Batch-1 BQ search latency on 10M x 768 (GPU box): per-query wall time and,
under rocprofv3 --kernel-trace --stats, the per-kernel split."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "grape-vector-db_amd")]
import torch  # noqa: E402

import gvdb  # noqa: E402

N, D = int(os.environ.get("N", 10_000_000)), 768
dev = torch.device("cuda", 0)
ix = gvdb.GpuVectorIndex(dimension=D, capacity_hint=N)
g = torch.Generator(device=dev).manual_seed(3)
for c0 in range(0, N, 1 << 20):
    n = min(1 << 20, N - c0)
    x = torch.randn((n, D), generator=g, device=dev)
    ix.add_device(x, torch.arange(c0, c0 + n, dtype=torch.int64, device=dev))
Q = torch.randn((int(os.environ.get("NQ", 200)), D), generator=g, device=dev)
oi = torch.zeros((1, 10), dtype=torch.int64, device=dev)
osc = torch.zeros((1, 10), device=dev)
p = gvdb.SearchParams(rescore_count=100)
for i in range(5):
    ix.search_device(Q[i:i + 1], 10, oi, osc, None, p)
torch.cuda.synchronize()
t = time.perf_counter()
for i in range(Q.shape[0]):
    ix.search_device(Q[i:i + 1], 10, oi, osc, None, p)
torch.cuda.synchronize()
t = time.perf_counter() - t
tag = os.environ.get("TAG", "")
print(f"batch-1{tag}: {1e3 * t / Q.shape[0]:.3f} ms/query, {Q.shape[0] / t:.0f} QPS", flush=True)
# concurrent single-query requests: S streams, each with its own output buffers
S = int(os.environ.get("STREAMS", 0))
if S > 1:
    streams = [torch.cuda.Stream() for _ in range(S)]
    outs = [(torch.zeros((1, 10), dtype=torch.int64, device=dev), torch.zeros((1, 10), device=dev)) for _ in range(S)]
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(Q.shape[0]):
        j = i % S
        ix.search_device(Q[i:i + 1], 10, outs[j][0], outs[j][1], None, p, stream=streams[j].cuda_stream)
    torch.cuda.synchronize()
    t = time.perf_counter() - t
    print(f"batch-1{tag} x{S} streams: {Q.shape[0] / t:.0f} QPS", flush=True)
