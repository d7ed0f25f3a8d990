"""GPU: the ABI's reentrancy promise under concurrent readers.

The reference shares its index as Arc<tokio::sync::RwLock<dyn VectorIndex>>
(src/lib.rs:238, 259-261): many concurrent `&self` searches, exclusive
writes.  include/gvdb.h promises the same: gvdb_index_search* are reentrant
(per-call workspace from a pool, per-index in-flight tracking), mutations take
the caller's exclusive lock.  Here 8 host threads (ctypes drops the GIL
during the foreign call) search one index at once -- host-buffer batch-1 and
batch-256 searches, and _device searches each on its own HIP stream -- and
every result must be bit-equal to the serial one.  Between rounds the writer
adds and removes rows with no reader active (the RwLock write side), and the
next round's serial references are recomputed.
"""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def g(gvdb_mod):
    import torch

    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return gvdb_mod


def test_concurrent_readers_equal_serial(g):
    import torch

    rng = np.random.default_rng(2024)
    N, D, T = 300_000, 768, 8
    x = rng.standard_normal((N, D)).astype(np.float32)
    ix = g.GpuVectorIndex(dimension=D, capacity_hint=N + 10_000)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    Q256 = rng.standard_normal((256, D)).astype(np.float32)
    Q1 = rng.standard_normal((T, D)).astype(np.float32)
    sp = g.SearchParams(rescore_count=100)
    k = 10
    qd = torch.from_numpy(Q256).cuda()

    def serial():
        ref = {}
        for t in range(T):
            ref[("b1", t)] = ix.search_batch(Q1[t:t + 1], k, sp)
        ref["b256"] = ix.search_batch(Q256, k, sp)
        return ref

    def reader(t, ref, errors, barrier):
        try:
            s = torch.cuda.Stream()
            oi = torch.zeros((256, k), dtype=torch.int64, device="cuda")
            osc = torch.zeros((256, k), dtype=torch.float32, device="cuda")
            on = torch.zeros(256, dtype=torch.int32, device="cuda")
            barrier.wait()
            for it in range(6):
                if (t + it) % 3 == 0:
                    got = ix.search_batch(Q1[t:t + 1], k, sp)
                    want = ref[("b1", t)]
                elif (t + it) % 3 == 1:
                    got = ix.search_batch(Q256, k, sp)
                    want = ref["b256"]
                else:
                    ix.search_device(qd, k, oi, osc, on, sp, stream=s.cuda_stream)
                    s.synchronize()
                    got = (oi.cpu().numpy().view(np.uint64), osc.cpu().numpy(), on.cpu().numpy().view(np.uint32))
                    want = ref["b256"]
                ok = ((got[0] == want[0]).all() and got[1].tobytes() == want[1].tobytes()
                      and (got[2] == want[2]).all())
                if not ok:
                    errors.append((t, it))
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append((t, repr(e)))

    next_id = N
    for rnd in range(3):
        ref = serial()
        errors = []
        barrier = threading.Barrier(T)
        th = [threading.Thread(target=reader, args=(t, ref, errors, barrier)) for t in range(T)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errors, (rnd, errors[:5])
        # the writer's turn (no reader active): add rows near some queries, remove others
        add = Q256[rnd * 8:rnd * 8 + 8] + 0.01 * rng.standard_normal((8, D)).astype(np.float32)
        ix.add_batch(np.arange(next_id, next_id + 8, dtype=np.uint64), add)
        next_id += 8
        for rid in (int(ref["b256"][0][rnd, 0]), int(ref["b256"][0][rnd + 1, 0])):
            assert ix.remove_vector_id(rid)
    # the last mutations are visible: the added rows are found
    ids, _, _ = ix.search_batch(Q256[16:24], 1, sp)
    assert set(int(v) for v in ids[:, 0]) <= set(range(N, next_id))


def test_concurrent_default_depth_device_searches_equal_serial(g):
    """The async certified default depth (R = 0.1 N, quantization.rs:27,178) runs
    its flat pass on a second pooled workspace whose failure word the certify
    pass reads later on the caller's stream (the word is now copied
    into the caller's own workspace before the pooled one is released).  Four
    threads, each on its own stream, interleave default-depth and FLAT-mode
    _device searches (the FLAT calls take pooled workspaces and clear their
    words) with no sync between enqueues; every result equals the serial
    host-buffer search bit for bit."""
    import torch

    rng = np.random.default_rng(77)
    N, D, B, T, k = 200_000, 768, 64, 4, 10
    x = rng.standard_normal((N, D)).astype(np.float32)
    ix = g.GpuVectorIndex(dimension=D, capacity_hint=N)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    Q = rng.standard_normal((T, B, D)).astype(np.float32)
    deep = g.SearchParams()  # mode BQ_RERANK, rescore_ratio 0.1 -> R = 20000
    flat = g.SearchParams(mode=g._ffi.GVDB_SEARCH_FLAT)
    ref = {(t, m): ix.search_batch(Q[t], k, sp) for t in range(T) for m, sp in (("deep", deep), ("flat", flat))}
    errors = []
    barrier = threading.Barrier(T)

    def worker(t):
        try:
            s = torch.cuda.Stream()
            outs = []
            with torch.cuda.stream(s):  # inputs, outputs and searches all ordered on s
                q = torch.from_numpy(Q[t]).cuda()
                s.synchronize()
                barrier.wait()
                for it in range(8):
                    m = "deep" if (t + it) % 2 == 0 else "flat"
                    oi = torch.zeros((B, k), dtype=torch.int64, device="cuda")
                    osc = torch.zeros((B, k), dtype=torch.float32, device="cuda")
                    on = torch.zeros(B, dtype=torch.int32, device="cuda")
                    ix.search_device(q, k, oi, osc, on, deep if m == "deep" else flat, stream=s.cuda_stream)
                    outs.append((m, oi, osc, on))
            s.synchronize()
            for m, oi, osc, on in outs:
                want = ref[(t, m)]
                got = (oi.cpu().numpy().view(np.uint64), osc.cpu().numpy(), on.cpu().numpy().view(np.uint32))
                if not ((got[0] == want[0]).all() and got[1].tobytes() == want[1].tobytes()
                        and (got[2] == want[2]).all()):
                    errors.append((t, m))
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append((t, repr(e)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[:5]


def test_concurrent_batch1_callers_coalesce_and_equal_serial(g):
    """Raw gvdb_index_search with B = 1 from many threads (the reference's
    concurrent readers, lib.rs:238 + index.rs:212-231) is coalesced inside the
    library: batches form while one executes, requests with a different k or
    params never share a batch, and every answer equals the serial call's."""
    import ctypes as C

    rng = np.random.default_rng(4242)
    N, D, T, per = 400_000, 768, 48, 6
    x = rng.standard_normal((N, D)).astype(np.float32)
    ix = g.GpuVectorIndex(dimension=D, capacity_hint=N)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    Q = rng.standard_normal((T * per, D)).astype(np.float32)
    Q[7] = x[123]
    sps = [g.SearchParams(rescore_count=100), g.SearchParams(rescore_count=300),
           g.SearchParams(mode=g._ffi.GVDB_SEARCH_FLAT)]
    ks = [10, 10, 5]
    ref = [ix.search_batch(Q[i:i + 1], ks[i % 3], sps[i % 3]) for i in range(T * per)]
    L = g.lib()
    L.gvdb_debug_b1_coalesce.argtypes = [C.POINTER(C.c_uint64)]
    before = (C.c_uint64 * 3)()
    L.gvdb_debug_b1_coalesce(before)
    errors = []
    barrier = threading.Barrier(T)

    def worker(t):
        try:
            barrier.wait()
            for j in range(per):
                i = t * per + j
                got = ix.search_batch(Q[i:i + 1], ks[i % 3], sps[i % 3])
                want = ref[i]
                if not ((got[0] == want[0]).all() and got[1].tobytes() == want[1].tobytes()
                        and (got[2] == want[2]).all()):
                    errors.append(i)
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append((t, repr(e)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[:5]
    after = (C.c_uint64 * 3)()
    L.gvdb_debug_b1_coalesce(after)
    nq = after[1] - before[1]
    assert nq == T * per
    assert after[0] - before[0] < nq  # some searches were shared
    assert int(ref[7][0][0, 0]) == 123
