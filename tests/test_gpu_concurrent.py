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
