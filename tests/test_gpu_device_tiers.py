"""GPU: the _device entry points return without a host sync in EVERY search mode
(VERDICT r04 item 4).  The fallback tiers are enqueued behind the tier they back
up and gated on the device by that tier's failure word (gvdb_device.h
gate_closed):

* FLAT (storage.rs:296-339 / index.rs:620-640): the i8 (or bf16) MFMA candidate
  tier, then the exact scan gated by its certificate;
* the reference's default depth R = 0.1 N (quantization.rs:27,178): the certified
  search, then the B x R rerank gated by the certificate;
* the deep sharded phase 2: the certified form, then the owned-row rerank gated.

Every test enqueues on a NON-default torch stream behind a long device-side
sleep, checks that the call returned while the stream was still busy (a host
sync inside would have drained it), waits on an event recorded after the search
(not a device sync), and compares ids / score bits with the host-buffer search
(whose tiers are decided on the host) and with the oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def g(gvdb_mod):
    import torch

    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return gvdb_mod


def rng_rows(seed, n, d, dup=0):
    r = np.random.default_rng(seed)
    x = r.standard_normal((n, d)).astype(np.float32)
    for i in range(dup):
        x[(7 * i + 11) % n] = x[(13 * i + 3) % n]
    return x


def same_f32(a, b):
    return np.array(a, np.float32).tobytes() == np.array(b, np.float32).tobytes()


def device_search_async(g, ix, Q, k, sp):
    """search_device on a side stream behind a long device-side sleep: returns
    (ids, scores, n, returned_while_busy).  A first call sizes the pooled
    workspace (growing a buffer frees the old one, which synchronises); the
    second -- the steady state -- is the one checked."""
    import torch

    st = torch.cuda.Stream()
    B = Q.shape[0]
    q = torch.from_numpy(Q).cuda()
    torch.cuda.synchronize()
    busy = False
    for rep in range(2):
        with torch.cuda.stream(st):
            oi = torch.full((B, k), -1, dtype=torch.int64, device="cuda")
            osc = torch.full((B, k), -1.0, dtype=torch.float32, device="cuda")
            on = torch.full((B,), -1, dtype=torch.int32, device="cuda")
            if rep:
                torch.cuda._sleep(20_000_000)  # device time before the search's work on this stream
            ix.search_device(q, k, oi, osc, on, sp, stream=st.cuda_stream)
            ev = torch.cuda.Event()
            ev.record(st)
        busy = not ev.query()  # the search's enqueue finished before the stream drained
        ev.synchronize()  # an event, not a device sync
    return oi.cpu().numpy().view(np.uint64), osc.cpu().numpy(), on.cpu().numpy().view(np.uint32), busy


def counts(g):
    import ctypes as C

    L = g.lib()
    L.gvdb_debug_deep_cert.argtypes = [C.POINTER(C.c_uint64)]
    out = (C.c_uint64 * 2)()
    assert L.gvdb_debug_deep_cert(out) == 0
    return {"flat": int(L.gvdb_flat_fallback_count()), "i8": int(L.gvdb_flat_i8_fallback_count()),
            "cert": int(out[0]), "rerank": int(out[1])}


@pytest.mark.parametrize("uncertifiable", [False, True])
def test_flat_device_tiers_no_host_sync(g, oracle_mod, monkeypatch, uncertifiable):
    """FLAT at B = 64, D = 768 (the i8 emit kernel): certified i8 batch, and a
    batch with a zero query (every row ties at 0.0: no certificate) that the
    gated exact scan answers on the device."""
    monkeypatch.setenv("GVDB_FLAT", "i8")
    N, D, B, k = 120_000, 768, 64, 10
    x = rng_rows(801, N, D, dup=40)
    Q = rng_rows(802, B, D)
    Q[:8] = x[:8] + 0.05 * Q[:8]
    if uncertifiable:
        Q[5] = 0.0
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    sp = g.SearchParams(mode=1, metric=0)
    hi, hs, hn = ix.search_batch(Q, k, sp)
    c0 = counts(g)
    di, ds, dn, busy = device_search_async(g, ix, Q, k, sp)
    c1 = counts(g)
    assert busy, "gvdb_index_search_device (FLAT) waited for the stream"
    assert (dn == hn).all() and (di == hi).all() and same_f32(ds, hs)
    # the device decided (two device calls): the exact tier ran iff the i8 tier failed
    assert (c1["i8"] - c0["i8"], c1["flat"] - c0["flat"]) == ((2, 2) if uncertifiable else (0, 0))
    ri, rs = oracle_mod.exact_topk_cosine_batch(Q, x, k, threads=16)
    assert (di == ri).all() and same_f32(ds, rs)


def test_default_depth_device_gated_rerank(g, oracle_mod):
    """The reference's default depth through gvdb_index_search_device: a batch
    whose certificate fails (planted rows of cosine ~0.84 at Hamming 400 > T fill
    the exact top-32 list) takes the B x R rerank, gated on the device; a batch
    without them is certified.  Both equal the host form and the oracle."""
    N, D, B, k = 100_000, 768, 6, 10
    r = np.random.default_rng(91)
    x = rng_rows(N + 21, N, D)
    Q = rng_rows(D + 23, B, D)
    for qi in range(2):
        q = Q[qi]
        base = q.copy()
        small = np.argsort(np.abs(q))[:400]
        base[small] = -q[small]
        for j in range(70):
            x[5000 * qi + 11 * j] = base + 0.01 * r.standard_normal(D).astype(np.float32)
    ix = g.GpuVectorIndex(dimension=D, capacity_hint=N)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    sp = g.SearchParams(rescore_ratio=0.1)
    R = int(np.float32(N) * np.float32(0.1))
    ri, rs = oracle_mod.multi_stage_search_batch_r(oracle_mod.quantize(Q), oracle_mod.quantize(x), Q, x, R)
    for Qb, fails in ((Q, True), (Q[2:], False)):
        hi, hs, hn = ix.search_batch(Qb, k, sp)
        c0 = counts(g)
        di, ds, dn, busy = device_search_async(g, ix, Qb, k, sp)
        c1 = counts(g)
        assert busy, "gvdb_index_search_device (default depth) waited for the stream"
        assert (dn == hn).all() and (di == hi).all() and same_f32(ds, hs)
        # two device calls, each certified or sent to the gated rerank by the device
        assert (c1["cert"] - c0["cert"], c1["rerank"] - c0["rerank"]) == ((0, 2) if fails else (2, 0))
        o = 0 if fails else 2
        assert (dn == k).all() and (di == ri[o:, :k]).all() and same_f32(ds, rs[o:, :k])


@pytest.mark.parametrize("shift", [0, 300])
def test_default_depth_device_byte_window(g, oracle_mod, monkeypatch, shift):
    """The byte form of the dense rule through gvdb_index_search_device: with
    the window on T the batch certifies on the device; with a window shifted
    off T (GVDB_DENSE8_SHIFT) the rule reports no rule, k_deep_certify fails
    the batch and the GATED rerank answers it -- no host sync either way, and
    both equal the host form and the oracle."""
    if shift:
        monkeypatch.setenv("GVDB_DENSE8_SHIFT", str(shift))
    N, D, B, k = 100_003, 768, 5, 10
    x = rng_rows(821, N, D, dup=60)
    Q = rng_rows(822, B, D)
    Q[0] = x[N - 1]
    ix = g.GpuVectorIndex(dimension=D, capacity_hint=N)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    sp = g.SearchParams(rescore_ratio=0.1)
    c0 = counts(g)
    di, ds, dn, busy = device_search_async(g, ix, Q, k, sp)
    c1 = counts(g)
    assert busy, "gvdb_index_search_device (default depth) waited for the stream"
    assert (c1["cert"] - c0["cert"], c1["rerank"] - c0["rerank"]) == ((0, 2) if shift else (2, 0))
    R = int(np.float32(N) * np.float32(0.1))
    ri, rs = oracle_mod.multi_stage_search_batch_r(oracle_mod.quantize(Q), oracle_mod.quantize(x), Q, x, R)
    assert (dn == k).all() and (di == ri[:, :k]).all() and same_f32(ds, rs[:, :k])
    assert di[0, 0] == N - 1
    hi, hs, hn = ix.search_batch(Q, k, sp)
    assert (hn == dn).all() and (hi == di).all() and same_f32(hs, ds)


def test_bq_device_search_no_host_sync(g, oracle_mod):
    """BQ R = 100 (the bench's mode) at batch 256 and batch 1: no host sync."""
    N, D, k = 150_000, 768, 10
    x = rng_rows(803, N, D)
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    sp = g.SearchParams(rescore_count=100)
    for B in (256, 1):
        Q = rng_rows(804 + B, B, D)
        hi, hs, hn = ix.search_batch(Q, k, sp)
        di, ds, dn, busy = device_search_async(g, ix, Q, k, sp)
        assert busy and (dn == hn).all() and (di == hi).all() and same_f32(ds, hs)


def test_default_depth_device_with_large_r_path_off(g, oracle_mod, monkeypatch):
    """with the batched large-R path disabled (GVDB_BIGR_OFF), a gated
    fallback could not honour its gate, so the async default depth must not take
    the certified form at all: the _device search runs the plain R = 0.1 N
    multi-stage search and still equals the host form and the oracle."""
    monkeypatch.setenv("GVDB_BIGR_OFF", "1")
    N, D, B, k = 90_000, 256, 3, 10
    x = rng_rows(811, N, D, dup=30)
    Q = rng_rows(812, B, D)
    Q[0] = x[17]
    ix = g.GpuVectorIndex(dimension=D, capacity_hint=N)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    sp = g.SearchParams(rescore_ratio=0.1)
    c0 = counts(g)
    di, ds, dn, _ = device_search_async(g, ix, Q, k, sp)
    c1 = counts(g)
    assert (c1["cert"], c1["rerank"]) == (c0["cert"], c0["rerank"])  # the certified form was not entered
    R = int(np.float32(N) * np.float32(0.1))
    ri, rs = oracle_mod.multi_stage_search_batch_r(oracle_mod.quantize(Q), oracle_mod.quantize(x), Q, x, R)
    assert (dn == k).all() and (di == ri[:, :k]).all() and same_f32(ds, rs[:, :k])
    hi, hs, hn = ix.search_batch(Q, k, sp)
    assert (hn == dn).all() and (hi == di).all() and same_f32(hs, ds)
