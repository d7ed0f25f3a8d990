"""Host mirrors of the reference API around the path: BinaryVectorStore
(quantization.rs:286-354, CPU) and QueryEngine::vector_search defaults
(query_engine.rs:23-30, 117-147; GPU)."""
import numpy as np
import pytest


def test_binary_vector_store_api(gvdb_mod):
    g = gvdb_mod
    st = g.BinaryVectorStore(g.BinaryQuantizationConfig(threshold=0.1))
    assert st.is_empty() and st.len() == 0 and st.get_vector(0) is None
    assert st.get_config().threshold == np.float32(0.1) or st.get_config().threshold == 0.1
    a = g.BinaryVector(bytes([0xA8]), 5)
    b = g.BinaryVector(bytes([0xFF, 0x01]), 9)
    st.add_vector(a, "doc-1")
    st.add_vector(b, "向量")  # multi-byte id: memory counts UTF-8 bytes (String::len)
    assert st.len() == 2 and not st.is_empty()
    assert st.get_vector(1) is b and st.get_vector(2) is None and st.get_vector(-1) is None
    assert st.memory_usage() == (1 + 2) + (5 + 6)
    st.validate_vector(a)
    with pytest.raises(g.InvalidVectorDimension):
        st.validate_vector(g.BinaryVector(b"", 0))


@pytest.mark.gpu
def test_query_engine_vector_search_defaults(gvdb_mod, oracle_mod):
    """limit None -> 10, threshold None -> 0.7: equal to the reference store
    search storage.rs:296-339 with Some(0.7) (the oracle), scores bit-exact."""
    import torch

    assert torch.cuda.is_available()
    g = gvdb_mod
    rng = np.random.default_rng(5)
    D, N = 32, 4000
    base = rng.standard_normal(D).astype(np.float32)
    x = (base + 0.6 * rng.standard_normal((N, D))).astype(np.float32)  # many rows above 0.7
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_vectors([(f"d{i}", x[i]) for i in range(N)])
    qe = g.QueryEngine(ix)
    got = qe.vector_search(base)
    ri, rs = oracle_mod.storage_vector_search(base, x, 10, threshold=0.7)
    assert [s for s, _ in got] == [f"d{int(i)}" for i in ri]
    assert np.array(rs, np.float32).tobytes() == np.array([v for _, v in got], np.float32).tobytes()
    assert all(v >= np.float32(0.7) for _, v in got)
    # explicit limit / threshold, and a threshold nothing passes
    got2 = qe.vector_search(base, limit=25, threshold=0.8)
    ri2, rs2 = oracle_mod.storage_vector_search(base, x, 25, threshold=0.8)
    assert [s for s, _ in got2] == [f"d{int(i)}" for i in ri2]
    assert qe.vector_search(-base, threshold=0.99) == []
    assert qe.vector_search(base) == got  # cached
