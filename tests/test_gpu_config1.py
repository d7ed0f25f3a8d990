"""GPU, BASELINE configs[0]: the MockEmbeddingProvider corpus (10k x 128,
embeddings.rs:222-266) through the index, BQ + rerank and flat, against the
oracle (multi_stage_search quantization.rs:151-193; storage.rs:296-339)."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))


def test_config1_mock_corpus_matches_oracle(gvdb_mod, oracle_mod):
    import torch

    from config1_mock import texts
    from gvdb.embeddings import MockEmbeddingProvider

    assert torch.cuda.is_available()
    g = gvdb_mod
    p = MockEmbeddingProvider(128)
    x = p.generate_embeddings(texts(10_000, 1))
    q = p.generate_embeddings(texts(64, 2))
    ix = g.GpuVectorIndex(dimension=128)
    ix.add_vectors([(f"doc{i}", x[i]) for i in range(len(x))])
    ids, sc, n = ix.search_batch(q, 10, g.SearchParams(rescore_count=100))
    ri, rs = oracle_mod.multi_stage_search_batch_r(oracle_mod.quantize(q), oracle_mod.quantize(x), q, x, 100, kind=0)
    assert (ids == ri[:, :10]).all() and sc.tobytes() == rs[:, :10].tobytes()
    # batch-1 path on the same corpus
    for b in range(0, 64, 9):
        i1, s1, n1 = ix.search_batch(q[b:b + 1], 10, g.SearchParams(rescore_count=100))
        assert (i1[0] == ri[b, :10]).all() and s1[0].tobytes() == rs[b, :10].tobytes()
    # exact flat (VectorStore::vector_search) with the QueryEngine defaults
    qe = g.QueryEngine(ix)
    for b in range(4):
        got = qe.vector_search(q[b])
        fi, fs = oracle_mod.storage_vector_search(q[b], x, 10, threshold=0.7)
        assert [s for s, _ in got] == [f"doc{int(i)}" for i in fi]
        assert np.array([v for _, v in got], np.float32).tobytes() == np.asarray(fs, np.float32).tobytes()
