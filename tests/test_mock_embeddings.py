"""Config 1 plumbing: MockEmbeddingProvider (src/embeddings.rs:222-266) against
a scalar restatement that steps through each f32 operation per text (the
reference's loop order), plus hand-checked known answers."""
import math
import struct

import numpy as np
import pytest


def f32(x):
    return struct.unpack("f", struct.pack("f", x))[0]


def scalar_mock(text, D):
    """embeddings.rs:236-257 step by step in f32."""
    b = text.encode()
    v = []
    for i in range(D):
        byte = f32(b[i % len(b)])
        t = f32(f32(byte / f32(255.0)) + f32(f32(i) * f32(0.01)))
        v.append(f32(f32(math.fmod(t, 1.0)) - f32(0.5)))
    s = -0.0
    for x in v:
        s = f32(s + f32(x * x))
    norm = f32(math.sqrt(s))
    if norm > 0:
        v = [f32(x / norm) for x in v]
    return np.array(v, np.float32)


@pytest.mark.parametrize("D", [1, 4, 128, 384])
def test_mock_matches_scalar_restatement(gvdb_mod, D):
    from gvdb.embeddings import MockEmbeddingProvider

    texts = ["a", "document 42", "向量数据库", "x" * 300, "doc 9999"]
    got = MockEmbeddingProvider(D).generate_embeddings(texts)
    for t, row in zip(texts, got):
        assert row.tobytes() == scalar_mock(t, D).tobytes(), t


def test_mock_known_answers(gvdb_mod):
    from gvdb.embeddings import MockEmbeddingProvider

    p = MockEmbeddingProvider(2)
    # "a" = 97: v0 = 97/255 - 0.5, v1 = (97/255 + 0.01) - 0.5, then normalised
    v0 = np.float32(97) / np.float32(255) - np.float32(0.5)
    v1 = (np.float32(97) / np.float32(255) + np.float32(0.01)) - np.float32(0.5)
    n = np.sqrt(np.float32(np.float32(np.float32(-0.0) + v0 * v0) + v1 * v1))
    assert p.generate_embedding("a").tobytes() == np.array([v0 / n, v1 / n], np.float32).tobytes()
    assert p.embedding_dimension() == 2
    with pytest.raises(ZeroDivisionError):
        p.generate_embedding("")
