"""MockEmbeddingProvider (src/embeddings.rs:222-266): the deterministic
text -> vector embedder the reference uses for tests and config 1 (10k x 128).

Per dimension i of a D-vector for text bytes b (embeddings.rs:236-244):
    v_i = (b[i % len(b)] as f32 / 255.0 + i as f32 * 0.01) % 1.0 - 0.5
then the vector is divided by its norm sqrt(sum v_i * v_i), the sum folded
left to right in f32 (246-252), when that norm is > 0.  Every operation here is
the same IEEE-754 single-precision operation, in the same order (numpy float32
scalars / columns, `%` = fmod), so the vectors are bit-identical to the
reference's.  Host code (no GPU): it produces the rows config 1 feeds to the
index.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np

__all__ = ["MockEmbeddingProvider"]


class MockEmbeddingProvider:
    def __init__(self, dimension: int):
        self.dimension = int(dimension)

    def embedding_dimension(self) -> int:
        return self.dimension

    def generate_embedding(self, text: str) -> np.ndarray:
        return self.generate_embeddings([text])[0]

    def generate_embeddings(self, texts: Sequence[str]) -> np.ndarray:
        """All texts at once: one f32 column per dimension, the norm folded
        across columns in order (the per-text fold of the reference)."""
        D, n = self.dimension, len(texts)
        out = np.zeros((n, D), np.float32)
        if n == 0 or D == 0:
            return out
        bs = [t.encode("utf-8") for t in texts]
        if any(len(b) == 0 for b in bs):
            raise ZeroDivisionError("empty text: `i % bytes.len()` panics in the reference (embeddings.rs:241)")
        lens = np.array([len(b) for b in bs], np.int64)
        flat = np.frombuffer(b"".join(bs), np.uint8)
        starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
        c255 = np.float32(255.0)
        c001 = np.float32(0.01)
        one = np.float32(1.0)
        half = np.float32(0.5)
        for i in range(D):
            byte = flat[starts + (i % lens)].astype(np.float32)
            v = np.fmod(byte / c255 + np.float32(i) * c001, one) - half
            out[:, i] = v.astype(np.float32)
        s = np.full(n, -0.0, np.float32)
        for i in range(D):
            s = (s + out[:, i] * out[:, i]).astype(np.float32)
        norm = np.sqrt(s).astype(np.float32)
        pos = norm > 0
        out[pos] = (out[pos] / norm[pos, None]).astype(np.float32)
        return out

    def generate_embedding_list(self, texts: Sequence[str]) -> List[np.ndarray]:
        return list(self.generate_embeddings(texts))
