"""CPU: the BM25 / RRF oracle (oracle/bm25_oracle.cpp; sparse.rs:71-222,
hybrid.rs:422-488) against the reference's own unit tests
(tests/golden/kat.json: sparse.rs:370-410, hybrid.rs:991-1025) and against an
independent pure-Python restatement that steps every f32 operation with numpy
float32 (adds, re-adds, removes, ties, negative idf).  The host-side pieces of
the Python mirror (SparseVector, SimpleTokenizer) are checked here too."""
import json
import math
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
KAT = json.load(open(os.path.join(HERE, "golden", "kat.json")))
f32 = np.float32


class PyBm25:
    """sparse.rs restated in pure Python with float32 steps (second opinion)."""

    def __init__(self, k1=1.2, b=0.75):
        self.k1, self.b = f32(k1), f32(b)
        self.slot_of, self.slot_id, self.entries = {}, [], []  # entries[slot] = [(term, tf, dl)] add order
        self.postings, self.df = {}, {}
        self.N = 0

    def avgdl(self):
        t = f32(0.0)
        for ents in self.entries:
            for term, tf, dl in sorted(ents, key=lambda e: e[0]):  # stable: (term, add order)
                t = f32(t + dl)
        return f32(t / f32(self.N)) if self.N else f32(0.0)

    def add(self, i, terms, tfs, dl):
        if i not in self.slot_of:
            self.slot_of[i] = len(self.slot_id)
            self.slot_id.append(i)
            self.entries.append([])
        s = self.slot_of[i]
        for t, v in zip(terms, tfs):
            self.entries[s].append((t, f32(v), f32(dl)))
            self.postings.setdefault(t, []).append(s)
            self.df[t] = self.df.get(t, 0) + 1
        self.N += 1
        self._avgdl = self.avgdl()

    def remove(self, i):
        if i not in self.slot_of:
            return False
        s, removed = self.slot_of[i], False
        for t in list(self.postings):
            pl = self.postings[t]
            if s in pl:
                pl.remove(s)
                removed = True
                for j, e in enumerate(self.entries[s]):
                    if e[0] == t:
                        del self.entries[s][j]
                        break
                if not pl:
                    self.df.pop(t, None)
        if removed:
            self.N = max(self.N - 1, 0)
            self._avgdl = self.avgdl() if self.N else f32(0.0)
        return removed

    def search(self, terms, vals, limit):
        if self.N == 0:
            return []
        score, order = {}, []
        for t, qv in zip(terms, vals):
            if t not in self.postings:
                continue
            dfv = self.df.get(t, 1)
            idf = f32(math.log(f32(f32(f32(f32(self.N) - f32(dfv)) + f32(0.5)) / f32(f32(dfv) + f32(0.5)))))
            seen = {}
            for s in self.postings[t]:
                kth = seen.get(s, 0)
                seen[s] = kth + 1
                e = [x for x in self.entries[s] if x[0] == t][kth]
                tf, dl = e[1], e[2]
                tfc = f32(f32(tf * f32(self.k1 + f32(1.0))) /
                          f32(tf + f32(self.k1 * f32(f32(f32(1.0) - self.b) + f32(self.b * f32(dl / self._avgdl))))))
                c = f32(f32(f32(qv) * tfc) * idf)
                if s not in score:
                    score[s] = f32(0.0)
                    order.append(s)
                score[s] = f32(score[s] + c)
        order.sort()
        order.sort(key=lambda s: (math.isnan(score[s]), -float(score[s]) if not math.isnan(score[s]) else 0.0))
        return [(self.slot_id[s], score[s]) for s in order[:limit]]


def zipf_docs(seed, n_docs, vocab, terms_per_doc, a=1.1):
    r = np.random.default_rng(seed)
    p = 1.0 / np.arange(1, vocab + 1) ** a
    p /= p.sum()
    docs = []
    for _ in range(n_docs):
        toks = r.choice(vocab, size=terms_per_doc, p=p)
        u, c = np.unique(toks, return_counts=True)
        tf = (c.astype(np.float32) / f32(terms_per_doc)).astype(np.float32)
        dl = f32(0.0)
        for v in tf:
            dl = f32(dl + v)
        docs.append((u.astype(np.uint32), tf, dl))
    return docs


def test_kat_sparse_vector():
    from gvdb.sparse import SparseVector

    c = KAT["sparse"][0]
    a, b = SparseVector(**c["a"]), SparseVector(**c["b"])
    assert a.dot_product(b) == c["dot"]
    assert (a.cosine_similarity(b) > 0) == c["cosine_positive"]
    with pytest.raises(ValueError):
        SparseVector([0, 11], [1.0, 1.0], 10)  # index out of range (types.rs:39-43)
    with pytest.raises(ValueError):
        SparseVector([0], [1.0, 2.0], 10)  # count mismatch (types.rs:33-37)


def test_kat_tokenizer():
    from gvdb.sparse import SimpleTokenizer

    c = KAT["tokenizer"][0]
    tok = SimpleTokenizer().tokenize(c["text"])
    assert all(w in tok for w in c["contains"]) and not any(w in tok for w in c["absent"])
    assert abs(sum(tok.values()) - 1.0) < 1e-6  # relative frequencies (sparse.rs:318-321)


def test_kat_sparse_index_stats(oracle_mod):
    from gvdb.sparse import SimpleTokenizer

    c = KAT["sparse_index"][0]
    tk = SimpleTokenizer()
    vocab = tk.build_vocabulary(c["docs"])
    d = tk.document_to_sparse_vector(c["add"][0], c["add"][1], vocab)
    o = oracle_mod.Bm25()
    o.add_document(1, list(d.term_frequencies), list(d.term_frequencies.values()), d.document_length)
    n, avgdl, v = o.stats()
    assert n == c["total_documents"] and (v > 0) == c["vocabulary_size_positive"]


def test_kat_rrf(oracle_mod):
    c = KAT["rrf"][0]
    names = {}
    ids = lambda lst: [(names.setdefault(s, len(names)), v) for s, v in lst]  # noqa: E731
    fused = oracle_mod.rrf_fusion(ids(c["dense"]), ids(c["sparse"]), ids(c["text"]), c["k"])
    sc = {i: s for i, s, *_ in fused}
    g, l = c["greater"]
    assert sc[names[g]] > sc[names[l]]
    assert sc[names["doc1"]] == f32(f32(1.0) / f32(61.0)) + f32(f32(1.0) / f32(61.0))


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_bm25_oracle_matches_python_restatement(oracle_mod, seed):
    docs = zipf_docs(seed, 300, 200, 12)
    o, p = oracle_mod.Bm25(), PyBm25()
    for i, (t, v, dl) in enumerate(docs):
        o.add_document(1000 + i, t, v, dl)
        p.add(1000 + i, t.tolist(), v.tolist(), dl)
    # re-add two ids, remove three (one of them re-added)
    for i in (5, 17):
        t, v, dl = docs[(i * 7) % len(docs)]
        o.add_document(1000 + i, t, v, dl)
        p.add(1000 + i, t.tolist(), v.tolist(), dl)
    for i in (17, 40, 41):
        assert o.remove_document(1000 + i) == p.remove(1000 + i)
    assert o.remove_document(99999) is False
    n, avgdl, _ = o.stats()
    assert n == p.N and avgdl == p._avgdl
    r = np.random.default_rng(seed + 100)
    for _ in range(25):
        qt = r.choice(200, size=r.integers(1, 9), replace=True).astype(np.uint32)  # repeats allowed
        qv = r.random(qt.size).astype(np.float32)
        ids, sc = o.search(qt, qv, 20)
        ref = p.search(qt.tolist(), qv.tolist(), 20)
        assert [int(i) for i in ids] == [i for i, _ in ref]
        assert sc.tobytes() == np.array([s for _, s in ref], np.float32).tobytes()


def test_bm25_negative_idf_and_empty(oracle_mod):
    o = oracle_mod.Bm25()
    assert o.search([1], [1.0], 5)[0].size == 0  # total_documents == 0 -> empty (sparse.rs:159-161)
    for i in range(3):
        o.add_document(i, [7], [0.5], 1.0)
    ids, sc = o.search([7, 8], [1.0, 1.0], 5)  # df = N: idf = ln(0.5/3.5) < 0, no floor
    assert list(ids) == [0, 1, 2] and np.all(sc < 0)


def test_rrf_oracle_matches_python(oracle_mod):
    r = np.random.default_rng(9)
    for _ in range(50):
        mk = lambda n: [(int(x), float(r.random())) for x in r.integers(0, 12, n)]  # noqa: E731
        d, s, t = mk(r.integers(0, 8)), mk(r.integers(0, 8)), mk(r.integers(0, 8))
        k = f32(60.0)
        acc, first = {}, []
        for lst, kind in ((d, 0), (s, 1), (t, 2)):
            for rank, (i, _) in enumerate(lst):
                rr = f32(f32(1.0) / f32(k + f32(rank + 1)))
                if i not in acc:
                    acc[i] = rr
                    first.append(i)
                elif kind == 0:
                    acc[i] = rr
                else:
                    acc[i] = f32(acc[i] + rr)
        want = sorted(first, key=lambda i: -float(acc[i]))
        got = oracle_mod.rrf_fusion(d, s, t, 60.0)
        assert [g[0] for g in got] == want
        assert [g[1] for g in got] == [acc[i] for i in want]
