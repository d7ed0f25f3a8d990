"""Host check of k_sample_mx's partial flush (grape-vector-db_amd/csrc/gvdb_kernels.hip):
each block adds to the global histogram only the bins up to its own target-th
smallest distance t_b (all bins below the cap when it never reaches target), and
k_threshold must still find exactly the threshold of the full histogram:
T = min{t : sum_b cnt_b(<= t) >= target}, or the last bin when never reached.
T <= t_b for every block that reached target, so bins above t_b cannot change it.
Pure numpy, no GPU; the GPU test is test_gpu_parity.py::
test_sample_histogram_mfma_thresholds_equal_valu."""
import numpy as np
import pytest


def threshold(hist, target):
    c = np.cumsum(hist)
    hit = np.nonzero(c >= target)[0]
    return int(hit[0]) if len(hit) else len(hist) - 1


def partial_flush(block_hists, target, cap):
    nb = block_hists.shape[1]
    out = np.zeros(nb, dtype=np.int64)
    for h in block_hists:
        c = np.cumsum(h[:cap])
        hit = np.nonzero(c >= target)[0]
        tb = int(hit[0]) if len(hit) else cap - 1
        out[: tb + 1] += h[: tb + 1]
    return out


@pytest.mark.parametrize("seed", range(40))
def test_partial_flush_gives_the_full_threshold(seed):
    rng = np.random.default_rng(seed)
    D = int(rng.choice([128, 256, 384, 768]))
    nb, cap = D + 1, min(D + 1, 384)
    blocks = int(rng.integers(1, 64))
    rows = int(rng.integers(1, 2000))
    target = int(rng.integers(1, 60))
    # distances of sampled rows: binomial around D/2, some blocks shifted (clustered data)
    shift = rng.integers(-D // 4, D // 8, size=blocks)
    d = np.clip(rng.binomial(D, 0.5, size=(blocks, rows)) + shift[:, None], 0, D)
    block_hists = np.stack([np.bincount(x[x < cap], minlength=nb) for x in d])  # bins >= cap never counted
    full = threshold(block_hists.sum(0), target)
    part = threshold(partial_flush(block_hists, target, cap), target)
    assert part == full
