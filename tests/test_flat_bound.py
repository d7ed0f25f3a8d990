"""CPU: the i8 candidate-pass certificate of K4 (gvdb_flat.hip, k_rows_to_i8 /
k_queries_to_i8).  With per-vector symmetric int8 quantisation
v^ = s*rint(v/s), s = max|v_i|/127, rho = |v - v^|/|v|, the MFMA pass scores
q^.x^ exactly (i32) and the certificate assumes

    |q.x - q^.x^| / (|q||x|)  <=  rho_q + (1 + rho_q) * rho_x.

This checks the inequality (and that it is not vacuous) on adversarial and
random vectors in fp64 — no GPU involved."""
import numpy as np
import pytest


def quant(v):
    amax = np.abs(v).max()
    if amax == 0:
        return np.zeros_like(v), 0.0
    s = np.float32(amax) / np.float32(127.0)
    inv = np.float32(127.0) / np.float32(amax)
    qi = np.clip(np.rint((v.astype(np.float32) * inv).astype(np.float32)), -127, 127)
    return qi.astype(np.float64) * np.float64(s), float(s)


@pytest.mark.parametrize("D", [64, 100, 768, 1100, 3072])
def test_i8_certificate_bound(D):
    r = np.random.default_rng(D)
    worst = 0.0
    for trial in range(300):
        kind = trial % 3
        q = r.standard_normal(D)
        x = r.standard_normal(D)
        if kind == 1:  # spiky vectors: one large coordinate dominates the scale
            q[r.integers(D)] *= 40.0
            x[r.integers(D)] *= 40.0
        elif kind == 2:  # near-parallel pair
            x = q + 0.01 * x
        q = q.astype(np.float32).astype(np.float64)
        x = x.astype(np.float32).astype(np.float64)
        qh, _ = quant(q)
        xh, _ = quant(x)
        nq, nx = np.linalg.norm(q), np.linalg.norm(x)
        rq = np.linalg.norm(q - qh) / nq
        rx = np.linalg.norm(x - xh) / nx
        err = abs(q @ x - qh @ xh) / (nq * nx)
        bound = rq + (1 + rq) * rx
        assert err <= bound * (1 + 1e-9), (trial, err, bound)
        worst = max(worst, err / bound)
    assert worst > 0.01  # the bound is not vacuous by orders of magnitude
