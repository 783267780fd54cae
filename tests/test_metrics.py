"""CPU: gncde.metrics.ndcg_at_k against scikit-learn's ndcg_score (what tgb's Evaluator calls, trainer_tgb.py:63-79),
with and without tied predictions and all-zero relevance rows."""
import numpy as np
import pytest

from gncde.metrics import ndcg_at_k

sk = pytest.importorskip("sklearn.metrics")


@pytest.mark.parametrize("ties", [False, True])
@pytest.mark.parametrize("k", [10, 3])
def test_ndcg_matches_sklearn(ties, k):
    rng = np.random.default_rng(7)
    yt = rng.random((17, 30)) * (rng.random((17, 30)) < 0.4)
    yt[3] = 0.0  # no relevant item: scores 0
    yp = rng.standard_normal((17, 30))
    if ties:
        yp = np.round(yp, 0)
    assert abs(ndcg_at_k(yt, yp, k) - sk.ndcg_score(yt, yp, k=k)) <= 1e-12
