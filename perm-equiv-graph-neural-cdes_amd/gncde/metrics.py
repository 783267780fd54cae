"""Evaluation metrics of the reference's trainers.

``ndcg_at_k`` restates what ``tgb.nodeproppred.evaluate.Evaluator(...).eval({..., "eval_metric": ["ndcg"]})``
reports at trainer_tgb.py:63-79: scikit-learn's ``ndcg_score(y_true, y_pred, k=10)`` — linear gains,
1/log2(rank+1) discounts cut at k, predictions tied in score share the average gain of their group, rows
whose ideal DCG is 0 score 0, mean over rows.  tgb and its evaluator are not installed here, so
this follows scikit-learn's published algorithm; tests/test_metrics.py checks it against scikit-learn itself.
Host-side: it runs on the (masked) predictions once per evaluation, not on the hot path.
"""
from __future__ import annotations

import numpy as np
import torch


def _dcg(y_true: np.ndarray, y_score: np.ndarray, k: int, ignore_ties: bool) -> np.ndarray:
    n = y_true.shape[1]
    discount = 1.0 / np.log2(np.arange(n) + 2.0)
    discount[k:] = 0.0
    if ignore_ties:
        order = np.argsort(-y_score, axis=1, kind="stable")
        return (np.take_along_axis(y_true, order, axis=1) * discount).sum(axis=1)
    cum = np.cumsum(discount)
    out = np.empty(y_true.shape[0])
    for r in range(y_true.shape[0]):
        _, inv, counts = np.unique(-y_score[r], return_inverse=True, return_counts=True)
        ranked = np.zeros(len(counts))
        np.add.at(ranked, inv, y_true[r])
        ranked /= counts
        groups = np.cumsum(counts) - 1
        sums = np.empty(len(counts))
        sums[0] = cum[groups[0]]
        sums[1:] = np.diff(cum[groups])
        out[r] = (ranked * sums).sum()
    return out


def ndcg_at_k(y_true, y_pred, k: int = 10) -> float:
    """Mean NDCG@k over rows of y_true / y_pred [rows, items] (torch or numpy)."""
    yt = (y_true.detach().double().cpu().numpy() if torch.is_tensor(y_true) else np.asarray(y_true, np.float64))
    yp = (y_pred.detach().double().cpu().numpy() if torch.is_tensor(y_pred) else np.asarray(y_pred, np.float64))
    if yt.ndim != 2 or yt.shape != yp.shape:
        raise ValueError(f"ndcg_at_k: shapes {yt.shape} vs {yp.shape}")
    if yt.shape[0] == 0:
        return float("nan")
    gain = _dcg(yt, yp, k, ignore_ties=False)
    ideal = _dcg(yt, yt, k, ignore_ties=True)
    ok = ideal > 0
    score = np.zeros_like(gain)
    score[ok] = gain[ok] / ideal[ok]
    return float(score.mean())
