"""Evaluation metrics (reference ``python/hetu/metrics.py:4-359``): AUC,
ROC/PR curves, accuracy, confusion matrix, precision/recall/F (one-hot)."""
from __future__ import annotations

import numpy as np


def _binary_clf_curve(y_true, y_score):
    y_true = np.asarray(y_true).reshape(-1).astype(np.float64)
    y_score = np.asarray(y_score).reshape(-1).astype(np.float64)
    order = np.argsort(-y_score, kind='mergesort')
    y_true, y_score = y_true[order], y_score[order]
    distinct = np.where(np.diff(y_score))[0]
    thr_idx = np.r_[distinct, y_true.size - 1]
    tps = np.cumsum(y_true)[thr_idx]
    fps = 1 + thr_idx - tps
    return fps, tps, y_score[thr_idx]


def roc_curve(y_true, y_score):
    fps, tps, thr = _binary_clf_curve(y_true, y_score)
    tps = np.r_[0, tps]
    fps = np.r_[0, fps]
    thr = np.r_[thr[0] + 1, thr]
    fpr = fps / fps[-1] if fps[-1] > 0 else np.zeros_like(fps)
    tpr = tps / tps[-1] if tps[-1] > 0 else np.zeros_like(tps)
    return fpr, tpr, thr


def auc(x, y):
    x, y = np.asarray(x), np.asarray(y)
    return float(np.trapz(y, x))


def roc_auc_score(y_true, y_score):
    fpr, tpr, _ = roc_curve(y_true, y_score)
    return auc(fpr, tpr)


def precision_recall_curve(y_true, y_score):
    fps, tps, thr = _binary_clf_curve(y_true, y_score)
    precision = tps / np.maximum(tps + fps, 1)
    recall = tps / tps[-1] if tps[-1] > 0 else np.ones_like(tps)
    last = tps.searchsorted(tps[-1])
    sl = slice(last, None, -1)
    return np.r_[precision[sl], 1], np.r_[recall[sl], 0], thr[sl]


def accuracy(y_pred, y_true):
    yp, yt = np.asarray(y_pred), np.asarray(y_true)
    if yp.ndim > 1 and yp.shape[-1] > 1:
        yp = yp.argmax(-1)
    if yt.ndim > 1 and yt.shape[-1] > 1:
        yt = yt.argmax(-1)
    return float(np.mean(yp.reshape(-1) == yt.reshape(-1)))


def confusion_matrix(y_pred, y_true, num_classes=None):
    yp, yt = np.asarray(y_pred), np.asarray(y_true)
    if yp.ndim > 1:
        yp = yp.argmax(-1)
    if yt.ndim > 1:
        yt = yt.argmax(-1)
    n = num_classes or int(max(yp.max(), yt.max()) + 1)
    m = np.zeros((n, n), dtype=np.int64)
    np.add.at(m, (yt.astype(np.int64), yp.astype(np.int64)), 1)
    return m


def precision_recall_fscore(y_pred, y_true, beta=1.0, average='macro'):
    m = confusion_matrix(y_pred, y_true).astype(np.float64)
    tp = np.diag(m)
    p = tp / np.maximum(m.sum(0), 1)
    r = tp / np.maximum(m.sum(1), 1)
    f = (1 + beta ** 2) * p * r / np.maximum(beta ** 2 * p + r, 1e-12)
    if average == 'macro':
        return float(p.mean()), float(r.mean()), float(f.mean())
    return p, r, f


def log_loss(y_true, y_prob, eps=1e-7):
    y = np.asarray(y_true, dtype=np.float64).reshape(-1)
    p = np.clip(np.asarray(y_prob, dtype=np.float64).reshape(-1), eps, 1 - eps)
    return float(-np.mean(y * np.log(p) + (1 - y) * np.log(1 - p)))
