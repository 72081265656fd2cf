"""Losses consumed by the 1vsAll / KvsAll jobs (kge/util/loss.py:29-274, the subset the
scoring path feeds): ``kl`` -- cross entropy for index labels, KL(softmax) for a label
matrix (loss.py:192-213) -- and ``bce`` (loss.py:137-189, mean/sum over all scores)."""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


class KgeLoss:
    def __init__(self, config):
        self.config = config

    @staticmethod
    def create(config):
        name = config.get("train.loss")
        if name == "kl":
            return KLDivWithSoftmaxKgeLoss(config)
        if name == "bce":
            return BCEWithLogitsKgeLoss(config)
        raise ValueError(f"invalid value train.loss={name}")

    def __call__(self, scores, labels, **kwargs):
        raise NotImplementedError

    def _labels_as_matrix(self, scores, labels):
        if labels.dim() == 2:
            return labels
        x = torch.zeros(scores.shape, dtype=torch.float, device=scores.device)
        x[range(len(scores)), labels] = 1.0
        return x


class KLDivWithSoftmaxKgeLoss(KgeLoss):
    def __init__(self, config, reduction="sum"):
        super().__init__(config)
        self._celoss = torch.nn.CrossEntropyLoss(reduction=reduction)
        self._klloss = torch.nn.KLDivLoss(reduction=reduction)

    def __call__(self, scores, labels, **kwargs):
        if labels.dim() == 1:  # index labels: KL == CE (entropy of a one-hot is 0)
            return self._celoss(scores, labels)
        return self._klloss(F.log_softmax(scores, dim=1), F.normalize(labels.float(), p=1, dim=1))


class BCEWithLogitsKgeLoss(KgeLoss):
    def __init__(self, config, reduction="sum"):
        super().__init__(config)
        offset = config.get("train.loss_arg")
        self._offset = 0.0 if (offset is None or (isinstance(offset, float) and math.isnan(offset))) else offset
        self._loss = torch.nn.BCEWithLogitsLoss(reduction=reduction)

    def __call__(self, scores, labels, **kwargs):
        labels = self._labels_as_matrix(scores, labels)
        return self._loss(scores.view(-1) + self._offset, labels.view(-1).float())
