"""Losses consumed by the 1vsAll / KvsAll / negative-sampling jobs (kge/util/loss.py:29-274):
``kl`` -- cross entropy for index labels, KL(softmax) for a label matrix (loss.py:192-213);
``bce`` / ``bce_mean`` (loss.py:137-189); ``margin_ranking`` for negative sampling
(loss.py:227-262); ``soft_margin`` (loss.py:216-224); ``se`` (loss.py:265-272).  All use
reduction "sum"; the jobs divide by the batch size.  The 1vsAll / KvsAll ``kl`` objective is
normally fused into the engine (engine.fused_loss) and never reaches these classes."""
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
        if name == "bce_mean":
            return BCEWithLogitsKgeLoss(config, mean=True)
        if name == "bce_self_adversarial":
            # the temperature is a user option (loss.py:64-67); 1 when it is not set
            try:
                temperature = float(config.get("user.bce_self_adversarial_temperature"))
            except KeyError:
                temperature = 1.0
            return BCEWithLogitsKgeLoss(config, mean=True, temperature=temperature)
        if name == "margin_ranking":
            return MarginRankingKgeLoss(config)
        if name == "soft_margin":
            return SoftMarginKgeLoss(config)
        if name == "se":
            return SEKgeLoss(config)
        raise ValueError(f"invalid value train.loss={name}")

    def __call__(self, scores, labels, **kwargs):
        raise NotImplementedError

    def _labels_as_matrix(self, scores, labels):
        if labels.dim() == 2:
            return labels
        x = torch.zeros(scores.shape, dtype=torch.float, device=scores.device)
        # scatter on the device: no host index list, so the step can be recorded into a graph
        x.scatter_(1, labels.view(-1, 1).to(device=scores.device, dtype=torch.int64), 1.0)
        return x

    def _labels_as_indexes(self, scores, labels):
        """Matrix labels with exactly one 1 per row -> the 1's column (loss.py:101-117)."""
        if labels.dim() == 1:
            return labels
        x = labels.nonzero()
        if not x[:, 0].equal(torch.arange(len(labels), device=labels.device)):
            raise ValueError("exactly one 1 per row required")
        return x[:, 1]


class KLDivWithSoftmaxKgeLoss(KgeLoss):
    def __init__(self, config, reduction="sum"):
        super().__init__(config)
        self._celoss = torch.nn.CrossEntropyLoss(reduction=reduction)
        self._klloss = torch.nn.KLDivLoss(reduction=reduction)

    def __call__(self, scores, labels, **kwargs):
        if labels.dim() == 1:  # index labels: KL == CE (entropy of a one-hot is 0)
            return self._celoss(scores, labels)
        return self._klloss(F.log_softmax(scores, dim=1), F.normalize(labels.float(), p=1, dim=1))


def _loss_arg(config, default):
    v = config.get("train.loss_arg")
    return default if (v is None or (isinstance(v, float) and math.isnan(v))) else float(v)


class BCEWithLogitsKgeLoss(KgeLoss):
    """bce: sum of BCE over all scores; bce_mean: (sum over positives + mean over each
    row's negatives) / 2; bce_self_adversarial: the negatives of a row averaged with the
    softmax of their own (detached) scores times a temperature instead of uniformly
    (loss.py:137-189).  loss_arg = offset added to the scores."""

    def __init__(self, config, mean=False, temperature=None):
        super().__init__(config)
        self._offset = _loss_arg(config, 0.0)
        self._mean = mean
        self._temperature = temperature  # None: uniform mean over the negatives
        self._loss = torch.nn.BCEWithLogitsLoss(reduction="none" if mean else "sum")

    def __call__(self, scores, labels, **kwargs):
        lm = self._labels_as_matrix(scores, labels)
        if self._offset != 0.0:
            scores = scores + self._offset
        losses = self._loss(scores.reshape(-1), lm.reshape(-1).float())
        if not self._mean:
            return losses
        idx = self._labels_as_indexes(scores, labels)
        n, k = scores.shape
        losses = losses.view(n, k)
        pos = losses.gather(1, idx.view(-1, 1)).sum()
        if self._temperature is None:
            neg = (losses.sum() - pos) / (k - 1)
        else:
            # every row has exactly one positive: its k - 1 negatives in column order
            keep = lm.reshape(n, k) == 0
            neg_scores = scores.detach()[keep].view(n, k - 1)  # the adversarial weights carry no gradient
            neg = (F.softmax(neg_scores * self._temperature, dim=1) * losses[keep].view(n, k - 1)).sum()
        return (pos + neg) / 2.0


class MarginRankingKgeLoss(KgeLoss):
    """Negative sampling only: each positive score paired with the negatives that follow it
    in its row, sum max(0, margin - (pos - neg)) (loss.py:227-262); loss_arg = margin (1)."""

    def __init__(self, config):
        super().__init__(config)
        self._train_type = config.get("train.type")
        self._loss = torch.nn.MarginRankingLoss(margin=_loss_arg(config, 1.0), reduction="sum")

    def __call__(self, scores, labels, **kwargs):
        if "negative_sampling" not in self._train_type:
            if self._train_type == "KvsAll":
                raise NotImplementedError("Margin ranking with KvsAll training not yet supported.")
            raise ValueError("train.type for margin ranking.")
        lm = self._labels_as_matrix(scores, labels).reshape(-1)
        pos_idx = lm.nonzero().view(-1)
        neg_idx = (lm == 0).nonzero().view(-1)
        pos_idx = pos_idx.view(-1, 1).repeat(1, kwargs["num_negatives"]).view(-1)
        positives = scores.reshape(-1)[pos_idx]
        negatives = scores.reshape(-1)[neg_idx]
        return self._loss(positives, negatives, torch.ones_like(positives))


class SoftMarginKgeLoss(KgeLoss):
    """SoftMarginLoss(sum) with labels mapped to +-1 (loss.py:216-224)."""

    def __init__(self, config):
        super().__init__(config)
        self._loss = torch.nn.SoftMarginLoss(reduction="sum")

    def __call__(self, scores, labels, **kwargs):
        lm = self._labels_as_matrix(scores, labels) * 2 - 1
        return self._loss(scores.reshape(-1), lm.reshape(-1))


class SEKgeLoss(KgeLoss):
    """Squared error against the 0/1 labels, sum (loss.py:265-272)."""

    def __init__(self, config):
        super().__init__(config)
        self._loss = torch.nn.MSELoss(reduction="sum")

    def __call__(self, scores, labels, **kwargs):
        return self._loss(scores, self._labels_as_matrix(scores, labels))
