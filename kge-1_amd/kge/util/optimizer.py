"""Optimizer / LR-scheduler factories (kge/util/optimizer.py:6-71): stock torch.optim
classes selected by name with ``train.optimizer_args``."""
from __future__ import annotations

import torch


class KgeOptimizer:
    @staticmethod
    def create(config, model):
        name = config.get("train.optimizer")
        try:
            cls = getattr(torch.optim, name)
        except AttributeError as e:
            raise ValueError(f"Could not create optimizer {name}") from e
        return cls([p for p in model.parameters() if p.requires_grad], **config.get("train.optimizer_args"))


class KgeLRScheduler:
    def __init__(self, config, optimizer):
        name = config.get("train.lr_scheduler")
        args = config.get("train.lr_scheduler_args")
        self._lr_scheduler = None
        self._metric_based = False
        if name != "":
            self._lr_scheduler = getattr(torch.optim.lr_scheduler, name)(optimizer, **args)
            self._metric_based = name in ["ReduceLROnPlateau"]

    def step(self, metric=None):
        if self._lr_scheduler is None:
            return
        if self._metric_based:
            if metric is not None:
                self._lr_scheduler.step(metrics=metric)
        else:
            self._lr_scheduler.step()
