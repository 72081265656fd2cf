"""Optimizer / LR-scheduler factories (kge/util/optimizer.py:6-71): torch.optim classes
selected by name with ``train.optimizer_args``; "Adagrad" runs on the engine's fused step
(engine.fused_optimizer, default on) with torch.optim.Adagrad's semantics and state, "Adam"
with device-side step counters so that the recorded training step can end in it."""
from __future__ import annotations

import torch


class FusedAdagrad(torch.optim.Adagrad):
    """torch.optim.Adagrad (same arguments, state_dict layout and per-element arithmetic)
    whose step runs one engine kernel per param group (kge_adagrad_step_multi: a single pass
    over param, grad and state sum of up to 8 tensors per launch) instead of the five-pass
    multi-tensor sequence.  Parameters
    the kernel does not take (not CUDA fp32 contiguous, sparse or complex gradients,
    differentiable mode) are stepped by torch."""

    @torch.no_grad()
    def step(self, closure=None):
        from .. import _lib

        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        rest = []
        for group in self.param_groups:
            fallback = []
            items = []  # (param, grad, state sum, minus_clr) of this group: one launch per 8
            for p in group["params"]:
                if p.grad is None:
                    continue
                g = p.grad
                st = self.state[p]
                if (group["differentiable"] or g.is_sparse or not p.is_cuda or p.dtype != torch.float32
                        or g.dtype != torch.float32 or not p.is_contiguous() or not g.is_contiguous()
                        or not st["sum"].is_contiguous() or st["step"].is_cuda):
                    fallback.append(p)
                    continue
                st["step"] += 1
                step = float(st["step"])
                lr = float(group["lr"])
                minus_clr = -lr / (1 + (step - 1) * group["lr_decay"])
                items.append((p, g, st["sum"], minus_clr))
            for i in range(0, len(items), _lib.ADAGRAD_MULTI_MAX):
                _lib.adagrad_step_multi(items[i:i + _lib.ADAGRAD_MULTI_MAX], group["eps"], group["weight_decay"],
                                        group["maximize"])
            if fallback:
                rest.append((group, fallback))
        for group, params in rest:  # torch's own step for what the kernel does not take
            saved = group["params"]
            group["params"] = params
            try:
                super().step()
            finally:
                group["params"] = saved
        return loss

    def graph_safe(self) -> bool:
        """True when every step issues the same device work with the same arguments, so it
        can be recorded once and replayed (TrainingJob graph_step): all parameters are
        stepped by the kernel and the effective learning rate does not depend on the step
        count (lr_decay 0).  The host-side step counters are advanced by advance_steps."""
        for group in self.param_groups:
            if group["differentiable"] or group["lr_decay"] != 0:
                return False
            for p in group["params"]:
                if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()
                        and not self.state[p]["step"].is_cuda):
                    return False
        return True

    def advance_steps(self, params):
        """The host-side part of step() for a replayed step: count it in the state of the
        parameters the recorded step updated (those that had a gradient)."""
        for p in params:
            self.state[p]["step"] += 1


class CapturableAdam(torch.optim.Adam):
    """torch.optim.Adam with its step counters on the device (capturable=True): every step
    issues the same device work with the same arguments, so a training step that ends in it can
    be recorded as a HIP graph and replayed (TrainingJob graph_step).  Same arithmetic and
    state_dict layout as torch.optim.Adam."""

    def __init__(self, params, **args):
        args.setdefault("capturable", True)
        super().__init__(params, **args)

    def graph_safe(self) -> bool:
        for group in self.param_groups:
            if not group["capturable"] or group["differentiable"]:
                return False
            if not all(p.is_cuda for p in group["params"]):
                return False
        return True

    def advance_steps(self, params):
        """Nothing to do on the host: the replayed step advances the device-side counters."""


class KgeOptimizer:
    @staticmethod
    def create(config, model=None, params=None):
        """The optimizer of train.optimizer over a model's trainable parameters, or over an
        explicit parameter list (a row-sharded job steps its shard of the entity table)."""
        name = config.get("train.optimizer")
        if params is None:
            params = [p for p in model.parameters() if p.requires_grad]
        args = config.get("train.optimizer_args")
        if name == "Adagrad" and config.get("engine.fused_optimizer"):
            return FusedAdagrad(params, **args)
        if (name == "Adam" and config.get("engine.graph_step") and params
                and all(p.is_cuda for p in params)):
            return CapturableAdam(params, **args)
        try:
            cls = getattr(torch.optim, name)
        except AttributeError as e:
            raise ValueError(f"Could not create optimizer {name}") from e
        return cls(params, **args)


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
