"""Job base (kge/job/job.py:16-179, the parts the scoring jobs use): hook lists, a
``run`` entry point and the ``create`` factory keyed by ``job.type``."""
from __future__ import annotations

from typing import Any, Callable, Dict, List


class Job:
    #: called with every job right after creation (job.py:37-43)
    job_created_hooks: List[Callable[["Job"], Any]] = []

    def __init__(self, config, dataset, parent_job=None):
        self.config = config
        self.dataset = dataset
        self.parent_job = parent_job
        self.device = config.get("job.device")
        self.pre_run_hooks: List[Callable[["Job"], Any]] = []
        self.post_run_hooks: List[Callable[["Job", Dict[str, Any]], Any]] = []
        self._is_prepared = False

    @staticmethod
    def create(config, dataset, parent_job=None, model=None) -> "Job":
        from .entity_ranking import EvaluationJob
        from .train import TrainingJob

        job_type = config.get("job.type")
        if job_type == "train":
            return TrainingJob.create(config, dataset, parent_job, model=model)
        if job_type == "eval":
            return EvaluationJob.create(config, dataset, parent_job, model=model)
        raise ValueError("unknown job type")

    def _prepare(self):
        pass

    def run(self) -> Any:
        if not self._is_prepared:
            self._prepare()
            self._is_prepared = True
        for f in self.pre_run_hooks:
            f(self)
        result = self._run()
        for f in self.post_run_hooks:
            f(self, result)
        return result

    def _run(self) -> Any:
        raise NotImplementedError

    def trace(self, **kwargs) -> Dict[str, Any]:
        return dict(kwargs)
