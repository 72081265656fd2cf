from .job import Job  # noqa: F401
from .train import TrainingJob, TrainingJob1vsAll, TrainingJobKvsAll  # noqa: F401
from .entity_ranking import EvaluationJob, EntityRankingJob  # noqa: F401
