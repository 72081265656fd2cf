"""cProfile of the host side of eager training steps (argv: model, train type; KGE_PROF_OPTIONS as
in prof_train.py): where the time of a step goes that is not replayed from a recorded graph."""
import cProfile
import os
import pstats
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "kge-1_amd"))
import torch  # noqa: E402

g = runpy.run_path(os.path.join(ROOT, "scripts", "dev", "prof_train.py"))
job, perm, B = g["job"], g["perm"], g["B"]
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for i in range(20, 40):
    job.train_step(i, job._collate(perm[i * B:(i + 1) * B]))
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(28)
