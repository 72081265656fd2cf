import sys, os, json
sys.path.insert(0, '.'); sys.path.insert(0, 'kge-1_amd'); sys.path.insert(0, 'tests')
import numpy as np, torch
from test_gpu_api import eval_job
f = np.load('tests/golden/eval_dyadic.npz')
for prec in ('fp32', 'bf16x3'):
    job, trace = eval_job(f, 'full', prec)
    for k, v in job.ranks.items():
        ref = f['full_' + k]
        print(prec, k, (v != ref).sum(), v[:8], ref[:8])
