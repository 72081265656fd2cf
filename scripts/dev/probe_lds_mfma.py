"""Dev probe: how fast the contraction kernel's LDS-read + MFMA loop runs without any staging
(libkgeprobe.so, kge_probe_mfma_lds): mode bit 0 = A fragment reads, bit 1 = B fragment reads,
bit 2 = a barrier per stage."""
import ctypes, os, sys
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
lib = ctypes.CDLL(os.path.join(ROOT, "kge-1_amd", "kge", "libkgeprobe.so"))
lib.kge_probe_mfma_lds.restype = ctypes.c_int64
lib.kge_probe_mfma_lds.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
lib.kge_probe_mfma.restype = ctypes.c_int64
lib.kge_probe_mfma.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
out = torch.empty(lib.kge_probe_cus() * 512, device="cuda")
st = torch.cuda.current_stream().cuda_stream


def timed(fn, reps=10, settle=3):
    for _ in range(settle):
        flops = fn()
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        flops = fn()
    b.record(); torch.cuda.synchronize()
    return flops / (a.elapsed_time(b) / reps / 1e3) / 1e12


stages = 1600  # 100 tiles' worth of K loop per launch (~3 ms)
for rnd in range(2):
    print(f"registers only, random: {timed(lambda: lib.kge_probe_mfma(8000, 1, out.data_ptr(), out.numel(), st)):.0f} TF/s")
    for mode in (0, 1, 2, 3, 7):
        tf = timed(lambda: lib.kge_probe_mfma_lds(mode, stages, out.data_ptr(), out.numel(), st))
        print(f"mode {mode} (A reads {mode & 1}, B reads {(mode >> 1) & 1}, barrier {(mode >> 2) & 1}): {tf:.0f} TF/s bf16", flush=True)
