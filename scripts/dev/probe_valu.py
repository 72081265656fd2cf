"""Dev: scalar-fp32 VALU issue rate of the chip (libkgeprobe.so kge_probe_valu): the L1-distance
inner loop on registers, independent FMA chains, and the L1 loop fed from LDS, at 1-4 waves per SIMD."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
lib = ctypes.CDLL(os.path.join(ROOT, "kge-1_amd", "kge", "libkgeprobe.so"))
lib.kge_probe_valu.restype = ctypes.c_int64
lib.kge_probe_valu.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
cus = lib.kge_probe_cus()
out = torch.zeros(1 + cus * 8 * 256, device="cuda")
st = torch.cuda.current_stream().cuda_stream
names = {0: "L1 sub + add|.| (registers)", 1: "independent v_fma_f32 chains", 2: "L1 loop fed from LDS",
         3: "L1 bwd: sub, med3(VGPR u), fmac(SGPR w)", 4: "L1 bwd: sub, med3(SGPR u), fmac(SGPR w)"}
only = [int(a) for a in sys.argv[1:]]
for variant in (only or (0, 1, 2, 3, 4)):
    for w in (1, 2, 3, 4):
        iters = 20000
        ops = lib.kge_probe_valu(variant, w, iters, out.data_ptr(), out.numel(), st)  # warm-up
        assert ops > 0
        a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(3):
            lib.kge_probe_valu(variant, w, iters, out.data_ptr(), out.numel(), st)
        b.record(); torch.cuda.synchronize()
        ms = a.elapsed_time(b) / 3
        print(f"{names[variant]:32s} {w} wave(s)/SIMD: {ops / ms / 1e9:.1f} T lane-ops/s = {ops / ms / 1e9 / 78.6:.3f} of 78.6 "
              f"({ms:.2f} ms)", flush=True)
