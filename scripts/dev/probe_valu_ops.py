"""Dev: issue cost of single VALU instruction forms (libkgeprobe.so kge_probe_valu_op), 4 waves per
SIMD: cycles per wave-instruction at an assumed 2.4 GHz, and lane-operations per second."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
lib = ctypes.CDLL(os.path.join(ROOT, "kge-1_amd", "kge", "libkgeprobe.so"))
lib.kge_probe_valu_op.restype = ctypes.c_int64
lib.kge_probe_valu_op.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
cus = lib.kge_probe_cus()
out = torch.zeros(1 + cus * 8 * 256, device="cuda")
st = torch.cuda.current_stream().cuda_stream
names = ["v_sub_f32 v,v,v", "v_add_f32 v,v,|v|", "v_fma_f32 v,v,v,v", "v_fmac_f32 v,v,v", "v_fmac_f32 v,s,v",
         "v_med3_f32 v,v,-v,v", "v_med3_f32 v,v,-s,s", "v_mul_f32 v,s,v", "v_sub_f32 v,s,v", "v_max_f32 v,v,v",
         "v_and_b32 v,v,v", "v_bfi_b32 v,s,v,v", "v_sad_u32 v,v,v,v", "v_cmp_lt_f32 + v_cndmask_b32", "v_mul_legacy_f32 v,v,v",
         "v_mul_f32 v,v,v", "v_add_f32 v,v,v", "v_sub_f32 v,v,v2 (no dst read)", "v_fma_f32 v,v,s,v", "v_mul_f32 v,2.0,v",
         "v_med3_f32 v,v,-1.0,1.0", "v_xor_b32 v,s,v", "v_cmp_lt_f32 vcc,v,v", "v_cndmask_b32 v,v,v,vcc"]
waves = int(sys.argv[1]) if len(sys.argv) > 1 else 4
for op, name in enumerate(names):
    iters = 20000
    ops = lib.kge_probe_valu_op(op, waves, iters, out.data_ptr(), out.numel(), st)
    assert ops > 0, op
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(3):
        lib.kge_probe_valu_op(op, waves, iters, out.data_ptr(), out.numel(), st)
    b.record(); torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 3
    rate = ops / ms / 1e9
    cyc = cus * 4 * 64 * 2.4e9 / (rate * 1e12)
    print(f"{op:2d} {name:34s} {rate:6.1f} T lane-ops/s  {cyc:.2f} cycles per wave-instruction at 2.4 GHz", flush=True)
lib.kge_probe_valu_bank.restype = ctypes.c_int64
lib.kge_probe_valu_bank.argtypes = lib.kge_probe_valu_op.argtypes
for mode, name in enumerate(["v_fma_f32, 3 sources in 3 banks", "v_fma_f32, 3 sources in 1 bank", "v_sub_f32, 2 sources in 2 banks",
                             "v_sub_f32, 2 sources in 1 bank", "v_fma_f32, src0/src1 in one bank"]):
    iters = 20000
    ops = lib.kge_probe_valu_bank(mode, waves, iters, out.data_ptr(), out.numel(), st)
    assert ops > 0, mode
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(3):
        lib.kge_probe_valu_bank(mode, waves, iters, out.data_ptr(), out.numel(), st)
    b.record(); torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 3
    rate = ops / ms / 1e9
    print(f"bank {mode} {name:34s} {rate:6.1f} T lane-ops/s", flush=True)
