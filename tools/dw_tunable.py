"""Weight-gradient shapes of the c3 step: our split-K GEMM (triad_amd.linear.weight_grad) vs
torch.mm(dy^T, x) with TunableOp searching every hipBLASLt / rocBLAS solution (tuning here, in
this process only). One JSON line per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    from triad_amd import _lib
    from triad_amd.linear import weight_grad
    _lib.load()
    tun = torch.cuda.tunable
    tun.set_filename("gpurun_out/dw_tunable_results.csv")
    tun.set_max_tuning_duration(80)
    tun.set_max_tuning_iterations(100)
    for M, O, K in ((50944, 768, 768), (50944, 3072, 768), (50944, 768, 3072), (50944, 2304, 768),
                    (8192, 768, 768), (8192, 3072, 768), (8192, 768, 3072), (8192, 2304, 768)):
        dy = torch.randn(M, O, device="cuda").to(torch.bfloat16)
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        ours = bench(lambda: weight_grad(dy, x))
        tun.enable(False)
        lib = bench(lambda: torch.mm(dy.t(), x))
        tun.enable(True)
        tun.tuning_enable(True)
        torch.mm(dy.t(), x)
        tun.tuning_enable(False)
        tuned = bench(lambda: torch.mm(dy.t(), x))
        tun.enable(False)
        print(json.dumps({"M": M, "O": O, "K": K, "ours_ms": round(ours, 4), "lib_ms": round(lib, 4),
                          "lib_tuned_ms": round(tuned, 4)}), flush=True)


if __name__ == "__main__":
    main()
