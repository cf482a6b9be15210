"""Why k_resim runs slower inside the default bench than standalone: time the kernel (HIP events,
3 launches) fresh, right after a heavy GPU phase (FC_large-like fp32 GEMM load for ~4 s), after the caching allocator
has been churned by large allocations, and again after an idle pause. python tools/resim_context.py"""
import os
import subprocess
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def clocks():
    try:
        out = subprocess.run(["rocm-smi", "--showclocks", "--showtemp", "--showpower"], capture_output=True,
                             text=True, timeout=20).stdout
        keep = [ln.strip() for ln in out.splitlines() if any(k in ln for k in ("sclk", "mclk", "Temperature",
                                                                                "Power", "(W)"))]
        return " | ".join(keep[:6])
    except Exception as e:  # noqa: BLE001
        return f"rocm-smi: {e}"


def main():
    from bench import FC_SMALL, resim_draws
    from bcnf_amd.resimulation import resimulate_device
    from bcnf_amd.utils import ParameterIndexMapping
    dev = torch.device("cuda")
    yh, dd = resim_draws(1024, 1000)
    pim = ParameterIndexMapping(FC_SMALL["global"]["parameter_selection"])
    y = torch.from_numpy(yh).to(dev).contiguous()

    def k_us(n=3):
        resimulate_device(y, 2.0, 1 / 15, dd, pim, break_on_impact=True, device=dev)
        st = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(n):
            resimulate_device(y, 2.0, 1 / 15, dd, pim, break_on_impact=True, device=dev)
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / n

    print("fresh", round(k_us(), 1), clocks(), flush=True)
    print("fresh again", round(k_us(), 1), flush=True)
    a = torch.randn(8192, 8192, device=dev)
    t0 = time.time()
    while time.time() - t0 < 4.0:
        for _ in range(20):
            a = (a @ a).clamp_(-1, 1)
        torch.cuda.synchronize()
    print("right after 4 s of GEMM load", round(k_us(), 1), clocks(), flush=True)
    del a
    big = [torch.empty(int(1.5e9) // 4, device=dev) for _ in range(8)]
    del big
    print("after allocator churn (12 GB)", round(k_us(), 1), flush=True)
    torch.cuda.empty_cache()
    print("after empty_cache", round(k_us(), 1), flush=True)
    time.sleep(5)
    print("after 5 s idle", round(k_us(), 1), clocks(), flush=True)


if __name__ == "__main__":
    main()
