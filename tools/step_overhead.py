"""Where the fixed cost of a short timed region goes (FC_small training, bench.py's default run_epoch path): for
each n in STEPS, the host wall time of run_epoch(n) bracketed by synchronize() as bench.py brackets it, the GPU time
between events recorded right before and after it, and the host time until the first graph launch returned.
A fit wall = a + b n separates the per-step time b from the fixed cost a. PREWARM=matmul MS=200 runs unrelated GEMMs
first; WARM = the run_epoch steps before the measurements (16); LR; FUSE_ADAM=0 keeps Adam out of the tail."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import FC_SMALL  # noqa: E402
from bcnf_amd import CondRealNVP_v2  # noqa: E402
from bcnf_amd.data import DeviceBatches  # noqa: E402
from bcnf_amd.train import TrainStep  # noqa: E402

STEPS = [8, 16, 48, 96, 200, 400]
B = 4096
dev = torch.device("cuda", 0)
torch.manual_seed(2024_03_25)
model = CondRealNVP_v2.from_config(FC_SMALL).to(dev)
model.train()
data = DeviceBatches(int(os.environ.get("POOL", "65536")), B, dev, seed=2024_03_25)
step = TrainStep(model, lr=float(os.environ.get("LR", "2e-4")), capture=True)
step.fuse_adam = os.environ.get("FUSE_ADAM", "1") == "1"     # 0: Adam in its own launch every step
step.set_pool(data.y, data.traj)
WARM = int(os.environ.get("WARM", "16"))
total = WARM + 3 * sum(STEPS) + 32
step.set_epoch(torch.cat([data.next_indices() for _ in range(total)]), B)
# PREWARM=matmul: ~MS ms of unrelated fp32 GEMMs before the first step (is the slow start the clock ramp?)
if os.environ.get("PREWARM") == "matmul":
    a = torch.randn(4096, 4096, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < float(os.environ.get("MS", "200")) / 1e3:
        for _ in range(10):
            a = (a @ a) * 1e-3
        torch.cuda.synchronize()
step.run_epoch(WARM)
step.prepare_epoch(8)
rows = []
for rep in range(3):
    for n in STEPS:
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        step.run_epoch(n)       # ends with a stream synchronize and the history read
        e1.record()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        gpu = e0.elapsed_time(e1)
        rows.append((n, wall, gpu))
        print(f"rep {rep} n {n:4d}: wall {wall:8.3f} ms ({wall / n * 1e3:7.2f} us/step)  gpu {gpu:8.3f} ms "
              f"({gpu / n * 1e3:7.2f} us/step)", flush=True)
a = np.array(rows)
for col, name in ((1, "wall"), (2, "gpu")):
    b, c = np.polyfit(a[:, 0], a[:, col], 1)
    print(f"{name}: {b * 1e3:.2f} us/step + {c * 1e3:.1f} us fixed")
# idle gap before the region: a bare synchronize, then the first multi-step graph alone, timed per launch
for gap_ms in (0.0, 1.0, 5.0):
    torch.cuda.synchronize()
    if gap_ms:
        time.sleep(gap_ms / 1e3)
    t0 = time.perf_counter()
    step.run_epoch(8)
    print(f"after {gap_ms:.0f} ms idle: one 8-step graph {(time.perf_counter() - t0) * 1e3:.3f} ms wall", flush=True)
