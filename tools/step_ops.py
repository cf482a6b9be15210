"""Which ops a wide training step issues besides the coupling stack (torch.profiler over eager TrainStep steps):
python tools/step_ops.py [lstm_large|fc_large] [steps]. Prints the top ops by device time and call counts per step,
so copies, casts and elementwise glue (around the MIOpen LSTM, or in the feature MLP) show up by name."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(workload="lstm_large", steps=3):
    from torch.profiler import ProfilerActivity, profile
    from bcnf_amd import CondRealNVP_v2
    from bcnf_amd.data import DeviceBatches
    from bcnf_amd.train import TrainStep
    from bench import FC_LARGE, LSTM_LARGE
    cfg, B = (LSTM_LARGE, 1024) if workload == "lstm_large" else (FC_LARGE, 2048)
    torch.manual_seed(2024_03_25)
    m = CondRealNVP_v2.from_config(cfg).cuda().train()
    data = DeviceBatches(8 * B, B, "cuda", seed=1)
    st = TrainStep(m, lr=2e-4, capture=False)
    st.set_pool(data.y, data.traj)
    idx = [data.next_indices() for _ in range(steps + 2)]
    for i in range(2):
        st.step_indexed(idx[i])
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        for i in range(steps):
            st.step_indexed(idx[2 + i])
        torch.cuda.synchronize()
    ka = prof.key_averages()
    rows = sorted(ka, key=lambda e: -getattr(e, "self_device_time_total", 0))
    print(workload)
    print(f"{'op':60s} {'calls/step':>10s} {'self dev ms/step':>16s}")
    for e in rows[:45]:
        t = getattr(e, "self_device_time_total", 0) / 1e3 / steps
        if t < 0.005:
            continue
        print(f"{e.key[:60]:60s} {e.count / steps:10.1f} {t:16.3f}")
    copies = [e for e in ka if "copy" in e.key.lower() or "Memcpy" in e.key]
    for e in sorted(copies, key=lambda e: -e.count)[:10]:
        print(f"  copy-like: {e.key[:70]:70s} {e.count / steps:8.1f} per step, cpu stack rows: {e.cpu_time_total / steps:.0f} us")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "lstm_large", int(sys.argv[2]) if len(sys.argv) > 2 else 3)
