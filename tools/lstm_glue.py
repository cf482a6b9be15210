"""Which ATen / MIOpen ops an LSTM_large training step issues besides the coupling stack (torch.profiler over eager
TrainStep steps, B = 1024): python tools/lstm_glue.py [steps]. Prints the top ops by device time and call counts per
step, so copies, casts and elementwise glue around the MIOpen LSTM show up by name."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(steps=3):
    from torch.profiler import ProfilerActivity, profile
    from bcnf_amd import CondRealNVP_v2
    from bcnf_amd.data import DeviceBatches
    from bcnf_amd.train import TrainStep
    from bench import LSTM_LARGE
    torch.manual_seed(2024_03_25)
    m = CondRealNVP_v2.from_config(LSTM_LARGE).cuda().train()
    data = DeviceBatches(8192, 1024, "cuda", seed=1)
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
    print(f"{'op':60s} {'calls/step':>10s} {'self dev ms/step':>16s}")
    for e in rows[:45]:
        t = getattr(e, "self_device_time_total", 0) / 1e3 / steps
        if t < 0.005:
            continue
        print(f"{e.key[:60]:60s} {e.count / steps:10.1f} {t:16.3f}")
    lstm = m.feature_network_stack.feature_networks[1].lstm
    print("lstm weights contiguous chunk:", all(w.is_contiguous() for w in lstm._flat_weights),
          [w.data_ptr() for w in lstm._flat_weights][:3])


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 3)
