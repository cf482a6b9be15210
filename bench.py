"""Benchmark: NLL-training samples/s of CondRealNVP_v2 trajectory_FC_small (B=4096 per GPU) on MI355X.

One step = bcnf.train.Trainer._train_batch semantics (src/bcnf/train/trainer.py:244-277): batch gather
from the device-resident pool, zero_grad, forward [FC feature net Linear on the HIP GEMM + fused coupling
stack with the NLL in the same launch], backward [fused NLL backward + deterministic slab reduce + Linear
weight-gradient GEMM], (N>1: RCCL all-reduce of the gradients), Adam step (one fused launch), clip_grad_norm_
after the step, one host sync for the three logged losses. The step is one HIP-graph replay.
Synthetic ballistic trajectories (bcnf_amd/data.py), device-resident, pre-shuffled; dropout active.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
N>1: either launched by torch.distributed.run (RANK / WORLD_SIZE in the environment), or run directly, in which
case this process -- before it touches the GPU -- starts `torch.distributed.run --nproc-per-node N` on itself as a
child process and exits with the child's status. Prints ONE JSON line on rank 0.
"""
import argparse
import json
import math
import os
import socket
import statistics
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "NLL-training samples/sec + log_prob max-abs-err vs ref, trajectory_FC_small"
FC_SMALL = {
    "global": {"parameter_selection": ['x0_x', 'x0_y', 'x0_z', 'v0_x', 'v0_y', 'v0_z', 'g', 'w_x', 'w_y', 'w_z',
                                       'b', 'm', 'a_x', 'a_y', 'a_z', 'r', 'A', 'Cd', 'rho']},
    "model": {"kwargs": {"size": 19, "nested_sizes": [16] * 7, "n_conditions": 80, "n_blocks": 32,
                         "dropout": 0.383, "act_norm": True}},
    "feature_networks": [
        {"type": "ConcatenateCondition", "kwargs": {"input_size": None, "output_size": 90}},
        {"type": "FullyConnected", "kwargs": {"sizes": [90, 80], "dropout": 0.244}},
    ],
}
# Algorithmic work per sample (recompute excluded). MAC counts for FC_small:
#   forward flow  = 32 * (90*16 + 6*16*16 + 16*18) + 31 * 19*19 = 115,639 MAC   (k_forward; the reference's count,
#                   the condition projection included -- k_forward computes it on its helper waves)
#   backward flow = dX (115,639) + dW of every Linear (32 * 3,264 = 104,448)      = 220,087 MAC for the whole backward;
#                   k_backward's own share excludes the W1 condition columns (dW1h and dL/dh: 2 * 32 * 16 * 80 =
#                   81,920 MAC, done by the tail's split-K): 138,167 MAC
FWD_FLOP_PER_SAMPLE = 2 * 115_639
# the pack-free forward (bcnf_fold_train_forward) also computes the feature Linear h = x Wf^T + bf of its rows
FEAT_FLOP_PER_SAMPLE = 2 * 90 * 80
BWD_FLOP_PER_SAMPLE = 2 * 220_087
KBWD_FLOP_PER_SAMPLE = 2 * (220_087 - 81_920)
# SURVEY §8d minimal HBM bytes per sample of per-block kernels (recompute in backward), nb = 32, D = 19, C = 80:
#   forward  nb * 4 * (2D + C + 2)                         = 15,360 B   (y, h in; z, ldj out, per block)
#   training nb * 4 * (5D + 4C + 2)                        = 53,376 B   -> backward share 53,376 - 15,360 = 38,016 B
FWD_ALG_BYTES_PER_SAMPLE = 32 * 4 * (2 * 19 + 80 + 2)
BWD_ALG_BYTES_PER_SAMPLE = 32 * 4 * (5 * 19 + 4 * 80 + 2) - FWD_ALG_BYTES_PER_SAMPLE
# trajectory_FC_large / trajectory_LSTM_large (configs/runs/old/*.yaml): the wide-MLP family (bcnf_wide.hip)
FC_LARGE = {
    "global": FC_SMALL["global"],
    "model": {"kwargs": {"size": 19, "nested_sizes": [526] * 5, "n_conditions": 1360, "n_blocks": 26,
                         "dropout": 0.407, "act_norm": True}},
    "feature_networks": [
        {"type": "ConcatenateCondition", "kwargs": {"input_size": None, "output_size": 90}},
        {"type": "FullyConnected", "kwargs": {"sizes": [90] + [310] * 7 + [1360], "dropout": 0.111}},
    ],
}
LSTM_LARGE = {
    "global": FC_SMALL["global"],
    "model": {"kwargs": {"size": 19, "nested_sizes": [526] * 5, "n_conditions": 1360, "n_blocks": 26,
                         "dropout": 0.407, "act_norm": True, "random_state": 2024_03_25}},
    "feature_networks": [
        {"type": "ConcatenateCondition", "kwargs": {"input_size": None, "output_size": 3}},
        {"type": "LSTM", "kwargs": {"input_size": 3, "hidden_size": 140, "output_size": 1360, "num_layers": 2,
                                    "dropout": 0.111, "bidirectional": True, "pooling": "mean", "pool_dim": 1}},
    ],
}
# training FLOPs per sample (2 x MAC, forward + dX + dW of every Linear of the flow; feature net excluded)
#   flow forward = 26 * (1370*526 + 4*526*526 + 526*18) + 25 * 19*19 = 47,765,617 MAC
WIDE_FWD_FLOP_PER_SAMPLE = 2 * 47_765_617
WIDE_TRAIN_FLOP_PER_SAMPLE = 3 * WIDE_FWD_FLOP_PER_SAMPLE
# SURVEY §8d per-block minimum for the training step, nb = 26, D = 19, C = 1360: nb * 4 * (5D + 4C + 2)
WIDE_ALG_BYTES_PER_SAMPLE = 26 * 4 * (5 * 19 + 4 * 1360 + 2)
# The FLOPs the wide training step EXECUTES, against the reference count above: the folded last feature
# Linear (x1 = [x | 1 | 0], Xp = round_up(X + 1, 4): FC_large X = 310 -> 312, LSTM_large X = 280 -> 284) replaces the
# 1360-wide condition GEMMs per sample by Xp-wide ones plus three per-step GEMMs of nb H C Xp MACs (Wcb = W0h wfb,
# dW0h = Gx wfb^T, [dWf | dbf] = W0h^T Gx). Per sample, MACs (nin = 10, nout = 18, H = 526):
#   forward  nb (nin H + Xp H + 4 H^2 + H nout) + (nb - 1) D^2
#   backward nb (4 H^2 + nout H + nin H          [dX of the hidden, last and Linear-1 y-part]
#                + 4 H (H + 1) + nout (H + 1) + H (nin + 1))   [dW / db]
#            + 2 nb H Xp (dL/dx = dZ0 Wcb, Gx = dZ0^T x1) + (nb - 1) D^2
WIDE_FOLD_X = {"fc_large": 310, "lstm_large": 280}


def wide_executed_flop(workload, B):
    nb, H, C, D, nin, nout = 26, 526, 1360, 19, 10, 18
    Xp = (WIDE_FOLD_X[workload] + 1 + 3) // 4 * 4
    fwd = nb * (nin * H + Xp * H + 4 * H * H + H * nout) + (nb - 1) * D * D
    bwd = nb * (4 * H * H + nout * H + nin * H + 4 * H * (H + 1) + nout * (H + 1) + H * (nin + 1)) \
        + 2 * nb * H * Xp + (nb - 1) * D * D
    return 2 * ((fwd + bwd) * B + 3 * nb * H * C * Xp)


WIDE_NAMES = {"fc_large": "trajectory_FC_large", "lstm_large": "trajectory_LSTM_large"}
WORKLOADS = {"fc_small": (FC_SMALL, 4096), "fc_large": (FC_LARGE, 2048), "lstm_large": (LSTM_LARGE, 1024),
             "sample": (FC_SMALL, 1024), "resimulate": (None, 1024)}
# Re-simulation (simulation/resimulation.py:21-59, notebooks/resimulation.ipynb: T = 2, dt = 1/15, m_samples = 1000,
# break_on_impact = True): executed fp64 work per Dormand-Prince attempt of bcnf_resim.hip, counted from its source:
# 6 right-hand sides x 28 (sqrt and reciprocal as 1 each) + stage combinations 138 + error norm 59
RESIM_FLOP_PER_ATTEMPT = 6 * 28 + 138 + 59
PEAK_FP64_TFLOPS = 78.6        # MI355X fp64 vector, AMD's product figure (not in MI355X_MICROARCH.md)
PEAK_FP32_TFLOPS = 157.3       # MI355X fp32 (vector = MFMA f32), MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="fc_small",
                    help="fc_small = the headline metric (configs[1]); fc_large / lstm_large = configs[2] / [3] per GPU")
    ap.add_argument("--batch", type=int, default=None, help="samples per GPU (weak scaling; default per workload)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--overlap-ranges", type=int, default=None,
                    help="wide workloads at world > 1: block ranges of the overlapped gradient all-reduce (default "
                         "4; 0 = one all-reduce after the backward, captured graphs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=12)
    ap.add_argument("--kernel-iters", type=int, default=20)
    ap.add_argument("--spinup-ms", type=float, default=150.0,
                    help="device spin-up before the warmup steps: the step's own kernels back to back for this long "
                         "(untimed, no parameter update), so the timed steps do not run inside the GPU's clock ramp "
                         "(the first ~40 ms of continuous work after idle run ~10 %% slower, DESIGN 3k); 0 = off")
    ap.add_argument("--indexed", action="store_true", help="per-step index copy instead of the device epoch cursor")
    ap.add_argument("--per-step-sync", action="store_true",
                    help="one host sync + logged-value read per step (the Trainer loop shape) instead of run_epoch")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the secondary figures (Trainer loop shape, unchanged-Trainer DataLoader)")
    ap.add_argument("--launch-check", action="store_true",
                    help="only bring up the N-rank process group (gloo without a GPU) and report the ranks seen")
    return ap.parse_args()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args):
    """`python bench.py --gpus N` (N > 1) outside torch.distributed.run: run N fresh worker processes through
    torch.distributed.run as a CHILD of this process (which has not touched the GPU: nothing before this point
    initialises HIP) and exit with its status. Returns when this process is itself a rank (or N == 1)."""
    if "WORLD_SIZE" in os.environ or args.gpus <= 1:
        return
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd, env=env))


def host_cores():
    """CPU cores this process may use: the scheduler affinity set, capped by a cgroup CPU quota (the GPU box's
    16-CPU share of a larger machine) -- what torch.set_num_threads can actually occupy."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit():
        n = min(n, int(omp))
    return max(1, n)


SHARED_DEVICES = False          # set by init_dist: more ranks than visible GPUs (a rehearsal, reported in the JSON)


def init_dist(args):
    """One process per GPU over RCCL (backend "nccl"). With fewer visible GPUs than ranks (a 1-GPU box rehearsing
    --gpus 2) the ranks share devices round-robin and talk over gloo -- RCCL refuses two ranks on one device -- and
    the JSON line says so ("shared_devices": true): such a number is not a scaling measurement."""
    global SHARED_DEVICES
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        ndev = torch.cuda.device_count()
        if args.launch_check and not torch.cuda.is_available():
            dist.init_process_group("gloo")
        elif ndev < world:
            SHARED_DEVICES = True
            local = local % max(ndev, 1)
            torch.cuda.set_device(local)
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"bench.py: process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")
    return world, rank, local


def ranks_seen(world, device):
    """Number of ranks that took part in the timed run (an all-reduce of ones), reported in the JSON line."""
    if world == 1:
        return 1
    t = torch.ones(1, device=device)
    dist.all_reduce(t)
    return int(t.item())


def launch_check(args):
    world, rank, _ = init_dist(args)
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0"))) if torch.cuda.is_available() else "cpu"
    seen = ranks_seen(world, dev)
    sub = run_sublines(args, world, rank, dev, dry=True)
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "ranks_seen": seen,
                          "backend": dist.get_backend() if world > 1 else None, "secondary": sub}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


N_SIMD = 1024                  # 256 CUs x 4 SIMDs
CLOCK_GHZ = 2.4


def pmc_utilisation(kernel, avg_us):
    """Matrix-pipe utilisation and occupancy of `kernel` from the committed rocprofv3 SQ counters of the same
    build (profiles/pmc_insts.json, tools/profile_round.sh): mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x
    launch cycles at 2.4 GHz), waves_per_simd = SQ_WAVES / SIMDs, and the per-launch instruction counts."""
    path = os.path.join(ROOT, "profiles", "pmc_insts.json")
    if not os.path.exists(path) or not (avg_us == avg_us):
        return {}
    with open(path) as f:
        c = json.load(f).get(kernel)
    if not c:
        return {}
    out = {"waves_per_simd": round(c.get("SQ_WAVES", 0.0) / N_SIMD, 3)}
    if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
        out["mfma_busy_frac"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (N_SIMD * avg_us * 1e3 * CLOCK_GHZ), 4)
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT"):
        if k in c:
            out[k.lower()] = c[k]
    return out


def log_prob_error(model, device):
    """log_prob max-abs-err vs the reference's own outputs (golden fixture produced by running psaegert/bcnf)."""
    path = os.path.join(ROOT, "tests", "golden", "g1_fc_small.npz")
    if not os.path.exists(path):
        return None, None
    g1 = np.load(path)
    sd = {k[3:]: torch.from_numpy(np.ascontiguousarray(g1[k])) for k in g1.keys() if k.startswith("sd/")}
    from bcnf_amd import CondRealNVP_v2
    torch.manual_seed(0)
    m = CondRealNVP_v2.from_config(FC_SMALL)
    m.load_state_dict(sd)
    m.to(device).eval()
    with torch.no_grad():
        lp = m.log_prob(torch.from_numpy(g1["y"]).to(device), torch.from_numpy(g1["traj"]).to(device)).double().cpu()
    ref = -torch.from_numpy(g1["nll"]).double() - 0.5 * 19 * math.log(2 * math.pi)
    err = (lp - ref).abs()
    return float(err.max()), float((err / ref.abs().clamp_min(1.0)).max())


def _proxy_sd(model, seed):
    """numpy-PCG64 weights in state_dict order, the orthonormal matrices kept (tests/golden/make_golden.py's
    large_proxy_state, the recipe the g7 fixture was made with)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    sd = {}
    for k, v in model.state_dict().items():
        if k.endswith("orthonormal_matrix"):
            sd[k] = v.detach().cpu().numpy()
            continue
        shape = tuple(v.shape)
        if k.endswith(".scale"):
            a = rng.uniform(0.7, 1.3, size=shape)
        elif len(shape) == 2:
            a = rng.uniform(-1.0, 1.0, size=shape) / np.sqrt(shape[1])
        else:
            a = rng.uniform(-0.05, 0.05, size=shape)
        sd[k] = a.astype(np.float32)
    return sd


def _lp_err(lp, z_ref, ldj_ref):
    ref = -(0.5 * (torch.from_numpy(z_ref).double() ** 2).sum(1) - torch.from_numpy(ldj_ref).double()) \
        - 0.5 * z_ref.shape[1] * math.log(2 * math.pi)
    err = (lp.double().cpu() - ref).abs()
    return float(err.max()), float((err / ref.abs().clamp_min(1.0)).max())


def log_prob_errors_more(device):
    """log_prob max-abs / max-rel error on the reference's other fixtures -- G7 (FC_large-shaped proxy:
    C = 1360, [526] x 5, 2 blocks, the wide kernel family) and G9 (physical ballistic trajectories from the
    reference's ODE simulator on the seeded FC_small init)."""
    from bcnf_amd import CondRealNVP_v2
    out = {}
    p9 = os.path.join(ROOT, "tests", "golden", "g9_ballistic.npz")
    if os.path.exists(p9):
        d = np.load(p9)
        torch.manual_seed(2024_03_25)
        m = CondRealNVP_v2.from_config(FC_SMALL).to(device).eval()
        with torch.no_grad():
            lp = m.log_prob(torch.from_numpy(d["y"]).to(device), torch.from_numpy(d["traj"]).to(device))
        out["g9"] = _lp_err(lp, d["z"], d["ldj"])
    p7 = os.path.join(ROOT, "tests", "golden", "g7_large_proxy.npz")
    if os.path.exists(p7):
        d = np.load(p7)
        shape = dict(size=19, nested_sizes=[526] * 5, n_blocks=2, n_conditions=1360, dropout=0.407, act_norm=True)
        cfg = {"global": {"parameter_selection": [f"p{i}" for i in range(19)]}, "model": {"kwargs": shape},
               "feature_networks": [
                   {"type": "ConcatenateCondition", "kwargs": {"input_size": None, "output_size": 90}},
                   {"type": "FullyConnected", "kwargs": {"sizes": [90, 1360], "dropout": 0.0}}]}
        torch.manual_seed(7)
        m = CondRealNVP_v2.from_config(cfg)
        sd = _proxy_sd(m, 2024_03_25)
        sd["layers.2.orthonormal_matrix"] = d["q/layers.2.orthonormal_matrix"]
        m.load_state_dict({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()})
        m.to(device).eval()
        with torch.no_grad():
            lp = m.log_prob(torch.from_numpy(d["y"]).to(device), torch.from_numpy(d["traj"]).to(device))
        out["g7"] = _lp_err(lp, d["z"], d["ldj"])
    return {f"{k}_{n}": v[i] for k, v in out.items() for i, n in enumerate(("max_abs", "max_rel"))}


def wide_fixture_error(workload, device):
    """log_prob max-abs / max-rel error of the wide workload's model at FULL depth (26 blocks) against the reference's
    own outputs: g11 (trajectory_FC_large, FC[90, 310 x 7, 1360]) or g10's pool-over-time outputs (trajectory_LSTM_large
    with pool_dim=1, the reference's own LSTM / Linear modules), both on PCG64 weights
    (tests/golden/make_golden.py: the same seeds rebuild the same model here), eval mode."""
    from bcnf_amd import CondRealNVP_v2
    lstm = workload == "lstm_large"
    path = os.path.join(ROOT, "tests", "golden", "g10_lstm_large.npz" if lstm else "g11_fc_large.npz")
    if not os.path.exists(path):
        return None
    d = np.load(path)
    cfg = json.loads(json.dumps(WORKLOADS[workload][0]))
    torch.manual_seed(2024_03_25 + (12 if lstm else 15))
    m = CondRealNVP_v2.from_config(cfg)
    sd = _proxy_sd(m, 2024_03_25 + (13 if lstm else 16))
    for k in sd:
        if k.endswith("orthonormal_matrix"):      # the reference's own Q bytes (host LAPACK rounding aside)
            sd[k] = d["q"] if lstm else d["q/" + k]
    m.load_state_dict({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()})
    m.to(device).eval()
    y, traj, z, ldj = (d["y1"], d["traj1"], d["z1"], d["ldj1"]) if lstm else (d["y"], d["traj"], d["z"], d["ldj"])
    with torch.no_grad():
        lp = m.log_prob(torch.from_numpy(y).to(device), torch.from_numpy(traj).to(device))
    mx, rel = _lp_err(lp, z, ldj)
    del m
    return {"fixture": os.path.basename(path), "rows": int(y.shape[0]), "log_prob_max_abs_err": mx,
            "log_prob_max_rel_err": rel}


def cpu_baseline(args):
    """The CPU oracle (PyTorch-eager restatement of the reference, pinned to its outputs) timed on this host's
    cores: same FC_small step at the same batch, bounded sample."""
    from oracle import cnf_oracle as O
    from bcnf_amd.data import simulate
    threads = host_cores()
    torch.set_num_threads(threads)
    torch.manual_seed(2024_03_25)
    from bcnf_amd import CondRealNVP_v2
    m = CondRealNVP_v2.from_config(FC_SMALL)
    sd = {k: v.detach().clone().requires_grad_(not k.endswith("orthonormal_matrix")) for k, v in m.state_dict().items()}
    opt = torch.optim.Adam([v for v in sd.values() if v.requires_grad], lr=2e-4)
    y, traj = simulate(args.batch, seed=7)
    y = torch.from_numpy(y)
    traj = torch.from_numpy(traj)
    y = (y - y.mean(0)) / (y.std(0) + 1e-6)
    traj = (traj - traj.mean((0, 1))) / (traj.std((0, 1)) + 1e-6)
    times = []
    for i in range(3 + args.cpu_steps):
        t0 = time.perf_counter()
        O.train_step_cpu(sd, O.FC_SMALL_SPEC, y, traj, opt, training=True)
        times.append(time.perf_counter() - t0)
    med = statistics.median(times[3:])
    return {"value": round(args.batch / med, 1), "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": f"oracle/cnf_oracle.train_step_cpu (PyTorch-eager CPU restatement pinned to the reference), "
                      f"FC_small B={args.batch}, dropout on, median of {args.cpu_steps} steps after 3 warmup, "
                      f"{threads} threads, {med * 1e3:.1f} ms/step"}


def spinup(fn, ms):
    """Run fn back to back until `ms` of wall time have passed (untimed device spin-up, --spinup-ms); returns the
    milliseconds spent. Nothing it runs touches the parameters or the optimizer state, and fn holds no collective:
    each rank runs it a different number of times."""
    if ms <= 0:
        return 0.0
    sync = torch.cuda.synchronize if torch.cuda.is_available() else (lambda: None)   # (CPU: the gloo tests)
    sync()
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        fn()
    sync()
    return round((time.perf_counter() - t0) * 1e3, 1)


def kernel_timing(model, data, args):
    """Average device time (us) of each launch of the NLL training pass on one batch, measured with HIP
    events on the launch stream around back-to-back launches (FusedStack.time_kernels)."""
    idx = data.next_indices()
    y, traj = data.y[idx], data.traj[idx]
    with torch.no_grad():
        h = model.feature_network_stack(traj).contiguous()
        w = model.fold_pool_width(traj) if hasattr(model, "fold_pool_width") else None
        lin = model._fold_linear() if hasattr(model, "_fold_linear") else None
    if lin is not None:                 # the folded step: x rows padded like TrainStep's pool
        X = traj[0].numel()
        xp = torch.zeros((traj.shape[0], w or X), dtype=traj.dtype, device=traj.device)
        xp[:, :X] = traj.reshape(traj.shape[0], X)
        fold = (xp[:, :X], lin.weight.detach(), None if lin.bias is None else lin.bias.detach())
        return model.fused.time_kernels(y, h, training=True, iters=args.kernel_iters, fold=fold)
    with torch.no_grad():
        wfold = model._wide_fold(y, (traj,)) if hasattr(model, "_wide_fold") else None
    if wfold is not None:               # the wide family's folded step (the last feature Linear in the projection)
        with torch.no_grad():
            x, lin = wfold
            fold = (x.contiguous(), lin.weight.detach(), None if lin.bias is None else lin.bias.detach())
            return model.fused.time_kernels(y, h, training=True, iters=args.kernel_iters, fold=fold)
    return model.fused.time_kernels(y, h, training=True, iters=args.kernel_iters)


def main():
    args = parse()
    launch_ranks(args)
    if args.launch_check:
        return launch_check(args)
    if args.batch is None:
        args.batch = WORKLOADS[args.workload][1]
    if args.workload == "sample":
        return main_sample(args)
    if args.workload == "resimulate":
        return main_resim(args)
    if args.workload != "fc_small":
        return main_wide(args)
    world, rank, local = init_dist(args)
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    from bcnf_amd import CondRealNVP_v2
    from bcnf_amd.data import DeviceBatches
    from bcnf_amd.train import TrainStep

    torch.manual_seed(2024_03_25)
    model = CondRealNVP_v2.from_config(FC_SMALL).to(device)
    model.train()
    model.fused.set_seed(2024_03_25 + 7919 * rank)
    data = DeviceBatches(65536, args.batch, device, seed=2024_03_25 + rank)
    step = TrainStep(model, lr=2e-4, capture=not args.no_graph)
    step.broadcast_parameters()
    step.set_pool(data.y, data.traj)
    # the shuffled batch order of the whole run lives on the device; the graph walks it with a device cursor
    batches = [data.next_indices() for _ in range(args.warmup + args.steps)]
    if not args.indexed:
        step.set_epoch(torch.cat(batches), args.batch)
    # default: the epoch's steps replayed back to back, logged values read once at the end (run_epoch);
    # --per-step-sync: the Trainer's loop shape, one host sync + read per step (step_epoch)
    if args.indexed or args.per_step_sync:
        run = (lambda i: step.step_indexed(batches[i])) if args.indexed else (lambda i: step.step_epoch())

        def run_range(a, b):
            out = None
            for i in range(a, b):
                out = run(i)
            return out
    else:
        def run_range(a, b):
            vals = step.run_epoch(b - a)
            return vals[-1] if vals else None

    if not (args.indexed or args.per_step_sync):
        # graph captures (host work, the GPU idle) before the spin-up and the warmup steps, so the timed steps follow
        # device work without an idle gap
        step.prepare_epoch(max(args.steps, args.warmup))
    spin = argparse.Namespace(**{**vars(args), "kernel_iters": 4})
    spun = spinup(lambda: kernel_timing(model, data, spin), args.spinup_ms)
    run_range(0, args.warmup)
    if not (args.indexed or args.per_step_sync):
        step.prepare_epoch(args.steps)      # (captured above: no capture lands in the timed region at any --warmup)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    losses = run_range(args.warmup, args.warmup + args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], device=device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    ms_per_step = dt / args.steps * 1e3
    value = world * args.batch * args.steps / dt
    seen = ranks_seen(world, device)

    kern = kernel_timing(model, data, args) if rank == 0 else {}
    line = None
    if rank == 0:
        B = args.batch
        lp_abs, lp_rel = log_prob_error(model, device)
        per_kernel = fc_small_rooflines(kern, B)
        dom = max(per_kernel, key=lambda k: per_kernel[k]["avg_us"])   # the longest single launch, measured
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "samples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "device_spinup_ms": spun, "ms_per_step": round(ms_per_step, 4),
            "ranks_seen": seen,
            **({"shared_devices": True} if SHARED_DEVICES else {}),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic ballistic trajectories (bcnf_amd/data.py RK4 restatement of physics.py), device-resident",
            "config": {"workload": "trajectory_FC_small NLL training step (configs[1])", "batch_per_gpu": B,
                       "global_batch": B * world, "parallelism": f"dp{world}", "hip_graph": not args.no_graph,
                       "n_blocks": 32, "nested_sizes": [16] * 7, "n_conditions": 80, "dropout": 0.383},
            "log_prob_max_abs_err": lp_abs, "log_prob_max_rel_err": lp_rel,
            "log_prob_err_other_fixtures": log_prob_errors_more(device),
            "last_loss": losses[0] if losses else None,
            "roofline": dict(per_kernel[dom], kernel=dom),
            "roofline_kernels": per_kernel,
            "kernels_us": {k: round(v, 2) for k, v in kern.items()},
        }
        if not args.no_secondary and world == 1 and not (args.indexed or args.per_step_sync):
            line["secondary"] = secondary_figures(step, args, device)
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline(args)
    if not args.no_secondary and not (args.indexed or args.per_step_sync):
        # configs[2], [3], [4] and re-simulation on every rank (the world's own scaling of each), each with its own
        # roofline and, at world 1, its own cpu_baseline (bounded)
        del step, model, data
        torch.cuda.empty_cache()
        sub = run_sublines(args, world, rank, device)
        if rank == 0:
            line.setdefault("secondary", {}).update(sub)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


# The sub-lines of the default run: (workload, timed steps). Per rank: FC_large 2048 / LSTM_large 1024 samples per step
# (weak scaling; at world > 1 the backward's bucket slices are all-reduced while it runs, TrainStep overlap_ranges),
# sampling's 1024 conditions and re-simulation's 1024 trajectories sharded over the ranks (strong scaling).
SUBLINES = (("fc_large", 8), ("lstm_large", 8), ("sample", 30), ("resimulate", 5))
OVERLAP_RANGES = 4


def run_sublines(args, world, rank, device, dry=False):
    """Every SUBLINES workload on every rank of the world (the collectives of each -- barriers, the max-over-ranks
    clock, the gradient / draw exchange -- need all of them); returns rank 0's {workload: JSON object}. dry=True
    (--launch-check, no GPU) walks the same sequence through the timing contract with an empty step."""
    out = {}
    cpu = not args.no_cpu_baseline and world == 1
    for wl, steps in SUBLINES:
        t_sub = time.perf_counter()
        try:
            if dry:
                res = run_dry(wl, steps, world, rank, device)
            elif wl == "resimulate":
                res = run_resim(WORKLOADS[wl][1], steps, 2, world, rank, device, cpu=cpu, spinup_ms=args.spinup_ms)
            elif wl == "sample":
                # 10 warm-up draws (~20 ms): the first launches after the FC_large / LSTM_large sub-lines
                # run while the clocks settle (k_inverse_mfma 1.81 -> 1.57 ms over 13 launches, r03i trace)
                res = run_sample(WORKLOADS[wl][1], steps, 10, world, rank, device, cpu=cpu, spinup_ms=args.spinup_ms)
            else:
                res = run_wide(wl, WORKLOADS[wl][1], steps, 3, world, rank, device, graph=not args.no_graph,
                               kernel_iters=3, cpu=cpu, cpu_batch=256 if wl == "fc_large" else 128, cpu_steps=2,
                               overlap_ranges=(args.overlap_ranges if args.overlap_ranges is not None
                                               else OVERLAP_RANGES) if world > 1 else 0, spinup_ms=args.spinup_ms)
        except Exception as e:           # a sub-line never takes the headline down with it
            res = {"error": f"{type(e).__name__}: {e}"}
        if rank == 0:
            res = res if res is not None else {"error": "rank 0 returned no line"}
            res["bench_wall_s"] = round(time.perf_counter() - t_sub, 1)
            out[wl] = res
        if not dry:
            torch.cuda.empty_cache()
    return out


def run_dry(workload, steps, world, rank, device):
    """--launch-check: one sub-line's distributed plumbing without a GPU -- the barrier-bracketed timed region, the
    max-over-ranks clock and ranks_seen -- so a CPU test can see that every sub-line runs on every rank."""
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], device=device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    seen = ranks_seen(world, device)
    if rank != 0:
        return None
    return {"metric": workload, "dry": True, "n_gpus": world, "steps": steps, "ranks_seen": seen}


def _pmc_traffic(kernel):
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(pmc):
        return None
    with open(pmc) as f:
        return json.load(f).get(kernel)


def fc_small_rooflines(kern, B):
    """Per-kernel roofline entries of the two single-launch FC_small kernels: achieved = the kernel's ALGORITHMIC
    FLOPs per launch (reference count) / its HIP-event duration; algorithmic_bytes = SURVEY §8d's per-block
    minimum x B; traffic = PMC FETCH (x2, gfx950) + WRITE bytes per launch of the same build (profiles/pmc_traffic.json,
    tools/profile_round.sh), traffic_ratio = traffic / algorithmic_bytes (> 1: bytes beyond the per-block minimum)."""
    raw = "k_pack_fold" not in kern            # the pack-free forward: no pack launch, the feature Linear inside
    spec = {"k_forward": (FWD_FLOP_PER_SAMPLE + (FEAT_FLOP_PER_SAMPLE if raw else 0), FWD_ALG_BYTES_PER_SAMPLE,
                          "whole-stack forward: ActNorm, nested MLP (DPP-rotation VALU), coupling, log-det, mix; "
                          "condition projection on fp32 MFMA helper waves; saves the activation records" +
                          ("; pack-free (bcnf_fold_train_forward): records gathered from the parameters, the feature "
                           "Linear h = x Wf^T + bf on the compute waves' matrix cores (its FLOPs counted)" if raw
                           else "")),
              "k_backward": (KBWD_FLOP_PER_SAMPLE, BWD_ALG_BYTES_PER_SAMPLE,
                             "whole-stack backward from the saved records: dX chain (DPP VALU) + dW tiles (fp32 "
                             "MFMA); the W1 condition-column gradients run in the tail (excluded from its FLOPs)")}
    out = {}
    for k, (fps, bps, what) in spec.items():
        us = kern.get(k, float("nan"))
        flop, alg = fps * B, bps * B
        achieved = flop / (us * 1e-6) / 1e12
        traffic = _pmc_traffic(k)
        out[k] = {"bound": "mfma", "achieved": round(achieved, 3), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                  "frac": round(achieved / PEAK_FP32_TFLOPS, 4), "traffic": traffic, "avg_us": round(us, 2),
                  "flop_per_launch": flop, "algorithmic_bytes": alg,
                  "traffic_ratio": round(traffic / alg, 3) if traffic else None,
                  "hbm_achieved_GBps": round(traffic / (us * 1e3), 1) if traffic else None,
                  "hbm_frac": round(traffic / (us * 1e3) / PEAK_HBM_GBS, 4) if traffic else None,
                  "alg_hbm_frac": round(alg / (us * 1e3) / PEAK_HBM_GBS, 4),
                  **pmc_utilisation(k, us), "what": what,
                  "note": "fp32 VALU + fp32 MFMA; peak = the fp32 vector = MFMA-f32 rate (MI355X_MICROARCH.md)"}
    return out


def secondary_figures(step, args, device, n_loop=50, n_trainer=12):
    """SURVEY §8d's two side figures, measured after the headline run (not part of `value`):
    * trainer_loop_shape: the same captured step replayed one batch at a time with a host sync and a read of the
      three logged values after every step -- the shape of Trainer.train's loop (trainer.py:164-173, the three
      .item() of trainer.py:277) -- instead of run_epoch's one sync per epoch;
    * unchanged_trainer: Trainer._train_batch (trainer.py:244-277) restated statement for statement over a host
      TensorDataset + DataLoader(batch_size=B, shuffle=True, num_workers=0, pin_memory=False) -- the settings of
      configs/runs/old/trajectory_FC_small.yaml:66-69 -- with torch.optim.Adam(lr=2e-4) and clip_grad_norm_ on a
      fresh bcnf_amd model: what a user gets by swapping the import and changing nothing else."""
    from bcnf_amd import CondRealNVP_v2, inn_nll_loss
    B = args.batch
    out = {}
    for _ in range(5):
        step.step_epoch()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n_loop):
        last = step.step_epoch()
    dt = time.perf_counter() - t0
    out["trainer_loop_shape"] = {"value": round(B * n_loop / dt, 1), "unit": "samples/s",
                                 "ms_per_step": round(dt / n_loop * 1e3, 4), "steps": n_loop, "last_loss": last[0],
                                 "what": "captured step + host sync + 3 logged values read per step"}
    from torch.utils.data import DataLoader, TensorDataset
    from bcnf_amd.data import simulate
    y, traj = simulate(B * 4, seed=11)
    y = torch.from_numpy(y)
    traj = torch.from_numpy(traj)
    y = (y - y.mean(0)) / (y.std(0) + 1e-6)
    traj = (traj - traj.mean((0, 1))) / (traj.std((0, 1)) + 1e-6)
    loader = DataLoader(TensorDataset(y, traj), batch_size=B, shuffle=True, num_workers=0, pin_memory=False)
    torch.manual_seed(2024_03_25)
    model = CondRealNVP_v2.from_config(FC_SMALL).to(device)
    model.train()
    optimizer = torch.optim.Adam(model.parameters(), lr=2e-4)
    times = []

    def train_batch(yb, *conditions):           # trainer.py:244-277, hybrid_weight = 0
        optimizer.zero_grad()
        z, h = model.forward(yb.to(model.device), *[c.to(model.device) for c in conditions], log_det_J=True,
                             return_features=True)
        mse_loss = torch.tensor(0.0)
        nll_loss = inn_nll_loss(z, model.log_det_J)
        loss = (nll_loss + mse_loss * 0.0) / (1 + 0.0)
        loss.backward()
        optimizer.step()
        torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0)
        return loss.item(), nll_loss.item(), mse_loss.item()

    done = 0
    while done < 3 + n_trainer:
        t_prev = time.perf_counter()
        for data in loader:                      # the DataLoader's fetch + collate is inside the timing
            yb, *conds = data
            last = train_batch(yb, *conds)
            now = time.perf_counter()
            times.append(now - t_prev)
            t_prev = now
            done += 1
            if done >= 3 + n_trainer:
                break
    med = statistics.median(times[3:])
    out["unchanged_trainer"] = {"value": round(B / med, 1), "unit": "samples/s", "ms_per_step": round(med * 1e3, 3),
                                "steps": n_trainer, "last_loss": last[0],
                                "what": "Trainer._train_batch restated + host DataLoader (num_workers=0), torch Adam"}
    return out


def cpu_baseline_wide(workload, cfg, batch=256, steps=4):
    """CPU oracle training step of the wide workload (FC_large / LSTM_large shapes; LSTM features through the oracle's
    LSTM restatement, pool_dim = 1 as on the GPU) on this host, bounded: a few steps at a small batch."""
    from oracle import cnf_oracle as O
    threads = host_cores()
    torch.set_num_threads(threads)
    torch.manual_seed(2024_03_25)
    from bcnf_amd import CondRealNVP_v2
    m = CondRealNVP_v2.from_config(cfg)
    kw = cfg["model"]["kwargs"]
    fn = cfg["feature_networks"][1]
    fk = fn["kwargs"]
    extra = ({"lstm": (fk["input_size"], fk["hidden_size"], fk["num_layers"], fk["bidirectional"], fk["pool_dim"])}
             if fn["type"] == "LSTM" else {"feature_sizes": fk["sizes"], "feature_dropout": fk["dropout"]})
    spec = O.StackSpec(size=19, nested_sizes=kw["nested_sizes"], n_blocks=kw["n_blocks"],
                       n_conditions=kw["n_conditions"], dropout=kw["dropout"], act_norm=kw["act_norm"], **extra)
    sd = {k: v.detach().clone().requires_grad_(not k.endswith("orthonormal_matrix")) for k, v in m.state_dict().items()}
    del m
    opt = torch.optim.Adam([v for v in sd.values() if v.requires_grad], lr=2e-4)
    g = torch.Generator().manual_seed(7)
    y = torch.randn(batch, 19, generator=g)
    traj = torch.randn(batch, 30, 3, generator=g)
    times = []
    for _ in range(1 + steps):
        t0 = time.perf_counter()
        O.train_step_cpu(sd, spec, y, traj, opt, training=True)
        times.append(time.perf_counter() - t0)
    med = statistics.median(times[1:])
    return {"value": round(batch / med, 1), "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": f"oracle/cnf_oracle.train_step_cpu, {workload} B={batch}, dropout on, median of {steps} "
                      f"steps after 1 warmup, {threads} threads, {med * 1e3:.0f} ms/step"}


def wide_mfma_busy(workload):
    """Matrix-pipe busy fractions of a wide workload's kernels from the committed SQ counters of a short run of the
    same build (profiles/pmc_wide.json, tools/pmc_wide.sh + tools/pmc_wide.py): SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x
    kernel-trace duration x 2.4 GHz) for the chain GEMMs (k_wbr: ACT / GRAD) and over all library kernels, with their
    VALU-per-MFMA instruction ratio (f32 MFMA and VALU do not co-issue on a SIMD)."""
    path = os.path.join(ROOT, "profiles", "pmc_wide.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f).get(workload)
    if not d:
        return None
    return {"chain_gemms": d.get("chain"), "all_library_kernels": d.get("library_kernels_mfma_busy_frac"),
            "source": "profiles/pmc_wide.json"}


def run_wide(workload, batch, steps, warmup, world, rank, device, graph=True, kernel_iters=20, cpu=True,
             cpu_batch=256, cpu_steps=4, overlap_ranges=0, spinup_ms=150.0):
    """NLL-training samples/s of a wide workload (trajectory_FC_large = configs[2], trajectory_LSTM_large =
    configs[3]) per GPU, same step definition and timing contract as main(). Returns rank 0's JSON object."""
    from bcnf_amd import CondRealNVP_v2
    from bcnf_amd.data import DeviceBatches
    from bcnf_amd.train import TrainStep
    cfg = WORKLOADS[workload][0]
    torch.manual_seed(2024_03_25)
    model = CondRealNVP_v2.from_config(cfg).to(device)
    model.train()
    model.fused.set_seed(2024_03_25 + 7919 * rank)
    data = DeviceBatches(max(16384, 4 * batch), batch, device, seed=2024_03_25 + rank)
    # world > 1: the backward in `overlap_ranges` block ranges, each range's gradient slice all-reduced while the
    # rest runs (eager steps: the collectives sit between kernel launches)
    step = TrainStep(model, lr=2e-4, capture=graph, overlap_ranges=overlap_ranges)
    step.broadcast_parameters()
    step.set_pool(data.y, data.traj)
    batches = [data.next_indices() for _ in range(warmup + steps)]
    step.set_epoch(torch.cat(batches), batch)

    class _A:                           # kernel_timing's argument shape
        pass
    ka = _A()
    ka.kernel_iters = 2
    step.prepare_epoch(max(steps, warmup))      # captures first, then spin-up and warmup without an idle gap
    spun = spinup(lambda: kernel_timing(model, data, ka), spinup_ms)
    step.run_epoch(warmup)
    step.prepare_epoch(steps)          # no graph capture inside the timed region
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    vals = step.run_epoch(steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], device=device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    value = world * batch * steps / dt
    seen = ranks_seen(world, device)
    if rank != 0:
        return None
    ka.kernel_iters = kernel_iters
    kern = kernel_timing(model, data, ka)
    B = batch
    flop_step = WIDE_TRAIN_FLOP_PER_SAMPLE * B
    achieved = flop_step / (dt / steps) / 1e12
    fb_us = kern.get("forward", float("nan")) + kern.get("backward", float("nan"))
    ach_fb = flop_step / (fb_us * 1e-6) / 1e12
    alg = WIDE_ALG_BYTES_PER_SAMPLE * B
    flop_exec = wide_executed_flop(workload, B)
    kw = cfg["model"]["kwargs"]
    line = {
        "metric": f"NLL-training samples/sec, {WIDE_NAMES[workload]}",
        "value": round(value, 1), "unit": "samples/s", "n_gpus": world, "steps": steps,
        "warmup": warmup, "device_spinup_ms": spun, "ms_per_step": round(dt / steps * 1e3, 4), "ranks_seen": seen,
        **({"shared_devices": True} if SHARED_DEVICES else {}),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic ballistic trajectories (bcnf_amd/data.py), device-resident",
        "config": {"workload": f"{WIDE_NAMES[workload]} NLL training step", "batch_per_gpu": B,
                   "global_batch": B * world, "parallelism": f"dp{world}", "hip_graph": step.capture,
                   "overlap_ranges": step.overlap_ranges,
                   "n_blocks": kw["n_blocks"], "nested_sizes": kw["nested_sizes"],
                   "n_conditions": kw["n_conditions"], "dropout": kw["dropout"]},
        "last_loss": vals[-1][0] if vals else None,
        "roofline": {"bound": "mfma", "kernel": "coupling stack forward + backward launches (fp32 MFMA GEMM chain + "
                                                "link kernels; HIP events over each launch sequence)",
                     "frac_executed": round(flop_exec / (fb_us * 1e-6) / 1e12 / PEAK_FP32_TFLOPS, 4),
                     "flop_executed_per_step": flop_exec,
                     "achieved": round(ach_fb, 3), "achieved_whole_step": round(achieved, 3),
                     "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s", "frac": round(ach_fb / PEAK_FP32_TFLOPS, 4),
                     "frac_whole_step": round(achieved / PEAK_FP32_TFLOPS, 4), "traffic": None,
                     "avg_us": round(fb_us, 2), "flop_per_step": flop_step, "algorithmic_bytes": alg,
                     "alg_hbm_frac": round(alg / (fb_us * 1e3) / PEAK_HBM_GBS, 4),
                     "note": "frac_executed = the FLOPs the folded step executes (bench.py wide_executed_flop, "
                             "DESIGN §3d) / launch time / peak: the figure to read against mfma_busy; achieved / frac "
                             "= SURVEY §8d reference count (3 x forward flow with 1360-wide condition GEMMs, feature "
                             "net excluded), which the fold does not execute"},
        "kernels_us": {k: round(v, 2) for k, v in kern.items()},
    }
    mb = wide_mfma_busy(workload)
    if mb:
        line["roofline"]["mfma_busy"] = mb
    del step, model, data
    torch.cuda.empty_cache()
    try:
        line["parity"] = wide_fixture_error(workload, device)
    except Exception as e:                   # parity evidence never takes the throughput line down
        line["parity"] = {"error": f"{type(e).__name__}: {e}"}
    torch.cuda.empty_cache()
    if cpu and world == 1:
        line["cpu_baseline"] = cpu_baseline_wide(workload, cfg, batch=cpu_batch, steps=cpu_steps)
    return line


def main_wide(args):
    world, rank, local = init_dist(args)
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    ov = args.overlap_ranges if args.overlap_ranges is not None else (OVERLAP_RANGES if world > 1 else 0)
    line = run_wide(args.workload, args.batch, args.steps, args.warmup, world, rank, device, graph=not args.no_graph,
                    kernel_iters=args.kernel_iters, cpu=not args.no_cpu_baseline, overlap_ranges=ov,
                    spinup_ms=args.spinup_ms)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def run_sample(n_cond, steps, warmup, world, rank, device, n_draws=500, cpu=True, cpu_conds=1024, spinup_ms=150.0):
    """Posterior draws/s (BASELINE configs[4]): 500 draws for each of `n_cond` conditions with trajectory_FC_small,
    the conditions sharded over the ranks (strong scaling of a fixed job; bcnf_amd/sampling.py), gathered at the end.
    One step = draw_sharded(500, all conditions) incl. feature net, device z draw, inverse, all-gather."""
    from bcnf_amd import CondRealNVP_v2
    from bcnf_amd.data import simulate
    from bcnf_amd.sampling import draw_sharded, shard_range
    torch.manual_seed(2024_03_25)
    model = CondRealNVP_v2.from_config(FC_SMALL).to(device).eval()
    _, traj = simulate(n_cond, seed=2024_03_25)
    traj = torch.from_numpy(traj)
    traj = ((traj - traj.mean((0, 1))) / (traj.std((0, 1)) + 1e-6)).to(device)
    gen = torch.Generator(device=device).manual_seed(17 + rank)
    with model.fused.reuse_pack():
        # this rank's shard only (gather=False): the spin-up is time-bounded, so ranks run different counts of it,
        # and a collective inside would pair up across ranks wrongly
        spun = spinup(lambda: draw_sharded(model, n_draws, traj, generator=gen, gather=False), spinup_ms)
        for _ in range(warmup):
            draw_sharded(model, n_draws, traj, generator=gen)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            out = draw_sharded(model, n_draws, traj, generator=gen)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        if world > 1:
            tt = torch.tensor([dt], device=device)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            dt = float(tt.item())
        # dominant kernel: the inverse of this rank's n_draws x N_local rows, HIP events on the launch stream
        a, b = shard_range(n_cond, rank, world)
        with torch.no_grad():
            h = model.feature_network_stack(traj[a:b]).contiguous()
            rows = n_draws * (b - a)
            z = torch.randn(rows, 19, device=device, generator=gen)
            idx = torch.arange(rows, device=device) % (b - a)
            model._inverse_indexed(z, h, idx)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                model._inverse_indexed(z, h, idx)
            e1.record()
            torch.cuda.synchronize()
            inv_us = e0.elapsed_time(e1) * 1e3 / 5
    value = n_draws * n_cond * steps / dt
    seen = ranks_seen(world, device)
    if rank != 0:
        return None
    flop = FWD_FLOP_PER_SAMPLE * rows
    achieved = flop / (inv_us * 1e-6) / 1e12
    # the reference repeats each condition per draw, so its per-row MLP includes the condition projection
    # (nb x 16 x C MACs); here k_hp computes it once per condition and k_inverse_mfma runs the rest
    proj_macs = 32 * 16 * 80
    flop_exec = 2 * ((FWD_FLOP_PER_SAMPLE // 2 - proj_macs) * rows + proj_macs * (b - a))
    # per-block minimum of the eval inverse (z in, y out per block, projection read per row; SURVEY §8d forward form)
    alg = FWD_ALG_BYTES_PER_SAMPLE * rows
    line = {
        "metric": "posterior draws/sec (inverse sampling, 500 draws x 1024 conditions), trajectory_FC_small",
        "value": round(value, 1), "unit": "draws/s", "n_gpus": world, "steps": steps, "warmup": warmup,
        "device_spinup_ms": spun,
        "ms_per_step": round(dt / steps * 1e3, 4), "ranks_seen": seen, "higher_is_better": True,
        **({"shared_devices": True} if SHARED_DEVICES else {}),
        "scaling": "strong",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic ballistic trajectories as conditions, device z",
        "config": {"workload": "CondRealNVP_v2.sample-equivalent draw (configs[4])", "conditions": n_cond,
                   "draws_per_condition": n_draws, "parallelism": f"condition shards x{world}",
                   "output": tuple(out.shape)},
        "roofline": {"bound": "mfma", "kernel": "k_inverse_mfma (this rank's rows)", "achieved": round(achieved, 3),
                     "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s", "frac": round(achieved / PEAK_FP32_TFLOPS, 4),
                     "traffic": _pmc_traffic("k_inverse_mfma"), "avg_us": round(inv_us, 2), "flop_per_launch": flop,
                     "flop_executed_per_launch": flop_exec, "algorithmic_bytes": alg,
                     "alg_hbm_frac": round(alg / (inv_us * 1e3) / PEAK_HBM_GBS, 4),
                     "frac_executed": round(flop_exec / (inv_us * 1e-6) / 1e12 / PEAK_FP32_TFLOPS, 4),
                     **pmc_utilisation("k_inverse_mfma", inv_us),
                     "note": "flop_per_launch counts the reference's per-row work (condition projection "
                             "repeated per draw); flop_executed: projection once per condition (k_hp) + "
                             "k_inverse_mfma (fp32 MFMA dense layers, VALU GELU / tanh / coupling)"},
    }
    if cpu and world == 1:
        # the oracle as the checker, outside the timed region (world 1, with the cpu_baseline leg): 8 conditions'
        # rows of the full 500 x 1024 launch vs the oracle's tiled inverse on the same z
        line["parity"] = sample_parity(model, traj, n_draws)
    del model
    torch.cuda.empty_cache()
    if cpu and world == 1:
        line["cpu_baseline"] = cpu_baseline_sample(n_draws, cpu_conds)
    return line


def sample_parity(model, traj, n_draws, n_check=8):
    """Max error of the configs[4] launch shape against the oracle: z for all n_draws x N rows, ONE draw over all N
    conditions (the benchmarked launch), then n_check conditions spread over [0, N) checked against the CPU oracle's
    inverse of the tiled features (cnf.py:577-582) on the same z rows, at the north star's 1e-5 gate."""
    from oracle import cnf_oracle as O
    from bcnf_amd.sampling import draw
    n = traj.shape[0]
    g = torch.Generator(device=traj.device).manual_seed(31)
    z = torch.randn(n_draws * n, 19, device=traj.device, generator=g)
    with torch.no_grad():
        got = draw(model, n_draws, traj, z=z)
    cols = torch.linspace(0, n - 1, n_check).round().long()
    got = got[:, cols.to(got.device)].cpu()
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    with torch.no_grad():
        h = O.feature_forward(sd, O.FC_SMALL_SPEC, traj[cols.to(traj.device)].cpu())
        zs = z.view(n_draws, n, 19)[:, cols.to(z.device)].reshape(-1, 19).cpu()
        ref = O.model_inverse(sd, O.FC_SMALL_SPEC, zs, h.repeat(n_draws, 1)).view(n_draws, n_check, 19)
    err = (got.double() - ref.double()).abs()
    tol = 1e-5 * ref.double().abs() + 1e-5 * max(1.0, ref.abs().max().item())
    return {"checker": "oracle/cnf_oracle.model_inverse (tiled features)", "conditions": cols.tolist(),
            "rows": n_draws * n_check, "of_launch": [n_draws, n], "max_abs_err": float(err.max()),
            "max_abs_ref": float(ref.abs().max()),
            "tol_ratio": float((err / tol).max()), "within_1e-5_gate": bool((err <= tol).all()),
            "gate": "|got - ref| <= 1e-5 |ref| + 1e-5 max(1, max |ref|) per element; tol_ratio = max of the quotient"}


def main_sample(args, n_draws=500):
    world, rank, local = init_dist(args)
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    line = run_sample(args.batch, args.steps, args.warmup, world, rank, device, n_draws=n_draws,
                      cpu=not args.no_cpu_baseline, spinup_ms=args.spinup_ms)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def cpu_baseline_sample(n_draws=500, n_cond=1024):
    """The oracle's sample(outer=True, batch_size=100) (CPU restatement of cnf.py:510-588) on the host, bounded."""
    from oracle import cnf_oracle as O
    threads = host_cores()
    torch.set_num_threads(threads)
    torch.manual_seed(2024_03_25)
    from bcnf_amd import CondRealNVP_v2
    m = CondRealNVP_v2.from_config(FC_SMALL)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    cond = torch.randn(n_cond, 30, 3, generator=torch.Generator().manual_seed(3))
    O.sample(sd, O.FC_SMALL_SPEC, 10, cond[:16], outer=True, batch_size=100)
    t0 = time.perf_counter()
    O.sample(sd, O.FC_SMALL_SPEC, n_draws, cond, outer=True, batch_size=100)
    dt = time.perf_counter() - t0
    return {"value": round(n_draws * n_cond / dt, 1), "unit": "draws/s", "cores": threads, "kind": "port",
            "sample": f"oracle.sample(outer=True, batch_size=100), {n_draws} draws x {n_cond} conditions, "
                      f"{threads} threads, {dt:.2f} s"}


def resim_draws(n_traj, n_draws, seed=2024_03_25):
    """(M, N, 19) float32 'posterior draws' of the FC_small parameters for N synthetic trajectories (bcnf_amd/data.py
    priors), each parameter jittered by 5% per draw, + the data_dict with the parameters the model does not predict."""
    from bcnf_amd.data import simulate
    y, _ = simulate(n_traj, seed=seed, T=0.1, dt=0.067)
    rng = np.random.Generator(np.random.PCG64(seed + 1))
    yh = y[None] * (1 + 0.05 * rng.standard_normal((n_draws, n_traj, y.shape[1]))).astype(np.float32)
    zeros = [0.0] * n_traj
    data_dict = {"g_x": zeros, "g_y": zeros, "g_z": list(y[:, 6].astype(np.float64))}
    return yh.astype(np.float32), data_dict


def run_resim(n_traj, steps, warmup, world, rank, device, n_draws=1000, cpu=True, T=2.0, dt=1 / 15, spinup_ms=150.0):
    """Re-simulated trajectories/s (resimulate with y_hat given, resimulation.py:21-59; notebooks/resimulation.ipynb
    sizes): n_draws x n_traj trajectories, the trajectories sharded over the ranks (independent, no collective).
    One step = bcnf_resimulate over this rank's draws, y_hat resident in HBM, (N, M, 30, 3) float64 written."""
    from bcnf_amd.resimulation import resimulate_device
    from bcnf_amd.sampling import shard_range
    from bcnf_amd.utils import ParameterIndexMapping
    yh, data_dict = resim_draws(n_traj, n_draws)
    a, b = shard_range(n_traj, rank, world)
    pim = ParameterIndexMapping(FC_SMALL["global"]["parameter_selection"])
    dd = {k: v[a:b] for k, v in data_dict.items()}
    y = torch.from_numpy(yh[:, a:b]).to(device).contiguous()
    st = torch.cuda.current_stream(device)
    spun = spinup(lambda: resimulate_device(y, T, dt, dd, pim, break_on_impact=True, device=device), spinup_ms)
    for _ in range(warmup):
        out = resimulate_device(y, T, dt, dd, pim, break_on_impact=True, device=device)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = resimulate_device(y, T, dt, dd, pim, break_on_impact=True, device=device)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([el], device=device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    # the kernel alone, HIP events on its launch stream; step attempts for the executed-work roofline. e0 is recorded
    # behind one launch already in the queue, so the host's per-call preparation (~60 us of Python + table upload)
    # overlaps a running kernel instead of leaving the GPU idle inside the window (round 3's 3-launch window started
    # on an empty queue: +20 us per launch against the kernel trace, tools/resim_context.py)
    _, att, stat = resimulate_device(y, T, dt, dd, pim, break_on_impact=True, device=device, return_status=True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n_k = 8
    resimulate_device(y, T, dt, dd, pim, break_on_impact=True, device=device)
    e0.record(st)
    for _ in range(n_k):
        resimulate_device(y, T, dt, dd, pim, break_on_impact=True, device=device)
    e1.record(st)
    torch.cuda.synchronize()
    k_us = e0.elapsed_time(e1) * 1e3 / n_k
    # the reference-compatible resimulate() also hands the (N, M, steps, 3) float64 positions to the host as numpy:
    # timed separately (same barrier / max-over-ranks contract), never part of `value`
    import types
    from bcnf_amd.resimulation import resimulate
    host_model = types.SimpleNamespace(parameter_index_mapping=pim, device=device)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(2):
        xh = resimulate(host_model, T, dt, dd, y, break_on_impact=True, verbose=False)
    if world > 1:
        dist.barrier()
    el_host = (time.perf_counter() - t0) / 2
    if world > 1:
        tt = torch.tensor([el_host], device=device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el_host = float(tt.item())
    host_bytes = xh.nbytes
    del xh
    value = n_draws * n_traj * steps / el
    seen = ranks_seen(world, device)
    if rank != 0:
        return None
    n_att = int(att.sum().item())
    n_bad = int((stat != 0).sum().item())
    flop = RESIM_FLOP_PER_ATTEMPT * n_att
    ach = flop / (k_us * 1e-6) / 1e12
    out_bytes = out.numel() * 8
    line = {
        "metric": "re-simulated trajectories/sec, device-resident (resimulate_device: y_hat in HBM, positions left "
                  "in HBM; 1000 draws x 1024 trajectories, T=2, dt=1/15, break_on_impact)",
        "value": round(value, 1), "unit": "trajectories/s", "n_gpus": world, "steps": steps, "warmup": warmup,
        "device_spinup_ms": spun,
        "ms_per_step": round(el / steps * 1e3, 4), "ranks_seen": seen, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic draws: bcnf_amd/data.py priors jittered 5% per draw, device-resident",
        "config": {"workload": "resimulate (simulation/resimulation.py:21-59), y_hat given", "trajectories": n_traj,
                   "draws": n_draws, "steps_per_trajectory": int(out.shape[2]), "parallelism": f"trajectory shards x{world}",
                   "output": list(out.shape)},
        "end_to_end": {"value": round(n_draws * n_traj / el_host, 1), "unit": "trajectories/s",
                       "ms_per_call": round(el_host * 1e3, 2), "host_bytes_per_rank": host_bytes,
                       "what": "resimulate() (the reference's signature and result): the same launch + the float64 "
                               "positions copied to a host numpy array (pageable device-to-host copy)"},
        "roofline": {"bound": "valu-fp64", "kernel": "k_resim", "achieved": round(ach, 3), "peak": PEAK_FP64_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(ach / PEAK_FP64_TFLOPS, 4), "traffic": _pmc_traffic("k_resim"),
                     "avg_us": round(k_us, 2), "flop_per_launch": flop, "attempts_per_trajectory":
                     round(n_att / (n_draws * (b - a)), 2), "not_ok_trajectories": n_bad,
                     "output_bytes": out_bytes, "hbm_floor_us": round(out_bytes / PEAK_HBM_GBS / 1e3, 2),
                     "note": "adaptive integrator: FLOPs are the executed Dormand-Prince attempts x "
                             f"{RESIM_FLOP_PER_ATTEMPT} (fp64 sqrt / division count 1 but are multi-instruction "
                             "sequences); the float64 positions written set an HBM floor (hbm_floor_us)"},
    }
    if cpu and world == 1:
        line["cpu_baseline"] = cpu_baseline_resim(yh, data_dict, pim.parameters, T, dt)
    return line


def main_resim(args):
    world, rank, local = init_dist(args)
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    line = run_resim(args.batch, args.steps, args.warmup, world, rank, device, cpu=not args.no_cpu_baseline,
                     spinup_ms=args.spinup_ms)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def cpu_baseline_resim(yh, data_dict, names, T, dt, n_traj=4):
    """The oracle (scipy odeint per (draw, trajectory), the reference's integrator) over all draws of the first
    n_traj trajectories, one process (the reference maps the same tasks over a ProcessPoolExecutor)."""
    import warnings
    from oracle import resim_oracle as RO
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        t0 = time.perf_counter()
        RO.resimulate(yh, list(names), data_dict, T, dt, True, traj=range(n_traj))
        el = time.perf_counter() - t0
    n = yh.shape[0] * n_traj
    return {"value": round(n / el, 1), "unit": "trajectories/s", "cores": 1, "kind": "port",
            "sample": f"oracle.resimulate (scipy odeint) over {yh.shape[0]} draws x {n_traj} trajectories, "
                      f"1 process, {el:.2f} s"}


if __name__ == "__main__":
    main()
