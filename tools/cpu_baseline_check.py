"""Is the CPU baseline honest? Times the REFERENCE's own training step -- bcnf.train.trainer.Trainer._train_batch
(/root/reference/src/bcnf/train/trainer.py:244-277), imported from /root/reference with throwaway stubs for the
modules it imports but never calls on this path (dynaconf, wandb, torchsummary) -- and the oracle's restatement
(oracle/cnf_oracle.train_step_cpu, the function bench.py's `cpu_baseline` times on the GPU box) on the same host, the
same threads, the same weights and batch, interleaved (reference, oracle, reference, ...) so that both see the same
host noise; medians over the alternations.

Test infrastructure only: runs in the build container, never on the GPU box (the reference does not
travel). Usage: python tools/cpu_baseline_check.py [--alternations 7] [--threads 8]
"""
import argparse
import os
import statistics
import sys
import tempfile
import time
import types

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
REF_SRC = "/root/reference/src"


def import_reference():
    stub = tempfile.mkdtemp(prefix="bcnf_stub_")
    for mod, body in (("dynaconf", "class Dynaconf:\n    def __init__(self, *a, **k):\n        raise RuntimeError('stub')\n"),
                      ("wandb", ""),
                      ("torchsummary", "def summary(*a, **k):\n    raise RuntimeError('stub')\n")):
        os.makedirs(os.path.join(stub, mod))
        with open(os.path.join(stub, mod, "__init__.py"), "w") as f:
            f.write(body)
    sys.dont_write_bytecode = True
    sys.path[:0] = [stub, REF_SRC]
    import bcnf.models.cnf as cnf  # noqa
    import bcnf.utils as utils  # noqa
    from bcnf.train.trainer import Trainer  # noqa
    return cnf, utils, Trainer


def run_case(name, cfg, spec_fn, batch, alternations, warmup, threads):
    from oracle import cnf_oracle as O
    cnf, utils, Trainer = import_reference()
    torch.set_num_threads(threads)
    torch.manual_seed(2024_03_25)
    ref = cnf.CondRealNVP_v2.from_config(cfg)
    ref.train()
    sd = {k: v.detach().clone().requires_grad_(not k.endswith("orthonormal_matrix")) for k, v in ref.state_dict().items()}
    opt_ref = torch.optim.Adam(ref.parameters(), lr=2e-4)
    opt_or = torch.optim.Adam([v for v in sd.values() if v.requires_grad], lr=2e-4)
    g = torch.Generator().manual_seed(7)
    y = torch.randn(batch, 19, generator=g)
    traj = torch.randn(batch, 30, 3, generator=g)
    # what Trainer._train_batch reads from `self` on this path (hybrid_weight 0: mse_loss is never called)
    trainer = types.SimpleNamespace(hybrid_weight=0, mse_loss=torch.nn.MSELoss())
    spec = spec_fn(O)

    def ref_step():
        return Trainer._train_batch(trainer, y, traj, model=ref, optimizer=opt_ref, loss_function=utils.inn_nll_loss)

    def oracle_step():
        return O.train_step_cpu(sd, spec, y, traj, opt_or, training=True)

    t_ref, t_or = [], []
    for i in range(warmup + alternations):
        for fn, acc in ((ref_step, t_ref), (oracle_step, t_or)):
            t0 = time.perf_counter()
            fn()
            dt = time.perf_counter() - t0
            if i >= warmup:
                acc.append(dt)
    mr, mo = statistics.median(t_ref), statistics.median(t_or)
    print(f"{name} B={batch} threads={threads} alternations={alternations}: reference _train_batch median "
          f"{mr * 1e3:.1f} ms ({batch / mr:.1f} samples/s), oracle train_step_cpu median {mo * 1e3:.1f} ms "
          f"({batch / mo:.1f} samples/s); oracle / reference time = {mo / mr:.3f}", flush=True)
    print(f"   reference ms: {[round(t * 1e3, 1) for t in t_ref]}", flush=True)
    print(f"   oracle ms:    {[round(t * 1e3, 1) for t in t_or]}", flush=True)
    return mo / mr


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--alternations", type=int, default=7)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    ap.add_argument("--cases", default="fc_small,fc_large")
    args = ap.parse_args()
    from bench import FC_LARGE, FC_SMALL
    cases = {
        "fc_small": (FC_SMALL, lambda O: O.FC_SMALL_SPEC, 4096),
        "fc_large": (FC_LARGE, lambda O: O.StackSpec(size=19, nested_sizes=[526] * 5, n_blocks=26, n_conditions=1360,
                                                      dropout=0.407, act_norm=True, feature_sizes=[90] + [310] * 7 + [1360],
                                                      feature_dropout=0.111), 256),
    }
    for name in args.cases.split(","):
        cfg, spec_fn, batch = cases[name]
        run_case(name, cfg, spec_fn, batch, args.alternations, args.warmup, args.threads)


if __name__ == "__main__":
    main()
