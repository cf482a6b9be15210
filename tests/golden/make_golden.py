"""Generate golden fixtures by running the REFERENCE (psaegert/bcnf @ /root/reference) on CPU.

Test infrastructure only. Run in the build container (the reference never travels to the GPU box):

    python tests/golden/make_golden.py

The reference imports `dynaconf` at module level (`src/bcnf/utils.py:9`) but never calls it on the
hot path, so a throwaway stub package is written to a temp dir and put on sys.path ahead of the
reference. Nothing from the reference is copied: only inputs/outputs (data) are written here.

Fixtures:
  g1_fc_small.npz    FC_small model (seeded init, ActNorm perturbed), eval forward: h, z, ldj, nll
                     + G2 inverse of a random z + G4 eval-mode grads + G5 one Adam step (+ clip after)
  g3_sample.npz      sample(500, traj[:8], outer=True, batch_size=100) under torch.manual_seed
  g6_two_way.npz     two_way coupling layer (D=7) and two_way model (D=19) fwd + (buggy) inverse
  g7_large_proxy.npz FC_large-shaped proxy (C=1360, H=[526]*5, nb=2) with numpy-PCG64 weights
  g8_q.npz           OrthonormalTransformation(19, random_state=2024_03_25) Q bytes
  g9_ballistic.npz   64 physical trajectories from the reference ODE simulator + forward on them
  g_init.npz         state_dict of CondRealNVP_v2.from_config(FC_small) right after torch.manual_seed
  g10_lstm_large.npz trajectory_LSTM_large at FULL depth (nb=26, random_state=2024_03_25, biLSTM 3->140 x2 +
                     Linear 280->1360) with numpy-PCG64 weights (large_proxy_state, LSTM included): the
                     reference-faithful pool over the batch axis at B=30 (the only batch it runs at,
                     feature_network.py:174) -> h, z, ldj, inverse; the documented pool_dim=1 fix at B=48 (the
                     reference's own LSTM + Linear modules, mean over the time axis) -> h, z, ldj; Q of one block
                     + whether all 25 Q are bit-identical (random_state reseeds, cnf.py:319-320)
  g11_fc_large.npz   trajectory_FC_large at FULL depth (nb=26, FC[90,310x7,1360]) with PCG64 weights, eval, B=48:
                     h, z, ldj, inverse(z), every Q
  g12_fft_enriched.npz  layer="LinearFFTEnriched" coupling stack (dev config, test size): z, ldj, inverse, the
                     state_dict and every parameter gradient of the eval NLL (reference autograd)
  g13_anyglu.npz     layer="AnyGLU" (Sigmoid gate) two_way coupling stack (dev config, test size): the same
  g14_resim.npz      physics_ODE_simulation (physics.py:53-160) on 40 parameter sets (priors of g9 + thrust, one zero
                     wind) at (T=2, dt=1/15) with and without break_on_impact and at (T=10, dt=0.1); and
                     resimulate(...) (resimulation.py:21-59) itself, y_hat given (M=6 draws x N=5 trajectories, the
                     FC_small parameter_selection, g_x / g_y / g_z from data_dict), break_on_impact=True, 2 processes
"""
import os
import sys
import tempfile

import numpy as np
import torch

REF_SRC = "/root/reference/src"
OUT = os.path.dirname(os.path.abspath(__file__))
SEED = 2024_03_25


def _import_reference():
    stub = tempfile.mkdtemp(prefix="bcnf_stub_")
    os.makedirs(os.path.join(stub, "dynaconf"))
    with open(os.path.join(stub, "dynaconf", "__init__.py"), "w") as f:
        f.write("class Dynaconf:\n    def __init__(self, *a, **k):\n        raise RuntimeError('stub')\n")
    sys.dont_write_bytecode = True
    sys.path[:0] = [stub, REF_SRC]
    import bcnf.models.cnf as cnf  # noqa
    import bcnf.utils as utils  # noqa
    import bcnf.simulation.physics as physics  # noqa
    return cnf, utils, physics


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


def sd_to_np(sd, prefix="sd/"):
    return {prefix + k: v.detach().cpu().numpy().copy() for k, v in sd.items()}


def perturb_actnorm(model, gen):
    with torch.no_grad():
        for name, p in model.named_parameters():
            if name.endswith(".scale"):
                mag = 0.5 + torch.rand(p.shape, generator=gen)
                sign = torch.where(torch.rand(p.shape, generator=gen) < 0.2, -1.0, 1.0)
                p.copy_(mag * sign)
            elif name.endswith(".bias") and p.dim() == 1 and p.numel() == model.size and "layers." in name \
                    and name.count(".") == 2:
                p.copy_(0.3 * torch.randn(p.shape, generator=gen))


def make_g1(cnf, utils):
    torch.manual_seed(SEED)
    model = cnf.CondRealNVP_v2.from_config(FC_SMALL)
    init_sd = {k: v.clone() for k, v in model.state_dict().items()}
    np.savez_compressed(os.path.join(OUT, "g_init.npz"), **sd_to_np(init_sd))

    gen = torch.Generator().manual_seed(SEED + 1)
    perturb_actnorm(model, gen)
    sd_before = sd_to_np(model.state_dict())  # state used for forward / inverse / grads / Adam
    model.eval()
    B = 256
    y = torch.randn(B, 19, generator=gen)
    traj = 5.0 * torch.randn(B, 30, 3, generator=gen)
    z, h = model.forward(y, traj, log_det_J=True, return_features=True)
    ldj = model.log_det_J.detach().clone()
    nll = utils.inn_nll_loss(z, model.log_det_J, reduction="none")
    # G2: inverse of a random latent and of z itself
    zr = torch.randn(B, 19, generator=gen)
    with torch.no_grad():
        inv_zr = model.inverse(zr, traj)
        inv_z = model.inverse(z.detach(), traj)
    # G4: eval-mode gradients (dropout off) of the mean NLL, plus dL/dh
    model.zero_grad()
    z2, h2 = model.forward(y, traj, log_det_J=True, return_features=True)
    h2.retain_grad()
    loss = utils.inn_nll_loss(z2, model.log_det_J)
    loss.backward()
    grads = {"grad/" + n: p.grad.detach().numpy().copy() for n, p in model.named_parameters() if p.grad is not None}
    dh = h2.grad.detach().numpy().copy()
    # G5: one Adam step (lr 2e-4) then clip_grad_norm_ after the step (trainer.py:271-275)
    opt = torch.optim.Adam(model.parameters(), lr=2e-4)
    opt.step()
    total_norm = torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0)
    after = {"after/" + n: p.detach().numpy().copy() for n, p in model.named_parameters()}
    out = dict(y=y.numpy(), traj=traj.numpy(), h=h.detach().numpy(), z=z.detach().numpy(), ldj=ldj.numpy(),
               nll=nll.detach().numpy(), loss=np.float32(loss.item()), zr=zr.numpy(), inv_zr=inv_zr.numpy(),
               inv_z=inv_z.numpy(), dh=dh, clip_total_norm=np.float32(total_norm.item()))
    out.update(sd_before)
    out.update(grads)
    out.update(after)
    np.savez_compressed(os.path.join(OUT, "g1_fc_small.npz"), **out)


def make_g3(cnf):
    torch.manual_seed(SEED)
    model = cnf.CondRealNVP_v2.from_config(FC_SMALL)
    gen = torch.Generator().manual_seed(SEED + 1)
    perturb_actnorm(model, gen)
    model.eval()
    traj = 5.0 * torch.randn(8, 30, 3, generator=torch.Generator().manual_seed(SEED + 3))
    torch.manual_seed(SEED + 4)
    s = model.sample(500, traj, outer=True, batch_size=100)
    # a chunked (non-divisible) case: n=250, sample_batch_size=64, 8 conditions in batches of 3
    torch.manual_seed(SEED + 5)
    s2 = model.sample(250, traj, outer=True, batch_size=3, sample_batch_size=64)
    # the model state is g1's "sd/*" (same seeded construction + ActNorm perturbation)
    np.savez_compressed(os.path.join(OUT, "g3_sample.npz"), traj=traj.numpy(), sample=s.numpy(), sample2=s2.numpy())


def make_g6(cnf):
    torch.manual_seed(SEED + 6)
    layer = cnf.ConditionalAffineCouplingLayer(input_size=7, nested_sizes=[19] * 5, n_conditions=5, two_way=True)
    layer.eval()
    x = torch.randn(17, 7)
    c = torch.randn(17, 5)
    with torch.no_grad():
        z = layer.forward(x, c, log_det_J=True)
        ldj = layer.log_det_J.clone()
        xi = layer.inverse(z, c)
    out = dict(x=x.numpy(), c=c.numpy(), z=z.numpy(), ldj=ldj.numpy(), inv=xi.numpy())
    out.update({"layer_sd/" + k: v.numpy() for k, v in layer.state_dict().items()})
    # one-way, no dropout (Sequential index stride 2) layer at the reference test's shapes (tests/test_cnf.py:18-32)
    torch.manual_seed(SEED + 7)
    l1 = cnf.ConditionalAffineCouplingLayer(input_size=7, nested_sizes=[19] * 5, n_conditions=5)
    l1.eval()
    with torch.no_grad():
        z1 = l1.forward(x, c, log_det_J=True)
        ldj1 = l1.log_det_J.clone()
        xi1 = l1.inverse(z1, c)
    out.update(dict(z1=z1.numpy(), ldj1=ldj1.numpy(), inv1=xi1.numpy()))
    out.update({"l1_sd/" + k: v.numpy() for k, v in l1.state_dict().items()})
    # two_way full model at D=19
    cfg = {"global": FC_SMALL["global"], "feature_networks": FC_SMALL["feature_networks"],
           "model": {"kwargs": {"size": 19, "nested_sizes": [16] * 3, "n_conditions": 80, "n_blocks": 4,
                                "dropout": 0.0, "act_norm": True, "two_way": True}}}
    torch.manual_seed(SEED + 8)
    m = cnf.CondRealNVP_v2.from_config(cfg)
    m.eval()
    y = torch.randn(33, 19)
    traj = torch.randn(33, 30, 3)
    with torch.no_grad():
        zm = m.forward(y, traj, log_det_J=True)
        ldjm = m.log_det_J.clone()
        invm = m.inverse(zm, traj)
    out.update(dict(m_y=y.numpy(), m_traj=traj.numpy(), m_z=zm.numpy(), m_ldj=ldjm.numpy(), m_inv=invm.numpy()))
    out.update({"m_sd/" + k: v.numpy() for k, v in m.state_dict().items()})
    np.savez_compressed(os.path.join(OUT, "g6_two_way.npz"), **out)


def large_proxy_state(model, seed=SEED):
    """Deterministic weights for the FC_large proxy from numpy PCG64 (documented, regenerated by the tests)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    sd = {}
    for k, v in model.state_dict().items():
        if k.endswith("orthonormal_matrix"):
            sd[k] = v.numpy()
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


def make_g7(cnf):
    cfg = {"global": FC_SMALL["global"],
           "feature_networks": [{"type": "ConcatenateCondition", "kwargs": {"input_size": None, "output_size": 90}},
                                {"type": "FullyConnected", "kwargs": {"sizes": [90, 1360], "dropout": 0.0}}],
           "model": {"kwargs": {"size": 19, "nested_sizes": [526] * 5, "n_conditions": 1360, "n_blocks": 2,
                                "dropout": 0.407, "act_norm": True}}}
    torch.manual_seed(SEED + 9)
    m = cnf.CondRealNVP_v2.from_config(cfg)
    sd = large_proxy_state(m)
    m.load_state_dict({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()})
    m.eval()
    rng = np.random.Generator(np.random.PCG64(SEED + 10))
    y = rng.standard_normal((64, 19)).astype(np.float32)
    traj = rng.standard_normal((64, 30, 3)).astype(np.float32)
    with torch.no_grad():
        z = m.forward(torch.from_numpy(y), torch.from_numpy(traj), log_det_J=True)
        ldj = m.log_det_J.clone()
        inv = m.inverse(z, torch.from_numpy(traj))
    q = {("q/" + k): v.numpy() for k, v in m.state_dict().items() if k.endswith("orthonormal_matrix")}
    np.savez_compressed(os.path.join(OUT, "g7_large_proxy.npz"), y=y, traj=traj, z=z.numpy(), ldj=ldj.numpy(),
                        inv=inv.numpy(), **q)


def make_g8(cnf):
    t = cnf.OrthonormalTransformation(19, random_state=SEED)
    np.savez_compressed(os.path.join(OUT, "g8_q.npz"), q=t.orthonormal_matrix.detach().numpy())


def make_g9(cnf, utils, physics):
    rng = np.random.Generator(np.random.PCG64(SEED + 11))
    n = 64
    trajs, params = [], []
    for _ in range(n):
        r_xy, phi = abs(rng.normal(0, 20)), rng.uniform(0, 2 * np.pi)
        v_xy, vphi = abs(rng.normal(0, 15)), rng.uniform(0, 2 * np.pi)
        w_xy, wphi = abs(rng.normal(0, 3)), rng.uniform(0, 2 * np.pi)
        p = dict(x0_x=r_xy * np.cos(phi), x0_y=r_xy * np.sin(phi), x0_z=rng.uniform(0.1, 2.5),
                 v0_x=v_xy * np.cos(vphi), v0_y=v_xy * np.sin(vphi), v0_z=rng.normal(7, 5),
                 g_x=0.0, g_y=0.0, g_z=-rng.gamma(9.81, 1.0),
                 w_x=w_xy * np.cos(wphi), w_y=w_xy * np.sin(wphi), w_z=rng.normal(0, 1),
                 rho=rng.gamma(3.5, 0.35), r=rng.gamma(1.75, 0.05), Cd=rng.gamma(2.0, 0.1),
                 m=rng.gamma(2.0, 0.5) + 0.05, a_x=0.0, a_y=0.0, a_z=0.0)
        A = np.pi * p["r"] ** 2
        b = 0.5 * p["rho"] * A * p["Cd"]
        traj = physics.physics_ODE_simulation(**p, b=b, T=2.0, dt=0.067, break_on_impact=False)
        trajs.append(traj)
        params.append([p["x0_x"], p["x0_y"], p["x0_z"], p["v0_x"], p["v0_y"], p["v0_z"], p["g_z"], p["w_x"],
                       p["w_y"], p["w_z"], b, p["m"], p["a_x"], p["a_y"], p["a_z"], p["r"], A, p["Cd"], p["rho"]])
    traj = np.asarray(trajs, dtype=np.float32)
    y = np.asarray(params, dtype=np.float32)
    torch.manual_seed(SEED)
    model = cnf.CondRealNVP_v2.from_config(FC_SMALL)
    model.eval()
    with torch.no_grad():
        z = model.forward(torch.from_numpy(y), torch.from_numpy(traj), log_det_J=True)
        ldj = model.log_det_J.clone()
        inv = model.inverse(z, torch.from_numpy(traj))
    np.savez_compressed(os.path.join(OUT, "g9_ballistic.npz"), y=y, traj=traj, z=z.numpy(), ldj=ldj.numpy(),
                        inv=inv.numpy())


LSTM_LARGE = {
    "global": FC_SMALL["global"],
    "model": {"kwargs": {"size": 19, "nested_sizes": [526] * 5, "n_conditions": 1360, "n_blocks": 26,
                         "dropout": 0.407, "act_norm": True, "layer": "Linear", "activation": "GELU",
                         "random_state": 2024_03_25}},
    "feature_networks": [
        {"type": "ConcatenateCondition", "kwargs": {"input_size": None, "output_size": 3}},
        {"type": "LSTM", "kwargs": {"input_size": 3, "hidden_size": 140, "output_size": 1360, "num_layers": 2,
                                    "dropout": 0.111, "bidirectional": True, "pooling": "mean"}},
    ],
}
FC_LARGE = {
    "global": FC_SMALL["global"],
    "model": {"kwargs": {"size": 19, "nested_sizes": [526] * 5, "n_conditions": 1360, "n_blocks": 26,
                         "dropout": 0.407, "act_norm": True}},
    "feature_networks": [
        {"type": "ConcatenateCondition", "kwargs": {"input_size": None, "output_size": 90}},
        {"type": "FullyConnected", "kwargs": {"sizes": [90] + [310] * 7 + [1360], "dropout": 0.111}},
    ],
}


def _load_proxy(m, seed):
    sd = large_proxy_state(m, seed)
    m.load_state_dict({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()})
    m.eval()


def make_g10(cnf):
    """configs/runs/old/trajectory_LSTM_large.yaml at full depth."""
    torch.manual_seed(SEED + 12)
    m = cnf.CondRealNVP_v2.from_config(LSTM_LARGE)
    _load_proxy(m, SEED + 13)
    qs = [v for k, v in m.state_dict().items() if k.endswith("orthonormal_matrix")]
    same_q = all(torch.equal(q, qs[0]) for q in qs)
    rng = np.random.Generator(np.random.PCG64(SEED + 14))
    y = rng.standard_normal((30, 19)).astype(np.float32)
    traj = rng.standard_normal((30, 30, 3)).astype(np.float32)
    with torch.no_grad():
        z, h = m.forward(torch.from_numpy(y), torch.from_numpy(traj), log_det_J=True, return_features=True)
        ldj = m.log_det_J.clone()
        inv = m.inverse(z, torch.from_numpy(traj))
    # the pool_dim=1 fix (bcnf_amd LSTMFeatureNetwork(pool_dim=1)): the reference's own LSTM and Linear modules,
    # pooled over the time axis instead of the batch axis, at a batch != 30
    fn = m.feature_network_stack.feature_networks[1]

    def pooled_over_time(x):
        out, _ = fn.lstm.forward(x)
        return fn.linear.forward(out).mean(dim=1)
    fn.forward = pooled_over_time
    y1 = rng.standard_normal((48, 19)).astype(np.float32)
    traj1 = rng.standard_normal((48, 30, 3)).astype(np.float32)
    with torch.no_grad():
        z1, h1 = m.forward(torch.from_numpy(y1), torch.from_numpy(traj1), log_det_J=True, return_features=True)
        ldj1 = m.log_det_J.clone()
    np.savez_compressed(os.path.join(OUT, "g10_lstm_large.npz"), y=y, traj=traj, h=h.numpy(), z=z.numpy(),
                        ldj=ldj.numpy(), inv=inv.numpy(), q=qs[0].numpy(), n_q=np.int32(len(qs)),
                        q_all_identical=np.bool_(same_q), y1=y1, traj1=traj1, h1=h1.numpy(), z1=z1.numpy(),
                        ldj1=ldj1.numpy())


def make_g11(cnf):
    """configs/runs/old/trajectory_FC_large.yaml at full depth."""
    torch.manual_seed(SEED + 15)
    m = cnf.CondRealNVP_v2.from_config(FC_LARGE)
    _load_proxy(m, SEED + 16)
    rng = np.random.Generator(np.random.PCG64(SEED + 17))
    y = rng.standard_normal((48, 19)).astype(np.float32)
    traj = rng.standard_normal((48, 30, 3)).astype(np.float32)
    with torch.no_grad():
        z, h = m.forward(torch.from_numpy(y), torch.from_numpy(traj), log_det_J=True, return_features=True)
        ldj = m.log_det_J.clone()
        inv = m.inverse(z, torch.from_numpy(traj))
    q = {("q/" + k): v.numpy() for k, v in m.state_dict().items() if k.endswith("orthonormal_matrix")}
    np.savez_compressed(os.path.join(OUT, "g11_fc_large.npz"), y=y, traj=traj, h=h.numpy(), z=z.numpy(),
                        ldj=ldj.numpy(), inv=inv.numpy(), **q)


def _variant_fixture(cnf, utils, cfg, init_seed, weight_seed, data_seed, name):
    """A variant-layer model (configs/runs/dev/*): PCG64 weights, eval mode, B = 48 with a ConcatenateCondition-only
    feature stack: z, ldj, inverse(z) and the gradients of inn_nll_loss w.r.t. every parameter (reference autograd)."""
    torch.manual_seed(init_seed)
    m = cnf.CondRealNVP_v2.from_config(cfg)
    _load_proxy(m, weight_seed)
    C = cfg["model"]["kwargs"]["n_conditions"]
    rng = np.random.Generator(np.random.PCG64(data_seed))
    y = rng.standard_normal((48, 19)).astype(np.float32)
    cond = rng.standard_normal((48, C)).astype(np.float32)
    z = m.forward(torch.from_numpy(y), torch.from_numpy(cond), log_det_J=True)
    ldj = m.log_det_J
    loss = utils.inn_nll_loss(z, ldj)
    loss.backward()
    grads = {("grad/" + k): p.grad.numpy() for k, p in m.named_parameters() if p.grad is not None}
    with torch.no_grad():
        inv = m.inverse(z.detach(), torch.from_numpy(cond))
    np.savez_compressed(os.path.join(OUT, name), y=y, cond=cond, z=z.detach().numpy(), ldj=ldj.detach().numpy(),
                        inv=inv.numpy(), loss=np.float64(loss.item()),
                        **sd_to_np({k: v for k, v in m.state_dict().items()}), **grads)


# configs/runs/dev/trajectory_LSTM_FFT_large_small_cond.yaml's coupling (layer LinearFFTEnriched, one-way, random_state)
# at a test size; the feature stack is a bare ConcatenateCondition
FFT_DEV = {"global": FC_SMALL["global"],
           "model": {"kwargs": {"size": 19, "nested_sizes": [40, 40, 40], "n_conditions": 12, "n_blocks": 3,
                                "dropout": 0.407, "act_norm": True, "layer": "LinearFFTEnriched", "activation": "GELU",
                                "random_state": SEED}},
           "feature_networks": [{"type": "ConcatenateCondition", "kwargs": {"input_size": None, "output_size": 12}}]}
# configs/runs/dev/trajectory_SFrExp_LSTM_SiGLU_GELU_2_large.yaml's coupling (AnyGLU with a Sigmoid gate, GELU,
# two_way, random_state) at a test size
GLU_DEV = {"global": FC_SMALL["global"],
           "model": {"kwargs": {"size": 19, "nested_sizes": [24, 24, 24], "n_conditions": 12, "n_blocks": 3,
                                "dropout": 0.407, "act_norm": True, "two_way": True, "layer": "AnyGLU",
                                "layer_kwargs": {"activation": "Sigmoid"}, "activation": "GELU",
                                "random_state": SEED}},
           "feature_networks": [{"type": "ConcatenateCondition", "kwargs": {"input_size": None, "output_size": 12}}]}


def make_g12(cnf, utils):
    _variant_fixture(cnf, utils, FFT_DEV, SEED + 18, SEED + 19, SEED + 20, "g12_fft_enriched.npz")


def make_g13(cnf, utils):
    _variant_fixture(cnf, utils, GLU_DEV, SEED + 21, SEED + 22, SEED + 23, "g13_anyglu.npz")


def _physics_draw(rng):
    r_xy, phi = abs(rng.normal(0, 20)), rng.uniform(0, 2 * np.pi)
    v_xy, vphi = abs(rng.normal(0, 15)), rng.uniform(0, 2 * np.pi)
    w_xy, wphi = abs(rng.normal(0, 3)), rng.uniform(0, 2 * np.pi)
    p = dict(x0_x=r_xy * np.cos(phi), x0_y=r_xy * np.sin(phi), x0_z=rng.uniform(0.1, 2.5),
             v0_x=v_xy * np.cos(vphi), v0_y=v_xy * np.sin(vphi), v0_z=rng.normal(7, 5),
             g_x=0.0, g_y=0.0, g_z=-rng.gamma(9.81, 1.0),
             w_x=w_xy * np.cos(wphi), w_y=w_xy * np.sin(wphi), w_z=rng.normal(0, 1),
             rho=rng.gamma(3.5, 0.35), r=rng.gamma(1.75, 0.05) + 1e-3, m=rng.gamma(2.0, 0.5) + 0.05,
             a_x=rng.normal(0, 0.5), a_y=rng.normal(0, 0.5), a_z=rng.normal(0, 0.5))
    p["b"] = 0.5 * p["rho"] * np.pi * p["r"] ** 2 * rng.gamma(2.0, 0.1)
    return p


PHYS = ("x0_x", "x0_y", "x0_z", "v0_x", "v0_y", "v0_z", "g_x", "g_y", "g_z", "w_x", "w_y", "w_z", "b", "m", "rho", "r",
        "a_x", "a_y", "a_z")


def make_g14(utils, physics):
    import types
    import warnings
    from bcnf.simulation import resimulation
    rng = np.random.Generator(np.random.PCG64(SEED + 24))
    n = 40
    P = np.zeros((n, len(PHYS)))
    for k in range(n):
        p = _physics_draw(rng)
        if k == 7:                                   # zero wind: w^2 w / |w| = 0/0 (physics.py:42)
            p.update(w_x=0.0, w_y=0.0, w_z=0.0)
        if k == 11:                                  # heavy and draggy
            p.update(m=0.06, b=0.02)
        P[k] = [p[q] for q in PHYS]
    out = {"params": P}
    grids = {"a": (2.0, 1 / 15), "c": (10.0, 0.1)}
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for tag, brk in (("a", False), ("b", True), ("c", False)):
            T, dt = grids.get(tag, grids["a"])
            out["x_" + tag] = np.stack([physics.physics_ODE_simulation(**dict(zip(PHYS, P[k])), T=T, dt=dt,
                                                                       break_on_impact=brk) for k in range(n)])
        # resimulate itself, y_hat given: the FC_small parameter_selection (g_x / g_y / g_z are not predicted, 'g',
        # 'A', 'Cd' are predicted but are no physics arguments)
        names = FC_SMALL["global"]["parameter_selection"]
        M, N = 6, 5
        base = [_physics_draw(rng) for _ in range(N)]
        data_dict = {q: [b[q] for b in base] for q in PHYS}
        data_dict.update(g=[b["g_z"] for b in base], A=[np.pi * b["r"] ** 2 for b in base], Cd=[0.2] * N,
                         trajectories=[np.zeros((30, 3)) for _ in range(N)])
        y_hat = np.zeros((M, N, len(names)), dtype=np.float32)
        for j in range(M):
            for i in range(N):
                for c, q in enumerate(names):
                    v = data_dict[q][i] if q in data_dict else 0.0
                    y_hat[j, i, c] = v * (1 + 0.05 * rng.standard_normal()) if q not in ("a_x", "a_y", "a_z") else v
        model = types.SimpleNamespace(parameter_index_mapping=utils.ParameterIndexMapping(names))
        X = resimulation.resimulate(model, 2, 1 / 15, data_dict, y_hat, break_on_impact=True, n_procs=2,
                                    verbose=False)
    fixed = np.array([[data_dict[q][i] for q in PHYS] for i in range(N)])
    np.savez_compressed(os.path.join(OUT, "g14_resim.npz"), **out, y_hat=y_hat, names=np.array(names),
                        fixed_phys=fixed, g_extra=np.array(data_dict["g"]), A_extra=np.array(data_dict["A"]),
                        resim=X)


def main():
    cnf, utils, physics = _import_reference()
    if len(sys.argv) > 1:                      # e.g. `make_golden.py g10 g11`: only those fixtures
        for name in sys.argv[1:]:
            {"g10": lambda: make_g10(cnf), "g11": lambda: make_g11(cnf), "g12": lambda: make_g12(cnf, utils),
             "g13": lambda: make_g13(cnf, utils), "g14": lambda: make_g14(utils, physics)}[name]()
        return
    torch.set_num_threads(8)
    make_g1(cnf, utils)
    make_g3(cnf)
    make_g6(cnf)
    make_g7(cnf)
    make_g8(cnf)
    make_g9(cnf, utils, physics)
    make_g10(cnf)
    make_g11(cnf)
    make_g12(cnf, utils)
    make_g13(cnf, utils)
    make_g14(utils, physics)
    for f in sorted(os.listdir(OUT)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(OUT, f)))


if __name__ == "__main__":
    main()
