"""GPU parity of the variant coupling layers (reference layers.py:9-78, dev configs) against the reference's own
outputs and autograd gradients (fixtures g12 / g13 made by running psaegert/bcnf, tests/golden/make_golden.py):

* layer="LinearFFTEnriched" (trajectory_LSTM_FFT_large_small_cond's coupling at a test size): the fused wide-MLP
  kernels on the folded weights W[:, :n] + W[:, n:] F (bcnf_amd/fft_stack.py);
* layer="AnyGLU" with a Sigmoid gate, two_way (trajectory_SFrExp_LSTM_SiGLU_GELU_2_large's coupling): the layerwise
  path (its Linear layers on the library's MFMA GEMMs).

Gates: values |got - ref| <= 1e-5 |ref| + 1e-5 max(1, max|ref|); gradients 1e-4 (same form)."""
import copy

import numpy as np
import pytest
import torch

from conftest import FC_SMALL_CFG, close, load_golden

pytestmark = pytest.mark.gpu
DEV = "cuda"
SEED = 2024_03_25
FFT_DEV = {"global": FC_SMALL_CFG["global"],
           "model": {"kwargs": {"size": 19, "nested_sizes": [40, 40, 40], "n_conditions": 12, "n_blocks": 3,
                                "dropout": 0.407, "act_norm": True, "layer": "LinearFFTEnriched", "activation": "GELU",
                                "random_state": SEED}},
           "feature_networks": [{"type": "ConcatenateCondition", "kwargs": {"input_size": None, "output_size": 12}}]}
GLU_DEV = {"global": FC_SMALL_CFG["global"],
           "model": {"kwargs": {"size": 19, "nested_sizes": [24, 24, 24], "n_conditions": 12, "n_blocks": 3,
                                "dropout": 0.407, "act_norm": True, "two_way": True, "layer": "AnyGLU",
                                "layer_kwargs": {"activation": "Sigmoid"}, "activation": "GELU",
                                "random_state": SEED}},
           "feature_networks": [{"type": "ConcatenateCondition", "kwargs": {"input_size": None, "output_size": 12}}]}
CASES = {"fft": (FFT_DEV, "g12_fft_enriched.npz", "FFTWideStack"), "anyglu": (GLU_DEV, "g13_anyglu.npz", "_LayerwiseStack")}


def _model(name):
    from bcnf_amd import CondRealNVP_v2
    cfg, fx, stack = CASES[name]
    d = load_golden(fx)
    m = CondRealNVP_v2.from_config(copy.deepcopy(cfg))
    assert type(m.fused).__name__ == stack
    m.load_state_dict({k[3:]: torch.from_numpy(np.ascontiguousarray(d[k])) for k in d.keys() if k.startswith("sd/")})
    return m.to(DEV).eval(), d


@pytest.mark.parametrize("name", sorted(CASES))
def test_variant_values_match_reference(name):
    m, d = _model(name)
    y, c = torch.from_numpy(d["y"]).to(DEV), torch.from_numpy(d["cond"]).to(DEV)
    with torch.no_grad():
        z = m.forward(y, c, log_det_J=True)
        ldj = m.log_det_J.clone()
        inv = m.inverse(torch.from_numpy(d["z"]).to(DEV), c)
        lp = m.log_prob(y, c)
    for key, got in (("z", z), ("ldj", ldj), ("inv", inv)):
        ok, err = close(got.cpu(), d[key])
        assert ok, (name, key, err)
    ref_lp = -(0.5 * (d["z"].astype(np.float64) ** 2).sum(1) - d["ldj"]) - 0.5 * 19 * np.log(2 * np.pi)
    ok, err = close(lp.cpu(), ref_lp)
    assert ok, (name, "log_prob", err)


@pytest.mark.parametrize("name", sorted(CASES))
def test_variant_gradients_match_reference(name):
    """Every parameter gradient of the eval NLL (for LinearFFTEnriched: the reference's widened weights, i.e. the
    effective-weight gradient mapped back through the rfft matrix) vs the reference's autograd."""
    from bcnf_amd import inn_nll_loss
    m, d = _model(name)
    y, c = torch.from_numpy(d["y"]).to(DEV), torch.from_numpy(d["cond"]).to(DEV)
    m.zero_grad(set_to_none=True)
    z = m.forward(y, c, log_det_J=True)
    loss = inn_nll_loss(z, m.log_det_J)
    loss.backward()
    assert abs(loss.item() - float(d["loss"])) <= 1e-5 * abs(float(d["loss"])) + 1e-5
    n = 0
    for k, p in m.named_parameters():
        if not p.requires_grad:                      # the frozen orthonormal matrices
            continue
        ref = d["grad/" + k]
        assert p.grad is not None, k
        ok, err = close(p.grad.cpu(), ref, rtol=1e-4, floor=1e-4)
        assert ok, (name, k, err)
        n += 1
    assert n == sum(1 for k in d.keys() if k.startswith("grad/"))


@pytest.mark.parametrize("name", sorted(CASES))
def test_variant_training_loss_paths_agree(name):
    """Training mode (dropout on): the fused / layerwise NLL (model.nll_loss, the Trainer's loss) and the
    forward + inn_nll_loss give gradients of the same size; the loss is finite and the masks change per call."""
    from bcnf_amd import inn_nll_loss
    m, d = _model(name)
    m.train()
    y, c = torch.from_numpy(d["y"]).to(DEV), torch.from_numpy(d["cond"]).to(DEV)
    vals = m.nll_loss(y, c)
    assert torch.isfinite(vals).all() and vals[0].item() == vals[1].item() and vals[2].item() == 0.0
    vals[0].backward()
    g = torch.cat([p.grad.reshape(-1) for p in m.parameters() if p.grad is not None])
    assert torch.isfinite(g).all() and g.abs().sum() > 0
    with torch.no_grad():
        z1 = m.forward(y, c)
        z2 = m.forward(y, c)
    assert not torch.equal(z1, z2)
    _ = inn_nll_loss


def test_fft_sampling_runs_on_the_wide_kernels():
    m, d = _model("fft")
    c = torch.from_numpy(d["cond"][:4]).to(DEV)
    torch.manual_seed(0)
    s = m.sample(20, c, outer=True, batch_size=4)
    assert tuple(s.shape) == (20, 4, 19) and torch.isfinite(s).all()


def test_anyglu_trainstep_matches_the_trainer_step():
    """TrainStep on an AnyGLU model (layerwise, eager: FusedAdam + the clip after the step over model.parameters())
    against the reference's Trainer._train_batch restated on a deep copy with torch.optim.Adam and
    torch.nn.utils.clip_grad_norm_ (trainer.py:244-277). Dropout off, so both runs see the same forward and the only
    difference is the optimizer's kernels: losses within 1e-6 relative, parameters within 1e-6 after 3 steps."""
    from bcnf_amd import CondRealNVP_v2, inn_nll_loss
    from bcnf_amd.train import TrainStep
    cfg = copy.deepcopy(GLU_DEV)
    cfg["model"]["kwargs"]["dropout"] = 0.0
    m = CondRealNVP_v2.from_config(cfg).to(DEV).train()
    ref = copy.deepcopy(m)
    assert type(ref.fused).__name__ == "_LayerwiseStack" and ref.fused._model is ref
    ts = TrainStep(m, lr=2e-4)
    assert ts.layerwise and not ts.capture
    opt = torch.optim.Adam(ref.parameters(), lr=2e-4)
    g = torch.Generator().manual_seed(5)
    for _ in range(3):
        y = torch.randn(64, 19, generator=g).to(DEV)
        c = torch.randn(64, 12, generator=g).to(DEV)
        loss, nll, mse = ts.step(y, c)
        opt.zero_grad()
        z = ref(y, c, log_det_J=True)
        rl = inn_nll_loss(z, ref.log_det_J)
        rl.backward()
        opt.step()
        torch.nn.utils.clip_grad_norm_(ref.parameters(), max_norm=1.0)
        assert abs(loss - rl.item()) <= 1e-6 * abs(rl.item()) + 1e-6 and nll == loss and mse == 0.0
    for (k, p), q in zip(m.named_parameters(), ref.parameters()):
        ok, err = close(p.detach().cpu(), q.detach().cpu().numpy(), rtol=1e-6, floor=1e-6)
        assert ok, (k, err)
