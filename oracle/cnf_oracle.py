"""CPU ORACLE for the CondRealNVP_v2 coupling-stack hot path — TEST INFRASTRUCTURE ONLY.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this module,
and only as the checker / CPU baseline. The product path (`bcnf_amd`) never imports it.

A functional, PyTorch-eager fp32 restatement of the reference's algorithm
(psaegert/bcnf @ /root/reference, `src/bcnf/models/cnf.py`), operating on a plain
`state_dict` (same key layout as the reference). The op order follows the reference so that fp32
results agree to rounding. Pinned against fixtures produced by running the reference itself
(`tests/golden/make_golden.py`): see `tests/test_oracle_golden.py`.

Reference anchors:
  * nested MLP            cnf.py:49-107   (Linear → GELU(erf) → Dropout …, final Linear; t, tanh(s))
  * affine coupling       cnf.py:165-213  (forward, and the (non-inverse for two_way) inverse)
  * orthonormal mix       cnf.py:312-339  (y @ Q, inverse z @ Q.T)
  * ActNorm               cnf.py:342-354  (scale*x + bias, log|scale| summed; inverse divides)
  * model forward/inverse cnf.py:467-508
  * sample/_sample        cnf.py:510-588
  * NLL                   utils.py:49-53
  * FC feature network    feature_network.py:114-145 (x.view(B,-1) → Sequential)
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch
import torch.nn.functional as F


@dataclass
class StackSpec:
    size: int
    nested_sizes: list
    n_blocks: int
    n_conditions: int
    dropout: float = 0.0
    act_norm: bool = False
    two_way: bool = False
    feature_sizes: list = field(default_factory=list)  # FullyConnected feature net sizes ([] = identity)
    feature_dropout: float = 0.0
    # LSTM feature net (feature_network.py:148-178); lstm = (input_size, hidden_size, num_layers, bidirectional,
    # pool_dim) replaces the FullyConnected one when set
    lstm: tuple | None = None

    @property
    def Da(self):
        return int(math.ceil(self.size / 2))

    @property
    def Db(self):
        return int(math.floor(self.size / 2))


def layer_kinds(spec: StackSpec):
    """Layer order of CondRealNVP_v2.__init__ (cnf.py:395-423)."""
    kinds = []
    for _ in range(spec.n_blocks - 1):
        if spec.act_norm:
            kinds.append("actnorm")
        kinds.append("coupling")
        kinds.append("ortho")
    kinds.append("coupling")
    return kinds


def mlp_linear_indices(spec: StackSpec):
    """Sequential indices of the Linear layers of a nested MLP (cnf.py:79-85: stride 3 with Dropout, else 2)."""
    stride = 3 if spec.dropout > 0.0 else 2
    n = len(spec.nested_sizes) + 1
    return [i * stride for i in range(n)]


def nested_mlp(sd, prefix, spec, y, h, training, gen=None):
    """ConditionalNestedNeuralNetwork.forward (cnf.py:98-107)."""
    if spec.n_conditions > 0:
        y = torch.cat([y, h], dim=1)                                  # cnf.py:101
    idx = mlp_linear_indices(spec)
    x = y
    for li, i in enumerate(idx):
        x = F.linear(x, sd[f"{prefix}.nn.{i}.weight"], sd[f"{prefix}.nn.{i}.bias"])
        if li < len(idx) - 1:
            x = F.gelu(x)                                             # nn.GELU(), approximate='none'
            if spec.dropout > 0.0 and training:
                if gen is None:
                    x = F.dropout(x, spec.dropout, True)
                else:
                    keep = (torch.rand(x.shape, generator=gen) >= spec.dropout).to(x.dtype)
                    x = x * keep / (1.0 - spec.dropout)
    t, s = x.chunk(2, dim=1)                                          # cnf.py:104
    return t, torch.tanh(s)                                           # cnf.py:107


def coupling_forward(sd, prefix, spec, y, h, training=False, gen=None):
    """ConditionalAffineCouplingLayer.forward (cnf.py:165-196). Returns (z, ldj)."""
    if y.dim() == 1:
        y = y.unsqueeze(0)
    if h is not None and h.dim() == 1:
        h = h.unsqueeze(0)
    ya, yb = y.chunk(2, dim=-1)
    t_a, s_a = nested_mlp(sd, prefix + ".nn_a", spec, ya, h, training, gen)
    zb = torch.exp(s_a) * yb + t_a
    if spec.two_way:
        t_b, s_b = nested_mlp(sd, prefix + ".nn_b", spec, zb, h, training, gen)
        za = torch.exp(s_b) * ya + t_b
    else:
        za = ya
    ldj = s_a.sum(dim=-1)
    if spec.two_way:
        ldj = ldj + s_b.sum(dim=-1)
    return torch.cat([za, zb], dim=-1), ldj


def coupling_inverse(sd, prefix, spec, z, h, training=False, gen=None):
    """ConditionalAffineCouplingLayer.inverse (cnf.py:198-213) — bug-compatible for two_way."""
    za, zb = z.chunk(2, dim=-1)
    t_a, s_a = nested_mlp(sd, prefix + ".nn_a", spec, za, h, training, gen)
    yb = (zb - t_a) * torch.exp(-s_a)
    if spec.two_way:
        t_b, s_b = nested_mlp(sd, prefix + ".nn_b", spec, yb, h, training, gen)
        ya = (za - t_b) * torch.exp(-s_b)
    else:
        ya = za
    return torch.cat([ya, yb], dim=-1)


def feature_forward(sd, spec, cond):
    """FeatureNetworkStack with ConcatenateCondition + FullyConnectedFeatureNetwork (feature_network.py:46-145), or
    + LSTMFeatureNetwork when spec.lstm is set."""
    if spec.lstm is not None:
        return lstm_feature_forward(sd, spec, cond)
    x = cond.reshape(cond.shape[0], -1)
    fs = spec.feature_sizes
    if len(fs) < 2:
        return x
    stride = 3 if spec.feature_dropout > 0.0 else 2
    n = len(fs) - 1
    for li in range(n):
        i = li * stride
        x = F.linear(x, sd[f"feature_network_stack.feature_networks.1.nn.{i}.weight"],
                     sd[f"feature_network_stack.feature_networks.1.nn.{i}.bias"])
        if li < n - 1:
            x = F.gelu(x)
    return x


def lstm_feature_forward(sd, spec, cond, prefix="feature_network_stack.feature_networks.1"):
    """LSTMFeatureNetwork.forward (feature_network.py:167-178): batch_first LSTM -> Linear -> mean pooling over
    `pool_dim` (the reference pools over dim 0, the batch axis; pool_dim=1 is the documented fix). The LSTM runs as
    torch.nn.LSTM with the state_dict's tensors bound functionally, so gradients reach sd's leaves. Mean pooling only
    (every shipped LSTM config)."""
    inp, hid, nl, bi, pool_dim = spec.lstm
    lstm = torch.nn.LSTM(inp, hid, num_layers=nl, bidirectional=bi, batch_first=True)
    params = {k[len(prefix) + 6:]: v for k, v in sd.items() if k.startswith(prefix + ".lstm.")}
    x, _ = torch.func.functional_call(lstm, params, (cond,))
    x = F.linear(x, sd[prefix + ".linear.weight"], sd[prefix + ".linear.bias"])
    return x.mean(dim=pool_dim)


def model_forward(sd, spec, y, h, training=False, gen=None):
    """CondRealNVP_v2.forward layer loop (cnf.py:476-488) given features h. Returns (z, ldj)."""
    ldj = torch.zeros(y.shape[0], dtype=y.dtype)
    for li, kind in enumerate(layer_kinds(spec)):
        p = f"layers.{li}"
        if kind == "actnorm":
            scale, bias = sd[p + ".scale"], sd[p + ".bias"]
            y = scale * y + bias                                      # cnf.py:349
            ldj = ldj + torch.sum(torch.log(torch.abs(scale)), dim=-1)  # cnf.py:350
        elif kind == "coupling":
            y, l = coupling_forward(sd, p, spec, y, h, training, gen)
            ldj = ldj + l
        else:
            y = y @ sd[p + ".orthonormal_matrix"]                     # cnf.py:335
            ldj = ldj + 0
    return y, ldj


def model_inverse(sd, spec, z, h, training=False, gen=None):
    """CondRealNVP_v2.inverse (cnf.py:495-508) given features h."""
    kinds = layer_kinds(spec)
    for li in reversed(range(len(kinds))):
        p = f"layers.{li}"
        kind = kinds[li]
        if kind == "actnorm":
            z = (z - sd[p + ".bias"]) / sd[p + ".scale"]              # cnf.py:353-354
        elif kind == "coupling":
            z = coupling_inverse(sd, p, spec, z, h, training, gen)
        else:
            z = z @ sd[p + ".orthonormal_matrix"].T                   # cnf.py:339
    return z


def inn_nll_loss(z, ldj, reduction="mean"):
    """utils.py:49-53."""
    if reduction == "mean":
        return torch.mean(0.5 * torch.sum(z ** 2, dim=1) - ldj)
    return 0.5 * torch.sum(z ** 2, dim=1) - ldj


def log_prob(z, ldj):
    """Build contract: log p(y|x) = -0.5|z|^2 + ldj - D/2 log(2π)."""
    D = z.shape[1]
    return -inn_nll_loss(z, ldj, reduction="none") - 0.5 * D * math.log(2.0 * math.pi)


def sample(sd, spec, n_samples, cond, sigma=1.0, outer=False, batch_size=100, sample_batch_size=None):
    """CondRealNVP_v2.sample / _sample (cnf.py:510-588), 2-D conditions, CPU generator stream."""
    if sample_batch_size is None:
        sample_batch_size = batch_size
    m_sizes = [sample_batch_size] * (n_samples // sample_batch_size) + [n_samples % sample_batch_size]
    rows = []
    with torch.no_grad():
        for b in range(0, len(cond), batch_size):
            c = cond[b:b + batch_size]
            rows.append([])
            for m in m_sizes:
                if m == 0:
                    continue
                if outer:
                    nc = c.shape[0]
                    z = sigma * torch.randn(m * nc, spec.size)          # cnf.py:578
                    rc = c.repeat(m, *([1] * (c.ndim - 1)))            # cnf.py:579
                    h = feature_forward(sd, spec, rc)
                    rows[-1].append(model_inverse(sd, spec, z, h).view(m, nc, spec.size))
                else:
                    z = sigma * torch.randn(m, spec.size)              # cnf.py:584
                    h = feature_forward(sd, spec, c)
                    rows[-1].append(model_inverse(sd, spec, z, h).view(m, spec.size))
    return torch.cat([torch.cat(r, dim=0) for r in rows], dim=1)


FC_SMALL_SPEC = StackSpec(size=19, nested_sizes=[16] * 7, n_blocks=32, n_conditions=80, dropout=0.383,
                          act_norm=True, feature_sizes=[90, 80], feature_dropout=0.244)


def train_step_cpu(sd_params, spec, y, traj, opt, training=True):
    """One Trainer._train_batch step (trainer.py:244-277) on the oracle: zero_grad, forward(log_det_J),
    NLL, backward, Adam.step, clip_grad_norm_ (after the step), .item() — the CPU baseline's unit of work."""
    opt.zero_grad()
    h = feature_forward(sd_params, spec, traj)
    z, ldj = model_forward(sd_params, spec, y, h, training=training)
    nll = inn_nll_loss(z, ldj)
    loss = nll
    loss.backward()
    opt.step()
    torch.nn.utils.clip_grad_norm_([p for p in sd_params.values() if p.requires_grad], max_norm=1.0)
    return loss.item(), nll.item(), 0.0
