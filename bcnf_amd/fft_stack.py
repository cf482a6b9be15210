"""Coupling stacks whose nested-MLP layers are `LinearFFTEnriched` (reference layers.py:60-78) on the fused wide-MLP
HIP kernels.

LinearFFTEnriched(x) = W cat(x, Re rfft(x), Im rfft(x)) + b with norm="forward"; the rfft is a fixed linear map F
(2 (n//2 + 1) x n, `bcnf_amd.layers.rfft_matrix`), so the layer is a Linear with the effective weight
    W_eff = W[:, :n] + W[:, n:] F.
`FFTWideStack` keeps the reference's parameters (W of width n + 2 (n//2 + 1)) in its canonical flat buffer -- what
state_dict and optimizers see -- and before every launch folds them into an effective flat buffer in the plain
Linear layout, which the unchanged wide kernels (bcnf_wide.hip) consume. Gradients come back in the effective
layout and are mapped to the reference's parameters as dW[:, :n] = G, dW[:, n:] = G F^T, db = db. Both maps are GEMMs
on the library's MFMA Linear kernel (bcnf_linear_forward), one launch per distinct input width.
The fold reassociates the reference's sum (x and F x are contracted with W in one sum instead of two), so outputs
agree with the reference to fp32 rounding (tests/test_gpu_variants.py, fixture g12).
"""
from __future__ import annotations

import torch

from bcnf_amd import _native as N
from bcnf_amd.layers import rfft_matrix
from bcnf_amd.wide import WideStack


def _linear(x, w):
    """y = x w^T on the library's MFMA Linear kernel (x rows x k, w n x k, both contiguous fp32 on one device)."""
    rows, k = x.shape
    n = w.shape[0]
    y = torch.empty((rows, n), dtype=torch.float32, device=x.device)
    if rows and n:
        N.check(N.lib().bcnf_linear_forward(N.ptr(x), N.ptr(w), None, rows, k, n, N.ptr(y), N.stream_handle(x.device)),
                "bcnf_linear_forward")
    return y


class FFTWideStack(WideStack):
    """WideStack over LinearFFTEnriched couplings. `fft_n[i]` = the input width n of trainable[i] when it is a
    LinearFFTEnriched weight (shape out x (n + 2 (n//2 + 1))), else None."""

    def __init__(self, cfg, trainable, frozen, fft_n, bind: bool = True):
        self.fft_n = list(fft_n)
        super().__init__(cfg, trainable, frozen, bind)

    def flatten(self):
        params = self.trainable
        dev = params[0].device
        ncan = sum(p.numel() for p in params)
        canon = torch.empty(ncan, dtype=torch.float32, device=dev)
        maps, off, eoff = [], 0, 0
        with torch.no_grad():
            for p, n in zip(params, self.fft_n):
                k = p.numel()
                canon[off:off + k].copy_(p.detach().reshape(-1))
                p.data = canon[off:off + k].view(p.shape)
                ek = p.shape[0] * n if n is not None else k
                maps.append((off, tuple(p.shape), eoff, n))
                off += k
                eoff += ek
        nq = sum(q.numel() for q in self.frozen)
        qflat = torch.empty(max(nq, 1), dtype=torch.float32, device=dev)
        qo = 0
        with torch.no_grad():
            for q in self.frozen:
                k = q.numel()
                qflat[qo:qo + k].copy_(q.detach().reshape(-1))
                q.data = qflat[qo:qo + k].view(q.shape)
                qo += k
        self.canon = canon
        self.flat = torch.empty(eoff, dtype=torch.float32, device=dev)    # what the kernels read (Linear layout)
        self.qflat = qflat
        self.flat_param = torch.nn.Parameter(canon, requires_grad=True)
        self.flat_param.register_post_accumulate_grad_hook(self._on_flat_grad)
        self._offsets = [(o, int(torch.Size(s).numel())) for o, s, _, _ in maps]
        self._maps = maps
        self._F = {n: rfft_matrix(n, device=dev) for n in set(x for x in self.fft_n if x is not None)}
        self._Ft = {n: f.t().contiguous() for n, f in self._F.items()}
        self._packed = None
        self._rng_state = None

    # ------------------------------------------------------------------ canonical <-> effective
    def refresh(self):
        """canonical (reference) parameters -> effective Linear-layout buffer: W_eff = W[:, :n] + W[:, n:] F.
        The fold GEMM reads raw device pointers, so the buffers are checked first: a model still on the CPU raises
        the same RuntimeError as every other entry point instead of handing host pointers to the HIP kernel."""
        self._check_device(self.canon)
        with torch.no_grad():
            groups = {}
            for (o, shape, e, n) in self._maps:
                k = int(torch.Size(shape).numel())
                if n is None:
                    self.flat[e:e + k].copy_(self.canon[o:o + k])
                else:
                    groups.setdefault(n, []).append((o, shape, e))
            for n, items in groups.items():
                W = [self.canon[o:o + int(torch.Size(s).numel())].view(s) for o, s, _ in items]
                wf = torch.cat([w[:, n:] for w in W], dim=0).contiguous()          # all weights of width n, stacked
                eff = _linear(wf, self._Ft[n])                                     # W[:, n:] F
                r = 0
                for w, (o, s, e) in zip(W, items):
                    out = s[0]
                    self.flat[e:e + out * n].view(out, n).copy_(eff[r:r + out] + w[:, :n])
                    r += out

    def unfold_grad(self, g_eff):
        """effective-layout gradient -> gradient of the reference parameters (canonical layout)."""
        g = torch.empty_like(self.canon)
        with torch.no_grad():
            groups = {}
            for (o, shape, e, n) in self._maps:
                k = int(torch.Size(shape).numel())
                if n is None:
                    g[o:o + k].copy_(g_eff[e:e + k])
                else:
                    groups.setdefault(n, []).append((o, shape, e))
            for n, items in groups.items():
                G = [g_eff[e:e + s[0] * n].view(s[0], n) for _, s, e in items]
                gc = torch.cat(G, dim=0).contiguous()
                gf = _linear(gc, self._F[n])                                       # G F^T
                r = 0
                for Gi, (o, s, e) in zip(G, items):
                    out, width = s
                    dst = g[o:o + out * width].view(out, width)
                    dst[:, :n].copy_(Gi)
                    dst[:, n:].copy_(gf[r:r + out])
                    r += out
        return g

    # ------------------------------------------------------------------ launches (fold before, unfold after)
    def launch_forward(self, y, h, training: bool, save: bool, want_logp: bool = False):
        self._check_inputs(y, h, "forward")
        self.refresh()
        return super().launch_forward(y, h, training, save, want_logp)

    def launch_nll_forward(self, y, h, training: bool, finalize: bool = True):
        self._check_inputs(y, h, "forward")
        self.refresh()
        return super().launch_nll_forward(y, h, training, finalize)

    def launch_backward(self, h, dz, dldj, training: bool, saved, want_dy: bool, want_dh: bool):
        dy, dh, dparams = super().launch_backward(h, dz, dldj, training, saved, want_dy, want_dh)
        return dy, dh, self.unfold_grad(dparams)

    def launch_nll_backward(self, h, z, dvals, training: bool, saved, want_dy: bool, want_dh: bool, **kw):
        dy, dh, dparams = super().launch_nll_backward(h, z, dvals, training, saved, want_dy, want_dh, **kw)
        return dy, dh, self.unfold_grad(dparams)

    def launch_inverse(self, z, h, cond_index=None, training: bool = False):
        self._check_inputs(z, h, "inverse")
        if not self._pack_frozen:
            self.refresh()
        return super().launch_inverse(z, h, cond_index, training)

    def reuse_pack(self):
        self.refresh()
        return super().reuse_pack()
