"""CPU restatement (torch fp32 + autograd) of Cool-chic's encoder overfit step.

TEST INFRASTRUCTURE ONLY: the parity checker for the GPU training kernels of libccmi
(cool-chic_amd/csrc/train_*.hip).  Only tests/ and bench.py's cpu_baseline leg may
import it.  Pinned against tests/golden/train_*.npz (tools/gen_golden_train.py runs the
reference modules here).

One step (enc/training/train.py:238-262):
  quantize (quantizer.py:16-232) -> CoolChicEncoder.forward in train mode
  (coolchic.py:291-479) -> FrameEncoder train-mode post-processing (frame.py:175-183:
  no rounding, 420 nearest, clamp) -> loss_function (loss.py) -> backward ->
  clip_grad_norm_(0.1) -> Adam (torch.optim.Adam defaults).
"""

from __future__ import annotations

import math

import torch
import torch.nn.functional as F

import forward_oracle as fo


def softround(x, t):
    """quantizer.py:16-41."""
    fx = torch.floor(x)
    d = x - fx - 0.5
    return fx + 0.5 * torch.tanh(d / t) / math.tanh(1.0 / (2.0 * t)) + 0.5


def kumaraswamy(u, a):
    """generate_kumaraswamy_noise (quantizer.py:60-102)."""
    b = (2 ** a * (a - 1) + 1) / a
    return (1 - (1 - u) ** (1 / b)) ** (1 / a) - 0.5


def quantize(x, qtype: str, t: float, noise=None):
    """quantize (quantizer.py:121-232); `noise` is the already-shaped additive noise."""
    n = 0.0 if noise is None else noise
    if qtype == "none":
        return x + n
    if qtype == "softround_alone":
        return softround(x, t)
    if qtype == "softround":
        return softround(softround(x, t) + n, t)
    if qtype == "ste":
        y = softround(x, t)
        return y - y.detach() + torch.round(x)
    if qtype == "true_ste":
        return x - x.detach() + torch.round(x)
    if qtype == "hardround":
        return torch.round(x)
    raise ValueError(qtype)


class TrainState:
    """Trainable tensors of one frame, in the reference's parameter order."""

    def __init__(self, mp: fo.ModelParams, latents):
        self.mp = mp
        self.lat = [x.clone().float().requires_grad_(True) for x in latents]
        self.arm = [(W.clone().requires_grad_(True), b.clone().requires_grad_(True)) for W, b in mp.arm]
        self.ups = [h.clone().requires_grad_(True) for h in mp.ups_half]
        self.pre = [h.clone().requires_grad_(True) for h in mp.pre_half]
        self.syn = [(W.clone().requires_grad_(True), b.clone().requires_grad_(True)) for W, b in mp.syn]

    def params(self):
        out = list(self.lat)
        for W, b in self.arm:
            out += [W, b]
        out += list(self.ups) + list(self.pre)
        for W, b in self.syn:
            out += [W, b]
        return out


def loss(st: TrainState, target, qtype, t, lmbda, yuv420, noise=None, keep=None):
    """Training forward + loss.  target: [3,H,W] (444) or dict(y, u, v).  Returns
    (loss, mse, rate_bit_sum).  keep (a dict, tests only): receives the ARM outputs mu and
    log_scale with their gradients retained, so a test can see the per-latent terms a
    bias gradient sums."""
    mp = st.mp
    flat = torch.cat([x.reshape(-1) for x in st.lat]) * mp.gain
    q = quantize(flat, qtype, t, noise)
    grids, o = [], 0
    for h, w in mp.sizes:
        grids.append(q[o:o + h * w].view(h, w))
        o += h * w
    ctx = torch.cat([fo.context(x, mp.dim_arm) for x in grids], dim=0)
    mu, scale, log_scale = fo.arm_mlp(ctx, st.arm)
    if keep is not None:
        mu.retain_grad()
        log_scale.retain_grad()
        keep.update(mu=mu, log_scale=log_scale)
    r = fo.rate(q, mu, scale)
    ups = fo.upsampling(grids, [fo.sym_kernel(h, mp.ups_k) for h in st.ups],
                        [fo.sym_kernel(h, mp.pre_k) for h in st.pre])
    raw = fo.synthesis(ups, mp.layers, st.syn)
    if yuv420:
        uv = F.interpolate(raw[None, 1:3], scale_factor=(0.5, 0.5), mode="nearest")[0]
        parts = [(raw[0].clamp(0, 1), target["y"]), (uv[0].clamp(0, 1), target["u"]),
                 (uv[1].clamp(0, 1), target["v"])]
        tot = sum(a.numel() for a, _ in parts)
        mse = sum(((a - b) ** 2).sum() for a, b in parts) / tot
    else:
        mse = ((raw.clamp(0, 1) - target) ** 2).mean()
    npx = mp.H * mp.W
    L = mse + lmbda * r.sum() / npx
    return L, mse, r.sum()


def grads(st: TrainState, *a, **k):
    for p in st.params():
        p.grad = None
    L, mse, r = loss(st, *a, **k)
    L.backward()
    return float(L.detach()), float(mse.detach()), float(r.detach())


class Adam:
    """torch.optim.Adam defaults (betas 0.9 / 0.999, eps 1e-8), restated."""

    def __init__(self, params, lr):
        self.p, self.lr, self.t = list(params), lr, 0
        self.m = [torch.zeros_like(x) for x in self.p]
        self.v = [torch.zeros_like(x) for x in self.p]

    @torch.no_grad()
    def step(self, clip=0.1):
        gs = [x.grad for x in self.p]
        norm = torch.sqrt(sum((g.double() ** 2).sum() for g in gs)).float()
        coef = torch.clamp(clip / (norm + 1e-6), max=1.0)
        self.t += 1
        b1, b2, eps = 0.9, 0.999, 1e-8
        bc1, bc2 = 1 - b1 ** self.t, 1 - b2 ** self.t
        for x, g, m, v in zip(self.p, gs, self.m, self.v):
            g = g * coef
            m.mul_(b1).add_(g, alpha=1 - b1)
            v.mul_(b2).addcmul_(g, g, value=1 - b2)
            denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
            x.addcdiv_(m, denom, value=-self.lr / bc1)


def from_golden(z):
    """(TrainState, target, qtype, t, lmbda, yuv420, meta) from a tests/golden/train_*.npz."""
    import ast
    meta = ast.literal_eval(str(z["meta"]))
    mp = fo.ModelParams.from_npz(z)
    lat = [torch.from_numpy(z[f"p/latent_grids.{i}.data"])[0, 0] for i in range(mp.n_grids)]
    st = TrainState(mp, lat)
    if meta["yuv420"]:
        target = {c: torch.from_numpy(z[f"t420_{c}"]) for c in "yuv"}
    else:
        target = torch.from_numpy(z["t444"])
    return st, target, meta


def golden_param_names(meta):
    """Reference parameter names in TrainState.params() order."""
    names = [f"latent_grids.{i}.data" for i in range(meta["n_grids"])]
    for i in range(meta["n_hidden_arm"] + 1):
        names += [f"arm.mlp.{2 * i}.weight", f"arm.mlp.{2 * i}.bias"]
    names += [f"upsampling.conv_transpose2ds.{i}.parametrizations.weight.original" for i in range(meta["n_grids"] - 1)]
    names += [f"upsampling.conv2ds.{i}.parametrizations.weight.original" for i in range(meta["n_grids"] - 1)]
    for i in range(len(meta["layers"].split("|"))):
        names += [f"synthesis.layers.{2 * i}.weight", f"synthesis.layers.{2 * i}.bias"]
    return names
