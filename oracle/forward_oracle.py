"""CPU restatement (torch fp32) of Cool-chic's float forward path (path A).

TEST INFRASTRUCTURE ONLY: the parity checker for the HIP kernels of libccmi
(cool-chic_amd/csrc/fwd_*.hip).  Only tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py may import it.

Pinned against tests/golden/forward_*.npz, produced by running the reference
PyTorch implementation (tools/gen_golden_forward.py, build container only).
Each function cites the reference code it restates.
"""

from __future__ import annotations

import ast
from pathlib import Path

import numpy as np
import torch
import torch.nn.functional as F

# Flattened 9x9-mask indices of the causal context pixels (arm.py:373-506).
CTX_INDEX = {
    8: [13, 22, 30, 31, 32, 37, 38, 39],
    16: [13, 14, 20, 21, 22, 23, 24, 28, 29, 30, 31, 32, 33, 37, 38, 39],
    24: [4, 11, 12, 13, 14, 15, 19, 20, 21, 22, 23, 24, 25, 28, 29, 30, 31, 32, 33, 34, 36, 37, 38, 39],
    32: [2, 3, 4, 5, 10, 11, 12, 13, 14, 15, 16, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33,
         34, 35, 36, 37, 38, 39],
}


def quantize(lat: torch.Tensor, gain: float) -> torch.Tensor:
    """quantizer.py:231-232 (eval 'hardround') applied to gain * y (coolchic.py:365-371)."""
    return torch.round(lat * gain)


def context(q: torch.Tensor, dim_arm: int) -> torch.Tensor:
    """_get_neighbor (arm.py:308-352): zero pad 4, 9x9 window, causal subset.  q [H, W] -> [H*W, d]."""
    H, W = q.shape
    qp = F.pad(q, (4, 4, 4, 4))
    cols = []
    for k in CTX_INDEX[dim_arm]:
        dy, dx = k // 9, k % 9
        cols.append(qp[dy:dy + H, dx:dx + W].reshape(-1))
    return torch.stack(cols, dim=1)


def arm_mlp(ctx: torch.Tensor, layers) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Arm.forward (arm.py:227-268) with ArmLinear (arm.py:86-101): residual hidden layers + ReLU."""
    x = ctx
    for W, b in layers[:-1]:
        x = torch.relu(F.linear(x, W, b) + x)
    W, b = layers[-1]
    out = F.linear(x, W, b)
    mu, log_scale = out[..., 0], out[..., 1]
    scale = torch.exp(torch.clamp(log_scale - 4, min=-4.6, max=5.0))
    return mu, scale, log_scale


def laplace_cdf(x, mu, scale):
    """arm.py:355-370."""
    s = x - mu
    return 0.5 - 0.5 * s.sign() * torch.expm1(-s.abs() / scale)


def rate(q, mu, scale):
    """coolchic.py:419-424."""
    p = torch.clamp_min(laplace_cdf(q + 0.5, mu, scale) - laplace_cdf(q - 0.5, mu, scale), 2 ** -16)
    return -torch.log2(p)


def sym_kernel(half: torch.Tensor, k: int) -> torch.Tensor:
    """_Parameterization_Symmetric_1d.forward (upsampling.py:46-68)."""
    return torch.cat([half, torch.flip(half, [0])[k % 2:]])


def refine(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """UpsamplingSeparableSymmetricConv2d.forward, eval (upsampling.py:205-209). x [B,1,H,W]."""
    k = w.numel()
    p = k // 2
    yw = F.conv2d(x, w.view(1, 1, 1, k), padding=(0, p))
    return F.conv2d(yw, w.view(1, 1, k, 1), padding=(p, 0)) + x


def upsample2(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """UpsamplingSeparableSymmetricConvTranspose2d.forward, eval (upsampling.py:337-353)."""
    k = w.numel()
    p0 = k // 2
    c = 2 * p0 - 1 + k // 2
    y = F.conv_transpose2d(F.pad(x, (p0, p0, 0, 0), mode="replicate"), w.view(1, 1, 1, k), stride=(1, 2))
    y = y[:, :, :, c:y.shape[-1] - c]
    y = F.conv_transpose2d(F.pad(y, (0, 0, p0, p0), mode="replicate"), w.view(1, 1, k, 1), stride=(2, 1))
    return y[:, :, c:y.shape[-2] - c, :]


def upsampling(grids, ups, pre) -> torch.Tensor:
    """Upsampling.forward (upsampling.py:476-506).  grids: list of [H_i, W_i] -> [L, H, W]."""
    rev = list(reversed(grids))
    cur = rev[0][None, None]
    for idx, tgt in enumerate(rev[1:]):
        x = upsample2(cur.transpose(0, 1), ups[idx % len(ups)]).transpose(0, 1)
        x = x[:, :, :tgt.shape[-2], :tgt.shape[-1]]
        hb = refine(tgt[None, None], pre[idx % len(pre)])
        cur = torch.cat((hb, x), dim=1)
    return cur[0]


def synthesis(x: torch.Tensor, layers, params) -> torch.Tensor:
    """Synthesis.forward (synthesis.py:264-277) with SynthesisConv2d (:69-84)."""
    y = x[None]
    for (n_out, ks, residual, relu), (W, b) in zip(layers, params):
        p = ks // 2
        z = F.conv2d(F.pad(y, (p, p, p, p), mode="replicate"), W, b)
        if residual:
            z = z + y
        y = torch.relu(z) if relu else z
    return y[0]


def post(x: torch.Tensor, bitdepth: int = 8, yuv420: bool = False):
    """FrameEncoder.forward eval post-processing (frame.py:175-183, yuv.py:275-299)."""
    m = 2 ** bitdepth - 1
    x = torch.round(x * m) / m
    if yuv420:
        uv = F.interpolate(x[None, 1:3], scale_factor=(0.5, 0.5), mode="nearest")[0]
        return {"y": x[0].clamp(0, 1), "u": uv[0].clamp(0, 1), "v": uv[1].clamp(0, 1)}
    return x.clamp(0, 1)


# ----------------------------------------------------------------------------- models


def parse_layers(desc: str):
    """'48-1-linear-relu' strings (synthesis.py:224-262) -> [(n_out, ks, residual, relu)]."""
    out = []
    for s in desc.split("|") if isinstance(desc, str) else desc:
        n, k, mode, nl = s.split("-")
        out.append((int(n), int(k), mode == "residual", nl == "relu"))
    return out


class ModelParams:
    """Float parameters of one Cool-chic frame, as the reference state_dict holds them."""

    def __init__(self, H, W, dim_arm, n_hidden, layers, n_grids, gain, arm, ups_half, pre_half, syn, ups_k=8, pre_k=7):
        self.H, self.W, self.dim_arm, self.n_hidden = H, W, dim_arm, n_hidden
        self.layers, self.n_grids, self.gain = layers, n_grids, gain
        self.arm, self.ups_half, self.pre_half, self.syn = arm, ups_half, pre_half, syn
        self.ups_k, self.pre_k = ups_k, pre_k

    @property
    def sizes(self):
        s, h, w = [], self.H, self.W
        for _ in range(self.n_grids):
            s.append((h, w))
            h, w = (h + 1) // 2, (w + 1) // 2
        return s

    def ups_full(self):
        return [sym_kernel(h, self.ups_k) for h in self.ups_half]

    def pre_full(self):
        return [sym_kernel(h, self.pre_k) for h in self.pre_half]

    @classmethod
    def from_npz(cls, z):
        meta = ast.literal_eval(str(z["meta"]))
        p = {k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("p/")}
        nh = meta["n_hidden_arm"]
        arm = [(p[f"arm.mlp.{2 * i}.weight"], p[f"arm.mlp.{2 * i}.bias"]) for i in range(nh + 1)]
        ng = meta["n_grids"]
        ups = [p[f"upsampling.conv_transpose2ds.{i}.parametrizations.weight.original"] for i in range(ng - 1)]
        pre = [p[f"upsampling.conv2ds.{i}.parametrizations.weight.original"] for i in range(ng - 1)]
        layers = parse_layers(meta["layers"])
        syn = [(p[f"synthesis.layers.{2 * i}.weight"], p[f"synthesis.layers.{2 * i}.bias"]) for i in range(len(layers))]
        return cls(meta["H"], meta["W"], meta["dim_arm"], nh, layers, ng, float(meta["encoder_gain"]), arm, ups, pre,
                   syn)

    @classmethod
    def random(cls, H, W, dim_arm=16, n_hidden=2, layers=None, n_grids=7, seed=0, gain=16.0):
        layers = layers or parse_layers("48-1-linear-relu|3-1-linear-none|3-3-residual-relu|3-3-residual-none")
        g = torch.Generator().manual_seed(seed)
        d = dim_arm
        arm = [(torch.randn(d, d, generator=g) / d, torch.randn(d, generator=g) * 0.1) for _ in range(n_hidden)]
        arm.append((torch.randn(2, d, generator=g) / d, torch.randn(2, generator=g) * 0.1))
        bic = torch.tensor([0.0351562, 0.1054687, -0.2617187, -0.8789063])
        ups = [bic + 0.02 * torch.randn(4, generator=g) for _ in range(n_grids - 1)]
        pre = [torch.tensor([0.0, 0.0, 0.0, 1.0]) * 0.1 + 0.02 * torch.randn(4, generator=g) for _ in range(n_grids - 1)]
        syn, c = [], n_grids
        for n_out, ks, _, _ in layers:
            syn.append((torch.randn(n_out, c, ks, ks, generator=g) / np.sqrt(c * ks * ks),
                        0.05 * torch.randn(n_out, generator=g)))
            c = n_out
        return cls(H, W, dim_arm, n_hidden, layers, n_grids, gain, arm, ups, pre, syn)


def forward(mp: ModelParams, latents):
    """CoolChicEncoder.forward in eval mode (coolchic.py:291-479) on float latents [H_i, W_i].
    Returns dict(q, mu, scale, log_scale, rate (flat), ups [L,H,W], syn [3,H,W])."""
    q = [quantize(x, mp.gain) for x in latents]
    ctx = torch.cat([context(x, mp.dim_arm) for x in q], dim=0)
    mu, scale, log_scale = arm_mlp(ctx, mp.arm)
    flat = torch.cat([x.reshape(-1) for x in q])
    r = rate(flat, mu, scale)
    ups = upsampling(q, mp.ups_full(), mp.pre_full())
    syn = synthesis(ups, mp.layers, mp.syn)
    return {"q": q, "mu": mu, "scale": scale, "log_scale": log_scale, "rate": r, "ups": ups, "syn": syn}


def golden_files():
    return sorted((Path(__file__).resolve().parents[1] / "tests" / "golden").glob("forward_*.npz"))
