"""Generate golden fixtures for the float forward path (path A) by running the
reference PyTorch implementation (imported from /root/reference, build container
only) on seeded synthetic inputs.

Writes tests/golden/forward_<name>.npz with
  inputs : lat{i} (float latents before gain/quantisation), and every parameter of
           the reference CoolChicEncoder (``p/<state_dict key>``), arch strings;
  outputs: q{i} (quantised latents), mu, scale, log_scale, rate (flat, [N]),
           ups ([L,H,W] upsampling output), syn ([3,H,W] raw synthesis output),
           dec ([3,H,W] FrameEncoder eval output after 8-bit rounding + clamp, 444),
           dec420_{y,u,v} (same with the 420 nearest conversion).

The reference's fvcore (FLOP counting) and wandb (logging) imports are stubbed:
both are instrumentation only and are not installed here.
"""

import sys
import types
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, "/root/reference")


def _stub_modules():
    fv = types.ModuleType("fvcore")
    fvnn = types.ModuleType("fvcore.nn")

    class _Flops:
        def __init__(self, *a, **k):
            pass

        def unsupported_ops_warnings(self, *_):
            pass

        def uncalled_modules_warnings(self, *_):
            pass

        def total(self):
            return 0

        def by_module(self):
            import collections
            return collections.defaultdict(int)

    fvnn.FlopCountAnalysis = _Flops
    fvnn.flop_count_table = lambda *a, **k: ""
    fv.nn = fvnn
    sys.modules["fvcore"] = fv
    sys.modules["fvcore.nn"] = fvnn
    sys.modules.setdefault("wandb", types.ModuleType("wandb"))


_stub_modules()

from coolchic.enc.component.coolchic import CoolChicEncoder, CoolChicEncoderParameter  # noqa: E402
from coolchic.enc.component.core.arm import _get_neighbor, _laplace_cdf  # noqa: E402
from coolchic.enc.io.format.yuv import convert_444_to_420  # noqa: E402

HOP = ["48-1-linear-relu", "3-1-linear-none", "3-3-residual-relu", "3-3-residual-none"]
MOP = ["16-1-linear-relu", "3-1-linear-none", "3-3-residual-relu", "3-3-residual-none"]

CASES = [
    # name, H, W, dim_arm, n_hidden, layers, n_grids
    ("hop_64x96", 64, 96, 16, 2, HOP, 7),
    ("hop_67x101", 67, 101, 16, 2, HOP, 7),
    ("mop_120x208", 120, 208, 16, 2, MOP, 7),
    ("arm8_33x50", 33, 50, 8, 1, ["8-1-linear-relu", "3-1-linear-none", "3-3-residual-none"], 5),
    ("arm24_48x40", 48, 40, 24, 2, ["12-1-linear-relu", "3-1-linear-none", "3-3-residual-relu"], 6),
    ("arm32_40x56", 40, 56, 32, 0, HOP, 7),
]


def build(h, w, dim_arm, n_hidden, layers, n_grids, seed):
    p = CoolChicEncoderParameter(layers_synthesis=layers, n_ft_per_res=[1] * n_grids,
                                 dim_arm=dim_arm, n_hidden_layers_arm=n_hidden)
    p.set_image_size((h, w))
    torch.manual_seed(seed)
    enc = CoolChicEncoder(p)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for name, prm in enc.named_parameters():
            if name.startswith("latent_grids"):
                prm.copy_(0.5 * torch.randn(prm.shape, generator=g))
            elif "upsampling" in name and "weight" in name:
                # perturb the bicubic / dirac init so every tap matters
                prm.add_(0.05 * torch.randn(prm.shape, generator=g))
            else:
                fan = prm[0].numel() if prm.dim() > 1 else 8
                prm.copy_(torch.randn(prm.shape, generator=g) / np.sqrt(max(fan, 1)))
    return enc.eval()


def run(enc):
    out = {}
    lat = [g.data.detach() for g in enc.latent_grids]
    with torch.no_grad():
        raw, rate, _ = enc.forward(quantizer_noise_type="none", quantizer_type="hardround")
        q = [torch.round(x * enc.encoder_gains) for x in lat]
        ctx = torch.cat([_get_neighbor(x, enc.mask_size, enc.non_zero_pixel_ctx_index) for x in q], dim=1)
        mu, scale, log_scale = enc.arm(ctx)
        flat = torch.cat([x.view(1, -1) for x in q], dim=1)
        ups = enc.upsampling(q)
        syn = enc.synthesis(ups)
        dec = torch.clamp(torch.round(raw * 255) / 255, 0.0, 1.0)
        d420 = convert_444_to_420(torch.round(raw * 255) / 255)
    assert torch.equal(syn, raw)
    p = torch.clamp_min(_laplace_cdf(flat + 0.5, mu, scale) - _laplace_cdf(flat - 0.5, mu, scale), 2 ** -16)
    assert torch.allclose(-torch.log2(p), rate)
    for i, (x, y) in enumerate(zip(lat, q)):
        out[f"lat{i}"] = x[0, 0].numpy()
        out[f"q{i}"] = y[0, 0].numpy()
    out["mu"], out["scale"], out["log_scale"] = mu[0].numpy(), scale[0].numpy(), log_scale[0].numpy()
    out["rate"] = rate[0].numpy()
    out["ups"] = ups[0].numpy()
    out["syn"] = raw[0].numpy()
    out["dec"] = dec[0].numpy()
    for k in ("y", "u", "v"):
        out[f"dec420_{k}"] = torch.clamp(d420[k], 0, 1)[0, 0].numpy()
    return out


def main():
    dst = ROOT / "tests" / "golden"
    dst.mkdir(parents=True, exist_ok=True)
    for i, (name, h, w, d, nh, layers, ng) in enumerate(CASES):
        enc = build(h, w, d, nh, layers, ng, seed=100 + i)
        res = run(enc)
        params = {f"p/{k}": v.detach().numpy() for k, v in enc.state_dict().items()
                  if not k.startswith("latent_grids")}
        meta = {"H": h, "W": w, "dim_arm": d, "n_hidden_arm": nh, "n_grids": ng,
                "layers": "|".join(layers), "encoder_gain": enc.encoder_gains}
        np.savez_compressed(dst / f"forward_{name}.npz", **res, **params,
                            meta=np.array(repr(meta)))
        print(name, {k: v.shape for k, v in list(res.items())[-6:]})


if __name__ == "__main__":
    main()
