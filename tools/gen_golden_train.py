"""Generate golden fixtures for the encoder overfit step (training forward + backward +
gradient clipping + Adam) by running the reference PyTorch implementation (imported
from /root/reference; build container only) on seeded synthetic inputs.

For each case, tests/golden/train_<name>.npz holds
  inputs : every parameter of the reference CoolChicEncoder (``p/<name>``, latents
           included), the target image (t444, or t420_y/u/v), meta (architecture,
           quantizer, temperature, lambda, lr);
  outputs: loss, mse, rate_bit (sum over latents) of the training forward
           (FrameEncoder train-mode post-processing + enc.training.loss.loss_function),
           ``g/<name>``: the gradient of every parameter after loss.backward(),
           ``s1/<name>`` / ``s2/<name>``: the parameters after one and two optimisation
           steps exactly as enc/training/train.py:238-262 runs them
           (clip_grad_norm_(1e-1) then torch.optim.Adam(lr)); ``g1/<name>``: the gradient
           at the step-1 parameters (before the second step's clipping).
The quantisation noise is zero (gaussian of std 0 / "none"; the reference draws it from torch's RNG, which a
GPU kernel cannot reproduce); noise paths are checked against the CPU oracle with a
shared noise tensor instead.
"""

import sys
import zlib
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent))
import gen_golden_forward as G  # noqa: E402  (stubs fvcore / wandb, imports the reference)

from coolchic.enc.io.format.yuv import convert_444_to_420, yuv_dict_clamp  # noqa: E402
from coolchic.enc.training.loss import loss_function  # noqa: E402
from torch.nn.utils import clip_grad_norm_  # noqa: E402

ROOT = G.ROOT

CASES = [
    # name, H, W, dim_arm, n_hidden, layers, n_grids, quantizer_type, temperature, lmbda, yuv420
    ("hop_sr_24x40", 24, 40, 16, 2, G.HOP, 7, "softround", 0.3, 1e-3, True),
    ("mop_ste_29x37", 29, 37, 16, 2, G.MOP, 6, "ste", 1e-4, 1e-2, True),
    ("arm8_sra_20x31", 20, 31, 8, 1, ["8-1-linear-relu", "3-1-linear-none", "3-3-residual-none"], 5,
     "softround_alone", 0.2, 4e-3, False),
    # a realistic size: every pyramid level has interior pixels, the 3x3 layers' adjoint and
    # the workgroup-level reductions see many tiles
    ("hop_sr_128x192", 128, 192, 16, 2, G.HOP, 7, "softround", 0.3, 1e-3, True),
]


def forward_loss(enc, target, qtype, temp, lmbda, yuv420):
    # "softround" needs a noise tensor (quantizer.py:206-213): gaussian noise of std 0 is exactly 0
    raw, rate, _ = enc.forward(quantizer_noise_type="gaussian" if qtype == "softround" else "none",
                               quantizer_type=qtype, soft_round_temperature=torch.tensor(temp),
                               noise_parameter=torch.tensor(0.0))
    # FrameEncoder.forward, train mode (frame.py:175-183): no rounding, 420 nearest, clamp
    if yuv420:
        dec = yuv_dict_clamp(convert_444_to_420(raw), min_val=0.0, max_val=1.0)
    else:
        dec = torch.clamp(raw, 0.0, 1.0)
    out = loss_function(dec, rate, target, lmbda=lmbda, rate_mlp_bit=0.0, compute_logs=True)
    return out, rate


def main():
    only = sys.argv[1:]  # case names to (re)generate; default: the ones without a file yet
    for name, h, w, d, nh, layers, ng, qtype, temp, lmbda, yuv420 in CASES:
        if (only and name not in only) or (not only and (ROOT / "tests" / "golden" / f"train_{name}.npz").exists()):
            continue
        enc = G.build(h, w, d, nh, layers, ng, seed=zlib.crc32(name.encode()) % 1000)
        with torch.no_grad():  # keep most of the output inside [0, 1] so the clamp passes gradients
            n_syn = len(layers)
            for i in range(n_syn):
                enc.synthesis.layers[2 * i].weight.mul_(0.5)
            enc.synthesis.layers[2 * (n_syn - 1)].bias.add_(0.5)
            for k, prm in enc.named_parameters():  # latents a few quantisation steps wide
                if k.startswith("latent_grids"):
                    prm.mul_(0.15)
        enc.train()
        g = torch.Generator().manual_seed(7)
        t444 = torch.rand(1, 3, h, w, generator=g)
        target = convert_444_to_420(t444) if yuv420 else t444
        params = [p for p in enc.parameters()]
        named = list(enc.named_parameters())
        z = {f"p/{k}": v.detach().numpy().copy() for k, v in named}
        if yuv420:
            for c in "yuv":
                z[f"t420_{c}"] = target[c][0, 0].numpy()
        else:
            z["t444"] = t444[0].numpy()
        out, rate = forward_loss(enc, target, qtype, temp, lmbda, yuv420)
        out.loss.backward()
        z["loss"] = np.float64(out.loss.item())
        z["mse"] = np.float64(out.mse)
        z["rate_bit"] = np.float64(rate.sum().item())
        with torch.no_grad():
            raw = enc.forward(quantizer_noise_type="none", quantizer_type="hardround")[0]
        print(name, "fraction of outputs inside [0, 1]:", float(((raw >= 0) & (raw <= 1)).float().mean()))
        for k, v in named:
            z[f"g/{k}"] = (v.grad if v.grad is not None else torch.zeros_like(v)).numpy().copy()
        # two optimisation steps, train.py:238-262
        lr = 1e-2
        for p in params:
            p.grad = None
        opt = torch.optim.Adam(enc.parameters(), lr=lr)
        for s in (1, 2):
            for p in params:
                p.grad = None
            out, _ = forward_loss(enc, target, qtype, temp, lmbda, yuv420)
            out.loss.backward()
            if s == 2:  # the gradient at the parameters after one step (before clipping)
                for k, v in named:
                    z[f"g1/{k}"] = (v.grad if v.grad is not None else torch.zeros_like(v)).numpy().copy()
            clip_grad_norm_(params, 1e-1, norm_type=2.0, error_if_nonfinite=False)
            opt.step()
            for k, v in named:
                z[f"s{s}/{k}"] = v.detach().numpy().copy()
        z["meta"] = repr({"H": h, "W": w, "dim_arm": d, "n_hidden_arm": nh, "layers": "|".join(layers),
                          "n_grids": ng, "encoder_gain": float(enc.encoder_gains), "quantizer_type": qtype,
                          "temperature": temp, "lmbda": lmbda, "yuv420": yuv420, "lr": lr})
        dst = ROOT / "tests" / "golden" / f"train_{name}.npz"
        np.savez_compressed(dst, **z)
        print(dst.name, "loss", z["loss"], "mse", z["mse"], "rate", z["rate_bit"])


if __name__ == "__main__":
    main()
