"""Worst rate error / tolerance (tests/test_forward.py's bound) of the HIP ARM over the
reference goldens and random 720p / 1080p frames -- margin check for rate-math changes.
Usage (GPU box): [CCMI_LIB=...] python tools/rate_margin.py"""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT / "cool-chic_amd", ROOT / "oracle", ROOT / "tests"):
    sys.path.insert(0, str(p))
import forward_oracle as fo  # noqa: E402
from test_forward import _hip_forward, _flat_q, _lat  # noqa: E402


def ratio(r, ref, mu, mu_ref, sc, sc_ref, q):
    f = lambda a: np.asarray(a, np.float64)
    r, ref, mu, mu_ref, sc, sc_ref, q = map(f, (r, ref, mu, mu_ref, sc, sc_ref, q))
    prop = (np.abs(mu - mu_ref) + np.abs(sc - sc_ref) * np.abs(q - mu_ref) / sc_ref) / (sc_ref * np.log(2))
    tol = 1e-4 + 2.4e-7 * np.exp2(ref) + 1.5 * prop
    return float((np.abs(r - ref) / tol).max())


dev = torch.device("cuda:0")
worst = 0.0
for path in fo.golden_files():
    z = np.load(path)
    mp = fo.ModelParams.from_npz(z)
    a, _, _ = _hip_forward([mp], [_lat(z, mp)], dev)
    v = ratio(a["rate"][0].cpu().numpy(), z["rate"], a["mu"][0].cpu().numpy(), z["mu"], a["scale"][0].cpu().numpy(),
              z["scale"], _flat_q([z[f"q{i}"] for i in range(mp.n_grids)]))
    print(path.stem, round(v, 4))
    worst = max(worst, v)
for H, W, seed in [(720, 1280, 1), (1080, 1920, 11), (37, 53, 2)]:
    mp = fo.ModelParams.random(H, W, seed=seed)
    g = torch.Generator().manual_seed(seed)
    lat = [0.5 * torch.randn(h, w, generator=g) for h, w in mp.sizes]
    ref = fo.forward(mp, lat)
    a, _, _ = _hip_forward([mp], [lat], dev)
    v = ratio(a["rate"][0].cpu().numpy(), ref["rate"].numpy(), a["mu"][0].cpu().numpy(), ref["mu"].numpy(),
              a["scale"][0].cpu().numpy(), ref["scale"].numpy(), _flat_q(ref["q"]))
    print(f"random {H}x{W}", round(v, 4))
    worst = max(worst, v)
print("WORST", round(worst, 4))
