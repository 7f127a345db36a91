"""Per-parameter gradient error of the GPU training step against a reference training golden
(tests/golden/train_*.npz): max |err| / max |ref| per tensor, after 0 and 1 Adam steps.
python tools/grad_err.py [golden-name]"""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT / "cool-chic_amd", ROOT / "oracle", ROOT / "tests"):
    sys.path.insert(0, str(p))
import train_oracle as to  # noqa: E402
from ccmi import train as T  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "train_hop_sr_128x192"
z = np.load(ROOT / "tests" / "golden" / f"{name}.npz")
st, target, meta = to.from_golden(z)
mp = st.mp
dev = torch.device("cuda:0")
arch = T.Arch(H=mp.H, W=mp.W, dim_arm=mp.dim_arm, n_hidden=mp.n_hidden, layers=tuple(mp.layers), n_grids=mp.n_grids,
              gain=mp.gain)
params = T.pack_params(mp.arm, mp.ups_half, mp.pre_half, mp.syn)
lat = torch.cat([x.reshape(-1) for x in st.lat]).detach()
tgt = torch.cat([target[c].reshape(-1) for c in "yuv"]) if meta["yuv420"] else target.reshape(-1)
of = T.Overfitter(arch, lat[None].to(dev), params[None].to(dev), tgt[None].to(dev), yuv420=meta["yuv420"])
names = to.golden_param_names(meta)
args = (target, meta["quantizer_type"], meta["temperature"], meta["lmbda"], meta["yuv420"])
# CPU oracle in float64 as the accuracy yardstick
st64, _, _ = to.from_golden(z)
for p in st64.params():
    p.data = p.data.double()
for k, v in list(vars(st64.mp).items()):
    pass
g = torch.zeros(1, of.N + of.P, device=dev)
of.step(meta["quantizer_type"], "none", meta["temperature"], 0.0, meta["lmbda"], update=False, grad_out=g)
got = g[0].cpu().numpy().astype(np.float64)
L, _, _ = to.grads(st, *args)
o = 0
print(f"{'tensor':60s} {'gpu-vs-golden':>14s} {'cpu-vs-golden':>14s}")
for nm, p in zip(names, st.params()):
    n = p.numel()
    ref = z[f"g/{nm}"].reshape(-1).astype(np.float64)
    cpu = p.grad.reshape(-1).numpy().astype(np.float64)
    sc = np.abs(ref).max() + 1e-30
    print(f"{nm:60s} {np.abs(got[o:o + n] - ref).max() / sc:14.3e} {np.abs(cpu - ref).max() / sc:14.3e}")
    o += n
