"""Per-tensor gradient error of the GPU training step against the oracle's autograd on small /
narrow frames (the shapes of tests/test_train_gpu.py::test_gpu_gradients_border_tile_shapes),
several seeds each: max |got - ref| / (the test's tolerance) per parameter tensor, and the
conditioning of the ARM output-bias gradient (sum of |per-latent dL/dmu| over |sum|).
Usage (GPU box): python tools/grad_border_diag.py"""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT / "oracle", ROOT / "cool-chic_amd"):
    sys.path.insert(0, str(p))

import forward_oracle as fo  # noqa: E402
import train_oracle as to  # noqa: E402
from ccmi import train as T  # noqa: E402


def case(H, W, seed, gpu):
    mp = fo.ModelParams.random(H, W, seed=seed)
    g = torch.Generator().manual_seed(1000 + seed)
    arch = T.Arch(H, W, dim_arm=mp.dim_arm, n_hidden=mp.n_hidden, layers=tuple(mp.layers), n_grids=mp.n_grids)
    lat = [0.05 * torch.randn(h, w, generator=g) for h, w in mp.sizes]
    img = torch.rand(3, H, W, generator=g)
    st = to.TrainState(mp, lat)
    noise = to.kumaraswamy(torch.rand(arch.n_latents, generator=g), 2.0)
    to.grads(st, img, "softround", 0.3, 1e-3, False, noise=noise)
    # per-latent dL/dmu for the conditioning of the ARM output-bias gradient
    flat = torch.cat([x.detach().reshape(-1) for x in st.lat]) * mp.gain
    q = to.quantize(flat, "softround", 0.3, noise)
    grids, o = [], 0
    for h, w in mp.sizes:
        grids.append(q[o:o + h * w].view(h, w))
        o += h * w
    ctx = torch.cat([fo.context(x, mp.dim_arm) for x in grids], 0)
    arm = [(Wt.detach(), b.detach().clone().requires_grad_(True)) for Wt, b in st.arm]
    mu, scale, _ = fo.arm_mlp(ctx, arm)
    mu.retain_grad()
    (1e-3 * fo.rate(q, mu, scale).sum() / (H * W)).backward()
    cond = float(mu.grad.abs().sum() / max(mu.grad.sum().abs(), 1e-30))
    of = T.Overfitter(arch, torch.cat([x.reshape(-1) for x in lat])[None].to(gpu),
                      T.pack_params(mp.arm, mp.ups_half, mp.pre_half, mp.syn)[None].to(gpu),
                      img.reshape(-1)[None].to(gpu))
    gout = torch.zeros(1, of.N + of.P, device=gpu)
    of.step("softround", "kumaraswamy", 0.3, 2.0, 1e-3, update=False, noise=noise[None].to(gpu), grad_out=gout)
    torch.cuda.synchronize()
    got = gout[0].cpu().numpy()
    worst, o = [], 0
    for i, p in enumerate(st.params()):
        n = p.numel()
        ref = p.grad.reshape(-1).numpy()
        tol = 2e-3 * np.abs(ref) + 1e-7 + 2e-4 * np.abs(ref).max()
        worst.append(float((np.abs(got[o:o + n] - ref) / tol).max()))
        o += n
    bad = [(i, round(w, 2)) for i, w in enumerate(worst) if w > 1]
    print(f"{H}x{W} seed {seed}: worst/tol {max(worst):.2f} bad {bad} arm-out-bias cond {cond:.0f}", flush=True)


def via_test(H, W, seed, gpu):
    """The test's own helper (tests/test_train_gpu.py::_random_arch_vs_oracle)."""
    sys.path.insert(0, str(ROOT / "tests"))
    import test_train_gpu as tt
    try:
        tt._random_arch_vs_oracle(gpu, H, W, seed)
        print(f"{H}x{W} seed {seed}: test helper passes", flush=True)
    except AssertionError as e:
        print(f"{H}x{W} seed {seed}: test helper FAILS: {str(e).splitlines()[-3:]}", flush=True)


if __name__ == "__main__":
    gpu = torch.device("cuda:0")
    if len(sys.argv) > 1 and sys.argv[1] == "--test-helper":
        for H, W in ((37, 58), (17, 1), (81, 129)):
            for s in range(3):
                via_test(H, W, 7 * H + W + 100 * s, gpu)
        sys.exit(0)
    for H, W in ((17, 1), (17, 2), (16, 1), (18, 1), (2, 1), (1, 70), (33, 65), (81, 129), (37, 58)):
        for s in range(4):
            case(H, W, 7 * H + W + 100 * s, gpu)
