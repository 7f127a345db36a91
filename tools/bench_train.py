"""Timing of the GPU encoder overfit step (ccmi_train_step) at Kodak size (512x768, c3x /
hop architecture, 7 grids): ms per iteration for batches of frames, plus the CPU oracle
(torch autograd, same math) for one iteration.  python tools/bench_train.py [B ...]"""
import json
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
# --lib PATH: time another libccmi build (A/B; set before ccmi is imported -- no env hop, so
# the command can run under rocprofv3)
if "--lib" in sys.argv:
    import os
    i = sys.argv.index("--lib")
    os.environ["CCMI_LIB"] = str((ROOT / sys.argv[i + 1]).resolve())
    del sys.argv[i:i + 2]
NO_CPU = "--no-cpu" in sys.argv
if NO_CPU:
    sys.argv.remove("--no-cpu")
# --default-arch: the reference's default decoder (ARM 24,2; synthesis head 40 wide) instead of hop
DEFAULT_ARCH = "--default-arch" in sys.argv
if DEFAULT_ARCH:
    sys.argv.remove("--default-arch")
sys.path.insert(0, str(ROOT / "cool-chic_amd"))
sys.path.insert(0, str(ROOT / "oracle"))

from ccmi import train as T  # noqa: E402


def gpu_ms(H, W, B, iters=20):
    import forward_oracle as fo
    dev = torch.device("cuda:0")
    rows = []
    if DEFAULT_ARCH:
        layers = ((40, 1, False, True), (3, 1, False, False), (3, 3, True, True), (3, 3, True, False))
        arch = T.Arch(H, W, dim_arm=24, n_hidden=2, layers=layers)
        for b in range(B):
            rows.append(T.init_params(arch, torch.Generator().manual_seed(b)))
    else:
        arch = T.Arch(H, W)
        for b in range(B):
            mp = fo.ModelParams.random(H, W, seed=b)
            rows.append(T.pack_params(mp.arm, mp.ups_half, mp.pre_half, mp.syn))
    g = torch.Generator().manual_seed(0)
    lat = 0.01 * torch.randn(B, arch.n_latents, generator=g)
    tgt = torch.rand(B, H * W + 2 * (H // 2) * (W // 2), generator=g)
    of = T.Overfitter(arch, lat.to(dev), torch.stack(rows).to(dev), tgt.to(dev), yuv420=True, seed=1)
    for _ in range(3):
        of.step("softround", "kumaraswamy", 0.3, 2.0, 1e-3)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        of.step("softround", "kumaraswamy", 0.3, 2.0, 1e-3)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def cpu_ms(H, W, iters=2):
    import forward_oracle as fo
    import train_oracle as to
    mp = fo.ModelParams.random(H, W, seed=0)
    g = torch.Generator().manual_seed(0)
    lat = [0.01 * torch.randn(h, w, generator=g) for h, w in mp.sizes]
    st = to.TrainState(mp, lat)
    tgt = {"y": torch.rand(H, W), "u": torch.rand(H // 2, W // 2), "v": torch.rand(H // 2, W // 2)}
    opt = to.Adam(st.params(), 1e-2)
    noise = to.kumaraswamy(torch.rand(sum(h * w for h, w in mp.sizes)), 2.0)
    to.grads(st, tgt, "softround", 0.3, 1e-3, True, noise=noise)
    t0 = time.perf_counter()
    for _ in range(iters):
        to.grads(st, tgt, "softround", 0.3, 1e-3, True, noise=noise)
        opt.step()
    return (time.perf_counter() - t0) / iters * 1e3


if __name__ == "__main__":
    H, W = 512, 768
    res = {"size": f"{H}x{W}", "gpu_ms_per_iter": {}}
    for B in [int(x) for x in (sys.argv[1:] or ["1", "8"])]:
        res["gpu_ms_per_iter"][B] = round(gpu_ms(H, W, B), 3)
        print(json.dumps(res), flush=True)
    if not NO_CPU:
        res["cpu_ms_per_iter"] = round(cpu_ms(H, W), 1)
        res["cpu_threads"] = torch.get_num_threads()
        print(json.dumps(res), flush=True)
