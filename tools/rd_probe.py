"""Seed spread of the GPU encoder on one image: python tools/rd_probe.py <image> <lambda,...> [n_seeds] [preset] [first_seed]
Images: kodim15_192x128 | kodim01_768x512 | kodim01_crop512 (as tests/test_rd_gpu.py builds them)."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "cool-chic_amd"))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    import torch
    from ccmi import io, rd, train
    from test_rd_gpu import HOP, _targets
    image, lms = sys.argv[1], [float(x) for x in sys.argv[2].split(",")]
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    preset = sys.argv[4] if len(sys.argv) > 4 else "debug"
    base = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    x = _targets()[image]
    H, W = x.shape[-2:]
    arch = train.Arch(H, W, dim_arm=16, n_hidden=2, layers=HOP)
    tgt = io.to_target(x, "rgb").cuda()
    for lm in lms:
        recs = rd.encode_points(tgt, H, W, [lm], arch, seeds=tuple(range(base, base + n)), preset=preset,
                                scale=0.1 if preset == "c3x" else 1.0, name=image)
        p = [r.psnr_db for r in recs]
        b = [r.rate_bpp for r in recs]
        print(f"{image} {preset} lambda {lm}: PSNR {np.mean(p):.3f} +- {np.std(p):.3f} "
              f"[{', '.join(f'{v:.2f}' for v in p)}]  rate {np.mean(b):.4f} "
              f"[{', '.join(f'{v:.3f}' for v in b)}]", flush=True)


if __name__ == "__main__":
    main()
