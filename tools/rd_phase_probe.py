"""Per-seed validation after every phase of the GPU encoding schedule (and before / after
quantize_model), to find where a seed falls behind.
usage: python tools/rd_phase_probe.py IMAGE LAMBDA [preset=debug] [arch=default|hop] [n_seeds=8]"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "cool-chic_amd"))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    import torch
    from ccmi import io, quantize, rd, train
    from test_rd_gpu import DEFAULT_ARCH, HOP, _targets
    image, lm = sys.argv[1], float(sys.argv[2])
    preset = sys.argv[3] if len(sys.argv) > 3 else "debug"
    arch_name = sys.argv[4] if len(sys.argv) > 4 else "default"
    n = int(sys.argv[5]) if len(sys.argv) > 5 else 8
    x = _targets()[image]
    H, W = x.shape[-2:]
    arch = train.Arch(H, W, **(DEFAULT_ARCH if arch_name == "default" else dict(dim_arm=16, n_hidden=2, layers=HOP)))
    tgt = io.to_target(x, "rgb").cuda()

    def psnr(v):
        return [round(float(10 * np.log10(1.0 / max(m, 1e-12))), 2) for m in v[:, 1].tolist()]

    run_phase0, qm0 = train.run_phase, quantize.quantize_model
    k = {"i": 0}

    def run_phase(of, ph, lmbda, scale=1.0):
        before = psnr(of.validate(lmbda))
        best = run_phase0(of, ph, lmbda, scale)
        print(f"phase {k['i']} ({ph.max_itr} its, {ph.quantizer_type}/{ph.quantizer_noise_type}, B={of.B}): "
              f"before {before} -> best {psnr(best)}", flush=True)
        k["i"] += 1
        return best

    def quantize_model(*a, **kw):
        qm = qm0(*a, **kw)
        print(f"  quantize_model: q_step {getattr(qm, 'q_step', None)}", flush=True)
        return qm

    train.run_phase, quantize.quantize_model = run_phase, quantize_model
    recs = rd.encode_points(tgt, H, W, (lm,), arch, yuv420=False, seeds=tuple(range(n)), preset=preset,
                            name=image)
    print("final", [round(r.psnr_db, 2) for r in recs], "rate", [round(r.rate_bpp, 3) for r in recs], flush=True)


if __name__ == "__main__":
    main()
