"""Rate-distortion reporting: Bjontegaard deltas and the per-image encoding records the
reference's result tables hold.

bd_rate / bd_psnr restate coolchic/utils/bjontegaard_metric.py:6-90 (a third-party file the
reference vendors, "Anserw/Bjontegaard_metric", downloaded 2024-11-15): a cubic fit of log
rate against PSNR (or PSNR against log rate) per curve, integrated over the overlapping
interval; piecewise=1 uses PCHIP interpolation and the trapezoid rule on 100 samples instead.
Pinned by tests/golden/rd_reference_*.json, whose "bd" entries the reference function
computed (tools/gen_golden_rd.py).

encode_points runs the GPU encoder (ccmi.train.overfit + quantize_model, as
enc/component/video.py:224-330 for one intra frame) and reports what the reference's test()
reports (enc/training/test.py:370-438): eval-mode PSNR, latent and network rate in bpp.
"""

from __future__ import annotations

import math
import time
from dataclasses import asdict, dataclass

import numpy as np
import torch


def _fit_integral(x, y, lo, hi, piecewise: int) -> float:
    x, y = np.asarray(x, dtype=np.float64), np.asarray(y, dtype=np.float64)
    if piecewise == 0:
        p = np.polyint(np.polyfit(x, y, 3))
        return float(np.polyval(p, hi) - np.polyval(p, lo))
    import scipy.interpolate
    samples, step = np.linspace(lo, hi, num=100, retstep=True)
    o = np.argsort(x)
    v = scipy.interpolate.pchip_interpolate(x[o], y[o], samples)
    return float(np.trapezoid(v, dx=float(step)))


def bd_rate(R1, PSNR1, R2, PSNR2, piecewise: int = 0) -> float:
    """Average rate difference (%) of curve 2 against curve 1 at equal PSNR
    (BD_RATE, bjontegaard_metric.py:48-90); negative = curve 2 needs fewer bits."""
    lR1, lR2 = np.log(np.asarray(R1, float)), np.log(np.asarray(R2, float))
    lo, hi = max(min(PSNR1), min(PSNR2)), min(max(PSNR1), max(PSNR2))
    i1 = _fit_integral(PSNR1, lR1, lo, hi, piecewise)
    i2 = _fit_integral(PSNR2, lR2, lo, hi, piecewise)
    return (math.exp((i2 - i1) / (hi - lo)) - 1) * 100


def bd_psnr(R1, PSNR1, R2, PSNR2, piecewise: int = 0) -> float:
    """Average PSNR difference (dB) of curve 2 against curve 1 at equal rate
    (BD_PSNR, bjontegaard_metric.py:6-45)."""
    lR1, lR2 = np.log(np.asarray(R1, float)), np.log(np.asarray(R2, float))
    lo, hi = max(lR1.min(), lR2.min()), min(lR1.max(), lR2.max())
    i1 = _fit_integral(lR1, PSNR1, lo, hi, piecewise)
    i2 = _fit_integral(lR2, PSNR2, lo, hi, piecewise)
    return (i2 - i1) / (hi - lo)


@dataclass
class Record:
    """One encoded image: the columns of the reference's results_best.tsv that BD-rate and
    the encoder-speed comparison use."""
    image: str
    lmbda: float
    seed: int
    psnr_db: float
    rate_bpp: float          # latent + networks (test()'s total_rate_bpp)
    rate_latent_bpp: float
    rate_nn_bpp: float
    iterations: int
    seconds: float
    cool_bpp: float = float("nan")   # size of the written .cool stream (when written)
    timing: dict | None = None        # the batch's schedule timing (ccmi.train.overfit), on its first record

    def as_dict(self):
        return asdict(self)


def encode_batch(targets: torch.Tensor, H: int, W: int, lmbda: float, arch, *, names=None, seeds=None,
                 yuv420: bool = False, preset: str = "debug", scale: float = 1.0, write: bool = False) -> list[Record]:
    """Overfit B frames of one geometry together (targets [B, n] flat ccmi.train targets on
    the GPU, one independent decoder per frame), then measure each as the reference's test()
    does (quantised model, hard-rounded latents): one Record per frame.  `seconds` is the
    batch's wall time divided by B."""
    from . import encode, quantize, train
    warm, phases = (train.DEBUG_WARMUP, train.DEBUG_PHASES) if preset == "debug" else (train.C3X_WARMUP, train.C3X_PHASES)
    B = targets.shape[0]
    names = list(names) if names is not None else [""] * B
    seeds = list(seeds) if seeds is not None else list(range(B))
    npx = H * W
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    of, _ = train.overfit(arch, targets, lmbda=float(lmbda), yuv420=yuv420, scale=scale, seed=int(seeds[0]),
                          warmup=warm, phases=phases)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # counted as the reference's iterations_counter: every warm-up candidate's iterations
    # (3 x 10 + 2 x 10 for debug), then each frame's phases up to its early stop
    out = []
    for b in range(B):
        mse, rate_lat = quantize.evaluate(arch, of.latents[b], of.params[b], of.targets[b], yuv420=yuv420, bitdepth=8)
        qm = of.quantized[b] if of.quantized else None
        nn_bits = sum(qm.nn_bits.values()) if qm else 0.0
        rec = Record(image=names[b], lmbda=float(lmbda), seed=int(seeds[b]), psnr_db=-10 * math.log10(mse + 1e-10),
                     rate_bpp=(rate_lat + nn_bits) / npx, rate_latent_bpp=rate_lat / npx, rate_nn_bpp=nn_bits / npx,
                     iterations=int(of.iterations[b]), seconds=dt / B)
        if write and qm is not None:
            rec.cool_bpp = 8 * len(encode.write_cool(arch, of.latents[b], qm, yuv420=yuv420)) / npx
        if b == 0:
            rec.timing = dict(getattr(of, "timing", {}), batch=B, total_s=dt)
        out.append(rec)
    return out


def encode_points(target: torch.Tensor, H: int, W: int, lambdas, arch, *, yuv420: bool = False, seeds=(0,),
                  preset: str = "debug", scale: float = 1.0, name: str = "", write: bool = False) -> list[Record]:
    """Encode one image (flat ccmi.train target on the GPU) at every lambda; the seeds of one
    lambda train together as one batch (independent initialisations and noise streams)."""
    out = []
    for lm in lambdas:
        tg = target.reshape(1, -1).repeat(len(seeds), 1).contiguous()
        out += encode_batch(tg, H, W, lm, arch, names=[name] * len(seeds), seeds=seeds, yuv420=yuv420,
                            preset=preset, scale=scale, write=write)
    return out


def curve(records, key="rate_bpp"):
    """Mean (rate, PSNR) per lambda over seeds, sorted by lambda."""
    by = {}
    for r in records:
        r = r if isinstance(r, dict) else r.as_dict()
        by.setdefault(r["lmbda"], []).append(r)
    lms = sorted(by)
    return ([float(np.mean([r[key] for r in by[l]])) for l in lms],
            [float(np.mean([r["psnr_db"] for r in by[l]])) for l in lms], lms)


__all__ = ["bd_rate", "bd_psnr", "Record", "encode_batch", "encode_points", "curve"]
