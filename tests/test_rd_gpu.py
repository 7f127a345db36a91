"""Matched rate-distortion: the GPU encoder against the reference encoder on the same images,
preset, architecture and lambdas (BASELINE configs 1 and 4).

Reference points: tests/golden/rd_reference_*.json, written by tools/gen_golden_rd.py, which
ran the reference's own warmup() / train() / quantize_model() / test() on CPU here:
  * kodim15_192x128 -- the image of the reference's sanity check (test/sanity_check.py:13);
  * kodim01_768x512 -- results/image/kodak/bitstreams/kodim01-lmbda-00001.cool decoded
    bit-exactly: Kodak geometry (config 4's content; the reference's 40.5 dB reconstruction
    stands in for the original image, which the reference tree does not hold);
  * kodim01_crop512 -- config 1: the same cropped to [0, 512) x [0, 512);
hop decoder (cfg/dec/hop.cfg), lambdas 0.02 / 0.004 / 0.001 / 0.0004, 2 seeds each.

The encoder is stochastic (random initialisation, quantisation noise): neither side can
reproduce the other's random draws, so the bar is statistical.  Per lambda the GPU's median PSNR and mean rate over
GPU_SEEDS must lie within the reference's own 2-seed spread widened by a fixed margin, and
the BD-rate of the GPU curve against the reference curve (ccmi.rd.bd_rate, the restatement of
bjontegaard_metric.py:48-90) must stay inside the BD_WORSE / BD_BETTER band.  Records are written to
gpurun_out/rd_gpu_<preset>.json for the bench / DESIGN.md tables.
"""
import json
import os
from pathlib import Path

import numpy as np
import pytest
import torch

GOLDEN = Path(__file__).resolve().parent / "golden"
ROOT = Path(__file__).resolve().parents[1]
HOP = ((48, 1, False, True), (3, 1, False, False), (3, 3, True, True), (3, 3, True, False))
LAMBDAS = (0.02, 0.004, 0.001, 0.0004)
# GPU seeds per lambda: encodes are cheap on the GPU (a debug-preset batch of 8 takes < 1 s at
# 512 x 512), and the short presets are bimodal (tools/rd_probe.py: at 512 x 512, lambda 1e-3,
# about one seed in five lands near 28 dB instead of 31), so 2 seeds are not a stable mean.
GPU_SEEDS = tuple(range(8))
PSNR_MARGIN_DB = 0.5   # on top of the reference's own seed-to-seed spread at that lambda
RATE_MARGIN = 0.15     # relative, on top of the reference's spread
# BD-rate band (percent, GPU curve against the reference curve, seed means): the GPU encoder
# may not need more than BD_WORSE % more bits at equal PSNR; a much lower rate would point at
# a rate-accounting bug, hence the lower bound.  Not on the 192 x 128 image: its
# 120-iteration curves are too noisy for a cubic fit (the reference's own seed 1 against its
# seed 0 gives -66.6 % there, -0.45 % on kodim01 at 768 x 512).
BD_WORSE, BD_BETTER = 10.0, 25.0
# Kodak geometry (768 x 512, config 4's content): the band narrowed to +-5 % (measured: c3x
# x0.1 +0.9 / +1.0 %, debug -0.65 %; profiles/r3_rd_gpu_summary.txt)
BD_KODAK = 5.0

pytestmark = pytest.mark.gpu


def _targets():
    from ccmi import decode, io
    img, bd = io.read_png(GOLDEN / "192x128_kodim15.png")
    assert bd == 8
    out, = decode.decode_batch([(GOLDEN / "cool" / "kodim01-lmbda-00001.cool").read_bytes()], as_yuv=False)
    k01, bd = io.parse_ppm(out)
    assert bd == 8
    k01 = k01[0].float()  # [3, 512, 768]
    out, = decode.decode_batch([(GOLDEN / "cool" / "kodim04-lmbda-00001.cool").read_bytes()], as_yuv=False)
    k04, bd = io.parse_ppm(out)
    assert bd == 8
    return {"kodim15_192x128": img[0].float(), "kodim01_768x512": k01.contiguous(),
            "kodim01_crop512": k01[:, :512, :512].contiguous(),
            "kodim04_512x768": k04[0].float().contiguous()}  # [3, 768, 512]: config 4's portrait batch


def _ref(preset_file):
    d = json.loads((GOLDEN / preset_file).read_text())
    return d["runs"]


def _check(image, ours, ref, bd_band):
    from ccmi import rd
    lines = []
    for lm in LAMBDAS:
        r = [x for x in ref if x["image"] == image and x["lmbda"] == lm]
        o = [x for x in ours if x.lmbda == lm]
        rp, rr = [x["psnr_db"] for x in r], [x["rate_bpp"] for x in r]
        # PSNR: the median over GPU seeds (outcomes are bimodal, see GPU_SEEDS), rate: the mean
        op, orr = np.median([x.psnr_db for x in o]), np.mean([x.rate_bpp for x in o])
        tol_p = PSNR_MARGIN_DB + (max(rp) - min(rp))
        tol_r = RATE_MARGIN + (max(rr) - min(rr)) / np.mean(rr)
        lines.append(f"{image} lambda {lm}: PSNR ref {np.mean(rp):.3f} gpu {op:.3f} (tol {tol_p:.2f}), "
                     f"rate ref {np.mean(rr):.4f} gpu {orr:.4f} (tol {tol_r:.2f})")
        assert abs(op - np.mean(rp)) <= tol_p, lines[-1]
        assert abs(orr / np.mean(rr) - 1) <= tol_r, lines[-1]
    R1, P1, _ = rd.curve([x for x in ref if x["image"] == image])
    R2, P2, _ = rd.curve(ours)
    bd = rd.bd_rate(R1, P1, R2, P2)
    lines.append(f"{image}: BD-rate GPU vs reference {bd:+.2f} %")
    print("\n" + "\n".join(lines))
    if bd_band:
        if isinstance(bd_band, tuple):
            lo, hi = bd_band
        else:
            lo, hi = (-BD_KODAK, BD_KODAK) if image == "kodim01_768x512" else (-BD_BETTER, BD_WORSE)
        assert lo <= bd <= hi, lines[-1] + f" (band {lo:+.1f} .. {hi:+.1f} %)"
    return bd


def _ref_seed_bd(ref, image):
    """BD-rate of the reference's own seed 1 curve against its seed 0 curve on `image`: how far
    two runs of the SAME encoder land apart with this preset and architecture."""
    from ccmi import rd
    c = {}
    for sd in (0, 1):
        rr = sorted([r for r in ref if r["image"] == image and r["seed"] == sd], key=lambda r: r["lmbda"])
        c[sd] = ([r["rate_bpp"] for r in rr], [r["psnr_db"] for r in rr])
    return rd.bd_rate(c[0][0], c[0][1], c[1][0], c[1][1])


@pytest.mark.parametrize("image", ["kodim15_192x128", "kodim01_768x512", "kodim01_crop512"])
def test_debug_preset_matches_reference_rd(image, gpu):
    from ccmi import io, rd, train
    ref = [r for r in _ref("rd_reference_debug.json") if r["image"] == image]
    assert ref, f"no reference points for {image}"
    x = _targets()[image]
    H, W = x.shape[-2:]
    arch = train.Arch(H, W, dim_arm=16, n_hidden=2, layers=HOP)
    tgt = io.to_target(x, "rgb").to(gpu)
    recs = rd.encode_points(tgt, H, W, LAMBDAS, arch, yuv420=False, seeds=GPU_SEEDS, preset="debug", name=image,
                            write=True)
    out = ROOT / "gpurun_out"
    out.mkdir(exist_ok=True)
    f = out / "rd_gpu_debug.json"
    prev = json.loads(f.read_text()) if f.exists() else {}
    prev[image] = [r.as_dict() for r in recs]
    f.write_text(json.dumps(prev, indent=1))
    bd = _check(image, recs, ref, bd_band=image != "kodim15_192x128")
    # the written .cool streams: what the bitstream really costs next to the estimate
    for r in recs:
        assert r.cool_bpp == r.cool_bpp and r.cool_bpp > 0
    assert np.isfinite(bd)


# The reference's DEFAULT decoder (coolchic/utils/types.py:120-143: synthesis
# 40-1-linear-relu,X-1-linear-none,X-3-residual-relu,X-3-residual-none, ARM "24,2"), debug
# preset: the dim-24 ARM is the VALU training kernel whose context-gradient gather reaches 4
# rows up (wrong until round 3's last commit), so its R-D is pinned end to end here against
# the reference encoder run with the same architecture (tools/gen_golden_rd.py debug_default).
DEFAULT_ARCH = dict(dim_arm=24, n_hidden=2,
                    layers=((40, 1, False, True), (3, 1, False, False), (3, 3, True, True), (3, 3, True, False)))


@pytest.mark.skipif(not (GOLDEN / "rd_reference_debug_default.json").exists(), reason="default-arch fixture absent")
@pytest.mark.parametrize("image", ["kodim15_192x128", "kodim01_768x512"])
def test_debug_preset_default_arch_matches_reference_rd(image, gpu):
    from ccmi import io, rd, train
    ref = [r for r in _ref("rd_reference_debug_default.json") if r["image"] == image and r["arch"] == "default"]
    if {r["lmbda"] for r in ref} != set(LAMBDAS):
        pytest.skip(f"default-arch fixture incomplete for {image}")
    x = _targets()[image]
    H, W = x.shape[-2:]
    arch = train.Arch(H, W, **DEFAULT_ARCH)
    tgt = io.to_target(x, "rgb").to(gpu)
    recs = rd.encode_points(tgt, H, W, LAMBDAS, arch, yuv420=False, seeds=GPU_SEEDS, preset="debug", name=image,
                            write=True)
    out = ROOT / "gpurun_out"
    out.mkdir(exist_ok=True)
    f = out / "rd_gpu_debug_default.json"
    prev = json.loads(f.read_text()) if f.exists() else {}
    prev[image] = [r.as_dict() for r in recs]
    f.write_text(json.dumps(prev, indent=1))
    # 120 iterations of a 40-wide head and a dim-24 ARM land far apart from seed to seed (the
    # reference's seed 1 against its seed 0: +18 % BD-rate on kodim01), so two reference seeds
    # could not pin it: since round 6 the fixture holds 6 seeds per lambda and the bands are the
    # pooled-sigma form of the c3x test (per lambda) plus a BD-rate band from the reference's own
    # seed-curve scatter (_check_pooled)
    if min(sum(1 for x in ref if x["lmbda"] == lm) for lm in LAMBDAS) >= 4:
        bd = _check_pooled(image, recs, ref, "debug default")
    else:  # the round-5 form (2 reference seeds): spread of the reference's two seed curves + 5 %
        spread = abs(_ref_seed_bd(ref, image))
        bd = _check(image, recs, ref, bd_band=(-(spread + BD_KODAK), spread + BD_KODAK) if image == "kodim01_768x512" else False)
    for r in recs:
        assert r.cool_bpp == r.cool_bpp and r.cool_bpp > 0
    assert np.isfinite(bd)


# pooled-sigma bands of the debug preset (round 6): per lambda the GPU mean within
# 3 sqrt(sigma_ref^2 / n_ref + sigma_gpu^2 / n_gpu) + DEBUG_PSNR_MARGIN_DB / + DEBUG_RATE_MARGIN of
# the reference mean, each sigma pooled over that side's four lambdas (the two-sample form: with the
# default decoder the GPU's 8 seeds scatter about twice as wide as the reference's 6 -- kodim01
# PSNR 0.95 vs 0.41 dB, rate 7.0 vs 4.7 % -- so one common sigma understated the difference's
# spread; gpurun_out/r6k, profiles/r6k_rd_debug_default.txt).  On the Kodak-geometry image also the BD-rate of
# the GPU's mean curve against the reference's mean curve: within 3 sd_half sqrt((1 / n_ref +
# 1 / n_gpu) / (2 / h)) + DEBUG_BD_MARGIN %, sd_half the scatter of the BD-rate between the mean
# curves of complementary halves (h seeds each) of the reference's own seeds.  (The 192 x 128 image's
# 120-iteration curves are too irregular for a cubic BD fit: its half-split BD-rates reach +1,000 %.)
DEBUG_PSNR_MARGIN_DB = 0.1
DEBUG_RATE_MARGIN = 0.03
DEBUG_BD_MARGIN = 2.0


def _half_split_bd_sd(ref):
    """Standard deviation of the BD-rate between the mean curves of complementary halves of the
    reference seeds (every split with seed 0 in the first half), and the half size."""
    import itertools
    from ccmi import rd
    seeds = sorted({r["seed"] for r in ref})
    h = len(seeds) // 2
    out = []
    for A in itertools.combinations(seeds, h):
        if seeds[0] not in A:
            continue
        B = [x for x in seeds if x not in A][:h]
        R1, P1, _ = rd.curve([r for r in ref if r["seed"] in A])
        R2, P2, _ = rd.curve([r for r in ref if r["seed"] in B])
        out.append(rd.bd_rate(R1, P1, R2, P2))
    return float(np.std(out, ddof=1)), h, out


def _check_pooled(image, recs, ref, tag):
    from ccmi import rd
    by_lm = {lm: [x for x in ref if x["lmbda"] == lm] for lm in LAMBDAS}
    assert all(len(v) >= 4 for v in by_lm.values()), "pooled bands need >= 4 reference seeds per lambda"
    sd_p = _pooled_sd([[x["psnr_db"] for x in r] for r in by_lm.values()])
    sd_r = _pooled_sd([[x["rate_bpp"] for x in r] for r in by_lm.values()], rel=True)
    go = {lm: [x for x in recs if x.lmbda == lm] for lm in LAMBDAS}
    gsd_p = _pooled_sd([[x.psnr_db for x in o] for o in go.values()])
    gsd_r = _pooled_sd([[x.rate_bpp for x in o] for o in go.values()], rel=True)
    lines = [f"{image} {tag}: pooled seed sigma reference PSNR {sd_p:.3f} dB rate {sd_r:.3f}, GPU {gsd_p:.3f} dB {gsd_r:.3f}"]
    for lm in LAMBDAS:
        r = by_lm[lm]
        rp, rr = [x["psnr_db"] for x in r], [x["rate_bpp"] for x in r]
        o = go[lm]
        op, orr = np.mean([x.psnr_db for x in o]), np.mean([x.rate_bpp for x in o])
        tol_p = DEBUG_PSNR_MARGIN_DB + 3.0 * np.sqrt(sd_p ** 2 / len(r) + gsd_p ** 2 / len(o))
        tol_r = DEBUG_RATE_MARGIN + 3.0 * np.sqrt(sd_r ** 2 / len(r) + gsd_r ** 2 / len(o))
        lines.append(f"{image} {tag} lambda {lm}: PSNR ref {np.mean(rp):.3f} ({len(rp)} seeds, {min(rp):.3f}..{max(rp):.3f}) "
                     f"gpu {op:.3f} (tol {tol_p:.2f}), rate ref {np.mean(rr):.4f} gpu {orr:.4f} (tol {tol_r:.3f})")
        assert abs(op - np.mean(rp)) <= tol_p, lines[-1]
        assert abs(orr / np.mean(rr) - 1) <= tol_r, lines[-1]
    R1, P1, _ = rd.curve(ref)
    R2, P2, _ = rd.curve(recs)
    bd = rd.bd_rate(R1, P1, R2, P2)
    if image == "kodim01_768x512":
        sd_h, h, splits = _half_split_bd_sd(ref)
        n_ref = min(len(v) for v in by_lm.values())
        n_gpu = len({x.seed for x in recs})
        band = 3.0 * sd_h * np.sqrt((1.0 / n_ref + 1.0 / n_gpu) / (2.0 / h)) + DEBUG_BD_MARGIN
        lines.append(f"{image} {tag}: BD-rate GPU vs reference {bd:+.2f} % (band +-{band:.1f}: reference half-split "
                     f"BD-rates {', '.join(f'{v:+.1f}' for v in splits)} %, sd {sd_h:.1f})")
        print("\n" + "\n".join(lines))
        assert abs(bd) <= band, lines[-1]
    else:
        lines.append(f"{image} {tag}: BD-rate GPU vs reference {bd:+.2f} % (reported, not banded)")
        print("\n" + "\n".join(lines))
    return bd


# c3x preset (preset_cfg/c3x.yaml) with every phase / warm-up / patience scaled by 0.1, as
# tools/gen_golden_rd.py ran it (C3X_SCALE).  The reference ran 2-6 seeds per lambda
# (kodim15: 6 since round 5; two seeds had put the GPU 0.29 dB "below" the reference at
# lambda 0.004, where the six seeds' mean is 0.03 dB from the GPU's).  Per lambda the GPU's
# mean (GPU_SEEDS) must lie within 3 standard deviations of the difference of two means of
# the reference mean, sigma = the reference's seed standard deviation pooled over the four
# lambdas of the image (sqrt(1 / n_ref + 1 / n_gpu) sigma), + 0.1 dB (PSNR) / + 3 % (rate,
# relative).  Round 4 allowed the largest two-seed spread + 0.3 dB / 8 %.
C3X_SCALE = 0.1
C3X_PSNR_MARGIN_DB = 0.1
C3X_RATE_MARGIN = 0.03


def _pooled_sd(groups, rel=False):
    """Standard deviation pooled over groups (within-group sample variances, ddof 1); rel:
    each group's values divided by the group mean first."""
    v = []
    for g in groups:
        a = np.asarray(g, dtype=np.float64)
        if rel:
            a = a / a.mean()
        if len(a) >= 2:
            v.append(a.var(ddof=1))
    return float(np.sqrt(np.mean(v)))


@pytest.mark.parametrize("image", ["kodim15_192x128", "kodim01_768x512"])
def test_c3x_preset_matches_reference_rd(image, gpu):
    from ccmi import io, rd, train
    d = json.loads((GOLDEN / "rd_reference_c3x.json").read_text())
    ref = [r for r in d["runs"] if r["image"] == image]
    assert {r["lmbda"] for r in ref} == set(LAMBDAS)
    assert all(len({r["seed"] for r in ref if r["lmbda"] == lm}) >= 2 for lm in LAMBDAS), "two reference seeds"
    x = _targets()[image]
    H, W = x.shape[-2:]
    arch = train.Arch(H, W, dim_arm=16, n_hidden=2, layers=HOP)
    tgt = io.to_target(x, "rgb").to(gpu)
    recs = rd.encode_points(tgt, H, W, LAMBDAS, arch, yuv420=False, seeds=GPU_SEEDS, preset="c3x", scale=C3X_SCALE,
                            name=image)
    out = ROOT / "gpurun_out"
    out.mkdir(exist_ok=True)
    f = out / "rd_gpu_c3x.json"
    prev = json.loads(f.read_text()) if f.exists() else {}
    prev[image] = [r.as_dict() for r in recs]
    f.write_text(json.dumps(prev, indent=1))
    lines = []
    by_lm = {lm: [x for x in ref if x["lmbda"] == lm] for lm in LAMBDAS}
    sd_p = _pooled_sd([[x["psnr_db"] for x in r] for r in by_lm.values()])
    sd_r = _pooled_sd([[x["rate_bpp"] for x in r] for r in by_lm.values()], rel=True)
    for lm in LAMBDAS:
        r = by_lm[lm]
        rp, rr, ri = [x["psnr_db"] for x in r], [x["rate_bpp"] for x in r], [x["iterations"] for x in r]
        o = [x for x in recs if x.lmbda == lm]
        op, orr = np.mean([x.psnr_db for x in o]), np.mean([x.rate_bpp for x in o])
        k = 3.0 * np.sqrt(1.0 / len(r) + 1.0 / len(o))
        tol_p = C3X_PSNR_MARGIN_DB + k * sd_p
        tol_r = C3X_RATE_MARGIN + k * sd_r
        its = int(np.median([x.iterations for x in o]))
        lines.append(f"{image} c3x lambda {lm}: PSNR ref {np.mean(rp):.3f} ({len(rp)} seeds, {min(rp):.3f}..{max(rp):.3f}) gpu {op:.3f} "
                     f"(tol {tol_p:.2f}), rate ref {np.mean(rr):.4f} gpu {orr:.4f} (tol {tol_r:.2f}), iterations ref "
                     f"{ri} gpu median {its} (min {min(x.iterations for x in o)}, max {max(x.iterations for x in o)})")
        assert abs(op - np.mean(rp)) <= tol_p, lines[-1]
        assert abs(orr / np.mean(rr) - 1) <= tol_r, lines[-1]
        # patience early stopping as train.py:226-240: the same iteration counts (the third
        # phase stops when its loss stops improving; 2 % covers a record taken at one more
        # validation)
        assert abs(its - np.mean(ri)) <= 0.02 * np.mean(ri), lines[-1]
    R1, P1, _ = rd.curve(ref)
    R2, P2, _ = rd.curve(recs)
    bd = rd.bd_rate(R1, P1, R2, P2)
    lines.append(f"{image} c3x: BD-rate GPU vs reference {bd:+.2f} %")
    print("\n" + "\n".join(lines))
    if image == "kodim01_768x512":
        assert -BD_KODAK <= bd <= BD_KODAK, lines[-1]
    elif image != "kodim15_192x128":
        assert -BD_BETTER <= bd <= BD_WORSE, lines[-1]


# The FULL c3x schedule (preset_cfg/c3x.yaml unscaled: warm-up 5 x 400 + 2 x 400 candidate
# iterations, phases 10,000 + 1,500 + 1,000 with patience; BASELINE config 4's operating
# point) on the Kodak-geometry target at lambda 1e-3: the reference encoder ran it twice here
# (seeds 0 and 1, tools/gen_golden_rd.py one kodim01_768x512 1.0 0.001 SEED ...; ~3.8 h each
# on 3 CPU threads), the GPU runs GPU_SEEDS.  Bar: the GPU's median PSNR within the
# reference's seed spread + 0.3 dB of the reference mean, its mean rate within the spread + 10 %,
# and the same iteration counts (patience stopping, train.py:226-240) within 2 %.  Since round 5
# the bands are 0.15 dB and 4 % of the reference mean (round 4 measured the GPU within 0.04 dB
# and 1.2 % at all three lambdas, against 0.3 dB + spread / 10 % + spread allowed).
FULL_PSNR_MARGIN_DB = 0.15
FULL_RATE_MARGIN = 0.04


FULL_CASES = [
    ("kodim01_768x512", "hop", 0.001),   # round 3
    ("kodim01_768x512", "hop", 0.0004),  # round 4
    ("kodim01_768x512", "hop", 0.004),   # round 4
    ("kodim04_512x768", "hop", 0.001),   # round 5: config 4's portrait geometry batch
    ("kodim01_768x512", "default", 0.001),  # round 5: the reference's default decoder (ARM 24,2; 40-wide head)
]


@pytest.mark.skipif(not (GOLDEN / "rd_reference_c3x_full.json").exists(), reason="full-schedule reference fixture absent")
@pytest.mark.parametrize("image,arch_name,lm", FULL_CASES, ids=[f"{i}-{a}-{lm}" for i, a, lm in FULL_CASES])
def test_c3x_full_schedule_matches_reference(image, arch_name, lm, gpu):
    """kodim01 768x512 with the hop decoder at lambda 1e-3 (round 3), 4e-4 and 4e-3 (round 4); the
    portrait kodim04 512x768 (hop) and kodim01 with the reference's default decoder at lambda 1e-3
    (round 5; its second reference seed round 6).  Two full-schedule reference seeds each."""
    from ccmi import io, rd, train
    ref = json.loads((GOLDEN / "rd_reference_c3x_full.json").read_text())["runs"]
    ref = [r for r in ref if r["image"] == image and r["lmbda"] == lm and r["preset"] == "c3x"
           and r.get("arch", "hop") == arch_name]
    if (image, arch_name, lm) != ("kodim01_768x512", "hop", 0.001) and not ref:
        pytest.skip(f"full-schedule reference for {image} / {arch_name} at lambda {lm} not generated yet")
    assert len(ref) >= 2, "two full-schedule reference seeds per case (round 6: every case has them)"
    x = _targets()[image]
    H, W = x.shape[-2:]
    arch = train.Arch(H, W, **(DEFAULT_ARCH if arch_name == "default" else dict(dim_arm=16, n_hidden=2, layers=HOP)))
    tgt = io.to_target(x, "rgb").to(gpu)
    recs = rd.encode_points(tgt, H, W, (lm,), arch, yuv420=False, seeds=GPU_SEEDS, preset="c3x", scale=1.0,
                            name=image)
    out = ROOT / "gpurun_out"
    out.mkdir(exist_ok=True)
    f = out / "rd_gpu_c3x_full.json"
    prev = json.loads(f.read_text()) if f.exists() else {}
    prev[f"{image}@{lm}" + ("" if arch_name == "hop" else f"@{arch_name}")] = [r.as_dict() for r in recs]
    f.write_text(json.dumps(prev, indent=1))
    rp, rr, ri = [r["psnr_db"] for r in ref], [r["rate_bpp"] for r in ref], [r["iterations"] for r in ref]
    op = float(np.median([r.psnr_db for r in recs]))
    orr = float(np.mean([r.rate_bpp for r in recs]))
    its = int(np.median([r.iterations for r in recs]))
    tol_p = FULL_PSNR_MARGIN_DB
    tol_r = FULL_RATE_MARGIN
    line = (f"{image} {arch_name} c3x full lambda {lm}: PSNR ref {np.mean(rp):.3f} ({len(rp)} seeds, {min(rp):.3f}..{max(rp):.3f}) gpu median "
            f"{op:.3f} (tol {tol_p:.2f}); rate ref {np.mean(rr):.4f} gpu {orr:.4f} (tol {tol_r:.2f}); iterations "
            f"ref {ri} gpu median {its} (min {min(r.iterations for r in recs)}, max {max(r.iterations for r in recs)})")
    print("\n" + line)
    assert abs(op - np.mean(rp)) <= tol_p, line
    assert abs(orr / np.mean(rr) - 1) <= tol_r, line
    assert abs(its - np.mean(ri)) <= 0.02 * np.mean(ri), line
