"""The reference's sanity check (test/sanity_check.py) on this framework.

The reference's own test image (test/data/192x128_kodim15.png, kept as
tests/golden/192x128_kodim15.png) is encoded on the GPU with the debug preset
(preset_cfg/debug.yaml, which enc/utils/manager.py loads -- its AVAILABLE_PRESETS lookup of the
class presets.py:380-432 is commented out: warm-up 3 x 10 then 2 x 10 candidate iterations with
kumaraswamy noise 2.0, phases 50 / 10 / 10, network quantisation after the second) and the vlop decoder (cfg/dec/vlop.cfg: ARM 8 x 1,
synthesis 8-1-linear-relu / X-1-linear-none / X-3-residual-none, upsampling 8 / 7), written as
a .cool stream and decoded by the bit-exact HIP decoder to a PPM.  The encoder's estimates
(results_best.tsv: eval-mode PSNR, latent + network rate) must match the decoded file with
the reference's thresholds (sanity_check.py:108-124): |dPSNR| < 0.1 dB, rate within 20 %."""
from pathlib import Path

import numpy as np
import pytest
import torch

GOLDEN = Path(__file__).resolve().parent / "golden"
VLOP = ((8, 1, False, True), (3, 1, False, False), (3, 3, True, False))


def test_debug_preset_is_the_reference_schedule():
    from ccmi import train
    assert [c for c, _ in train.DEBUG_WARMUP] == [3, 2]
    assert [p.max_itr for _, p in train.DEBUG_WARMUP] == [10, 10]
    assert all(p.noise_parameter == (2.0, 2.0) and p.quantizer_noise_type == "kumaraswamy"
               and p.freq_valid == 400 and p.patience == 100000 for _, p in train.DEBUG_WARMUP)
    assert [p.max_itr for p in train.DEBUG_PHASES] == [50, 10, 10]
    assert [p.quantize_model for p in train.DEBUG_PHASES] == [False, True, False]
    assert train.DEBUG_PHASES[2].optimized_module == "latent"
    assert train.DEBUG_PHASES[0].quantizer_noise_type == "gaussian" and train.DEBUG_PHASES[1].quantizer_type == "ste"


@pytest.mark.gpu
def test_sanity_check_kodim15(gpu):
    from ccmi import decode, encode, io, quantize, train
    img, bd = io.read_png(GOLDEN / "192x128_kodim15.png")
    H, W = img.shape[-2:]
    arch = train.Arch(H, W, dim_arm=8, n_hidden=1, layers=VLOP)
    tgt = io.to_target(img, "rgb")[None].to(gpu)
    of, _ = train.overfit(arch, tgt, lmbda=1e-3, yuv420=False, warmup=train.DEBUG_WARMUP,
                          phases=train.DEBUG_PHASES)
    qm = of.quantized[0]
    stream = encode.write_cool(arch, of.latents[0], qm, yuv420=False)

    # encoder side (test(): eval forward of the quantised model)
    mse_enc, rate_latent = quantize.evaluate(arch, of.latents[0], of.params[0], tgt[0], yuv420=False, bitdepth=8)
    npx = H * W
    enc_psnr = -10 * np.log10(mse_enc)
    enc_bpp = (rate_latent + sum(qm.nn_bits.values())) / npx

    # decoder side: the bit-exact decoder's PPM against the original 8-bit image
    out, = decode.decode_batch([stream], as_yuv=False)
    dec, dbd = io.parse_ppm(out)
    assert dbd == 8 and dec.shape == img.shape
    a, b = torch.round(img * 255).double(), torch.round(dec * 255).double()
    dec_psnr = 10 * np.log10(255 ** 2 / float(((a - b) ** 2).mean()))
    dec_bpp = len(stream) * 8 / npx
    print(f"\nsanity: PSNR enc {enc_psnr:.3f} dB / dec {dec_psnr:.3f} dB, rate enc {enc_bpp:.3f} / dec {dec_bpp:.3f} bpp")
    assert abs(enc_psnr - dec_psnr) < 0.1, (enc_psnr, dec_psnr)
    assert abs(dec_bpp - enc_bpp) / enc_bpp < 0.2, (enc_bpp, dec_bpp)
