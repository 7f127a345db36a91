"""End-to-end intra codec on the GPU: overfit (c3x schedule, shortened) -> quantize_model
(batched candidate search) -> .cool writer -> bit-exact decoder.

Checks: the written stream decodes on the GPU to exactly the bytes the C oracle (pinned
to the reference decoder) produces from it; the decoded picture's PSNR is within 0.3 dB
of the float eval PSNR of the quantised model (fixed-point decoder vs float forward);
the quantisation search picks valid steps.  Unit checks of exp_golomb_nbins / layouts run
on the CPU."""
from pathlib import Path

import numpy as np
import pytest
import torch


def test_exp_golomb_nbins_matches_definition():
    from ccmi.quantize import exp_golomb_nbins
    # count 0: 0 -> 1 bit, +-1 -> 3 + sign, +-2 -> 3 + sign, 3 -> 5 + sign (misc.py:248-268)
    assert exp_golomb_nbins(np.array([0]), 0) == 1
    assert exp_golomb_nbins(np.array([1]), 0) == 4
    assert exp_golomb_nbins(np.array([-2]), 0) == 4
    assert exp_golomb_nbins(np.array([3]), 0) == 6
    assert exp_golomb_nbins(np.array([3]), 2) == 4


def test_layout_covers_parameter_block():
    from ccmi.quantize import Layout
    from ccmi.train import Arch, init_params
    a = Arch(32, 48)
    lay = Layout.of(a)
    idx = np.concatenate([lay.arm_w, lay.arm_b, lay.ups_w, lay.syn_w, lay.syn_b])
    assert np.array_equal(np.sort(idx), np.arange(lay.P))
    assert lay.P == init_params(a).numel()


def _image(H, W, seed=0):
    g = torch.Generator().manual_seed(seed)
    yy, xx = torch.meshgrid(torch.linspace(0, 1, H), torch.linspace(0, 1, W), indexing="ij")
    img = torch.stack([0.5 + 0.3 * torch.sin(7 * xx) * torch.cos(4 * yy), 0.5 + 0.1 * torch.cos(5 * yy),
                       0.5 + 0.1 * torch.sin(3 * xx)])
    img = torch.round((img + 0.01 * torch.randn(img.shape, generator=g)).clamp(0, 1) * 255) / 255
    return torch.cat([img[0].reshape(-1), img[1, ::2, ::2].reshape(-1), img[2, ::2, ::2].reshape(-1)])


@pytest.mark.gpu
def test_gpu_encode_quantize_write_decode(gpu, oracle_c, tmp_path):
    from ccmi import decode, encode, quantize, train
    H, W = 64, 96
    arch = train.Arch(H, W)
    tgt = _image(H, W)[None].to(gpu)
    # c3x (shortened): quantize_model runs after its second phase, the last phase trains
    # the latents against the quantised networks
    of, best = train.overfit(arch, tgt, lmbda=1e-3, scale=0.05, seed=0)
    qm = of.quantized[0]
    for m in ("arm", "synthesis", "upsampling"):
        assert m in qm.q_index and m in qm.expgol and qm.nn_bits[m] > 0
    assert np.array_equal(of.params[0].cpu().numpy(), qm.params)
    stream = encode.write_cool(arch, of.latents[0], qm, yuv420=True)
    assert 100 < len(stream) < H * W  # far below 8 bpp
    # bit-exact decode: GPU decoder == C oracle (== reference decoder)
    y_gpu, = decode.decode_batch([stream])
    p = tmp_path / "e2e.cool"
    p.write_bytes(stream)
    assert oracle_c.cco_decode_file(str(p).encode(), str(tmp_path / "o.yuv").encode(), 0, 0, 0) == 0
    assert y_gpu == (tmp_path / "o.yuv").read_bytes()
    ref = Path(__file__).resolve().parents[1] / "oracle" / "_ref" / "ccdec_ref"
    if ref.exists():  # the reference decoder itself, compiled from its sources (oracle/Makefile)
        import subprocess
        subprocess.run([str(ref), f"--input={p}", f"--output={tmp_path / 'r.yuv'}"], check=True,
                       stdout=subprocess.DEVNULL)
        assert y_gpu == (tmp_path / "r.yuv").read_bytes()
    # quality: decoded 8-bit picture vs the float eval of the quantised model
    dec = torch.frombuffer(bytearray(y_gpu), dtype=torch.uint8).float() / 255
    mse_dec = float(((dec - tgt[0].cpu()) ** 2).mean())
    of2 = train.Overfitter(arch, of.latents[:1].clone(), torch.from_numpy(qm.params)[None].to(gpu), tgt)
    mse_eval = float(of2.validate(1e-3)[0, 1])
    psnr_dec, psnr_eval = -10 * np.log10(mse_dec), -10 * np.log10(mse_eval)
    assert abs(psnr_dec - psnr_eval) < 0.3, (psnr_dec, psnr_eval)
    assert psnr_dec > 25
