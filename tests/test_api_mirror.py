"""The drop-in module surface (cool-chic_amd/coolchic, CCLIB) loads the reference's
state_dicts unchanged and reproduces the reference outputs through the HIP kernels."""
import ast
import hashlib
import json
from pathlib import Path

import numpy as np
import pytest
import torch

import forward_oracle as fo

GOLDEN = fo.golden_files()
GDIR = Path(__file__).resolve().parent / "golden"


def _build(z):
    from coolchic.enc.component.coolchic import CoolChicEncoder, CoolChicEncoderParameter
    meta = ast.literal_eval(str(z["meta"]))
    p = CoolChicEncoderParameter(layers_synthesis=meta["layers"].split("|"), n_ft_per_res=[1] * meta["n_grids"],
                                 dim_arm=meta["dim_arm"], n_hidden_layers_arm=meta["n_hidden_arm"])
    p.set_image_size((meta["H"], meta["W"]))
    enc = CoolChicEncoder(p)
    sd = {k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("p/")}
    for i in range(meta["n_grids"]):
        sd[f"latent_grids.{i}.data"] = torch.from_numpy(z[f"lat{i}"])[None, None]
    missing, unexpected = enc.load_state_dict(sd, strict=True), None
    return enc.eval(), meta


@pytest.mark.parametrize("path", GOLDEN[:3], ids=[p.stem for p in GOLDEN[:3]])
def test_reference_state_dict_loads_strictly(path):
    z = np.load(path)
    enc, meta = _build(z)
    ref_keys = {k[2:] for k in z.files if k.startswith("p/")}
    mine = {k for k in enc.state_dict() if not k.startswith("latent_grids")}
    assert mine == ref_keys


def test_forward_on_cpu_tensors_is_refused_loudly():
    """No CPU path: a module left on the CPU raises in train and in eval mode."""
    z = np.load(GOLDEN[0])
    enc, _ = _build(z)
    enc.train()
    with pytest.raises((ValueError, RuntimeError)):
        enc.forward()
    enc.eval()
    with pytest.raises((ValueError, RuntimeError)):
        enc.forward(quantizer_noise_type="none", quantizer_type="hardround")


@pytest.mark.gpu
@pytest.mark.parametrize("path", GOLDEN, ids=[p.stem for p in GOLDEN])
def test_coolchic_encoder_forward_matches_reference(path, gpu, ccmi_lib):
    z = np.load(path)
    enc, meta = _build(z)
    enc = enc.to(gpu)
    raw, rate, add = enc.forward(quantizer_noise_type="none", quantizer_type="hardround",
                                 flag_additional_outputs=True)
    tol = 2e-5 * (1 + float(np.abs(z["syn"]).max()))
    np.testing.assert_allclose(raw[0].cpu().numpy(), z["syn"], atol=tol)
    np.testing.assert_allclose(torch.cat([m.reshape(-1) for m in add["detailed_mu"]]).cpu().numpy(), z["mu"],
                               atol=2e-5 * (1 + float(np.abs(z["mu"]).max())))
    assert rate.shape == (1, z["rate"].size)
    assert abs(float(rate.sum()) - float(z["rate"].sum())) <= 1e-5 * float(z["rate"].sum()) + 1e-3


@pytest.mark.gpu
def test_module_forwards_match_reference(gpu, ccmi_lib):
    from coolchic.enc.component.core.arm import _get_neighbor
    z = np.load([p for p in GOLDEN if "hop_67x101" in p.name][0])
    enc, meta = _build(z)
    enc = enc.to(gpu)
    q = [torch.from_numpy(z[f"q{i}"])[None, None].to(gpu) for i in range(meta["n_grids"])]
    ctx = torch.cat([_get_neighbor(x, 9, enc.non_zero_pixel_ctx_index) for x in q], dim=1)
    mu, scale, log_scale = enc.arm(ctx)
    np.testing.assert_allclose(mu[0].cpu().numpy(), z["mu"], atol=2e-5 * (1 + float(np.abs(z["mu"]).max())))
    ups = enc.upsampling(q)
    np.testing.assert_allclose(ups[0].cpu().numpy(), z["ups"], atol=2e-5 * (1 + float(np.abs(z["ups"]).max())))
    syn = enc.synthesis(ups)
    np.testing.assert_allclose(syn[0].cpu().numpy(), z["syn"], atol=2e-5 * (1 + float(np.abs(z["syn"]).max())))


@pytest.mark.gpu
def test_frame_encoder_yuv420(gpu, ccmi_lib):
    from coolchic.enc.component.frame import FrameEncoder
    z = np.load([p for p in GOLDEN if "mop" in p.name][0])
    enc, meta = _build(z)
    fe = FrameEncoder(enc.param, frame_data_type="yuv420").eval()
    fe.coolchic_encoder = enc
    fe = fe.to(gpu)
    out = fe.forward()
    for k in "yuv":
        assert np.mean(out.decoded_image[k][0, 0].cpu().numpy() != z[f"dec420_{k}"]) < 1e-3


@pytest.mark.gpu
def test_cclib_shim_and_cli_decode(gpu, ccmi_lib, tmp_path):
    from CCLIB.ccdecapi_avx2 import cc_decode_avx2
    from CCLIB.ccdecapi_cpu import cc_decode_cpu
    from coolchic.decode import main
    md5 = json.loads((GDIR / "ref_md5.json").read_text())
    f = sorted((GDIR / "cool").glob("D-*.cool"))[0]
    for fn in (cc_decode_cpu, cc_decode_avx2):
        out = tmp_path / f"{fn.__name__}.yuv"
        assert fn(str(f), str(out), 0, 0, 0) == 0
        assert hashlib.md5(out.read_bytes()).hexdigest() == md5["jvet/" + f.name]["md5"]
    out = tmp_path / "cli.yuv"
    assert main(["-i", str(f), "-o", str(out)]) == 0
    assert hashlib.md5(out.read_bytes()).hexdigest() == md5["jvet/" + f.name]["md5"]
