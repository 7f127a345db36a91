"""Path A (float forward) parity.

CPU tests pin the torch-fp32 oracle (oracle/forward_oracle.py) to the golden vectors
produced by the reference implementation (tests/golden/forward_*.npz,
tools/gen_golden_forward.py).  GPU tests run the HIP kernels of libccmi through the
C ABI and compare them with the golden vectors and with the oracle.

Tolerances (fp32 everywhere; summation order differs from PyTorch's conv/linear):
  mu, log_scale, upsampling, synthesis: |err| <= 2e-5 * (1 + |ref|_max)
  rate (bits), per latent: |err| <= 1e-4 + 2.4e-7 * 2**rate + 1.5 * (|dmu| + |dscale| |q - mu| / scale)
               / (scale ln 2): the fp32 cancellation bound of the reference formula
               p = F(q+.5) - F(q-.5) (two CDF values near 0 or 1, one ulp of 1.0 each, over
               p ln 2) plus first-order propagation of the measured mu / scale differences
               (d rate / d mu <= 1 / (scale ln 2)); and |sum err| <= 1e-5 * sum.
  decoded 8-bit image: PSNR difference <= 1e-5 dB (north_star bar); every 8-bit value that
               differs from the reference's is a rounding tie of the reference's float output
               (|255 x - k - 1/2| within 255 x the float tolerance).
  realistic-target PSNR (720p, 1080p): the float synthesis output against the reference's
               output plus N(0, 0.01) noise (a ~40 dB operating point): PSNR within 1e-5 dB.
"""

import numpy as np
import pytest
import torch

import forward_oracle as fo

GOLDEN = fo.golden_files()
assert GOLDEN, "tests/golden/forward_*.npz missing"


def _tol(ref):
    return 2e-5 * (1.0 + float(np.abs(ref).max()))


def _rate_ok(r, ref, mu, mu_ref, sc, sc_ref, q):
    f = lambda a: np.asarray(a, np.float64)
    r, ref, mu, mu_ref, sc, sc_ref, q = map(f, (r, ref, mu, mu_ref, sc, sc_ref, q))
    prop = (np.abs(mu - mu_ref) + np.abs(sc - sc_ref) * np.abs(q - mu_ref) / sc_ref) / (sc_ref * np.log(2))
    tol = 1e-4 + 2.4e-7 * np.exp2(ref) + 1.5 * prop
    err = np.abs(r - ref)
    assert np.all(err <= tol), (float(err.max()), float((err - tol).max()))
    assert abs(r.sum() - ref.sum()) <= 1e-5 * ref.sum() + 1e-3


def _flat_q(qs):
    return np.concatenate([np.asarray(q).reshape(-1) for q in qs])


def _lat(z, mp):
    return [torch.from_numpy(z[f"lat{i}"]) for i in range(mp.n_grids)]


# ----------------------------------------------------------------------------- CPU: oracle pinned


@pytest.mark.parametrize("path", GOLDEN, ids=[p.stem for p in GOLDEN])
def test_oracle_matches_reference_golden(path):
    z = np.load(path)
    mp = fo.ModelParams.from_npz(z)
    r = fo.forward(mp, _lat(z, mp))
    for k in ("mu", "scale", "log_scale", "rate", "ups", "syn"):
        np.testing.assert_allclose(r[k].numpy(), z[k], rtol=0, atol=_tol(z[k]), err_msg=k)
    for i, q in enumerate(r["q"]):
        np.testing.assert_array_equal(q.numpy(), z[f"q{i}"])
    np.testing.assert_allclose(fo.post(r["syn"]).numpy(), z["dec"], atol=1e-6)
    d420 = fo.post(r["syn"], 8, True)
    for k in "yuv":
        np.testing.assert_allclose(d420[k].numpy(), z[f"dec420_{k}"], atol=1e-6)


def test_context_offsets_match_c_decoder_table():
    """The float path's 9x9 mask indices and the C decoder's stride offsets
    (cc-frame-decoder.cpp:111-154) describe the same causal neighbourhoods."""
    c16 = [(-3, 0), (-3, 1), (-2, -2), (-2, -1), (-2, 0), (-2, 1), (-2, 2), (-1, -3), (-1, -2), (-1, -1),
           (-1, 0), (-1, 1), (-1, 2), (0, -3), (0, -2), (0, -1)]
    assert [(k // 9 - 4, k % 9 - 4) for k in fo.CTX_INDEX[16]] == c16
    for d, idx in fo.CTX_INDEX.items():
        assert len(idx) == d and all(k < 40 for k in idx)  # strictly causal


# ----------------------------------------------------------------------------- GPU: HIP kernels


def _hip_forward(mp_list, lat_list, dev, quantize=True, want=("mu", "scale", "log_scale", "rate")):
    from ccmi import forward as F
    mp0 = mp_list[0]
    lat = torch.stack([torch.cat([x.reshape(-1) for x in lats]) for lats in lat_list]).to(dev)
    arm_p = torch.stack([F.pack_arm(mp.arm) for mp in mp_list]).to(dev)
    ups_p = torch.stack([F.pack_ups(mp.ups_full(), mp.pre_full()) for mp in mp_list]).to(dev)
    syn_p = torch.stack([F.pack_syn(mp.syn) for mp in mp_list]).to(dev)
    a = F.arm_forward(lat, mp0.sizes, arm_p, mp0.dim_arm, mp0.n_hidden, mp0.gain, quantize, want)
    u = F.ups_forward(lat, mp0.sizes, ups_p, mp0.ups_k, len(mp0.ups_half), mp0.pre_k, len(mp0.pre_half), mp0.gain,
                      quantize)
    s = F.syn_forward(u, mp0.layers, syn_p)
    torch.cuda.synchronize()
    return a, u, s


@pytest.mark.gpu
@pytest.mark.parametrize("path", GOLDEN, ids=[p.stem for p in GOLDEN])
def test_hip_forward_matches_reference_golden(path, gpu, ccmi_lib):
    from ccmi import forward as F
    z = np.load(path)
    mp = fo.ModelParams.from_npz(z)
    a, u, s = _hip_forward([mp], [_lat(z, mp)], gpu)
    for k in ("mu", "log_scale", "scale"):
        np.testing.assert_allclose(a[k][0].cpu().numpy(), z[k], rtol=0, atol=_tol(z[k]), err_msg=k)
    _rate_ok(a["rate"][0].cpu().numpy(), z["rate"], a["mu"][0].cpu().numpy(), z["mu"],
             a["scale"][0].cpu().numpy(), z["scale"], _flat_q([z[f"q{i}"] for i in range(mp.n_grids)]))
    np.testing.assert_allclose(u[0].cpu().numpy(), z["ups"], rtol=0, atol=_tol(z["ups"]))
    np.testing.assert_allclose(s[0].cpu().numpy(), z["syn"], rtol=0, atol=_tol(z["syn"]))
    dec = F.post_forward(s, 8, False)[0].cpu().numpy()
    assert np.mean(dec != z["dec"]) < 1e-3
    _ties_only(dec, z["syn"], _tol(z["syn"]))
    d420 = F.split_420(F.post_forward(s, 8, True)[0], mp.H, mp.W)
    for k in "yuv":
        assert np.mean(d420[k].cpu().numpy() != z[f"dec420_{k}"]) < 1e-3


def _ties_only(dec, ref_raw, tol, qmax=255.0):
    """Every 8-bit value of `dec` that differs from round(ref_raw) is a rounding tie of the
    reference's float output: |qmax x - k - 1/2| <= qmax * tol (k = floor(qmax x))."""
    ref = np.clip(np.round(ref_raw * qmax) / qmax, 0, 1)
    bad = dec != ref
    if not bad.any():
        return 0
    v = ref_raw[bad].astype(np.float64) * qmax
    dist = np.abs(v - np.floor(v) - 0.5)
    assert np.all(dist <= qmax * tol), (int(bad.sum()), float(dist.max()), qmax * tol)
    return int(bad.sum())


def _psnr(x, t):
    return float(10 * np.log10(1.0 / np.mean((x.astype(np.float64) - t) ** 2)))


@pytest.mark.gpu
@pytest.mark.parametrize("H,W,seed", [(720, 1280, 21), (1080, 1920, 22)])
def test_fused_psnr_realistic_target(H, W, seed, gpu, ccmi_lib):
    """north_star bar at a realistic operating point: the fused kernel's float synthesis output
    and the oracle's, each scored against the oracle's output plus N(0, 0.01) noise (~40 dB),
    agree within 1e-5 dB; the 8-bit frames differ only on rounding ties."""
    mp = fo.ModelParams.random(H, W, seed=seed)
    g = torch.Generator().manual_seed(seed)
    lat = [0.5 * torch.randn(h, w, generator=g) for h, w in mp.sizes]
    ref = fo.forward(mp, lat)["syn"].numpy()
    raw = _fused([mp], [lat], gpu, 0, False)[0].cpu().numpy()
    target = np.clip(ref + np.random.default_rng(seed).normal(0, 0.01, ref.shape), 0, 1)
    clip = lambda a: np.clip(a, 0, 1)  # noqa: E731
    p_ref, p_gpu = _psnr(clip(ref), target), _psnr(clip(raw), target)
    print(f"\n{H}x{W}: PSNR oracle {p_ref:.6f} dB, HIP {p_gpu:.6f} dB, diff {p_gpu - p_ref:.2e} dB, "
          f"max |err| {np.abs(raw - ref).max():.2e}")
    assert 30 < p_ref < 60  # the noise sets ~40 dB; clipping at [0, 1] removes part of it
    assert abs(p_gpu - p_ref) <= 1e-5
    dec = _fused([mp], [lat], gpu, 8, False)[0].cpu().numpy()
    n = _ties_only(dec, ref, _tol(ref))
    print(f"8-bit values off the oracle's: {n} of {dec.size}, all rounding ties")


@pytest.mark.gpu
@pytest.mark.parametrize("H,W,seed", [(720, 1280, 1), (1080, 1920, 11), (37, 53, 2), (1, 1, 3), (2, 130, 4),
                                      (129, 3, 5)])
def test_hip_forward_matches_oracle_random(H, W, seed, gpu, ccmi_lib):
    mp = fo.ModelParams.random(H, W, seed=seed)
    g = torch.Generator().manual_seed(seed)
    lat = [0.5 * torch.randn(h, w, generator=g) for h, w in mp.sizes]
    ref = fo.forward(mp, lat)
    a, u, s = _hip_forward([mp], [lat], gpu)
    np.testing.assert_allclose(a["mu"][0].cpu().numpy(), ref["mu"].numpy(), atol=_tol(ref["mu"].numpy()))
    _rate_ok(a["rate"][0].cpu().numpy(), ref["rate"].numpy(), a["mu"][0].cpu().numpy(), ref["mu"].numpy(),
             a["scale"][0].cpu().numpy(), ref["scale"].numpy(), _flat_q(ref["q"]))
    np.testing.assert_allclose(u[0].cpu().numpy(), ref["ups"].numpy(), atol=_tol(ref["ups"].numpy()))
    np.testing.assert_allclose(s[0].cpu().numpy(), ref["syn"].numpy(), atol=_tol(ref["syn"].numpy()))


def _with_kernel_sizes(mp, K, Kp, seed):
    """mp with random upsampling (K taps, even) and refine (Kp taps, odd) half kernels: the
    reference's --ups_k_size / --ups_preconcat_k_size (upsampling.py:233-292, :110-150)."""
    g = torch.Generator().manual_seed(100 + seed)
    hu, hp = (K + 1) // 2, (Kp + 1) // 2
    mp.ups_half = [0.3 * torch.randn(hu, generator=g) for _ in mp.ups_half]
    mp.pre_half = [0.1 * torch.randn(hp, generator=g) for _ in mp.pre_half]
    mp.ups_k, mp.pre_k = K, Kp
    return mp


@pytest.mark.gpu
@pytest.mark.parametrize("K,Kp", [(4, 1), (4, 3), (6, 5), (8, 1), (8, 9), (10, 7)])
def test_hip_upsampling_kernel_sizes(K, Kp, gpu, ccmi_lib):
    """Every upsampling / refine kernel size the reference's CLI allows (not only the default
    8 / 7): the per-level launch against the oracle, at an odd size that exercises the crop."""
    mp = _with_kernel_sizes(fo.ModelParams.random(45, 83, seed=K + Kp), K, Kp, K * Kp)
    g = torch.Generator().manual_seed(K + Kp)
    lat = [0.5 * torch.randn(h, w, generator=g) for h, w in mp.sizes]
    ref = fo.forward(mp, lat)
    a, u, s = _hip_forward([mp], [lat], gpu)
    np.testing.assert_allclose(u[0].cpu().numpy(), ref["ups"].numpy(), atol=_tol(ref["ups"].numpy()))
    np.testing.assert_allclose(s[0].cpu().numpy(), ref["syn"].numpy(), atol=_tol(ref["syn"].numpy()))


@pytest.mark.gpu
def test_hip_batch_of_frames_with_own_weights(gpu, ccmi_lib):
    """A batch of independent frames, each with its own network, in one launch sequence."""
    mps = [fo.ModelParams.random(96, 160, seed=10 + i) for i in range(3)]
    lats = []
    for i, mp in enumerate(mps):
        g = torch.Generator().manual_seed(100 + i)
        lats.append([0.5 * torch.randn(h, w, generator=g) for h, w in mp.sizes])
    a, u, s = _hip_forward(mps, lats, gpu)
    for i, (mp, lat) in enumerate(zip(mps, lats)):
        ref = fo.forward(mp, lat)
        np.testing.assert_allclose(s[i].cpu().numpy(), ref["syn"].numpy(), atol=_tol(ref["syn"].numpy()))
        _rate_ok(a["rate"][i].cpu().numpy(), ref["rate"].numpy(), a["mu"][i].cpu().numpy(), ref["mu"].numpy(),
                 a["scale"][i].cpu().numpy(), ref["scale"].numpy(), _flat_q(ref["q"]))


@pytest.mark.gpu
@pytest.mark.parametrize("layers", [
    "40-1-linear-relu|3-1-linear-none|3-3-residual-relu|3-3-residual-none",   # hop-like, other width
    "3-1-linear-none|3-3-residual-relu",                                      # single-layer head
    "16-1-linear-relu|3-1-linear-none",                                       # no 3x3
    "9-1-linear-relu|6-3-linear-relu|3-5-linear-none",                        # generic path (ks 5)
    "8-3-linear-relu|3-1-linear-none",                                        # spatial first -> generic
])
def test_hip_synthesis_architectures(layers, gpu, ccmi_lib):
    from ccmi import forward as F
    L = fo.parse_layers(layers)
    mp = fo.ModelParams.random(45, 70, layers=L, seed=7)
    x = torch.randn(7, 45, 70, generator=torch.Generator().manual_seed(3)) * 20
    ref = fo.synthesis(x, L, mp.syn)
    out = F.syn_forward(x.to(gpu), L, F.pack_syn(mp.syn).to(gpu))
    np.testing.assert_allclose(out.cpu().numpy(), ref.numpy(), atol=_tol(ref.numpy()))


@pytest.mark.gpu
def test_hip_rejects_cpu_tensors(ccmi_lib):
    from ccmi import forward as F
    mp = fo.ModelParams.random(8, 8, n_grids=2)
    with pytest.raises(ValueError):
        F.syn_forward(torch.zeros(2, 8, 8), mp.layers, F.pack_syn(mp.syn))


HEADS = (1, 2)  # ccmi.HEAD_VALU, ccmi.HEAD_MFMA: the fused kernel's two 1x1-head forms


def _fused(mps, lats, dev, bitdepth, yuv420, head=0, fold=False):
    from ccmi import forward as F
    mp0 = mps[0]
    lat = torch.stack([torch.cat([x.reshape(-1) for x in l]) for l in lats]).to(dev)
    ups_p = torch.stack([F.pack_ups(mp.ups_full(), mp.pre_full()) for mp in mps]).to(dev)
    syn_p = torch.stack([F.pack_syn(mp.syn) for mp in mps]).to(dev)
    return F.decode_forward(lat, mp0.sizes, ups_p, mp0.ups_k, len(mp0.ups_half), mp0.pre_k, len(mp0.pre_half),
                            mp0.layers, syn_p, mp0.gain, True, bitdepth, yuv420, head, fold)


@pytest.mark.gpu
@pytest.mark.parametrize("head", HEADS)
@pytest.mark.parametrize("path", GOLDEN, ids=[p.stem for p in GOLDEN])
def test_fused_decode_matches_reference_golden(path, head, gpu, ccmi_lib):
    """ccmi_decode_forward_f32 (upsampling + synthesis + post in one kernel) against the
    reference's synthesis output and decoded frames, with either head form (the MFMA form
    applies to the 48-wide 7-grid decoders and falls back to the VALU head otherwise)."""
    from ccmi import forward as F
    z = np.load(path)
    mp = fo.ModelParams.from_npz(z)
    raw = _fused([mp], [_lat(z, mp)], gpu, 0, False, head)
    np.testing.assert_allclose(raw[0].cpu().numpy(), z["syn"], rtol=0, atol=_tol(z["syn"]))
    dec = _fused([mp], [_lat(z, mp)], gpu, 8, False, head)[0].cpu().numpy()
    assert np.mean(dec != z["dec"]) < 1e-3
    _ties_only(dec, z["syn"], _tol(z["syn"]))
    d420 = F.split_420(_fused([mp], [_lat(z, mp)], gpu, 8, True, head)[0], mp.H, mp.W)
    for k in "yuv":
        assert np.mean(d420[k].cpu().numpy() != z[f"dec420_{k}"]) < 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("path", [p for p in GOLDEN if "hop" in p.stem or "arm32" in p.stem], ids=lambda p: p.stem)
def test_unrolled_head_bitwise_generic(path, gpu, ccmi_lib):
    """The unrolled 48-wide head with its scaled ReLU (hidden weights x 2^-32, output weights
    x 2^32, ReLU as the fma clamp; fwd_syn.hip unit()) against the runtime-width head without
    the scaling (CCMI_HEAD_GENERIC), bit for bit, on the reference's 48-wide 7-grid decoder weights
    and a 1080p random hop decoder (both heads sum in the same order)."""
    import ccmi
    z = np.load(path)
    mp = fo.ModelParams.from_npz(z)
    assert mp.layers[0][0] == 48 and mp.n_grids == 7  # the unrolled head's shape
    for bd, yuv in ((0, False), (8, False), (10, True)):
        a = _fused([mp], [_lat(z, mp)], gpu, bd, yuv, ccmi.HEAD_DEFAULT)
        b = _fused([mp], [_lat(z, mp)], gpu, bd, yuv, ccmi.HEAD_GENERIC)
        assert torch.equal(a, b)
    mp = fo.ModelParams.random(1080, 1920, seed=31)
    g = torch.Generator().manual_seed(31)
    lat = [0.5 * torch.randn(h, w, generator=g) for h, w in mp.sizes]
    assert torch.equal(_fused([mp], [lat], gpu, 0, False, ccmi.HEAD_DEFAULT),
                       _fused([mp], [lat], gpu, 0, False, ccmi.HEAD_GENERIC))


@pytest.mark.gpu
@pytest.mark.parametrize("H,W,seed", [(720, 1280, 1), (1080, 1920, 11), (37, 53, 2), (1, 1, 3), (2, 130, 4),
                                      (129, 3, 5), (45, 70, 6), (1365, 2048, 12), (1725, 1145, 13)])
def test_fused_level2_fold_bitwise_unfolded(H, W, seed, gpu, ccmi_lib):
    """The level-2 -> 1 upsampling step evaluated inside the fused kernel (opt-in, stages bit 3,
    for the 7-grid 48-wide-head decoders) against the same kernel reading that level from the
    pyramid's HBM stack: the fold repeats ups_level_fixed's operation
    order, so raw synthesis and post-processed 420 output are identical bit for bit, at sizes
    whose windows clamp at every border (upsampling.py:476-506)."""
    mp = fo.ModelParams.random(H, W, seed=seed)
    assert mp.n_grids == 7 and mp.layers[0][0] == 48
    g = torch.Generator().manual_seed(seed)
    lat = [0.5 * torch.randn(h, w, generator=g) for h, w in mp.sizes]
    for bd, yuv in ((0, False), (8, True)):
        a = _fused([mp], [lat], gpu, bd, yuv, 1, True)
        b = _fused([mp], [lat], gpu, bd, yuv, 1, False)
        assert torch.equal(a, b), (H, W, bd)


@pytest.mark.gpu
def test_fused_level2_fold_batch_own_weights(gpu, ccmi_lib):
    """Per-frame parameter blocks and latents in one folded launch: frame b's output equals a
    batch-of-1 unfolded run of frame b."""
    mps = [fo.ModelParams.random(96, 160, seed=40 + i) for i in range(3)]
    lats = []
    for i, mp in enumerate(mps):
        g = torch.Generator().manual_seed(400 + i)
        lats.append([0.5 * torch.randn(h, w, generator=g) for h, w in mp.sizes])
    both = _fused(mps, lats, gpu, 8, True, 1, True)
    for i in range(3):
        assert torch.equal(both[i], _fused([mps[i]], [lats[i]], gpu, 8, True, 1, False)[0]), i


@pytest.mark.gpu
@pytest.mark.parametrize("H,W,seed,layers", [
    (720, 1280, 1, None), (1080, 1920, 11, None), (37, 53, 2, None), (1, 1, 3, None), (2, 130, 4, None), (129, 3, 5, None),
    (1365, 2048, 12, None), (1725, 1145, 13, None),  # CLIC20-pro-valid geometries (config 5 content)
    (45, 70, 6, "3-1-linear-none|3-3-residual-relu"),
    (45, 70, 7, "16-1-linear-relu|3-1-linear-none"),
    (64, 96, 8, "16-1-linear-relu|4-1-linear-none|4-3-residual-relu|4-3-residual-none|4-3-linear-none"),
])
@pytest.mark.parametrize("head", HEADS)
def test_fused_decode_matches_oracle_random(H, W, seed, layers, head, gpu, ccmi_lib):
    """Fused path vs the staged path's reference (oracle), across sizes whose windows clamp
    at every border, and head-only / single-layer-head / 4-channel synthesis stacks."""
    kw = {} if layers is None else {"layers": fo.parse_layers(layers)}
    mp = fo.ModelParams.random(H, W, seed=seed, **kw)
    g = torch.Generator().manual_seed(seed)
    lat = [0.5 * torch.randn(h, w, generator=g) for h, w in mp.sizes]
    ref = fo.forward(mp, lat)
    raw = _fused([mp], [lat], gpu, 0, False, head)
    np.testing.assert_allclose(raw[0].cpu().numpy(), ref["syn"].numpy(), atol=_tol(ref["syn"].numpy()))
    if mp.layers[-1][0] == 3:
        post = fo.post(ref["syn"], 8)
        dec = _fused([mp], [lat], gpu, 8, False, head)[0].cpu().numpy()
        assert np.mean(dec != post.numpy()) < 1e-3
        _ties_only(dec, ref["syn"].numpy(), _tol(ref["syn"].numpy()))


@pytest.mark.gpu
@pytest.mark.parametrize("head", HEADS)
def test_fused_decode_batch_own_weights_and_two_grids(head, gpu, ccmi_lib):
    mps = [fo.ModelParams.random(96, 160, seed=20 + i) for i in range(3)]
    lats = []
    for i, mp in enumerate(mps):
        g = torch.Generator().manual_seed(200 + i)
        lats.append([0.5 * torch.randn(h, w, generator=g) for h, w in mp.sizes])
    raw = _fused(mps, lats, gpu, 0, False, head)
    for i, (mp, lat) in enumerate(zip(mps, lats)):
        ref = fo.forward(mp, lat)
        np.testing.assert_allclose(raw[i].cpu().numpy(), ref["syn"].numpy(), atol=_tol(ref["syn"].numpy()))
    mp = fo.ModelParams.random(33, 47, n_grids=2, seed=9)   # fused step reads the raw coarsest grid
    g = torch.Generator().manual_seed(9)
    lat = [0.5 * torch.randn(h, w, generator=g) for h, w in mp.sizes]
    ref = fo.forward(mp, lat)
    raw = _fused([mp], [lat], gpu, 0, False)
    np.testing.assert_allclose(raw[0].cpu().numpy(), ref["syn"].numpy(), atol=_tol(ref["syn"].numpy()))
