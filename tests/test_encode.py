"""Path B writer (.cool encoder): byte-exact against the reference's own bitstreams.

The shipped .cool files (tests/golden/cool/, taken from the reference's results/) were
written by the reference encoder (encode.py:221-623 + ccencapi.cpp).  Their latents,
network integers and header fields are recovered (latents by the C oracle's decode,
pinned to the reference decoder by test_oracle_bitstream.py; headers / network integers
by ccmi_cool_parse), then re-encoded here.  Reproducing every substream byte for byte
pins the CABAC encoder, code_val, the flat-block analysis, the Exp-Golomb weight coder
and both header writers.

CPU tests: host CABAC + header writer, with the oracle's ARM parameters (cco_arm_params,
test infrastructure).  GPU tests: the GPU integer ARM (ccmi_arm_forward_i32) against the
oracle, and the full writer ccmi_encode_frame against the shipped files.
"""
import ctypes as C
from pathlib import Path

import numpy as np
import pytest

GOLDEN = Path(__file__).resolve().parent / "golden"
FILES = sorted((GOLDEN / "cool").glob("*.cool"))
SMALL = [f for f in FILES if f.name.startswith(("D-", "kodim"))]
E720 = [f for f in FILES if f.name.startswith("E-")]


class _Frame(C.Structure):
    _fields_ = [("h", C.c_int), ("w", C.c_int), ("frame_data_type", C.c_int), ("bitdepth", C.c_int),
                ("n_layers", C.c_int), ("lh", C.c_int * 8), ("lw", C.c_int * 8),
                ("lat", C.POINTER(C.c_int32) * 8), ("syn_in", C.POINTER(C.c_int32)), ("n_out", C.c_int),
                ("syn_out", C.POINTER(C.c_int32)), ("t_arm", C.c_double), ("t_ups", C.c_double),
                ("t_syn", C.c_double)]


def oracle_latents(oracle_c, data: bytes, with_params: bool = True):
    """Decoded integer latents (and encoder-side mu / log_scale) per grid, from the oracle."""
    fr = _Frame()
    buf = C.create_string_buffer(data, len(data))
    assert oracle_c.cco_decode_frame_mem(buf, len(data), C.byref(fr)) == 0
    try:
        lat = []
        for l in range(fr.n_layers):
            n = fr.lh[l] * fr.lw[l]
            lat.append(np.ctypeslib.as_array(fr.lat[l], shape=(n,)).copy() >> 8)
        mus = lss = None
        if with_params:
            mus = [np.zeros(fr.lh[l] * fr.lw[l], np.int32) for l in range(fr.n_layers)]
            lss = [np.zeros_like(m) for m in mus]
            mp = (C.POINTER(C.c_int32) * 8)(*[m.ctypes.data_as(C.POINTER(C.c_int32)) for m in mus])
            lp = (C.POINTER(C.c_int32) * 8)(*[m.ctypes.data_as(C.POINTER(C.c_int32)) for m in lss])
            assert oracle_c.cco_arm_params(buf, len(data), C.byref(fr), mp, lp) == 0
        sizes = [(fr.lh[l], fr.lw[l]) for l in range(fr.n_layers)]
        return sizes, lat, mus, lss
    finally:
        oracle_c.cco_frame_free(C.byref(fr))


def substreams(frame, data: bytes):
    """(network substreams by slot, latent substreams by grid, header bytes) of a shipped file."""
    d = frame.desc
    hdr = 9 + ((data[9] << 8) | data[10])
    p, nets, lats = hdr, [], []
    for k in range(6):
        nets.append(data[p: p + d.n_bytes_nn[k]])
        p += d.n_bytes_nn[k]
    for l in range(d.n_grids):
        lats.append(data[p: p + d.n_bytes_latent[l]])
        p += d.n_bytes_latent[l]
    assert p == len(data)
    return nets, lats, data[:hdr]


@pytest.fixture(scope="module")
def enc(ccmi_lib):
    from ccmi import encode
    return encode


@pytest.mark.parametrize("f", SMALL + E720[:3], ids=lambda f: f.stem[:36])
def test_latent_substreams_reencode_bit_exact(f, enc, oracle_c):
    data = f.read_bytes()
    fr = enc.parse(data)
    _, lats, _ = substreams(fr, data)
    sizes, lat, mus, lss = oracle_latents(oracle_c, data)
    for l, (h, w) in enumerate(sizes):
        if not lat[l].any():
            assert lats[l] == b""
            continue
        got = enc.code_latent_layer(lat[l], mus[l], lss[l], h, w, fr.desc.hls_sig_blksize)
        assert got == lats[l], f"grid {l} ({h}x{w}): {len(got)} vs {len(lats[l])} bytes"


@pytest.mark.parametrize("f", FILES, ids=lambda f: f.stem[:36])
def test_network_substreams_and_headers_reencode_bit_exact(f, enc):
    data = f.read_bytes()
    fr = enc.parse(data)
    nets, _, hdr = substreams(fr, data)
    d = fr.desc
    for k, name in enumerate(enc.NN_SLOTS):
        if d.nn_len[k] == 0:
            assert nets[k] == b""
            continue
        got, used = enc.code_wb(fr.nn[name], d.expgol_count[k])
        assert used == d.expgol_count[k]
        assert got == nets[k], name
        # and the integers decode back (cc_decode_wb)
        back = enc.decode_wb(got, [(d.nn_len[k], d.expgol_count[k])])[0]
        np.testing.assert_array_equal(back, fr.nn[name])


def test_count_search_never_worse_than_shipped(enc):
    data = (GOLDEN / "cool" / "kodim01-lmbda-0001.cool").read_bytes()
    fr = enc.parse(data)
    nets, _, _ = substreams(fr, data)
    for k, name in enumerate(enc.NN_SLOTS):
        if fr.desc.nn_len[k]:
            got, used = enc.code_wb(fr.nn[name], -1)
            assert 0 <= used <= 12 and len(got) <= len(nets[k])


def test_cclib_ccencapi_surface(enc, tmp_path):
    from CCLIB import ccencapi
    x = [0, 3, -7, 12, 0, 0, -1, 255, -1024]
    p = tmp_path / "w"
    used = ccencapi.cc_code_wb_bac(str(p), x, -1)
    d = ccencapi.cc_decode_wb(str(p))
    assert d.decode_wb_continue(4, used) == x[:4]
    assert d.decode_wb_continue(5, used) == x[4:]
    q = tmp_path / "l"
    h, w = 5, 7
    rng = np.random.default_rng(0)
    lat = rng.integers(-9, 10, h * w).tolist()
    ccencapi.cc_code_latent_layer_bac(str(q), lat, [0] * (h * w), [-256] * (h * w), h, w, 0)
    assert q.stat().st_size > 0


def test_encoder_errors_are_reported(enc):
    import ccmi
    with pytest.raises(ValueError):
        enc.code_latent_layer([1, 2], [0, 0], [0, 0], 3, 3, 0)
    with pytest.raises(ccmi.CcmiError):
        enc.code_latent_layer([], [], [], 0, 0, 0)
    with pytest.raises(ccmi.CcmiError):
        enc.parse(b"\x00\x09" + b"\x00" * 5)


# ---------------------------------------------------------------- GPU: integer ARM + full writer
@pytest.mark.gpu
@pytest.mark.parametrize("f", SMALL[::3] + E720[:2], ids=lambda f: f.stem[:36])
def test_gpu_arm_i32_matches_oracle(f, enc, oracle_c, gpu):
    import torch
    data = f.read_bytes()
    fr = enc.parse(data)
    sizes, lat, mus, lss = oracle_latents(oracle_c, data)
    x = torch.from_numpy(np.concatenate(lat).astype(np.int32)).to(gpu)
    p = torch.from_numpy(fr.arm_params()).to(gpu)
    mu, ls = enc.arm_forward_i32(x, sizes, fr.desc.dim_arm, fr.desc.n_hidden_arm, p)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(mu.cpu().numpy(), np.concatenate(mus))
    np.testing.assert_array_equal(ls.cpu().numpy(), np.concatenate(lss))


@pytest.mark.gpu
@pytest.mark.parametrize("f", FILES, ids=lambda f: f.stem[:36])
def test_gpu_encode_frame_reproduces_shipped_stream(f, enc, oracle_c, gpu):
    import torch
    data = f.read_bytes()
    fr = enc.parse(data)
    sizes, lat, _, _ = oracle_latents(oracle_c, data, with_params=False)
    x = torch.from_numpy(np.concatenate(lat).astype(np.int32)).to(gpu)
    out = enc.encode_frame(fr, x)
    assert out == data
    with pytest.raises(ValueError):   # short latent buffer: refused before any device read
        enc.encode_frame(enc.parse(data), x[:-1].clone())


@pytest.mark.gpu
def test_gpu_encode_decode_round_trip_synthetic(enc, oracle_c, gpu, tmp_path):
    """A synthetic frame (seeded latents, shipped networks) written by the GPU writer:
    the oracle decoder recovers exactly those latents, the GPU decoder's output bytes
    equal the oracle's, and parse -> encode is a fixed point."""
    import torch
    from ccmi import decode
    data = (GOLDEN / "cool" / "D-BQSquare-lmbda-0001_416x240_60p_yuv420_8b.cool").read_bytes()
    fr = enc.parse(data)
    g = torch.Generator().manual_seed(0)
    lat = [torch.round(2.0 * torch.randn(h * w, generator=g)).to(torch.int32) for h, w in fr.grid_sizes]
    lat[-1].zero_()  # an all-zero grid -> empty substream
    x = torch.cat(lat).to(gpu)
    s1 = enc.encode_frame(fr, x, search_counts=True)
    assert fr.desc.n_bytes_latent[len(lat) - 1] == 0
    _, back, _, _ = oracle_latents(oracle_c, s1, with_params=False)
    for a, b in zip(back, lat):
        np.testing.assert_array_equal(a, b.numpy())
    s2 = enc.encode_frame(enc.parse(s1), x)
    assert s1 == s2
    y_gpu, = decode.decode_batch([s1])
    p = tmp_path / "s.cool"
    p.write_bytes(s1)
    assert oracle_c.cco_decode_file(str(p).encode(), str(tmp_path / "o.yuv").encode(), 0, 0, 0) == 0
    assert y_gpu == (tmp_path / "o.yuv").read_bytes()


@pytest.mark.gpu
@pytest.mark.parametrize("f", SMALL[::4] + E720[:1], ids=lambda f: f.stem[:36])
def test_gpu_decode_latents_match_oracle(f, enc, oracle_c, gpu):
    from ccmi import decode
    data = f.read_bytes()
    _, ref, _, _ = oracle_latents(oracle_c, data, with_params=False)
    got = decode.decode_latents(data)
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a, b)
