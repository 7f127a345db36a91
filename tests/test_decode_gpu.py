"""Path B parity: the HIP fixed-point decoder reproduces the reference decoder's output
bytes exactly (md5 of the YUV/PPM written by the reference ccdec, tests/golden/ref_md5.json)
and the C oracle's bytes for the output variants the md5 list does not cover."""
import hashlib
import json
from pathlib import Path

import pytest

GOLDEN = Path(__file__).resolve().parent / "golden"
MD5 = json.loads((GOLDEN / "ref_md5.json").read_text())
FILES = sorted((GOLDEN / "cool").glob("*.cool"))
# CLIC20-pro-valid (BASELINE config 5 content): 5 geometries from 384 x 512 to 1725 x 1145
# (portrait) at lambda 0.02, and one 1360 x 2048 stream at lambda 1e-4 (~1.1 bpp)
CLIC = sorted((GOLDEN / "cool" / "clic").glob("*.cool"))


def _key(f):
    if f.parent.name == "clic":
        return "clic20-pro-valid/" + f.name
    return ("kodak/" if f.name.startswith("kodim") else "jvet/") + f.name


@pytest.mark.gpu
@pytest.mark.parametrize("f", FILES, ids=[f.stem[:40] for f in FILES])
def test_hip_decode_file_bit_exact(f, gpu, ccmi_lib, tmp_path):
    from ccmi import decode
    e = MD5[_key(f)]
    out = tmp_path / ("o" + e["ext"])
    rc = decode.decode_file(str(f), str(out))
    assert rc == 0, decode.lib().ccmi_last_error()
    data = out.read_bytes()
    assert len(data) == e["bytes"]
    assert hashlib.md5(data).hexdigest() == e["md5"]


@pytest.mark.gpu
@pytest.mark.parametrize("f", CLIC, ids=[f.stem[:40] for f in CLIC])
def test_hip_decode_clic_bit_exact(f, gpu, ccmi_lib, tmp_path):
    test_hip_decode_file_bit_exact(f, gpu, ccmi_lib, tmp_path)


@pytest.mark.gpu
def test_hip_decode_batch_caller_workspace(gpu, ccmi_lib):
    """ccmi_decode_batch_ws: the caller sizes and owns the device workspace; same bytes."""
    import torch
    from ccmi import decode
    for fs, yuv in (([f for f in FILES if f.name[:2] in ("E-", "D-")][:8], True), (CLIC, False)):  # CLIC: rgb -> PPM
        data = [f.read_bytes() for f in fs]
        nb = decode.decode_batch_workspace_bytes(data, as_yuv=yuv)
        ws = torch.empty(nb, dtype=torch.uint8, device=gpu)
        outs = decode.decode_batch(data, as_yuv=yuv, workspace=ws)
        for f, o in zip(fs, outs):
            assert hashlib.md5(o).hexdigest() == MD5[_key(f)]["md5"], f.name
        with pytest.raises(decode.CcmiError):  # too small
            decode.decode_batch(data, as_yuv=yuv, workspace=ws[: nb // 2])


def _oracle_stages(oracle_c, data):
    import ctypes as C
    import numpy as np
    from test_encode import _Frame
    fr = _Frame()
    buf = C.create_string_buffer(data, len(data))
    assert oracle_c.cco_decode_frame_mem(buf, len(data), C.byref(fr)) == 0
    try:
        sizes = [(fr.lh[l], fr.lw[l]) for l in range(fr.n_layers)]
        lat = np.concatenate([np.ctypeslib.as_array(fr.lat[l], shape=(h * w,)).copy() for l, (h, w) in enumerate(sizes)])
        n = fr.n_layers * fr.h * fr.w
        syn_in = np.ctypeslib.as_array(fr.syn_in, shape=(n,)).copy().reshape(fr.n_layers, fr.h, fr.w)
        syn_out = np.ctypeslib.as_array(fr.syn_out, shape=(fr.n_out * fr.h * fr.w,)).copy().reshape(fr.n_out, fr.h, fr.w)
        return sizes, lat, syn_in, syn_out
    finally:
        oracle_c.cco_frame_free(C.byref(fr))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["D-BQSquare-lmbda-0001", "kodim01-lmbda-00001", "E-Johnny-lmbda-00004",
                                  "clic/todd-quackenbush-222-lmbda-002"])
def test_integer_stage_entry_points_match_oracle(name, gpu, ccmi_lib, oracle_c):
    """ccmi_decode_weights_i32 -> ccmi_ups_forward_i32 -> ccmi_syn_forward_i32 on the
    decoded latents reproduce the oracle's synthesis input and output planes bit for bit."""
    import numpy as np
    import torch
    from ccmi import decode, encode
    f = [g for g in FILES + CLIC if (g.parent.name + "/" + g.stem if g.parent.name == "clic" else g.stem).startswith(name)][0]
    data = f.read_bytes()
    sizes, lat, syn_in, syn_out = _oracle_stages(oracle_c, data)
    arm, ups, syn = decode.weights_i32(data)
    d = encode.parse(data).desc
    got_in = decode.ups_forward_i32(torch.from_numpy(lat).to(gpu), sizes, torch.from_numpy(ups).to(gpu), d.ups_k,
                                    d.n_ups, d.pre_k, d.n_pre)
    assert np.array_equal(got_in.cpu().numpy(), syn_in)
    layers = [(int(d.syn_out[i]), int(d.syn_ks[i]), int(d.syn_type[i]) // 16 == 1, int(d.syn_type[i]) % 16 == 1)
              for i in range(d.n_syn_layers)]
    if d.n_branches == 1:
        got_out = decode.syn_forward_i32(torch.from_numpy(syn_in).to(gpu), layers, torch.from_numpy(syn).to(gpu))
        assert np.array_equal(got_out.cpu().numpy(), syn_out)


@pytest.mark.gpu
def test_hip_decode_batch_bit_exact(gpu, ccmi_lib):
    """All 720p class-E + 240p class-D streams (mixed sizes / architectures) in one batch."""
    from ccmi import decode
    fs = [f for f in FILES if f.name[:2] in ("E-", "D-")]
    outs = decode.decode_batch([f.read_bytes() for f in fs])
    for f, o in zip(fs, outs):
        assert hashlib.md5(o).hexdigest() == MD5[_key(f)]["md5"], f.name


@pytest.mark.gpu
def test_hip_decode_batch_repeated_streams(gpu, ccmi_lib):
    """Copies of the same streams in one call: the batched decoder tail runs each geometry
    as one group (grid.y = frame); every copy stays bit-exact."""
    from ccmi import decode
    fs = [f for f in FILES if f.name[:2] in ("E-", "D-")][:6]
    outs = decode.decode_batch([f.read_bytes() for f in fs] * 3)
    for f, o in zip(fs * 3, outs):
        assert hashlib.md5(o).hexdigest() == MD5[_key(f)]["md5"], f.name


@pytest.mark.gpu
def test_hip_decode_batch_chunked_mixed_geometries(gpu, ccmi_lib):
    """A batch of >= 64 streams takes the overlapped path (dec_host.cpp: frames in two
    cost-ordered chunks, each chunk's ARM launch and decoder tail on its own HIP stream): the
    committed JVET B / D / E streams (1080p, 240p, 720p; YUV output) twice over in ONE call, and
    the Kodak + CLIC streams (768 x 512 to 2048 x 1365, portrait included; RGB -> PPM) eight
    times over in another, so that both chunks hold several geometries and copies of one stream
    land in either chunk; every output equals the reference decoder's."""
    from ccmi import decode
    jvet = [f for f in FILES if f.name[:2] in ("B-", "D-", "E-")]
    rgb = [f for f in FILES if f.name.startswith("kodim")] + CLIC
    for fs, yuv in ((jvet * 2, True), (rgb * 8, False)):
        assert len(fs) >= 64
        outs = decode.decode_batch([f.read_bytes() for f in fs], as_yuv=yuv)
        for f, o in zip(fs, outs):
            assert hashlib.md5(o).hexdigest() == MD5[_key(f)]["md5"], f.name
        t = decode.last_timing()
        assert t["arm_cabac"] > 0 and t["ups_syn_out"] >= 0


@pytest.mark.gpu
def test_hip_decode_batch_c_abi_pageable_and_views(gpu, ccmi_lib):
    """ccmi_decode_batch itself (library-allocated workspace, caller's pageable output buffers,
    sizes from ccmi_decode_batch_plan) on >= 64 streams, i.e. the two-chunk path with its
    per-chunk downloads; then decode_batch(views=True) (pinned pool, no copies) on the same
    streams, twice, so the second call reuses the pool.  Every output equals the reference's."""
    import ctypes as C
    import torch
    from ccmi import decode
    fs = [f for f in FILES if f.name[:2] in ("D-", "E-")] * 2
    assert len(fs) >= 64
    data = [f.read_bytes() for f in fs]
    n = len(data)
    L = decode._bind()
    bufs = [C.create_string_buffer(d, len(d)) for d in data]
    sp = (C.c_void_p * n)(*[C.cast(b, C.c_void_p) for b in bufs])
    ln = (C.c_size_t * n)(*[len(d) for d in data])
    cap, need = (C.c_size_t * n)(), C.c_size_t(0)
    assert L.ccmi_decode_batch_plan(sp, ln, n, 0, 0, 1, cap, C.byref(need)) == 0
    assert need.value > 0 and all(int(c) == MD5[_key(f)]["bytes"] for f, c in zip(fs, cap))
    outs = [C.create_string_buffer(int(c)) for c in cap]
    op = (C.c_void_p * n)(*[C.cast(o, C.c_void_p) for o in outs])
    got = (C.c_size_t * n)()
    rc = ccmi_lib.ccmi_decode_batch(sp, ln, n, op, cap, got, 0, 0, 1, C.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0, decode.lib().ccmi_last_error()
    for f, o, g in zip(fs, outs, got):
        assert hashlib.md5(o.raw[:g]).hexdigest() == MD5[_key(f)]["md5"], f.name
    for _ in range(2):
        views = decode.decode_batch(data, views=True)
        for f, v in zip(fs, views):
            assert isinstance(v, memoryview) and hashlib.md5(v).hexdigest() == MD5[_key(f)]["md5"], f.name


@pytest.mark.gpu
@pytest.mark.parametrize("bd,chroma,ext", [(10, 420, ".yuv"), (8, 444, ".yuv"), (10, 444, ".yuv"), (8, 0, ".ppm"),
                                           (16, 0, ".ppm")])
def test_hip_output_variants_match_oracle(bd, chroma, ext, gpu, ccmi_lib, oracle_c, tmp_path):
    from ccmi import decode
    f = [f for f in FILES if f.name.startswith("D-")][0]
    a, b = tmp_path / ("g" + ext), tmp_path / ("c" + ext)
    assert decode.decode_file(str(f), str(a), bd, chroma) == 0, decode.lib().ccmi_last_error()
    assert oracle_c.cco_decode_file(str(f).encode(), str(b).encode(), bd, chroma, 0) == 0
    assert a.read_bytes() == b.read_bytes()


@pytest.mark.gpu
def test_hip_decode_rejects_bad_input(gpu, ccmi_lib, tmp_path):
    from ccmi import decode
    f = FILES[0]
    bad = tmp_path / "bad.cool"
    bad.write_bytes(f.read_bytes()[:60])
    assert decode.decode_file(str(bad), str(tmp_path / "o.yuv")) == 1
    assert decode.decode_file(str(tmp_path / "missing.cool"), str(tmp_path / "o.yuv")) == 1
    with pytest.raises(decode.CcmiError):
        decode.decode_batch([f.read_bytes()[:60]])
