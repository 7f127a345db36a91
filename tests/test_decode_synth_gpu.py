"""Path B parity where no shipped stream goes: the ARM decode kernels' 32-bit forms.

Every committed .cool stream decodes with |q| < 2^14 and ARM weights < 2^23, so the
decoder's 24-bit fast forms carry all of them; tests/synth_streams.py builds streams that
force each wider form of each kernel (the chain kernel's mid-row switch at |q| > 16383 and
its helper's 32-bit preG, the all-32-bit form for weights >= 2^23, the speculative and
one-latent kernels' 32-bit layer 0 at |q| >= 2^15; d = 8 / 16 / 24 / 32, 0-3 hidden layers,
three block-map modes).  Each stream, written by the GPU writer, must
  * equal the committed fixture byte for byte (the writer is deterministic),
  * decode on the GPU to the latents it was written from, and to the oracle's latents,
  * decode to the reference decoder's md5 (tests/golden/synth_md5.json, from
    oracle/_ref/ccdec_ref run on the committed fixture) and to the oracle's bytes,
  * report through ccmi_decode_last_arm_flags exactly the multiply forms the case targets.
The reference's int32 ARM: coolchic/cpp/arm_cpu.cpp:65-95 (one form for every value).
CPU part: the oracle (test infrastructure) on the committed fixtures against the reference
md5 and the case latents.
"""
import hashlib
import json

import numpy as np
import pytest

import synth_streams as S

MD5 = json.loads((S.GOLDEN / "synth_md5.json").read_text())["streams"] if (S.GOLDEN / "synth_md5.json").exists() else {}
NAMES = list(S.CASES)


@pytest.fixture(scope="module")
def enc(ccmi_lib):
    from ccmi import encode
    return encode


def _oracle_yuv(oracle_c, data: bytes, tmp_path) -> bytes:
    p = tmp_path / "s.cool"
    p.write_bytes(data)
    assert oracle_c.cco_decode_file(str(p).encode(), str(tmp_path / "o.yuv").encode(), 0, 0, 0) == 0
    return (tmp_path / "o.yuv").read_bytes()


@pytest.mark.parametrize("name", NAMES)
def test_oracle_decodes_synthetic_fixture_to_reference_md5(name, enc, oracle_c, tmp_path):
    from test_encode import oracle_latents
    f = S.SYNTH / f"{name}.cool"
    if not f.exists() or name not in MD5:
        pytest.skip("fixture not generated yet (tools/gen_synth_streams.py)")
    data = f.read_bytes()
    y = _oracle_yuv(oracle_c, data, tmp_path)
    assert hashlib.md5(y).hexdigest() == MD5[name]["md5"] == MD5[name]["md5_avx2"]
    _, lat = S.build(name, enc)
    _, back, _, _ = oracle_latents(oracle_c, data, with_params=False)
    for a, b in zip(back, lat):
        np.testing.assert_array_equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_decode_synthetic_stream_wide_forms(name, enc, oracle_c, gpu, tmp_path):
    import torch
    from ccmi import decode
    from test_encode import oracle_latents
    fr, lat = S.build(name, enc)
    data = enc.encode_frame(fr, torch.from_numpy(np.concatenate(lat)).to(gpu), search_counts=True)
    f = S.SYNTH / f"{name}.cool"
    if f.exists():
        assert data == f.read_bytes(), "the GPU writer no longer reproduces the committed stream"
    got = decode.decode_latents(data)
    flags = decode.last_arm_flags()
    _, ref, _, _ = oracle_latents(oracle_c, data, with_params=False)
    for g, r, a in zip(got, ref, lat):
        np.testing.assert_array_equal(r, a)
        np.testing.assert_array_equal(g, a)
    assert flags == [S.CASES[name][5]], (S.kernel_of(name), flags)
    y, = decode.decode_batch([data])
    assert y == _oracle_yuv(oracle_c, data, tmp_path)
    if name in MD5:
        assert hashlib.md5(y).hexdigest() == MD5[name]["md5"]


@pytest.mark.gpu
def test_gpu_synthetic_streams_in_one_batch(enc, gpu, tmp_path, oracle_c):
    """All cases in one ccmi_decode_batch (one launch per (d, nh) group, mixed forms side by
    side in one launch): same bytes, per-stream flags in input order."""
    import torch
    from ccmi import decode
    data = []
    for name in NAMES:
        fr, lat = S.build(name, enc)
        data.append(enc.encode_frame(fr, torch.from_numpy(np.concatenate(lat)).to(gpu), search_counts=True))
    outs = decode.decode_batch(data)
    assert decode.last_arm_flags() == [S.CASES[n][5] for n in NAMES]
    for name, d, o in zip(NAMES, data, outs):
        assert o == _oracle_yuv(oracle_c, d, tmp_path), name


@pytest.mark.gpu
def test_gpu_chain_wait_limit_is_an_error(enc, gpu, monkeypatch):
    """A two-wave hand-off that gives up (forced: CCMI_DEC_SPIN_CAP=0, every wait gives up at
    once) is reported -- the call fails, the stream's flags carry TIMEOUT -- instead of
    returning a decode built from unsynchronised data; the next call with the default limit
    is clean."""
    from ccmi import decode
    data = (S.GOLDEN / "cool" / "D-BQSquare-lmbda-0001_416x240_60p_yuv420_8b.cool").read_bytes()
    monkeypatch.setenv("CCMI_DEC_SPIN_CAP", "0")
    with pytest.raises(decode.CcmiError, match="hand-off"):
        decode.decode_batch([data])
    assert decode.last_arm_flags()[0] & decode.ARM_FLAG_TIMEOUT
    monkeypatch.delenv("CCMI_DEC_SPIN_CAP")
    decode.decode_batch([data])
    assert decode.last_arm_flags() == [0]
