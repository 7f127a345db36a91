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


def _key(f):
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
