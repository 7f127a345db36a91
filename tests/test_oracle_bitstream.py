"""The C restatement of the fixed-point decoder (oracle/) reproduces the reference
decoder's outputs on the shipped .cool bitstreams (md5 of the YUV/PPM bytes written
by the reference ccdec, tests/golden/ref_md5.json; tools/make_ref_md5.py)."""
import hashlib
import json
from pathlib import Path

import pytest

GOLDEN = Path(__file__).resolve().parent / "golden"
MD5 = json.loads((GOLDEN / "ref_md5.json").read_text())
FILES = sorted((GOLDEN / "cool").glob("*.cool"))


def _key(f):
    ds = "kodak" if f.name.startswith("kodim") else "jvet"
    return f"{ds}/{f.name}"


@pytest.mark.parametrize("f", FILES, ids=[f.stem[:40] for f in FILES])
def test_oracle_bit_exact_vs_reference(f, oracle_c, tmp_path):
    e = MD5[_key(f)]
    out = tmp_path / ("o" + e["ext"])
    assert oracle_c.cco_decode_file(str(f).encode(), str(out).encode(), 0, 0, 0) == 0
    data = out.read_bytes()
    assert len(data) == e["bytes"]
    assert hashlib.md5(data).hexdigest() == e["md5"]


def test_oracle_rejects_truncated_stream(oracle_c, tmp_path):
    f = FILES[0]
    bad = tmp_path / "bad.cool"
    bad.write_bytes(f.read_bytes()[:50])
    assert oracle_c.cco_decode_file(str(bad).encode(), str(tmp_path / "o.yuv").encode(), 0, 0, 0) != 0
