"""Rate-distortion reporting on the CPU: the BD-rate / BD-PSNR restatement (ccmi.rd) against
the reference's own bjontegaard_metric.py outputs (tests/golden/bd_reference.json, written by
tools/gen_golden_rd.py), and the shape of the reference R-D fixtures the GPU test uses."""
import json
from pathlib import Path

import numpy as np
import pytest

GOLDEN = Path(__file__).resolve().parent / "golden"


def _cases():
    return json.loads((GOLDEN / "bd_reference.json").read_text())["cases"]


@pytest.mark.parametrize("pw", [0, 1])
def test_bd_rate_matches_reference(pw):
    from ccmi import rd
    for c in _cases():
        got = rd.bd_rate(c["R1"], c["PSNR1"], c["R2"], c["PSNR2"], piecewise=pw)
        np.testing.assert_allclose(got, c[f"bd_rate_pw{pw}"], rtol=1e-9, atol=1e-9)
        got = rd.bd_psnr(c["R1"], c["PSNR1"], c["R2"], c["PSNR2"], piecewise=pw)
        np.testing.assert_allclose(got, c[f"bd_psnr_pw{pw}"], rtol=1e-9, atol=1e-9)


def test_bd_rate_identities():
    from ccmi import rd
    r = [0.1, 0.3, 0.8, 1.6]
    p = [27.0, 30.5, 33.8, 36.9]
    assert abs(rd.bd_rate(r, p, r, p)) < 1e-9
    assert abs(rd.bd_rate(r, p, [x * 1.1 for x in r], p) - 10.0) < 1e-6   # 10 % more bits everywhere
    assert abs(rd.bd_psnr(r, p, r, [x + 0.5 for x in p]) - 0.5) < 1e-9


def test_reference_rd_fixtures_are_complete():
    d = json.loads((GOLDEN / "rd_reference_debug.json").read_text())
    keys = {(r["image"], r["lmbda"], r["seed"]) for r in d["runs"]}
    for img in ("kodim15_192x128", "kodim01_768x512", "kodim01_crop512"):
        for lm in (0.02, 0.004, 0.001, 0.0004):
            for s in (0, 1):
                assert (img, lm, s) in keys
    for r in d["runs"]:
        assert r["iterations"] == 120          # debug preset: 3 x 10 + 2 x 10 warm-up (counted per
        assert 15 < r["psnr_db"] < 45           # candidate as the reference does) + 50 + 10 + 10
        assert abs(r["rate_bpp"] - r["rate_latent_bpp"] - r["rate_nn_bpp"]) < 1e-6
