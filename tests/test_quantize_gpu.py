"""quantize_model (ccmi.quantize, batched GPU search) against the reference's own search
(enc/training/quantizemodel.py:119-309) on the same trained model.

tests/golden/quantize_ref_kodim15_hop.npz (tools/gen_golden_rd.py quant) holds a hop model the
reference trained on kodim15 with the debug preset (lambda 1e-3), the image, and the loss of
EVERY (q_w, q_b) candidate the reference tried per module, with its choice and Exp-Golomb counts.
The GPU search drops the loss terms that do not depend on the module under search, so its
candidate losses must equal the reference's up to one constant per module; the chosen steps
must be the reference's, or tie with them within float noise."""
import ast
from pathlib import Path

import numpy as np
import pytest
import torch

GOLDEN = Path(__file__).resolve().parent / "golden"
pytestmark = pytest.mark.gpu


def test_quantize_model_matches_reference_search(gpu):
    import forward_oracle as fo
    from ccmi import quantize as Q
    from ccmi import train as T
    z = np.load(GOLDEN / "quantize_ref_kodim15_hop.npz")
    meta = ast.literal_eval(str(z["meta"]))
    mp = fo.ModelParams.from_npz(z)
    arch = T.Arch(meta["H"], meta["W"], dim_arm=mp.dim_arm, n_hidden=mp.n_hidden, layers=tuple(mp.layers),
                  n_grids=mp.n_grids, gain=mp.gain)
    params = T.pack_params(mp.arm, mp.ups_half, mp.pre_half, mp.syn)
    lat = torch.cat([torch.from_numpy(z[f"p/latent_grids.{i}.data"]).reshape(-1) for i in range(mp.n_grids)])
    tgt = torch.from_numpy(z["target"]).reshape(-1).float()
    qm = Q.quantize_model(arch, lat.to(gpu), params.to(gpu), tgt.to(gpu), meta["lmbda"], yuv420=False, bitdepth=8)
    for m in ("arm", "synthesis", "upsampling"):
        ref = z[f"table/{m}"]
        got = np.array(qm.table[m], dtype=np.float64)
        # same candidates, same order (skips of |q| > 65535 included)
        np.testing.assert_array_equal(got[:, :2], ref[:, :2], err_msg=m)
        off = got[:, 2] - ref[:, 2]
        spread = float(np.abs(off - np.median(off)).max())
        print(f"\n{m}: {len(ref)} candidates, loss offset spread {spread:.3g} (loss ~{ref[:, 2].min():.4g}); "
              f"chosen ref {tuple(z[f'chosen/{m}'])} gpu {qm.q_step[m]}")
        assert spread <= 1e-6 * float(np.abs(ref[:, 2]).max()), (m, spread)
        chosen = tuple(float(v) for v in z[f"chosen/{m}"])
        if tuple(qm.q_step[m]) != chosen:  # only a float-noise tie may flip the choice
            row = ref[(ref[:, 0] == qm.q_step[m][0]) & (ref[:, 1] == qm.q_step[m][1])]
            assert row[0, 2] - ref[:, 2].min() <= 2 * spread + 1e-12, (m, qm.q_step[m], chosen)
        else:
            assert tuple(qm.expgol[m]) == tuple(int(v) for v in z[f"expgol/{m}"]), m


def test_train_and_eval_rate_forms_agree(gpu):
    """The Laplace rate (arm.py:355-370, coolchic.py:419-424) exists in two fp32 forms: the
    training step (train.hip arm_rate: expm1f and an IEEE division, as torch evaluates it) and
    the eval forward that quantize_model / test() use (fwd_arm.hip laplace_cdf: v_exp_f32 - 1
    and one v_rcp_f32 shared by both CDF terms, 5 % faster).  On the reference-trained model
    of the quantize fixture, the two total rates (hard-rounded latents, the same network)
    must agree within 2e-6 relative -- well inside the 1e-5 rate tolerance of the parity
    tests and far below what moves a quantize_model choice (the loss-offset spread above is
    1e-6 of the loss); the measured difference is printed."""
    import forward_oracle as fo
    from ccmi import quantize as Q
    from ccmi import train as T
    z = np.load(GOLDEN / "quantize_ref_kodim15_hop.npz")
    meta = ast.literal_eval(str(z["meta"]))
    mp = fo.ModelParams.from_npz(z)
    arch = T.Arch(meta["H"], meta["W"], dim_arm=mp.dim_arm, n_hidden=mp.n_hidden, layers=tuple(mp.layers),
                  n_grids=mp.n_grids, gain=mp.gain)
    params = T.pack_params(mp.arm, mp.ups_half, mp.pre_half, mp.syn).to(gpu)
    lat = torch.cat([torch.from_numpy(z[f"p/latent_grids.{i}.data"]).reshape(-1) for i in range(mp.n_grids)]).to(gpu)
    tgt = torch.from_numpy(z["target"]).reshape(-1).float().to(gpu)
    _, rate_eval = Q.evaluate(arch, lat, params, tgt, yuv420=False, bitdepth=8)
    of = T.Overfitter(arch, lat[None], params[None], tgt[None], yuv420=False)
    rate_train = float(of.validate(meta["lmbda"])[0, 2])
    rel = abs(rate_eval - rate_train) / rate_train
    print(f"\nrate: eval form {rate_eval:.4f} bits, train form {rate_train:.4f} bits, relative difference {rel:.3g}")
    assert rel <= 2e-6, rel
