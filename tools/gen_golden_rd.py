"""Reference rate-distortion fixtures for the encoder (BASELINE configs 1 and 4).

Runs the REFERENCE encoder (imported from /root/reference; build container only, CPU) end
to end on real content and records what its own test() reports, so the GPU encoder can be
held to the same operating points on the GPU box, which has no reference:

    warmup()  (enc/training/warmup.py:22-158)
    train()   per preset phase (enc/training/train.py:57-374)
    quantize_model() after the phase flagged quantize_model (video.py:302-310)
    test()    (enc/training/test.py:370-438) -> psnr_db, rate bpp (latent + NN)

Content
  kodim15_192x128 : test/data/192x128_kodim15.png, the image of the reference's own
                    sanity check (test/sanity_check.py:13), committed as
                    tests/golden/192x128_kodim15.png;
  kodim01_768x512 : results/image/kodak/bitstreams/kodim01-lmbda-00001.cool decoded
                    bit-exactly (the C oracle, md5 = the reference decoder): Kodak geometry
                    (BASELINE config 4's content; the reference's 40.5 dB reconstruction
                    stands in for the original, which is not in the tree);
  kodim01_crop512 : SURVEY §8d config 1: the same, cropped to rows/cols [0, 512).

Schedules: the `debug` preset (preset_cfg/debug.yaml) at 4 lambdas and 2 seeds (the
seed-to-seed spread of the reference itself sets the test tolerance), and the c3x preset
(preset_cfg/c3x.yaml) with every phase / warm-up length scaled by C3X_SCALE.
Architecture: hop (cfg/dec/hop.cfg).

Also written: tests/golden/quantize_ref_<name>.npz -- the inputs and the reference's
quantize_model search (every candidate's loss, the chosen (q_w, q_b) and Exp-Golomb counts
per module) for one trained model, to pin ccmi.quantize.quantize_model; and the CPU
calibration of oracle/train_oracle.py against the reference's own training iteration
(BASELINE.md §3.3).

Usage: python tools/gen_golden_rd.py [debug|c3x|quant|calib|bd|all]
"""

from __future__ import annotations

import copy
import json
import subprocess
import sys
import tempfile
import time
import types
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent))
import gen_golden_forward as G  # noqa: E402  (stubs fvcore / wandb, imports the reference)

_wb = sys.modules["wandb"]
for _n in ("log", "init", "finish"):
    setattr(_wb, _n, lambda *a, **k: None)

import yaml  # noqa: E402

from coolchic.enc.component.coolchic import CoolChicEncoderParameter  # noqa: E402
from coolchic.enc.component.frame import FrameEncoder  # noqa: E402
from coolchic.enc.training import quantizemodel as QM  # noqa: E402
from coolchic.enc.training.test import test  # noqa: E402
from coolchic.enc.training.train import train  # noqa: E402
from coolchic.enc.training.warmup import warmup  # noqa: E402
from coolchic.enc.utils.codingstructure import Frame, FrameData  # noqa: E402
from coolchic.enc.utils.manager import FrameEncoderManager  # noqa: E402
from coolchic.utils.types import PresetConfig  # noqa: E402

ROOT = G.ROOT
sys.path.insert(0, str(ROOT / "cool-chic_amd"))
from ccmi import io as cio  # noqa: E402

REF = Path("/root/reference")
GOLD = ROOT / "tests" / "golden"
HOP = dict(layers=["48-1-linear-relu", "3-1-linear-none", "3-3-residual-relu", "3-3-residual-none"],
           dim_arm=16, n_hidden=2)
# the reference's default decoder (coolchic/utils/types.py:120-143): 40-wide synthesis head,
# ARM "24,2" -- the dim-24 ARM whose training gradients take the 4-rows-up context path
DEFAULT_ARCH = dict(layers=["40-1-linear-relu", "3-1-linear-none", "3-3-residual-relu", "3-3-residual-none"],
                    dim_arm=24, n_hidden=2)
ARCHS = {"hop": HOP, "default": DEFAULT_ARCH}
LAMBDAS = [0.02, 0.004, 0.001, 0.0004]
SEEDS = [0, 1]
C3X_SCALE = 0.1


def load_targets() -> dict:
    """name -> [3, H, W] float in [0, 1] (rgb, 8-bit)."""
    out = {}
    x, bd = cio.read_png(GOLD / "192x128_kodim15.png")
    assert bd == 8
    out["kodim15_192x128"] = x[0].float()  # [3, 128, 192]
    oracle = ROOT / "oracle" / "_build" / "ccdec_oracle"
    if not oracle.exists():
        subprocess.run(["make", "-s", "-C", str(ROOT / "oracle")], check=True)
    def dec(stream: str):
        with tempfile.TemporaryDirectory() as td:
            ppm = Path(td) / "k.ppm"
            subprocess.run([str(oracle), str(GOLD / "cool" / stream), str(ppm)], check=True,
                           stdout=subprocess.DEVNULL)
            k, bd = cio.read_ppm(ppm)
        assert bd == 8
        return k[0].float()

    k = dec("kodim01-lmbda-00001.cool")  # [3, 512, 768]
    out["kodim01_768x512"] = k.contiguous()                      # Kodak geometry (config 4 content)
    out["kodim01_crop512"] = k[:, :512, :512].contiguous()
    # the portrait Kodak geometry (config 4's second geometry batch: kodim04/09/10/17/18/19)
    out["kodim04_512x768"] = dec("kodim04-lmbda-00001.cool").contiguous()  # [3, 768, 512]
    return out


def preset(name: str, scale: float = 1.0) -> PresetConfig:
    with open(REF / "preset_cfg" / f"{name}.yaml") as f:
        d = yaml.safe_load(f)
    if scale != 1.0:
        for ph in d["warmup"]["phases"]:
            tp = ph["training_phase"]
            tp["max_itr"] = max(1, int(tp["max_itr"] * scale))
            tp["freq_valid"] = max(1, int(tp.get("freq_valid", 100) * scale))
        for tp in d["all_phases"]:
            tp["max_itr"] = max(1, int(tp["max_itr"] * scale))
            tp["freq_valid"] = max(1, int(tp.get("freq_valid", 100) * scale))
            tp["patience"] = max(1, int(tp.get("patience", 10000) * scale))
    return PresetConfig(**d)


def make_frame(x: torch.Tensor) -> Frame:
    fr = Frame(coding_order=0, display_order=0, seq_name="rd")
    fr.data = FrameData(8, "rgb", x[None].clone())
    fr.refs_data = []
    return fr


def encode(x: torch.Tensor, preset_cfg: PresetConfig, lmbda: float, seed: int, arch=HOP,
           keep_before_quant: dict | None = None) -> dict:
    """The reference's single-image encoding loop (encode_simpler.py / video.py:224-330)."""
    torch.manual_seed(seed)
    frame = make_frame(x)
    mgr = FrameEncoderManager(preset_config=preset_cfg, lmbda=lmbda)
    H, W = x.shape[-2:]
    p = CoolChicEncoderParameter(layers_synthesis=list(arch["layers"]), n_ft_per_res=[1] * 7,
                                 dim_arm=arch["dim_arm"], n_hidden_layers_arm=arch["n_hidden"])
    p.set_image_size((H, W))
    t0 = time.time()
    cands = [FrameEncoder(coolchic_encoder_param=p, frame_type="I", frame_data_type="rgb", bitdepth=8)
             for _ in range(mgr.preset.warmup.phases[0].candidates)]
    fe = warmup(frame_encoder_manager=mgr, list_candidates=cands, frame=frame, device="cpu")
    phase_its = [int(mgr.iterations_counter)]  # warm-up (every candidate's iterations)
    for ph in mgr.preset.all_phases:
        before = int(mgr.iterations_counter)
        fe = train(frame_encoder=fe, frame=frame, frame_encoder_manager=mgr, start_lr=ph.lr,
                   end_lr=ph.end_lr if ph.end_lr is not None else 1e-5, cosine_scheduling_lr=ph.schedule_lr,
                   max_iterations=ph.max_itr, frequency_validation=ph.freq_valid, patience=ph.patience,
                   optimized_module=ph.optimized_module, quantizer_type=ph.quantizer_type,
                   quantizer_noise_type=ph.quantizer_noise_type, softround_temperature=ph.softround_temperature,
                   noise_parameter=ph.noise_parameter)
        phase_its.append(int(mgr.iterations_counter) - before)
        if ph.quantize_model:
            if keep_before_quant is not None:
                keep_before_quant["fe"] = copy.deepcopy(fe)
                keep_before_quant["frame"] = frame
                keep_before_quant["mgr"] = copy.deepcopy(mgr)
            fe.coolchic_encoder._store_full_precision_param()
            fe = QM.quantize_model(fe, frame, mgr)
    logs = test(fe, frame, mgr)
    dt = time.time() - t0
    return {"psnr_db": float(logs.psnr_db), "rate_bpp": float(logs.total_rate_bpp),
            "rate_latent_bpp": float(logs.rate_latent_bpp), "rate_nn_bpp": float(logs.rate_nn_bpp),
            "loss": float(logs.loss), "iterations": int(mgr.iterations_counter), "phase_iterations": phase_its,
            "seconds": dt,
            "q_step": {k: {kk: float(vv) for kk, vv in v.items()} for k, v in
                       fe.coolchic_encoder.get_network_quantization_step().items()}}


def run_rd(kind: str, out_path: Path, images=None, lambdas=None, seeds=None, scale: float = C3X_SCALE,
           arch: str = "hop"):
    """kind: "debug" (debug preset) or "c3x" (c3x preset, every length x scale); arch: a key
    of ARCHS.  Runs already in out_path are skipped, so an interrupted run resumes."""
    targets = load_targets()
    res = json.loads(out_path.read_text()) if out_path.exists() else {"runs": []}
    done = {(r["image"], r["preset"], r["lmbda"], r["seed"]) for r in res["runs"]}
    seeds = seeds if seeds is not None else (SEEDS if kind == "debug" else [0])
    cfg = preset("debug") if kind == "debug" else preset("c3x", scale)
    tag = "debug" if kind == "debug" else ("c3x" if scale == 1.0 else f"c3x_x{scale}")
    for name, x in targets.items():
        if images is not None and name not in images:
            continue
        if images is None and kind != "debug" and name != "kodim15_192x128":
            continue  # c3x on CPU: the small image only by default (~17 min per point at Kodak size)
        for lm in (lambdas or LAMBDAS):
            for s in seeds:
                key = (name, tag, lm, s)
                if key in done:
                    continue
                r = encode(x, cfg, lm, s, arch=ARCHS[arch])
                r.update(image=name, preset=key[1], lmbda=lm, seed=s, H=int(x.shape[1]), W=int(x.shape[2]),
                         arch=arch)
                print(json.dumps(r), flush=True)
                res["runs"].append(r)
                out_path.write_text(json.dumps(res, indent=1))


class _LossRecorder:
    """Wraps quantizemodel.loss_function to record every candidate's loss with the
    (module, q_w, q_b) being tried (quantizemodel.py:183-263)."""

    def __init__(self, fe):
        self.fe, self.rows, self.orig = fe, [], QM.loss_function

    def __call__(self, *a, **k):
        out = self.orig(*a, **k)
        cc = self.fe.coolchic_encoder
        self.rows.append((dict((m, dict(v)) for m, v in cc.nn_q_step.items()), float(out.loss)))
        return out


def gen_quant():
    """Reference quantize_model on a model trained with the debug preset (kodim15, lambda
    1e-3): inputs and the whole candidate loss table."""
    targets = load_targets()
    x = targets["kodim15_192x128"]
    keep = {}
    encode(x, preset("debug"), 1e-3, 0, keep_before_quant=keep)
    fe, frame, mgr = keep["fe"], keep["frame"], keep["mgr"]
    cc = fe.coolchic_encoder
    z = {f"p/{k}": v.detach().numpy().copy() for k, v in cc.named_parameters()}
    z["target"] = x.numpy()
    fe.coolchic_encoder._store_full_precision_param()
    rec = _LossRecorder(fe)
    QM.loss_function = rec
    try:
        fe = QM.quantize_model(fe, frame, mgr)
    finally:
        QM.loss_function = rec.orig
    chosen = fe.coolchic_encoder.get_network_quantization_step()
    counts = fe.coolchic_encoder.nn_expgol_cnt
    # rows arrive module by module in sorted order (quantizemodel.py:181); a module's block
    # ends after its last (q_w, q_b) pair in itertools.product order, and candidates with
    # |q| > 65535 are skipped: split the rows where the searched module's own step pair
    # (the one that changes from row to row) returns to its first value
    mods = sorted(chosen.keys())
    rows_by_mod, cur = {m: [] for m in mods}, 0
    for qs, loss in rec.rows:
        while True:
            m = mods[cur]
            q = (float(qs[m]["weight"]), float(qs[m]["bias"]))
            prev = rows_by_mod[m][-1][:2] if rows_by_mod[m] else None
            last = (float(QM.POSSIBLE_Q_STEP[m]["weight"][-1]), float(QM.POSSIBLE_Q_STEP[m]["bias"][-1]))
            if prev is not None and prev == last:
                cur += 1  # the previous module's block is complete
                continue
            rows_by_mod[m].append((q[0], q[1], loss))
            break
    for m in mods:
        arr = np.array(rows_by_mod[m], dtype=np.float64).reshape(-1, 3)
        z[f"table/{m}"] = arr
        z[f"chosen/{m}"] = np.array([chosen[m]["weight"], chosen[m]["bias"]], dtype=np.float64)
        z[f"expgol/{m}"] = np.array([counts[m]["weight"], counts[m]["bias"]], dtype=np.int64)
    z["meta"] = repr({"H": int(x.shape[1]), "W": int(x.shape[2]), "lmbda": 1e-3, "arch": "hop", "dim_arm": 16,
                      "n_hidden_arm": 2, "n_grids": 7, "layers": "|".join(HOP["layers"]), "encoder_gain": 16,
                      "frame_data_type": "rgb", "bitdepth": 8})
    np.savez_compressed(GOLD / "quantize_ref_kodim15_hop.npz", **z)
    print("quantize fixture:", {m: z[f"chosen/{m}"].tolist() for m in mods})


def gen_calib(out_path: Path):
    """Per-iteration CPU time of the reference's training step vs oracle/train_oracle.py on
    the same size, same threads (BASELINE.md §3.3 calibration)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import forward_oracle as fo
    import train_oracle as to
    from coolchic.enc.training.loss import loss_function
    res = {"threads": torch.get_num_threads()}
    for H, W in ((512, 512), (512, 768)):
        x = torch.rand(3, H, W, generator=torch.Generator().manual_seed(0))
        frame = make_frame(x)
        p = CoolChicEncoderParameter(layers_synthesis=list(HOP["layers"]), n_ft_per_res=[1] * 7, dim_arm=16,
                                     n_hidden_layers_arm=2)
        p.set_image_size((H, W))
        torch.manual_seed(0)
        fe = FrameEncoder(coolchic_encoder_param=p, frame_type="I", frame_data_type="rgb", bitdepth=8)
        fe.set_to_train()
        opt = torch.optim.Adam(fe.parameters(), lr=1e-2)
        ts = []
        for it in range(6):
            t0 = time.perf_counter()
            for q in fe.parameters():
                q.grad = None
            out = fe.forward(reference_frames=[], quantizer_noise_type="kumaraswamy", quantizer_type="softround",
                             soft_round_temperature=torch.tensor(0.3), noise_parameter=torch.tensor(1.0))
            lo = loss_function(out.decoded_image, out.rate, frame.data.data, lmbda=1e-3, rate_mlp_bit=0.0,
                               compute_logs=False)
            lo.loss.backward()
            torch.nn.utils.clip_grad_norm_(list(fe.parameters()), 1e-1)
            opt.step()
            ts.append(time.perf_counter() - t0)
        ref_s = float(np.median(ts[1:]))
        mp = fo.ModelParams.random(H, W, seed=0)
        g = torch.Generator().manual_seed(0)
        st = to.TrainState(mp, [0.01 * torch.randn(h, w, generator=g) for h, w in mp.sizes])
        opt = to.Adam(st.params(), 1e-2)
        ts = []
        for it in range(6):
            t0 = time.perf_counter()
            to.grads(st, x, "softround", 0.3, 1e-3, False)
            opt.step()
            ts.append(time.perf_counter() - t0)
        port_s = float(np.median(ts[1:]))
        res[f"{H}x{W}"] = {"reference_s_per_iter": ref_s, "port_s_per_iter": port_s, "port_over_reference": port_s / ref_s}
        print(H, W, res[f"{H}x{W}"], flush=True)
    out_path.write_text(json.dumps(res, indent=1))


def gen_calib_forward(out_path: Path, threads: int):
    """Per-frame CPU time of the reference's eval forward (FrameEncoder.forward after
    set_to_eval(), the call of test.py:402-411 under test()'s no_grad: quantize, ARM + rate,
    upsampling, synthesis, 8-bit rounding, 444 -> 420) against oracle/forward_oracle.py's
    forward + post (bench.py's cpu_baseline) on the same 1280x720 hop frame, same threads.
    Merged into out_path under "forward_720p" (BASELINE.md §3.3 calibration)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import forward_oracle as fo
    torch.set_num_threads(threads)
    H, W = 720, 1280
    p = CoolChicEncoderParameter(layers_synthesis=list(HOP["layers"]), n_ft_per_res=[1] * 7, dim_arm=16,
                                 n_hidden_layers_arm=2)
    p.set_image_size((H, W))
    torch.manual_seed(0)
    fe = FrameEncoder(coolchic_encoder_param=p, frame_type="I", frame_data_type="yuv420", bitdepth=8)
    fe.set_to_eval()
    ts = []
    with torch.no_grad():
        for _ in range(4):
            t0 = time.perf_counter()
            fe.forward(reference_frames=[], quantizer_noise_type="none", quantizer_type="hardround", AC_MAX_VAL=-1,
                       flag_additional_outputs=True)
            ts.append(time.perf_counter() - t0)
    ref_s = float(np.median(ts[1:]))
    mp = fo.ModelParams.random(H, W, seed=0)
    g = torch.Generator().manual_seed(0)
    lats = [0.5 * torch.randn(h, w, generator=g) for h, w in mp.sizes]
    ts = []
    for _ in range(4):
        t0 = time.perf_counter()
        r = fo.forward(mp, lats)
        fo.post(r["syn"], 8, True)
        ts.append(time.perf_counter() - t0)
    port_s = float(np.median(ts[1:]))
    res = json.loads(out_path.read_text()) if out_path.exists() else {}
    res["forward_720p"] = {"threads": threads, "reference_s_per_frame": ref_s, "port_s_per_frame": port_s,
                           "port_over_reference": port_s / ref_s,
                           "what": "reference FrameEncoder.forward eval (hardround, yuv420 8-bit) vs "
                                   "oracle/forward_oracle.py forward + post, one 1280x720 hop frame, median of 3"}
    print(res["forward_720p"], flush=True)
    out_path.write_text(json.dumps(res, indent=1))


def gen_bd(out_path: Path):
    """Golden vectors for the BD-rate restatement: the reference's own BD_RATE / BD_PSNR
    (coolchic/utils/bjontegaard_metric.py) on seeded curve pairs, both integration modes."""
    sys.path.insert(0, str(REF / "coolchic" / "utils"))
    import bjontegaard_metric as bj
    g = np.random.default_rng(0)
    cases = []
    for k in range(6):
        n = 4 + k % 3
        r1 = np.sort(g.uniform(0.05, 2.0, n))
        p1 = 30 + 6 * np.log(r1) + g.normal(0, 0.1, n)
        r2 = r1 * g.uniform(0.8, 1.25) * np.exp(g.normal(0, 0.03, n))
        p2 = 30 + 6 * np.log(r1) + g.normal(0, 0.2, n) + g.uniform(-0.5, 0.5)
        case = {"R1": r1.tolist(), "PSNR1": p1.tolist(), "R2": r2.tolist(), "PSNR2": p2.tolist()}
        for pw in (0, 1):
            case[f"bd_rate_pw{pw}"] = float(bj.BD_RATE(r1, p1, r2, p2, piecewise=pw))
            case[f"bd_psnr_pw{pw}"] = float(bj.BD_PSNR(r1, p1, r2, p2, piecewise=pw))
        cases.append(case)
    out_path.write_text(json.dumps({"source": "coolchic/utils/bjontegaard_metric.py (reference tree)", "cases": cases},
                                   indent=1))
    print("bd fixtures:", len(cases))


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    if what == "one":
        # one (image, preset scale, lambda, seed) point into its own file, so several can run
        # side by side: python tools/gen_golden_rd.py one IMAGE SCALE LAMBDA SEED THREADS OUT [ARCH]
        # (SEED may be a comma list, run in order into the same file)
        img, sc, lm, sd, th, out = sys.argv[2:8]
        arch = sys.argv[8] if len(sys.argv) > 8 else "hop"
        torch.set_num_threads(int(th))
        run_rd("c3x", Path(out), images=[img], lambdas=[float(x) for x in lm.split(",")],
               seeds=[int(x) for x in sd.split(",")], scale=float(sc), arch=arch)
        sys.exit(0)
    if what in ("bd", "all"):
        gen_bd(GOLD / "bd_reference.json")
    if what in ("debug", "all"):
        run_rd("debug", GOLD / "rd_reference_debug.json")
    if what == "debug_seeds":
        # more reference seeds for the debug preset into their own file (merged by hand):
        # python tools/gen_golden_rd.py debug_seeds IMAGE SEEDS THREADS OUT ARCH
        img, sd, th, out, arch = sys.argv[2:7]
        torch.set_num_threads(int(th))
        run_rd("debug", Path(out), images=[img], seeds=[int(x) for x in sd.split(",")], arch=arch)
        sys.exit(0)
    if what == "debug_default":  # the reference's default decoder (arm 24,2; 40-wide head)
        if len(sys.argv) > 2:
            torch.set_num_threads(int(sys.argv[2]))
        run_rd("debug", GOLD / "rd_reference_debug_default.json", images=["kodim15_192x128", "kodim01_768x512"],
               arch="default")
    if what in ("quant", "all"):
        gen_quant()
    if what in ("c3x", "all"):
        run_rd("c3x", GOLD / "rd_reference_c3x.json")
    if what in ("calib", "all"):
        gen_calib(GOLD / "cpu_calibration.json")
    if what == "calib_forward":  # python tools/gen_golden_rd.py calib_forward THREADS
        gen_calib_forward(GOLD / "cpu_calibration.json", int(sys.argv[2]) if len(sys.argv) > 2 else 2)
