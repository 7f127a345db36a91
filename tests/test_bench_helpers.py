"""bench.py's measurement arithmetic on CPU: the algorithmic FLOP / byte counts the roofline
fractions divide by, the committed-profile readers (PMC traffic, historical kernel traces and
their source provenance), path B's tail work from stream headers, and the encoder's per-rank
shard.  No GPU: these are the numbers the bench line is built from."""
import json
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "cool-chic_amd"))

bench = pytest.importorskip("bench")


def test_grid_sizes_halve_with_ceil():
    s = bench.sizes(720, 1280)
    assert len(s) == 7 and s[0] == (720, 1280) and s[1] == (360, 640)
    assert s[-1] == (12, 20)  # 720 -> 360 -> 180 -> 90 -> 45 -> 23 -> 12 (ceil halving, as the latent grids)


def test_arm_and_synthesis_flops_per_frame():
    fl = bench.flops_per_frame(720, 1280)
    n_lat = sum(h * w for h, w in bench.sizes(720, 1280))
    assert fl["n_lat"] == n_lat
    # ARM: 2 hidden 16 x 16 layers + the 16 -> 2 output layer per latent, 2 FLOP per MAC
    assert fl["arm"] == 2 * n_lat * (2 * 16 * 16 + 2 * 16)
    # hop synthesis: 7 -> 48 (1x1), 48 -> 3 (1x1), 3 -> 3 (3x3) twice
    npx = 720 * 1280
    assert fl["syn"] == 2 * npx * (7 * 48 + 48 * 3 + 3 * 3 * 9 + 3 * 3 * 9)


def test_fused_bytes_match_the_committed_bench_line():
    """The algorithmic bytes of the fused launch in the committed final bench line are
    bytes_per_frame x frames (what roofline.traffic is compared against)."""
    d = json.loads((ROOT / "profiles/r6z_bench.json").read_text())
    frames = d["config"]["frames_per_step_per_gpu"]
    bench.Pipeline.fold = False
    assert d["roofline"]["algorithmic_bytes_per_launch"] == bench.bytes_per_frame()["decode_fused"] * frames
    assert d["roofline"]["algorithmic_flop_per_launch"] == bench.flops_fused_per_frame(fold=False) * frames


def test_pmc_traffic_reads_the_newest_summary_and_rescales():
    v32, src = bench.pmc_traffic("decode_fused", 32)
    v8, _ = bench.pmc_traffic("decode_fused", 8)
    assert src and src.endswith("pmc.json")
    assert v32 == pytest.approx(4 * v8)
    bench.Pipeline.fold = False
    alg = bench.bytes_per_frame()["decode_fused"] * 32
    assert 0.95 <= v32 / alg <= 1.10  # the XCD-aware window order: HBM ~1.00x the algorithmic bytes
    assert bench.pmc_traffic("no_such_stage", 32) == (None, None)


def test_profile_provenance_detects_changed_sources(tmp_path, monkeypatch):
    import hashlib
    (tmp_path / "profiles").mkdir()
    src = tmp_path / "k.hip"
    src.write_text("kernel v1\n")
    csv_path = "profiles/p.csv"
    (tmp_path / csv_path).write_text("Name,Calls,AverageNs,TotalDurationNs\n")
    side = {"commit": "abc1234", "sha256": {"k.hip": hashlib.sha256(src.read_bytes()).hexdigest()}}
    (tmp_path / (csv_path + ".sources.json")).write_text(json.dumps(side))
    monkeypatch.setattr(bench, "ROOT", tmp_path)
    p = bench.profile_provenance(csv_path)
    assert p["sources_match_current"] is True and p["changed"] == [] and p["measured_at_commit"] == "abc1234"
    src.write_text("kernel v2\n")
    p = bench.profile_provenance(csv_path)
    assert p["sources_match_current"] is False and p["changed"] == ["k.hip"]
    (tmp_path / (csv_path + ".sources.json")).unlink()
    assert bench.profile_provenance(csv_path)["sources_match_current"] is None


def test_train_kernel_rooflines_from_the_committed_trace():
    rows = bench.train_kernel_rooflines()
    names = [r["kernel"] for r in rows]
    assert any(n.startswith("t_head_bwd") for n in names) and any(n.startswith("t_arm16") for n in names)
    for r in rows:
        assert 0.0 < r["frac"] < 1.0 and r["avg_us"] > 0
        assert r["source"]["profile"] == bench.TRAIN_PROFILE
        assert r["achieved"] == pytest.approx(r["flop_per_launch"] / (r["avg_us"] * 1e-6) / 1e12, rel=1e-3)


def test_path_b_tail_work_from_stream_headers():
    from ccmi import encode
    f = sorted((ROOT / "tests/golden/cool").glob("E-*.cool"))[0]
    data = f.read_bytes()
    wk1 = bench.path_b_tail_work([data])
    wk2 = bench.path_b_tail_work([data, data])
    assert wk2["syn_ops"] == 2 * wk1["syn_ops"] and wk2["ups_bytes"] == 2 * wk1["ups_bytes"]
    d = encode.parse(data).desc
    npx = d.h * d.w
    c, ops = d.n_grids, 0
    for i in range(d.n_syn_layers):
        ops += 2 * npx * c * d.syn_out[i] * d.syn_ks[i] ** 2
        c = d.syn_out[i]
    assert wk1["syn_ops"] == ops > 0
    # every pyramid step writes at least the destination level's C + 1 planes
    assert wk1["ups_bytes"] > 4 * npx * 2


def test_encoder_shard_covers_the_reference_lambdas_across_ranks():
    lms = {bench.encoder_shard(r)[0][0] for r in range(5)}
    assert lms == set(bench.REF_LAMBDAS)
    assert bench.encoder_shard(7) == ([bench.REF_LAMBDAS[2]], 1)
    assert bench.encoder_shard(3, [0.02, 0.001]) == ([0.02, 0.001], 3)
