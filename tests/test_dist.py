"""Image-parallel multi-process path (ccmi.dist) with world_size 2 on the gloo backend (CPU):
sharding covers every image exactly once, records gather to every rank, counters reduce."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch.distributed as dist

    from ccmi import dist as cd
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        images = [f"kodim{i:02d}" for i in range(1, 25)]
        mine = cd.shard(images, rank, world)
        recs = [{"name": n, "rank": rank, "pixels": 768 * 512} for n in mine]
        allrec = cd.gather_records(recs)
        tot = cd.reduce_counters({"pixels": sum(r["pixels"] for r in recs), "frames": len(recs)})
        mx = cd.reduce_counters({"seconds": 1.0 + rank}, op="max")
        q.put((rank, mine, allrec, tot, mx))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_sharding_and_aggregation():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    shards = [set(r[1]) for r in res]
    assert not shards[0] & shards[1]
    assert len(shards[0] | shards[1]) == 24
    for rank, _, allrec, tot, mx in res:
        assert sorted(r["name"] for r in allrec) == sorted(f"kodim{i:02d}" for i in range(1, 25))
        assert tot == {"frames": 24.0, "pixels": 24.0 * 768 * 512}
        assert mx == {"seconds": 2.0}


def test_shard_validates_rank():
    from ccmi import dist as cd
    with pytest.raises(ValueError):
        cd.shard([1, 2], 2, 2)
    assert cd.shard(list(range(5)), 1, 2) == [1, 3]


def test_bench_inputs_come_from_the_product_side():
    """bench.py's timed legs build their frames with ccmi.synthetic (no oracle import); the
    CPU baseline converts the same tensors, which equal the oracle's own random init."""
    from pathlib import Path

    import torch

    import forward_oracle as fo
    from ccmi import synthetic as S
    a = S.random_frame(64, 96, seed=3)
    b = fo.ModelParams.random(64, 96, seed=3)
    for (w1, b1), (w2, b2) in zip(a.arm + a.syn, b.arm + b.syn):
        assert torch.equal(w1, w2) and torch.equal(b1, b2)
    for x, y in zip(a.ups_full() + a.pre_full(), b.ups_full() + b.pre_full()):
        assert torch.equal(x, y)
    src = (Path(__file__).resolve().parents[1] / "bench.py").read_text()
    head = src[:src.index("def _oracle(")]
    assert "forward_oracle" not in head and "sys.path.insert(0, str(ROOT / \"oracle\"))" not in head


def test_bench_reference_comparison_and_proxies():
    import importlib.util
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    spec = importlib.util.spec_from_file_location("bench_mod", root / "bench.py")
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    px = bench.kodak_proxies()
    assert [n for n, _ in px] == [f"kodim{i:02d}" for i in range(1, 25)]
    rows = {(r["seq_name"], r["lmbda"]): r for r in bench.kodak_reference_rows()}
    lms = [0.02, 0.004, 0.001, 0.0004]
    # the reference's own points, fed back as "ours": deltas 0, BD-rate 0
    recs = [{"image": n, "lmbda": lm, "psnr_db": rows[(n, lm)]["psnr_db"], "rate_bpp": rows[(n, lm)]["rate_bpp"]}
            for n in ("kodim01", "kodim07") for lm in lms]
    c = bench.compare_with_reference(recs, lms)
    assert c["bd_rate_images"] == 2 and abs(c["bd_rate_vs_results_tsv_on_proxies_pct_mean"]) < 1e-6
    for v in c["per_lambda"].values():
        assert v["psnr_db_mean"] == v["reference_psnr_db_mean"] and v["images"] == 2


def test_bench_encoder_shards_are_weak_scaled():
    """A rank's encoder work depends on its rank only: the Kodak-24 at REF_LAMBDAS[r % 5] with
    seed r // 5, so rank R of any N-GPU job does the work of --as-rank R; 8 ranks cover the
    reference's 5 operating points with distinct (lambda, seed) pairs."""
    import importlib.util
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    spec = importlib.util.spec_from_file_location("bench_mod2", root / "bench.py")
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    shards = [bench.encoder_shard(r) for r in range(8)]
    assert shards[0] == ([0.001], 0)
    assert len({(lm[0], sd) for lm, sd in shards}) == 8
    assert {lm[0] for lm, _ in shards} == {0.0001, 0.0004, 0.001, 0.004, 0.02}
    assert bench.encoder_shard(3, [0.02, 0.001]) == ([0.02, 0.001], 3)
    # seeds of one (image, lambda) are averaged before the BD fit
    rows = {(r["seq_name"], r["lmbda"]): r for r in bench.kodak_reference_rows()}
    lms = [0.02, 0.004, 0.001, 0.0004]
    recs = [{"image": "kodim05", "lmbda": lm, "psnr_db": rows[("kodim05", lm)]["psnr_db"] + d,
             "rate_bpp": rows[("kodim05", lm)]["rate_bpp"]} for lm in lms for d in (-0.1, 0.1)]
    c = bench.compare_with_reference(recs, None)
    assert c["bd_rate_images"] == 1 and abs(c["bd_rate_vs_results_tsv_on_proxies_pct_mean"]) < 1e-6


@pytest.mark.gpu
def test_bench_two_ranks_gloo_on_one_gpu(tmp_path):
    """bench.py's multi-rank path end to end: torch.distributed.run with 2 ranks on the one
    card (CCMI_BENCH_BACKEND=gloo), tiny legs; the line reports the whole job of both ranks."""
    import json
    import subprocess
    import sys
    from pathlib import Path

    import torch
    assert torch.cuda.device_count() >= 1   # counts without initialising HIP in this process
    root = Path(__file__).resolve().parents[1]
    env = dict(os.environ, CCMI_BENCH_BACKEND="gloo", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(root / "bench.py"), "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--batch", "2", "--hd-steps", "0", "--decode-reps", "1",
           "--hd-decode-reps", "1", "--encode-images", "3", "--encode-scale", "0.002", "--no-cpu-baseline",
           "--no-single-stream"]
    p = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, p.stdout[-2000:]
    r = json.loads(line[0])
    assert r["n_gpus"] == 2 and r["per_gpu"] * 2 == pytest.approx(r["value"], rel=1e-3)
    # weak scaling: every rank decodes its own copy of the stream set, encodes the 3 images
    # at its own lambda (rank 0: 1e-3, rank 1: 4e-4)
    assert r["bitexact_decode"]["frames"] == 30 and r["bitexact_decode"]["bit_exact_vs_reference_md5"]
    assert r["bitexact_decode"]["frames_per_gpu"] == 15
    assert r["bitexact_decode_1080p"]["frames"] == 10
    assert r["bitexact_encode"]["identical_to_shipped_streams"] and r["bitexact_encode"]["frames"] == 60
    e = r["encoder_overfit"]
    assert e["encodes"] == 6 and e["encodes_per_gpu"] == 3
    assert sorted((x["image"], x["lmbda"]) for x in e["records"]) == sorted(
        (f"kodim0{i}", lm) for i in (1, 2, 3) for lm in (0.001, 0.0004))


@pytest.mark.gpu
def test_bench_as_rank_runs_one_shard():
    """--as-rank R --as-world N: rank R's shard of an N-GPU job alone on this GPU (no
    torch.distributed); the encoder leg takes rank R's operating point."""
    import json
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    cmd = [sys.executable, str(root / "bench.py"), "--as-rank", "6", "--as-world", "8", "--steps", "2", "--warmup",
           "1", "--batch", "2", "--hd-steps", "0", "--decode-reps", "1", "--hd-decode-reps", "0", "--encode-images",
           "2", "--encode-scale", "0.002", "--no-cpu-baseline", "--no-single-stream"]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    p = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    r = json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][0])
    assert r["n_gpus"] == 1 and r["as_rank"]["rank"] == 6 and r["as_rank"]["world"] == 8
    assert r["bitexact_decode"]["frames"] == 15 and r["bitexact_decode"]["bit_exact_vs_reference_md5"]
    e = r["encoder_overfit"]
    assert e["shard"] == {"lambdas": [0.0004], "seed": 1, "rank": 6}
    assert sorted(x["image"] for x in e["records"]) == ["kodim01", "kodim02"]
