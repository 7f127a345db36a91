"""Benchmark: decoded Mpixel/s (whole job, all GPUs; `per_gpu` alongside) of Cool-chic's
forward/decode hot path (ARM probability model + rate, upsampling, synthesis, 420
post-processing) on synthetic 1280x720 frames, hop/c3x decoder architecture, float32.

A step = one batch of `--batch` independent 720p frames (each with its own network,
as Cool-chic overfits one per image) pushed through the libccmi HIP kernels, inputs
resident in HBM.  With N GPUs (torchrun, one process per GPU) every rank decodes its
own frames: weak scaling, no data-path collective; the step time is the max over
ranks and `value` counts the pixels of all ranks.

Prints ONE JSON line (rank 0).  Also reports:
  roofline     -- the dominant kernel's algorithmic FLOP/s (HIP events on the launch
                  stream) vs the FP32 peak, plus HBM traffic from the committed PMC
                  profile (profiles/*pmc*.json) when present;
  cpu_baseline -- the CPU oracle (torch fp32 restatement of the reference forward) on
                  a bounded sample of the same workload, on this host's cores.
Side legs (same line): 1080p float forward, bit-exact .cool decode / encode (path B, a
fixed number of streams per rank) with one-stream-at-a-time latency on the class-E / B /
CLIC streams, and the encoder overfit on the Kodak-24 proxies (every rank the whole
Kodak-24 at its own operating point, per-image R-D records gathered to rank 0, compared
with the reference's results/image/kodak/results.tsv rows).  Every leg is weak-scaled: a
rank's work depends on its rank, never on the world size, so `--as-rank R --as-world N`
runs exactly rank R's share of an N-GPU job on one GPU.  Only the cpu_baseline legs import
oracle/ (and run oracle/_ref); the timed legs run libccmi alone.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "cool-chic_amd"))

H, W = 720, 1280
HOP = [(48, 1, False, True), (3, 1, False, False), (3, 3, True, True), (3, 3, True, False)]
DIM_ARM, N_HIDDEN, N_GRIDS, GAIN = 16, 2, 7, 16.0
PEAK_FP32_TFLOPS = 157.3  # MI355X FP32 (vector == f32-MFMA rate), MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0
# int32 multiply-add on the VALU: v_mad_i32_i24 / v_mad_u32_u24 issue one per lane per clock,
# unpacked -- half the packed-f32 FMA rate of PEAK_FP32_TFLOPS (MI355X_MICROARCH.md lists no
# integer VALU peak; this is the f32 vector peak without v_pk_fma_f32's second lane), counted
# as 2 ops per multiply-add like the FLOPs.  v_mul_lo_u32 (the 32-bit form) is quarter rate.
PEAK_INT32_TOPS = PEAK_FP32_TFLOPS / 2


def sizes(h=H, w=W, n=N_GRIDS):
    out = []
    for _ in range(n):
        out.append((h, w))
        h, w = (h + 1) // 2, (w + 1) // 2
    return out


def flops_per_frame(H=H, W=W):
    s = sizes(H, W)
    n_lat = sum(h * w for h, w in s)
    npx = H * W
    d = DIM_ARM
    arm_mac = n_lat * (N_HIDDEN * d * d + 2 * d)
    syn_mac, c = 0, N_GRIDS
    for n_out, ks, _, _ in HOP:
        syn_mac += npx * n_out * c * ks * ks
        c = n_out
    # upsampling, polyphase: refine 2*7 taps per output, 2x upsample 2*4 taps per output
    ups_mac = 0
    for k in range(N_GRIDS - 1):  # destination level k receives (N_GRIDS-1-k) upsampled channels + 1 refined
        hk, wk = s[k]
        ups_mac += hk * wk * (14 + 8 * (N_GRIDS - 1 - k))
    return {"arm": 2 * arm_mac, "ups": 2 * ups_mac, "syn": 2 * syn_mac, "n_lat": n_lat}


def flops_fused_per_frame(H=H, W=W, fold=None):
    """The fused kernel: last upsampling step (level 1 -> 0) + synthesis (+ post, no flops);
    with the fold also the level-2 -> 1 step (each counted once, halo recompute not)."""
    fold = Pipeline.fold if fold is None else fold
    fl = flops_per_frame(H, W)
    s = sizes(H, W)
    h0, w0 = s[0]
    last_ups = 2 * h0 * w0 * (14 + 8 * (N_GRIDS - 1))
    if fold:
        last_ups += 2 * s[1][0] * s[1][1] * (14 + 8 * (N_GRIDS - 2))
    return last_ups + fl["syn"]


def bytes_per_frame(H=H, W=W):
    s = sizes(H, W)
    n_lat = sum(h * w for h, w in s)
    npx = H * W
    h1, w1 = s[1]
    return {"arm": 4 * n_lat * 2,                       # read latents, write rate
            "ups": 4 * (n_lat + N_GRIDS * npx),          # read latents, write dense synthesis input
            "syn": 4 * (N_GRIDS * npx + 3 * npx),        # read dense input, write 3 planes
            "post": 4 * (3 * npx + npx * 3 // 2),
            # fused: read the level-1 stack + full-res latent, write the 420 frame; folded: the
            # level-2 stack + the level-1 and full-res latents instead of the level-1 stack
            "decode_fused": 4 * ((N_GRIDS - 2) * s[2][0] * s[2][1] + h1 * w1 + npx + npx * 3 // 2) if Pipeline.fold
            else 4 * ((N_GRIDS - 1) * h1 * w1 + npx + npx * 3 // 2)}


def _oracle():
    """The CPU oracle, for the cpu_baseline legs only (test infrastructure, never timed as ours)."""
    if str(ROOT / "oracle") not in sys.path:
        sys.path.insert(0, str(ROOT / "oracle"))
    import forward_oracle
    import train_oracle
    return forward_oracle, train_oracle


def make_inputs(B, dev, seed, H=H, W=W):
    from ccmi import forward as F
    from ccmi import synthetic as S
    lat = S.random_latents(B, H, W, N_GRIDS, seed=seed)
    fws = [S.random_frame(H, W, DIM_ARM, N_HIDDEN, HOP, N_GRIDS, seed=seed + i, gain=GAIN) for i in range(B)]
    arm = torch.stack([F.pack_arm(m.arm) for m in fws])
    ups = torch.stack([F.pack_ups(m.ups_full(), m.pre_full()) for m in fws])
    syn = torch.stack([F.pack_syn(m.syn) for m in fws])
    return {"lat": lat.to(dev), "arm": arm.to(dev), "ups": ups.to(dev), "syn": syn.to(dev), "frames": fws,
            "lat_cpu": lat, "H": H, "W": W}


class Pipeline:
    """Preallocated buffers + direct C-ABI launches (no per-step allocation)."""

    head = 0  # ccmi_decode_args.head (CCMI_HEAD_*), set from --head
    fold = False  # --fold: the pyramid's level-2 -> 1 step inside the fused kernel (stages bit 3, opt-in)

    def __init__(self, inp, B, dev):
        import ctypes
        import ccmi
        from ccmi import forward as F
        self.L = ccmi.lib()
        self.B = B
        H, W = inp["H"], inp["W"]
        s = sizes(H, W)
        n = sum(h * w for h, w in s)
        self.rate = torch.empty(B, n, device=dev)
        self.dense = torch.empty(B, N_GRIDS, H, W, device=dev)
        self.syn = torch.empty(B, 3, H, W, device=dev)
        self.yuv = torch.empty(B, H * W + 2 * (H // 2) * (W // 2), device=dev)
        h, w = F._grid_arrays(s)
        nws = self.L.ccmi_ups_workspace_bytes(N_GRIDS, h, w, B)
        self.ws = torch.empty(nws, device=dev, dtype=torch.uint8)
        p = ccmi.ptr
        self.arm = ccmi.ArmArgs(latent=p(inp["lat"]), latent_stride=n, n_grids=N_GRIDS, h=h, w=w, gain=GAIN,
                                quantize=1, dim_arm=DIM_ARM, n_hidden=N_HIDDEN, params=p(inp["arm"]),
                                param_stride=inp["arm"].shape[1], mu=None, scale=None, log_scale=None,
                                rate=p(self.rate), out_stride=n, batch=B)
        self.ups = ccmi.UpsArgs(latent=p(inp["lat"]), latent_stride=n, n_grids=N_GRIDS, h=h, w=w, gain=GAIN,
                                quantize=1, ups_k=8, n_ups=N_GRIDS - 1, pre_k=7, n_pre=N_GRIDS - 1,
                                params=p(inp["ups"]), param_stride=inp["ups"].shape[1], out=p(self.dense),
                                out_stride=N_GRIDS * H * W, workspace=p(self.ws), workspace_bytes=nws, batch=B)
        self.synargs = F._syn_args(self.dense, HOP, inp["syn"], self.syn, B, N_GRIDS, H, W)
        self.post = ccmi.PostArgs(in_=p(self.syn), in_stride=3 * H * W, h=H, w=W, bitdepth=8, yuv420=1,
                                  out=p(self.yuv), out_stride=self.yuv.shape[1], batch=B)
        # fused decode tail: pyramid (levels 6 -> 1) then ONE kernel for the last
        # upsampling step + synthesis + 420 post (no dense stack, no raw synthesis output)
        self.dec = [ccmi.DecodeArgs(ups=self.ups, syn=self.synargs, bitdepth=8, yuv420=1, out=p(self.yuv),
                                    out_stride=self.yuv.shape[1], stages=st | (8 if Pipeline.fold else 0),
                                    head=Pipeline.head) for st in (1, 2)]
        self.byref = ctypes.byref
        self.stream = torch.cuda.current_stream(dev)
        # the ARM (rate) and the decode tail (pixels) only share the latents: with overlap
        # on, the ARM runs on a second HIP stream concurrently with the decode tail
        self.side = torch.cuda.Stream(dev)
        self.fork = torch.cuda.Event()
        self.join = torch.cuda.Event()

    STAGES = {"fused": ["arm", "ups_pyramid", "decode_fused"], "staged": ["arm", "ups", "syn", "post"]}

    join_before_last = False  # overlap: the ARM joins before the last kernel (pyramid || ARM)

    def step(self, events=None, mode="fused", overlap=True):
        """events: len(STAGES[mode]) + 1 (+ 2 with overlap: the ARM's own pair on the side stream)."""
        import ccmi
        L, br = self.L, self.byref
        if mode == "fused":
            calls = [(L.ccmi_arm_forward_f32, self.arm), (L.ccmi_decode_forward_f32, self.dec[0]),
                     (L.ccmi_decode_forward_f32, self.dec[1])]
        else:
            calls = [(L.ccmi_arm_forward_f32, self.arm), (L.ccmi_ups_forward_f32, self.ups),
                     (L.ccmi_syn_forward_f32, self.synargs), (L.ccmi_post_f32, self.post)]
        if not overlap:
            for i, (fn, a) in enumerate(calls):
                if events: events[i].record(self.stream)
                ccmi.check(fn(br(a), self.stream.cuda_stream))
            if events: events[len(calls)].record(self.stream)
            return
        n = len(calls)
        self.fork.record(self.stream)
        self.side.wait_event(self.fork)
        if events: events[n + 1].record(self.side)
        ccmi.check(calls[0][0](br(calls[0][1]), self.side.cuda_stream))
        if events: events[n + 2].record(self.side)
        self.join.record(self.side)
        for i, (fn, a) in enumerate(calls[1:], start=1):
            if self.join_before_last and i == n - 1:
                self.stream.wait_event(self.join)
            if events: events[i].record(self.stream)
            ccmi.check(fn(br(a), self.stream.cuda_stream))
        if events: events[n].record(self.stream)
        self.stream.wait_event(self.join)


def measure_path_a(inp, B, steps, warmup, mode, overlap, dist, dev, join_before_last=False):
    """Time `steps` pipeline steps (after `warmup`), barrier + synchronize on both sides;
    returns (max-over-ranks seconds, per-stage ms per step from HIP events)."""
    pipe = Pipeline(inp, B, dev)
    pipe.join_before_last = join_before_last
    names = Pipeline.STAGES[mode]
    for _ in range(warmup):
        pipe.step(mode=mode, overlap=overlap)
    torch.cuda.synchronize()
    # per-stage HIP events over the timed region (recorded on the stream each kernel runs on)
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(len(names) + 3)] for _ in range(steps)]
    if dist: dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        pipe.step(ev[k], mode, overlap)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if dist: dist.barrier()
    dt = t1 - t0
    if dist:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    nn = len(names)
    # per-step durations (first to last event of each step on the main stream): the median is
    # the statistic SURVEY 8d asks for; the throughput above is the whole timed region
    first = 1 if overlap else 0  # with overlap the ARM's events are on the side stream
    per_step = sorted(ev[k][first].elapsed_time(ev[k][nn]) for k in range(steps))
    measure_path_a.median_ms = per_step[len(per_step) // 2] if steps % 2 else \
        0.5 * (per_step[steps // 2 - 1] + per_step[steps // 2])
    if overlap:  # ARM timed by its own pair of events on the side stream
        stage_ms = {"arm": sum(ev[k][nn + 1].elapsed_time(ev[k][nn + 2]) for k in range(steps)) / steps}
        stage_ms.update({n: sum(ev[k][i].elapsed_time(ev[k][i + 1]) for k in range(steps)) / steps
                         for i, n in enumerate(names) if i > 0})
    else:
        stage_ms = {n: sum(ev[k][i].elapsed_time(ev[k][i + 1]) for k in range(steps)) / steps
                    for i, n in enumerate(names)}
    return dt, stage_ms


def measure_path_a_graph(inp, B, steps, warmup, dist, dev, per_graph=10, overlap=False):
    """The fused pipeline captured in a HIP graph (`per_graph` steps per graph, one stream):
    replays remove the host launch gaps between the step's small pyramid kernels.  Returns
    the max-over-ranks seconds for `steps` steps (a multiple of per_graph)."""
    pipe = Pipeline(inp, B, dev)
    pipe.join_before_last = overlap
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    g = torch.cuda.CUDAGraph()
    err = None
    try:
        with torch.cuda.stream(s):
            pipe.stream = s
            pipe.step(mode="fused", overlap=overlap)
            s.synchronize()
            ref = (pipe.yuv.clone(), pipe.rate.clone())  # eager outputs, to check the replays
            # thread_local: the process group's watchdog thread may query events meanwhile
            with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                for _ in range(per_graph):
                    pipe.step(mode="fused", overlap=overlap)
        torch.cuda.synchronize()
    except Exception as e:
        err = f"{type(e).__name__}: {e}"
    if dist:  # every rank takes the same branch, so the collectives below stay matched
        ok = torch.tensor([0 if err else 1], device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if not int(ok.item()) and not err:
            err = "graph capture failed on another rank"
    if err:
        raise RuntimeError(err)
    for _ in range(max(1, warmup // per_graph)):
        g.replay()
    torch.cuda.synchronize()
    reps = max(1, steps // per_graph)
    if dist: dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dist: dist.barrier()
    if dist:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    # a replay recomputes the outputs from scratch: clear them, replay once, compare
    pipe.yuv.zero_()
    pipe.rate.zero_()
    g.replay()
    torch.cuda.synchronize()
    same = bool(torch.equal(pipe.yuv, ref[0]) and torch.equal(pipe.rate, ref[1]))
    return dt, reps * per_graph, same


def bench_path_a_hd(B, steps, warmup, rank, world, dist, dev):
    """The same fused float forward on synthetic 1920x1080 frames (BASELINE config 5's
    geometry, fp32): whole-job Mpixel/s and the fused kernel's FP32 roofline fraction."""
    Hh, Wh = 1080, 1920
    inp = make_inputs(B, dev, seed=1000 * rank + 7, H=Hh, W=Wh)
    dt, st = measure_path_a(inp, B, steps, warmup, "fused", False, dist, dev)
    ach = flops_fused_per_frame(Hh, Wh) * B / (st["decode_fused"] * 1e-3) / 1e12
    return {"metric": "decoded Mpixel/s (Synth+ARM+upsample) @1920x1080, all GPUs",
            "value": round(B * steps * world * Hh * Wh / dt / 1e6, 2), "unit": "Mpixel/s",
            "frames_per_step_per_gpu": B, "steps": steps, "ms_per_step": round(dt / steps * 1e3, 4),
            "stage_ms_per_step": {k: round(v, 4) for k, v in st.items()},
            "roofline": {"bound": "valu-fp32", "kernel": "decode_fused", "achieved": round(ach, 3),
                         "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s", "frac": round(ach / PEAK_FP32_TFLOPS, 4)},
            "data": "synthetic (seeded N(0,0.5) latents, random-init hop weights per frame), 7 latent grids"}


def cpu_baseline(inp, budget_s=12.0, max_frames=64):
    """Oracle (torch fp32 CPU restatement of the reference forward) on whole 720p frames."""
    fo, _ = _oracle()
    s = sizes()
    mps = [fo.ModelParams(m.H, m.W, m.dim_arm, m.n_hidden, list(m.layers), m.n_grids, m.gain, m.arm, m.ups_half,
                          m.pre_half, m.syn) for m in inp["frames"][:4]]
    frames, t0 = 0, time.perf_counter()
    while frames < max_frames and (time.perf_counter() - t0) < budget_s:
        i = frames % len(mps)
        flat = inp["lat_cpu"][i]
        lats, o = [], 0
        for h, w in s:
            lats.append(flat[o:o + h * w].view(h, w))
            o += h * w
        r = fo.forward(mps[i], lats)
        fo.post(r["syn"], 8, True)
        frames += 1
    dt = time.perf_counter() - t0
    value = frames * H * W / dt / 1e6
    out = {"value": round(value, 3), "unit": "Mpixel/s", "cores": torch.get_num_threads(),
           "kind": "port",
           "sample": f"{frames} synthetic 1280x720 hop frames, full float forward + 420 post "
                     f"(oracle/forward_oracle.py, torch fp32 CPU, {torch.get_num_threads()} threads), {dt:.1f} s"}
    # the port timed against the reference's own eval forward on one host
    # (tests/golden/cpu_calibration.json "forward_720p", tools/gen_golden_rd.py calib_forward)
    cal = json.loads((ROOT / "tests" / "golden" / "cpu_calibration.json").read_text()).get("forward_720p")
    if cal:
        out["port_over_reference_time"] = round(cal["port_s_per_frame"] / cal["reference_s_per_frame"], 3)
        out["reference_equivalent_value"] = round(value * out["port_over_reference_time"], 3)
    return out


def _reduce(counters: dict, dist, dev, op="sum"):
    from ccmi import dist as D
    return D.reduce_counters(counters, op=op, device=dev) if dist else dict(counters)


REF_DEC_TIMES = ROOT / "tests/golden/ref_dec_times.json"


def _stream_set(cls: str):
    """Committed streams of a class: "E" / "B" / "D" (JVET) or "CLIC" -> [(key in ref_md5.json, path)]."""
    if cls == "CLIC":
        fs = sorted((ROOT / "tests/golden/cool/clic").glob("*.cool"))
        return [("clic20-pro-valid/" + f.name, f) for f in fs]
    return [("jvet/" + f.name, f) for f in sorted((ROOT / "tests/golden/cool").glob(f"{cls}-*.cool"))]


def _time_ref_one_core(path: Path, out: Path, reps: int):
    """The reference decoder (oracle/_ref/ccdec_ref, built from the reference's own sources) on
    one core, one stream: mean wall seconds over `reps` runs, or None when it is absent."""
    import subprocess
    ref = ROOT / "oracle" / "_ref" / "ccdec_ref"
    if not ref.exists():
        return None
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        subprocess.run([str(ref), f"--input={path}", f"--output={out}", "--avx2"], check=True,
                       stdout=subprocess.DEVNULL)
        ts.append(time.perf_counter() - t0)
    return sum(ts) / len(ts)


def bench_single_stream_decode(cls: str = "E", reps: int = 3, ref_reps: int = 2):
    """Path B latency, the drop-in case: ccmi_decode_file (cc_decode_cpu's replacement, file in
    -> .yuv / .ppm out: parse, upload, kernels, download, write) on each committed class-`cls`
    stream, ONE stream at a time: mean and best of `reps` wall-clock runs per stream, md5 checked
    against the reference decoder's.  Compared per stream with the reference decoder on one
    core: its own results.tsv time (the authors' host, tests/golden/ref_dec_times.json) and, when
    oracle/_ref is present, ccdec_ref --avx2 timed here on one core (mean of `ref_reps`)."""
    import hashlib
    import statistics
    import tempfile
    import ccmi
    md5 = json.loads((ROOT / "tests/golden/ref_md5.json").read_text())
    tsv = json.loads(REF_DEC_TIMES.read_text())["streams"]
    files = _stream_set(cls)
    L = ccmi.lib()
    per, exact = [], True
    with tempfile.TemporaryDirectory() as td:
        for key, f in files:
            out = Path(td) / ("o" + md5[key]["ext"])
            assert L.ccmi_decode_file(str(f).encode(), str(out).encode(), 0, 0, 0, 0) == 0, ccmi.last_error()  # warm
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                rc = L.ccmi_decode_file(str(f).encode(), str(out).encode(), 0, 0, 0, 0)
                ts.append(time.perf_counter() - t0)
                assert rc == 0, ccmi.last_error()
            exact &= hashlib.md5(out.read_bytes()).hexdigest() == md5[key]["md5"]
            rel = str(f.relative_to(ROOT / "tests/golden/cool"))
            r = {"stream": f.name, "mean_ms": round(statistics.mean(ts) * 1e3, 2), "best_ms": round(min(ts) * 1e3, 2),
                 "reference_results_tsv_ms": round(tsv[rel]["dec_time_all_sec"] * 1e3, 2) if rel in tsv else None}
            rt = _time_ref_one_core(f, Path(td) / ("r" + md5[key]["ext"]), ref_reps)
            r["reference_1core_here_ms"] = round(rt * 1e3, 2) if rt is not None else None
            per.append(r)
    mean = statistics.mean(r["mean_ms"] for r in per)
    out = {"metric": f"ccmi_decode_file wall ms per stream, one stream at a time (mean of {reps} runs; best alongside)",
           "class": cls, "streams": len(per), "mean_ms": round(mean, 2),
           "best_mean_ms": round(statistics.mean(r["best_ms"] for r in per), 2),
           "max_ms": max(r["mean_ms"] for r in per), "bit_exact_vs_reference_md5": exact, "per_stream": per}
    for k, name in (("reference_results_tsv_ms", "reference_results_tsv"), ("reference_1core_here_ms", "reference_1core_here")):
        if all(r[k] for r in per):
            ref = statistics.mean(r[k] for r in per)
            out[f"{name}_mean_ms"] = round(ref, 2)
            out[f"speedup_vs_{name}"] = round(ref / mean, 3)
            out[f"streams_not_slower_than_{name}"] = sum(r["mean_ms"] <= r[k] for r in per)
    return out


# committed rocprofv3 kernel traces of the path-B batch decode (tools/bench_decode.py under
# rocprofv3 --kernel-trace --stats), per class; historical, with a sources sidecar
DECODE_PROFILE = {"E": "profiles/r6d_decode_E_kernel_stats.csv", "B": "profiles/r6d_decode_B_kernel_stats.csv"}


def path_b_tail_work(streams) -> dict:
    """Algorithmic work of the integer decoder tail per batch (from the streams' headers):
    syn_ops -- 2 x the synthesis multiply-adds (every layer n_in x n_out x ks^2 per pixel,
    synfused_cpu.hpp / syn_cpu.hpp); ups_bytes -- HBM bytes of the pyramid steps (each
    dec_ups_level reads the level-k stack and the level-(k-1) latent and writes the C+1
    channels of level k-1, int32; ups_refine_cpu.hpp / ups_upsample_cpu.hpp)."""
    from ccmi import encode
    syn_ops = ups_bytes = 0
    for data in streams:
        fr = encode.parse(data)
        d = fr.desc
        sz = fr.grid_sizes
        npx = d.h * d.w
        c = d.n_grids
        for i in range(d.n_syn_layers):
            syn_ops += 2 * npx * c * d.syn_out[i] * d.syn_ks[i] * d.syn_ks[i]
            c = d.syn_out[i]
        L = d.n_grids
        for j in range(L - 2, -1, -1):  # destination level j from the (L-1-j)-channel stack of level j+1
            C = L - 1 - j
            ups_bytes += 4 * (C * sz[j + 1][0] * sz[j + 1][1] + sz[j][0] * sz[j][1] + (C + 1) * sz[j][0] * sz[j][1])
    return {"syn_ops": syn_ops, "ups_bytes": ups_bytes}


def path_b_tail_roofline(streams, cls: str, tail_ms: float) -> dict:
    """Roofline of the data-parallel int32 tail of path B: the dominant tail kernel
    (dec_syn_fused_batch, int32 VALU-bound) and the pyramid (dec_ups_level_batch, HBM), each as
    algorithmic work / its total time in the committed trace of the same batch (every launch of
    that kernel summed: one per geometry group and pyramid step), plus the live tail stage of
    this run (ccmi_decode_last_timing: upsampling + synthesis + output together)."""
    import csv
    wk = path_b_tail_work(streams)
    out = {"syn_ops_per_batch": wk["syn_ops"], "ups_hbm_bytes_per_batch": wk["ups_bytes"],
           "live_tail_stage": {"ms": round(tail_ms, 3),
                               "int32_tops_syn_only": round(wk["syn_ops"] / (tail_ms * 1e-3) / 1e12, 3)}}
    path = DECODE_PROFILE.get(cls)
    if path and (ROOT / path).exists():
        rows = list(csv.DictReader((ROOT / path).open()))
        meta = json.loads((ROOT / (path + ".sources.json")).read_text()) if (ROOT / (path + ".sources.json")).exists() else {}
        frames_prof = int(meta.get("frames", 0)) or None
        scale = len(streams) / frames_prof if frames_prof else None
        def tot(key):
            r = next((r for r in rows if key in r["Name"]), None)
            return (float(r["TotalDurationNs"]) * 1e-9, int(r["Calls"])) if r else (None, 0)
        ts, ns = tot("dec_syn_fused_batch")
        tu, nu = tot("dec_ups_level_batch")
        if ts and scale:
            ach = wk["syn_ops"] / scale / ts / 1e12
            out.update(bound="int32-valu", kernel="dec_syn_fused_batch", achieved=round(ach, 3), peak=PEAK_INT32_TOPS,
                       unit="TOPS (int32, 2 per multiply-add)", frac=round(ach / PEAK_INT32_TOPS, 4),
                       kernel_ms_per_batch=round(ts * 1e3, 3), launches=ns)
        if tu and scale:
            gbs = wk["ups_bytes"] / scale / tu / 1e9
            out["pyramid"] = {"kernel": "dec_ups_level_batch", "bound": "hbm", "achieved": round(gbs, 1),
                              "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(gbs / PEAK_HBM_GBS, 4),
                              "ms_per_batch": round(tu * 1e3, 3), "launches": nu}
        out["source"] = profile_provenance(path)
        out["profiled_frames"] = frames_prof
        out["note"] = ("batches of >= 64 streams run in two cost-ordered chunks: the cheap chunk's tail kernels "
                       "share the CUs with the other chunk's ARM chains (dec_host.cpp), so these kernel times "
                       "include that sharing")
    return out


def bench_bitexact_decode(reps: int, cls: str = "E", H=H, W=W, rank=0, world=1, dist=None, dev=None):
    """Path B: the bit-exact HIP decoder on the shipped JVET class-`cls` .cool streams
    (class E: 15 files at 1280x720; class B: 5 committed files at 1920x1080).  Weak scaling:
    every rank decodes its own `reps` copies of every stream (a fixed number of frames per
    GPU) in ONE ccmi_decode_batch call; output bytes are checked against the reference
    decoder's md5s.  Whole-job rate = all ranks' frames / the slowest rank's time."""
    import hashlib
    from ccmi import decode
    md5 = json.loads((ROOT / "tests/golden/ref_md5.json").read_text())
    files = sorted((ROOT / "tests/golden/cool").glob(f"{cls}-*.cool"))
    job = [f for _ in range(reps) for f in files]
    streams = [f.read_bytes() for f in job]
    # warm-up: the whole batch once (sizes the pinned output pool and the cached device
    # workspace, as a long-running decoder would have them), then the timed call
    decode.decode_batch(streams, views=True)
    if dist: dist.barrier()
    t0 = time.perf_counter()
    outs = decode.decode_batch(streams, views=True)
    wall = time.perf_counter() - t0
    tm = decode.last_timing()
    exact = all(hashlib.md5(o).hexdigest() == md5["jvet/" + f.name]["md5"] for f, o in zip(job, outs))
    c = _reduce({"frames": len(job), "exact": int(exact)}, dist, dev)
    t = _reduce({"kern_s": (tm["arm_cabac"] + tm["ups_syn_out"]) / 1e3, "wall": wall}, dist, dev, op="max")
    n = int(c["frames"])
    return {"metric": f"bit-exact .cool decode Mpixel/s (batch of independent {W}x{H} streams, all GPUs)",
            "frames": n, "frames_per_gpu": len(job), "n_gpus": world,
            "value_kernels": round(n * H * W / t["kern_s"] / 1e6, 2),
            "value_wall_pcie_inclusive": round(n * H * W / t["wall"] / 1e6, 2), "unit": "Mpixel/s",
            "wall_note": "host streams in -> decoded bytes in host memory (pinned pool, per-chunk downloads "
                         "overlapped with the other chunk's ARM), header parse + weight decode included",
            "per_gpu_kernels": round(len(job) * H * W / t["kern_s"] / 1e6, 2),
            "per_gpu_wall": round(len(job) * H * W / t["wall"] / 1e6, 2),
            "stage_ms": {k: round(v, 3) for k, v in tm.items()},
            "roofline": path_b_tail_roofline(streams, cls, tm["ups_syn_out"]),
            "bit_exact_vs_reference_md5": int(c["exact"]) == world,
            "scaling": "weak",
            "data": f"{len(files)} shipped JVET class-{cls} .cool bitstreams (results/image/jvet), x{reps} per GPU"}


def bench_bitexact_encode(reps: int = 2, rank=0, world=1, dist=None, dev=None):
    """Path B writer: ccmi_encode_frame (GPU integer ARM over all latents + host CABAC, one
    thread per latent grid) re-encoding the shipped class-E streams from their decoded
    latents (every rank all 15: weak scaling); the output must equal the shipped bytes."""
    from ccmi import decode, encode
    import numpy as np
    files = sorted((ROOT / "tests/golden/cool").glob("E-*.cool"))
    jobs = []
    for f in files:
        data = f.read_bytes()
        fr = encode.parse(data)
        lat = decode.decode_latents(data)
        jobs.append((data, fr, torch.from_numpy(np.concatenate(lat)).to(torch.int32).cuda()))
    encode.encode_frame(jobs[0][1], jobs[0][2])
    torch.cuda.synchronize()
    if dist: dist.barrier()
    t0 = time.perf_counter()
    exact = True
    for _ in range(reps):
        for data, fr, x in jobs:
            exact &= encode.encode_frame(fr, x) == data
    dt = time.perf_counter() - t0
    c = _reduce({"frames": reps * len(jobs), "exact": int(exact)}, dist, dev)
    dt = _reduce({"s": dt}, dist, dev, op="max")["s"]
    n = int(c["frames"])
    return {"metric": "bit-exact .cool encode Mpixel/s (GPU ARM contexts + host CABAC, one frame at a time per GPU, "
                      "all GPUs)",
            "frames": n, "value": round(n * H * W / dt / 1e6, 2), "unit": "Mpixel/s",
            "ms_per_frame_per_gpu": round(dt / max(1, reps * len(jobs)) * 1e3, 3),
            "identical_to_shipped_streams": int(c["exact"]) == world,
            "data": "15 shipped JVET class-E .cool bitstreams re-encoded from their decoded latents"}


KODAK_SHIPPED = ROOT / "tests/golden/cool"


def kodak_proxies():
    """The Kodak-24 content this tree holds: the reference's own lambda = 1e-4 encodings
    (results/image/kodak/bitstreams/kodimNN-lmbda-00001.cool, 35-46 dB) decoded bit-exactly
    by libccmi -- the originals are not in the reference tree.  Returns [(name, stream)]."""
    out = []
    for i in range(1, 25):
        n = f"kodim{i:02d}"
        f = KODAK_SHIPPED / f"{n}-lmbda-00001.cool"
        if not f.exists():
            f = KODAK_SHIPPED / "kodak" / f"{n}-lmbda-00001.cool"
        out.append((n, f.read_bytes()))
    return out


def encoder_flops_per_iteration(Hh, Wh):
    """Algorithmic FLOPs of one training iteration of one frame: forward (ARM + upsampling +
    synthesis, flops_per_frame) x 3 (forward + backward w.r.t. activations and weights)."""
    fl = flops_per_frame(Hh, Wh)
    return 3 * (fl["arm"] + fl["ups"] + fl["syn"])


# the reference's Kodak operating points (results/image/kodak/results.tsv), in the order ranks
# take them: rank r of an N-GPU job encodes the Kodak-24 at REF_LAMBDAS[r % 5] with seed r // 5
REF_LAMBDAS = (0.001, 0.0004, 0.004, 0.0001, 0.02)


def encoder_shard(rank: int, lambdas=None):
    """What one rank encodes (weak scaling, SURVEY §8e: images are independent units): the whole
    Kodak-24 at its own operating point -- REF_LAMBDAS[rank % 5], seed rank // 5 -- so every rank
    keeps full geometry batches (18 landscape + 6 portrait) and an N-GPU job covers the
    reference's lambda set (N >= 5) as the reference's one-image-per-GPU SLURM array does
    (sbatch-files/submit-coolchic-encoding.sh).  With explicit `lambdas`, every rank encodes
    every image at each of them, seed = rank.  Returns ([lambda...], seed)."""
    if lambdas:
        return list(lambdas), rank
    return [REF_LAMBDAS[rank % len(REF_LAMBDAS)]], rank // len(REF_LAMBDAS)


# Per-kernel rooflines of the encoder's training step, from a committed rocprofv3 kernel trace
# of tools/bench_train.py 8 with CCMI_ARM_OVERLAP=0 (every kernel alone; 8 frames of 512 x 768,
# hop, c3x; one launch per iteration each).  A HISTORICAL profile, not this run: its sidecar
# <csv>.sources.json records the sha256 of the kernel sources it was measured on, and the
# bench line says whether today's sources still match (profile_provenance).
TRAIN_PROFILE = "profiles/r6m_train_iso_kernel_stats.csv"
TRAIN_FRAMES, TRAIN_H, TRAIN_W = 8, 512, 768


def profile_provenance(csv_path: str) -> dict:
    """Which sources a committed profile was measured on, and whether they are still today's:
    {"profile", "measured_at_commit", "sources_match_current": bool | None, "changed": [...]}."""
    import hashlib
    side = ROOT / (csv_path + ".sources.json")
    out = {"profile": csv_path, "kind": "historical rocprofv3 trace (committed), not measured by this run"}
    if not side.exists():
        out["sources_match_current"] = None
        return out
    meta = json.loads(side.read_text())
    changed = [f for f, h in meta.get("sha256", {}).items()
               if not (ROOT / f).exists() or hashlib.sha256((ROOT / f).read_bytes()).hexdigest() != h]
    out.update(measured_at_commit=meta.get("commit"), sources_match_current=not changed, changed=changed)
    if changed:
        print(f"warning: {csv_path} was measured on other sources than today's ({', '.join(changed)})", file=sys.stderr)
    return out


def train_kernel_rooflines(csv_path: str = TRAIN_PROFILE) -> list:
    """FLOPs per launch / average launch duration for the two largest training kernels.
    t_head_bwd(_t)<7, 3>: per pixel the hidden-layer recompute (48 x 7 MAC), g_h (48 x 3), g_x (7 x 48),
    dW1 (3 x 48) and dW0 (48 x 7): 1,296 MAC = 2,592 FLOP.  t_arm16<2>: per latent 3 x the ARM
    forward (dim 16, 2 hidden layers + the 2-wide output: 544 MAC) = 3,264 FLOP (forward +
    input and weight gradients)."""
    import csv
    npx = TRAIN_H * TRAIN_W
    nlat = sum((TRAIN_H >> k) * (TRAIN_W >> k) for k in range(7))
    flops = {"t_head_bwd": 2592 * npx * TRAIN_FRAMES, "t_arm16<2>": 3264 * nlat * TRAIN_FRAMES}
    out = []
    path = ROOT / csv_path
    if not path.exists():
        return out
    rows = list(csv.DictReader(path.open()))
    for key, fl in flops.items():
        r = next((r for r in rows if key in r["Name"]), None)
        if r is None:
            continue
        us = float(r["AverageNs"]) / 1e3
        ach = fl / (us * 1e-6) / 1e12
        name = r["Name"].replace("void (anonymous namespace)::", "")
        out.append({"kernel": name[:name.index(">") + 1] if ">" in name else name.split("(")[0],
                    "flop_per_launch": fl, "avg_us": round(us, 2), "achieved": round(ach, 3),
                    "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s", "frac": round(ach / PEAK_FP32_TFLOPS, 4),
                    "launch": f"{TRAIN_FRAMES} frames {TRAIN_H}x{TRAIN_W}, one per iteration",
                    "source": profile_provenance(csv_path)})
    return out


def bench_encoder(images: int, scale: float, lambdas, rank: int, world: int, dist, dev):
    """Encoder overfit (BASELINE config 4): the c3x schedule (warm-up candidates + 3 phases +
    quantize_model, ccmi.train.overfit) on the first `images` Kodak proxies, RGB, hop decoder.
    Every rank overfits its own encoder_shard (fixed work per GPU), grouped by geometry
    (768x512 landscape / 512x768 portrait), one batch per group and lambda; the geometry
    batches run concurrently (one host thread + HIP stream each).  Per-image records are
    gathered to every rank (ccmi.dist.gather_records)."""
    from ccmi import decode, io, rd
    from ccmi import dist as D
    from ccmi import train as T
    lms, seed = encoder_shard(rank, lambdas)
    mine = kodak_proxies()[:images]
    recs, secs, kern = [], 0.0, 0.0
    if mine:
        outs = decode.decode_batch([s for _, s in mine], as_yuv=False)
        imgs = [io.parse_ppm(o)[0][0].float() for o in outs]
        groups = {}
        for (n, _), x in zip(mine, imgs):
            groups.setdefault(tuple(x.shape[-2:]), []).append((n, x))
        # one batch per geometry, the batches of different geometries run concurrently, each
        # from its own host thread on its own HIP stream (the small portrait batch alone
        # would leave most of the GPU idle)
        def run_group(key, stream):
            (Hh, Wh), items = key
            arch = T.Arch(Hh, Wh, dim_arm=DIM_ARM, n_hidden=N_HIDDEN, layers=HOP)
            out, flop = [], 0.0
            with torch.cuda.stream(stream):
                tg = torch.stack([io.to_target(x, "rgb") for _, x in items]).to(dev)
                for lm in lms:
                    r = rd.encode_batch(tg, Hh, Wh, lm, arch, names=[n for n, _ in items], seeds=[seed] * len(items),
                                        preset="c3x", scale=scale)
                    flop += encoder_flops_per_iteration(Hh, Wh) * sum(x.iterations for x in r)
                    out += r
            return out, flop
        keys = sorted(groups.items())
        torch.cuda.synchronize()
        if dist: dist.barrier()
        t0 = time.perf_counter()
        from concurrent.futures import ThreadPoolExecutor
        streams = [torch.cuda.Stream(dev) for _ in keys]
        with ThreadPoolExecutor(len(keys)) as ex:
            results = list(ex.map(run_group, keys, streams))
        torch.cuda.synchronize()
        secs = time.perf_counter() - t0
        for r, f in results:
            recs += r
            kern += f
    recs = D.gather_records([r.as_dict() for r in recs]) if dist else [r.as_dict() for r in recs]
    c = _reduce({"flop": kern}, dist, dev)
    t = _reduce({"s": secs}, dist, dev, op="max")
    return recs, t["s"], c["flop"], secs, {"lambdas": lms, "seed": seed}


def kodak_reference_rows():
    d = json.loads((ROOT / "tests/golden/kodak_results.json").read_text())
    return d["rows"]


def compare_with_reference(recs, lambdas):
    """Per image: our (bpp, PSNR) against the reference's results.tsv row at the same lambda;
    with >= 4 lambdas also the per-image BD-rate (ccmi.rd.bd_rate, bjontegaard_metric.py)."""
    import numpy as np
    from ccmi import rd
    ref = {(r["seq_name"], round(r["lmbda"], 6)): r for r in kodak_reference_rows()}
    lambdas = sorted({r["lmbda"] for r in recs}) if lambdas is None else lambdas
    out = {"lmbda": list(lambdas), "per_lambda": {}}
    for lm in lambdas:
        mine = [r for r in recs if abs(r["lmbda"] - lm) < 1e-9]
        pairs = [(r, ref[(r["image"], round(lm, 6))]) for r in mine if (r["image"], round(lm, 6)) in ref]
        if not pairs:
            continue
        out["per_lambda"][str(lm)] = {
            "images": len(pairs),
            "psnr_db_mean": round(float(np.mean([a["psnr_db"] for a, _ in pairs])), 3),
            "rate_bpp_mean": round(float(np.mean([a["rate_bpp"] for a, _ in pairs])), 4),
            "reference_psnr_db_mean": round(float(np.mean([b["psnr_db"] for _, b in pairs])), 3),
            "reference_rate_bpp_mean": round(float(np.mean([b["rate_bpp"] for _, b in pairs])), 4)}
    if len(lambdas) >= 4:
        bds = []
        for name in sorted({r["image"] for r in recs}):
            R2, P2, lms = rd.curve([r for r in recs if r["image"] == name])  # seed means per lambda
            rr = [ref.get((name, round(lm, 6))) for lm in lms]
            if None in rr or len(lms) < 4:
                continue
            bds.append(rd.bd_rate([r["rate_bpp"] for r in rr], [r["psnr_db"] for r in rr], R2, P2))
        if bds:
            # proxies: encoded from the reference's own lambda = 1e-4 reconstructions, while
            # results.tsv was measured on the originals -- an operating-point check, not matched R-D
            out["bd_rate_vs_results_tsv_on_proxies_pct_mean"] = round(float(np.mean(bds)), 3)
            out["bd_rate_images"] = len(bds)
    return out


def cpu_encoder_baseline(iters: int = 10, warm: int = 2):
    """The CPU oracle (torch fp32 autograd restatement of the training step, same math) at
    512x768: seconds per iteration on this host's cores, projected onto the c3x schedule.
    Also the reference-equivalent rate: the reference encoder's own s/iteration was measured
    against the same port on one host (tests/golden/cpu_calibration.json, tools/gen_golden_rd.py
    calib), and that ratio rescales the port's images/hr."""
    fo, to = _oracle()
    mp = fo.ModelParams.random(512, 768, seed=0)
    g = torch.Generator().manual_seed(0)
    st = to.TrainState(mp, [0.01 * torch.randn(h, w, generator=g) for h, w in mp.sizes])
    tgt = {"y": torch.rand(512, 768), "u": torch.rand(256, 384), "v": torch.rand(256, 384)}
    opt = to.Adam(st.params(), 1e-2)
    ts = []
    for it in range(warm + iters):
        t0 = time.perf_counter()
        to.grads(st, tgt, "softround", 0.3, 1e-3, True)
        opt.step()
        ts.append(time.perf_counter() - t0)
    ts = ts[warm:]
    per = sum(ts) / iters
    # per image: 5 x 400 + 2 x 400 warm-up candidate iterations + 13,100 phase iterations
    per_image = per * (5 * 400 + 2 * 400 + 13100)
    cal = json.loads((ROOT / "tests/golden/cpu_calibration.json").read_text())["512x768"]
    ratio = cal["port_over_reference"]
    return {"value": round(3600.0 / per_image, 3), "unit": "images/hr", "cores": torch.get_num_threads(),
            "kind": "port", "sample": f"{iters} training iterations at 512x768 after {warm} untimed ones "
                                      f"(oracle/train_oracle.py, torch fp32 autograd on CPU, {torch.get_num_threads()} "
                                      f"threads): mean {per * 1e3:.0f} ms/iteration (min {min(ts) * 1e3:.0f}, max "
                                      f"{max(ts) * 1e3:.0f}), projected onto the 15,900 image-iterations of c3x",
            "reference_equivalent_value": round(3600.0 / per_image * ratio, 3),
            "calibration": {"port_over_reference_s_per_iter": round(ratio, 4), "threads": 8,
                            "source": "tests/golden/cpu_calibration.json (reference train step vs oracle, same host)"}}


def cpu_decode_baseline(budget_s=10.0, cls="E", H=H, W=W):
    """The reference C decoder (oracle/_ref, built from /root/reference sources) -- or the C oracle
    when that binary is absent -- decoding the class-`cls` streams, one process per core."""
    import subprocess
    import tempfile
    ref = ROOT / "oracle" / "_ref" / "ccdec_ref"
    orc = ROOT / "oracle" / "_build" / "ccdec_oracle"
    files = sorted((ROOT / "tests/golden/cool").glob(f"{cls}-*.cool"))
    ncores = max(1, min(16, os.cpu_count() or 1))
    kind = "reference" if ref.exists() else "port"
    with tempfile.TemporaryDirectory() as td:
        def cmd(f, i):
            out = f"{td}/o{i}.yuv"
            return [str(ref), f"--input={f}", f"--output={out}", "--avx2"] if kind == "reference" else \
                [str(orc), str(f), out]
        frames, t0, k, procs = 0, time.perf_counter(), 0, []
        while True:
            while len(procs) < ncores and time.perf_counter() - t0 < budget_s:
                procs.append(subprocess.Popen(cmd(files[k % len(files)], len(procs)), stdout=subprocess.DEVNULL))
                k += 1
            if not procs:
                break
            procs.pop(0).wait()
            frames += 1
        dt = time.perf_counter() - t0
    return {"value": round(frames * H * W / dt / 1e6, 3), "unit": "Mpixel/s", "cores": ncores, "kind": kind,
            "sample": f"{frames} decodes of the {len(files)} class-{cls} {W}x{H} streams, {ncores} concurrent single-threaded "
                      f"processes ({'reference ccdec --avx2' if kind == 'reference' else 'C oracle'}), {dt:.1f} s"}


def pmc_traffic(stage: str, frames: int):
    """HBM bytes of one `stage` launch over `frames` frames, from the newest committed PMC
    summary (its per-launch bytes rescaled by the frames per launch it was measured at;
    summaries without that field were measured at 8), or None."""
    for f in sorted((ROOT / "profiles").glob("*pmc*.json"), reverse=True):
        try:
            d = json.loads(f.read_text())
            v = d.get("per_launch_hbm_bytes", {}).get(stage)
            if v:
                return float(v) * frames / float(d.get("frames_per_launch", 8)), f.name
        except Exception:
            pass
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=32, help="frames per step per GPU (720p headline and 1080p leg)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--decode-reps", type=int, default=64, help="class-E stream copies for the bit-exact decode leg")
    ap.add_argument("--staged", action="store_true",
                    help="run upsampling / synthesis / post as separate kernels (module-boundary path)")
    ap.add_argument("--encode-images", type=int, default=24,
                    help="Kodak proxies overfitted (the first N of kodim01..24, sharded over ranks; 0: skip)")
    ap.add_argument("--encode-scale", type=float, default=1.0, help="fraction of the c3x schedule to run")
    ap.add_argument("--encode-lambdas", default="",
                    help="comma-separated lambdas of the encoder leg, every rank all of them (default: rank r "
                         "encodes at REF_LAMBDAS[r %% 5]; 4 or more lambdas: per-image BD-rate vs results.tsv)")
    ap.add_argument("--as-rank", type=int, default=None,
                    help="run exactly rank R's shard of an --as-world N job on this one GPU, without "
                         "torch.distributed (the per-GPU rate of one rank of the N-GPU job)")
    ap.add_argument("--as-world", type=int, default=None)
    ap.add_argument("--no-single-stream", action="store_true",
                    help="skip the one-stream-at-a-time class-B / CLIC latency legs")
    ap.add_argument("--overlap", action="store_true",
                    help="run the ARM on a second HIP stream concurrently with the decode tail (the "
                         "step rate is the same within noise on MI355X; kernels then share CUs, so the "
                         "roofline kernel's duration is no longer its own)")
    ap.add_argument("--serial", action="store_true", help="(default) one stream, kernels back to back")
    ap.add_argument("--overlap-pyramid", action="store_true",
                    help="ARM on a second stream concurrent with the upsampling pyramid only; the fused "
                         "kernel starts after both (it then runs alone, so its roofline stays its own)")
    ap.add_argument("--no-graph", action="store_true",
                    help="time the eager launches instead of HIP-graph replays of the fused pipeline")
    ap.add_argument("--hd-steps", type=int, default=20, help="steps of the 1920x1080 float-forward leg (0: skip)")
    ap.add_argument("--fold", action="store_true",
                    help="evaluate the level-2 -> 1 upsampling step inside the fused kernel (opt-in; measured slower)")
    ap.add_argument("--head", choices=("default", "valu", "mfma"), default="default",
                    help="the fused kernel's 1x1 synthesis head: fp32 VALU or f32 MFMA (CCMI_HEAD_*)")
    ap.add_argument("--hd-decode-reps", type=int, default=64,
                    help="class-B (1080p) stream copies for the bit-exact decode leg (0: skip)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    as_rank = None
    if args.as_rank is not None:
        # one rank's shard alone: every leg is weak-scaled (a rank's work depends on its rank,
        # never on the world size), so this GPU does exactly what rank R of the N-GPU job does
        if world != 1:
            raise SystemExit("--as-rank runs one process (no torchrun)")
        n = args.as_world or 8
        if not 0 <= args.as_rank < n:
            raise SystemExit(f"--as-rank must lie in [0, {n})")
        as_rank = {"rank": args.as_rank, "world": n,
                   "note": "one GPU running rank R's shard of an N-GPU job without torch.distributed; every "
                           "number is this one GPU's (n_gpus 1)"}
        rank = args.as_rank
    # CCMI_BENCH_BACKEND=gloo: rehearsal of the multi-rank path with several ranks on one
    # card (RCCL needs one GPU per rank); the driver's runs use the default, RCCL
    backend = os.environ.get("CCMI_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % torch.cuda.device_count()
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    B = args.batch
    Pipeline.head = {"default": 0, "valu": 1, "mfma": 2}[args.head]
    Pipeline.fold = args.fold and args.head != "mfma"
    inp = make_inputs(B, dev, seed=1000 * rank + 1)
    mode = "staged" if args.staged else "fused"
    ovp = args.overlap_pyramid and not args.serial and mode == "fused"
    overlap = (args.overlap or ovp) and not args.serial
    dt, stage_ms = measure_path_a(inp, B, args.steps, args.warmup, mode, overlap, dist, dev, join_before_last=ovp)
    fl = flops_per_frame()
    fl["decode_fused"] = flops_fused_per_frame()
    by = bytes_per_frame()
    dom = max(("arm", "decode_fused" if mode == "fused" else "syn"), key=lambda n: stage_ms[n])
    achieved = fl[dom] * B / (stage_ms[dom] * 1e-3) / 1e12
    traffic, src = pmc_traffic(dom, B)

    eager, graph_error, graph_same = None, None, None
    graph = not (args.no_graph or args.staged or (overlap and not ovp))
    if graph:
        # headline: the same K steps replayed from HIP graphs (per-stage times and the
        # roofline above come from the event-instrumented eager pass)
        eager = {"value": round(B * args.steps * world * H * W / dt / 1e6, 2),
                 "ms_per_step": round(dt / args.steps * 1e3, 4)}
        per = 10 if args.steps % 10 == 0 else 1
        try:
            dt, n_done, graph_same = measure_path_a_graph(inp, B, args.steps, args.warmup, dist, dev, per, ovp)
            assert n_done == args.steps
        except Exception as e:  # report the eager timing, and say so in the line
            graph_error = f"{type(e).__name__}: {e}"[:200]
            graph = False
    launch = "HIP graph replays (10 steps per graph)" if graph else (
        "eager launches" + (f" (graph capture failed: {graph_error})" if graph_error else ""))
    n_frames = B * args.steps * world
    value = n_frames * H * W / dt / 1e6
    res = {
        "metric": "decoded Mpixel/s (Synth+ARM+upsample) @1280x720, all GPUs",
        "value": round(value, 2),
        "unit": "Mpixel/s",
        "per_gpu": round(value / world, 2),
        "baseline_metric": "BASELINE.json quotes this per GPU: per_gpu; value is the whole job (bench contract)",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "as_rank": as_rank,
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded N(0,0.5) latents, random-init hop weights per frame)",
        "config": {"workload": "1280x720 YUV420 8-bit frames, hop/c3x decoder (arm 16x2, syn 48-1/3-1/3-3r/3-3r, "
                               "7 latent grids), float forward ARM+rate -> upsampling -> synthesis -> 420 post",
                   "frames_per_step_per_gpu": B, "parallelism": f"image-parallel x{world}",
                   "kernels": (("ARM | upsampling pyramid (to level 2) | fused level-2->1 + last upsampling + synthesis + post"
                                if Pipeline.fold else "ARM | upsampling pyramid | fused last-upsampling+synthesis+post")
                               if mode == "fused"
                               else "ARM | upsampling | synthesis | post")
                   + (" (ARM on a second stream, concurrent with the pyramid)" if ovp else
                      " (ARM on a second stream, concurrent)" if overlap else " (one stream)")},
        "stage_ms_per_step": {k: round(v, 4) for k, v in stage_ms.items()},
        "launch": launch,
        "graph_outputs_equal_eager": graph_same,
        "eager": eager,
        "ms_per_step_median_eager": round(measure_path_a.median_ms, 4),
        "roofline": {"bound": "valu-fp32", "kernel": dom, "achieved": round(achieved, 3), "peak": PEAK_FP32_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(achieved / PEAK_FP32_TFLOPS, 4),
                     "traffic": traffic, "traffic_source": src,
                     "algorithmic_flop_per_launch": fl[dom] * B,
                     "algorithmic_bytes_per_launch": by[dom] * B,
                     "note": "FP32 VALU-bound fused kernel; peak = FP32 vector rate (= f32 MFMA rate, the same "
                             "datapath on gfx950: profiles/r3_mfma_valu_overlap.txt) on MI355X"},
    }
    if args.hd_steps > 0:
        res["path_a_1080p"] = bench_path_a_hd(B, args.hd_steps, args.warmup, rank, world, dist, dev)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(inp)
    if args.decode_reps > 0:
        dec = bench_bitexact_decode(args.decode_reps, rank=rank, world=world, dist=dist, dev=dev)
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            dec["cpu_baseline"] = cpu_decode_baseline()
        if rank == 0:  # latency: one stream at a time through the drop-in entry point
            dec["single_stream"] = bench_single_stream_decode("E")
        res["bitexact_decode"] = dec
        res["bitexact_encode"] = bench_bitexact_encode(rank=rank, world=world, dist=dist, dev=dev)
    if args.hd_decode_reps > 0:
        dec = bench_bitexact_decode(args.hd_decode_reps, "B", 1080, 1920, rank=rank, world=world, dist=dist, dev=dev)
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            dec["cpu_baseline"] = cpu_decode_baseline(cls="B", H=1080, W=1920)
        if rank == 0 and not args.no_single_stream:
            dec["single_stream"] = bench_single_stream_decode("B")
            dec["single_stream_clic"] = bench_single_stream_decode("CLIC")
        res["bitexact_decode_1080p"] = dec
    if args.encode_images > 0:
        lambdas = [float(x) for x in args.encode_lambdas.split(",") if x] or None
        recs, secs, flop, my_secs, shard = bench_encoder(args.encode_images, args.encode_scale, lambdas, rank, world,
                                                         dist, dev)
        tot = len(recs) / secs * 3600.0
        ach = flop / secs / 1e12
        import numpy as np
        res["encoder_overfit"] = {
            "metric": "encoder images/hr (c3x schedule, Kodak-24 proxies 768x512 RGB, hop, all GPUs)",
            "value": round(tot, 2), "per_gpu": round(tot / world, 2), "unit": "images/hr", "n_gpus": world,
            "scaling": "weak", "encodes": len(recs), "encodes_per_gpu": len(recs) // max(1, world),
            "shard": dict(shard, rank=rank), "lambdas": sorted({r["lmbda"] for r in recs}),
            "seconds_max_over_ranks": round(secs, 2),
            "schedule": f"c3x x{args.encode_scale:g}: warm-up 5x400 + 2x400 candidates, phases 10600 + 1500 + 1000 "
                        f"iterations (mean {np.mean([r['iterations'] for r in recs]) if recs else 0:.0f} per image, "
                        f"patience early stops included); quantize_model after "
                        f"the second phase; images of one geometry and lambda overfit together as one batch, "
                        f"the geometry batches concurrently on separate HIP streams; rank r encodes the "
                        f"Kodak-24 at lambda {list(REF_LAMBDAS)}[r % 5], seed r // 5 (fixed work per GPU)",
            "psnr_db_mean": round(float(np.mean([r["psnr_db"] for r in recs])), 3),
            "rate_bpp_mean": round(float(np.mean([r["rate_bpp"] for r in recs])), 4),
            "vs_reference_results": compare_with_reference(recs, None),
            "records": [{k: (round(v, 5) if isinstance(v, float) else v) for k, v in r.items()
                         if k in ("image", "lmbda", "seed", "psnr_db", "rate_bpp", "iterations")} for r in recs],
            "batch_timing": [r["timing"] for r in recs if r.get("timing")],
            "roofline": {"bound": "valu-fp32", "kernel": "whole overfit (all training kernels + host loop)",
                         "achieved": round(ach, 3), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(ach / PEAK_FP32_TFLOPS, 4),
                         "note": "algorithmic FLOPs = 3 x forward (ARM + upsampling + synthesis) per iteration",
                         "kernels": train_kernel_rooflines()},
            "data": "Kodak-24 proxies: the reference's own lambda=1e-4 Kodak .cool streams (35-46 dB) decoded "
                    "bit-exactly (the originals are not in the reference tree); PSNR is measured against the "
                    "proxy, results.tsv against the original"}
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            res["encoder_overfit"]["cpu_baseline"] = cpu_encoder_baseline()
    if rank == 0 or as_rank is not None:  # the process that speaks for the job
        print(json.dumps(res), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
