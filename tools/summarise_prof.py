"""Summarise a rocprofv3 run of bench.py (tools/rocprof_bench.sh) into profiles/.

  profiles/<tag>_kernel_stats.csv   -- rocprofv3 --kernel-trace --stats summary (copied)
  profiles/<tag>_pmc.json           -- per-launch HBM bytes per stage from the FETCH_SIZE and
                                       WRITE_SIZE passes, with the gfx950 correction of
                                       MI355X_MICROARCH.md section HBM: FETCH_SIZE counts half
                                       the bytes of wide coalesced reads -> x2; WRITE_SIZE
                                       taken as is.  Both counters are in KiB.

usage: python tools/summarise_prof.py gpurun_out/prof_r1 r1 [frames_per_launch=8]
"""

import csv
import re
import json
import shutil
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
STAGES = {"arm_fwd_kernel": "arm", "ups_level_kernel": "ups", "ups_level_fixed": "ups", "syn_fused_kernel": "syn",
          "syn_layer_kernel": "syn", "post_kernel": "post", "dec_arm": "dec_arm", "dec_ups": "dec_ups",
          "dec_syn": "dec_syn"}
FUSED = False  # set from the trace: a fused-decode run (syn_fused_kernel<..., true>) present


def find(src: Path, dirs, suffix: str) -> Path:
    """The rocprofv3 output file ending in `suffix` under src/<dir> (any run sub-directory;
    tools/rocprof_bench.sh and tools/gpu_round.sh lay them out differently)."""
    for d in ([dirs] if isinstance(dirs, str) else dirs):
        hits = sorted((src / d).rglob(f"*{suffix}"))
        if hits:
            return hits[0]
    raise FileNotFoundError(f"no *{suffix} under {src}/{dirs}")


def stage_of(name: str):
    # the fused decode tail: syn_fused_kernel<CIN, CMID, true> ("Lb1E" in the mangled name)
    if "syn_fused_kernel" in name and ("Lb1E" in name or re.search(r"syn_fused_kernel<\d+, \d+, true", name)):
        return "decode_fused"
    for k, v in STAGES.items():
        if k in name:
            if v == "ups" and FUSED:
                return "ups_pyramid"
            return v
    return None


def per_step_counter(path: Path, counter: str, steps_hint: int = None):
    rows = list(csv.DictReader(path.open()))
    by_stage = defaultdict(list)
    for r in rows:
        if r["Counter_Name"] != counter:
            continue
        st = stage_of(r["Kernel_Name"])
        if st:
            by_stage[st].append(float(r["Counter_Value"]))
    # a 'launch' of a stage = all its dispatches of one step (ups = one dispatch per pyramid level)
    arm_calls = len(by_stage.get("arm", [])) or 1
    out = {}
    for st, vals in by_stage.items():
        out[st] = sum(vals) / arm_calls
    return out


def main(src: str, tag: str, frames: int = 8):
    src = Path(src)
    prof = ROOT / "profiles"
    prof.mkdir(exist_ok=True)
    global FUSED
    stats_csv = find(src, "trace", "kernel_stats.csv")
    shutil.copy(stats_csv, prof / f"{tag}_kernel_stats.csv")
    FUSED = any(stage_of(r["Name"]) == "decode_fused" for r in csv.DictReader(stats_csv.open()))
    fetch = per_step_counter(find(src, ("pmc_fetch", "pmc_size"), "counter_collection.csv"), "FETCH_SIZE")
    write = per_step_counter(find(src, "pmc_write", "counter_collection.csv"), "WRITE_SIZE")
    stats = {r["Name"]: r for r in csv.DictReader(stats_csv.open())}
    avg_ns = {}
    for name, r in stats.items():
        st = stage_of(name)
        if st:
            avg_ns.setdefault(st, 0.0)
            avg_ns[st] += float(r["TotalDurationNs"])
    calls = {stage_of(n): int(r["Calls"]) for n, r in stats.items() if stage_of(n) == "arm"}
    n_steps = calls.get("arm", 1)
    res = {
        "source": str(src),
        "frames_per_launch": frames,
        "note": "per launch = one bench step (batch of frames); ups / ups_pyramid sum their per-level dispatches. "
                "hbm = 2 * FETCH_SIZE + WRITE_SIZE (KiB -> bytes), gfx950 FETCH_SIZE halving corrected "
                "as MI355X_MICROARCH.md prescribes for wide reads (dword-wide accesses are uncalibrated).",
        "fetch_kib_raw": fetch,
        "write_kib_raw": write,
        "per_launch_hbm_bytes": {st: 1024.0 * (2 * fetch.get(st, 0.0) + write.get(st, 0.0)) for st in fetch},
        "avg_ms_per_launch_trace": {st: v / n_steps / 1e6 for st, v in avg_ns.items()},
    }
    (prof / f"{tag}_pmc.json").write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 8)
