"""Summarise a GPU session directory written by tools/gpu_lib.sh: one line per step log that
ends in a JSON line (bench.py, tools/decode_latency.py, tools/bench_train.py, ...), with the
fields that matter for A/B reading.  Usage: python tools/ab_summary.py gpurun_out/r6b"""
import json
import sys
from pathlib import Path


def last_json(p: Path):
    for line in reversed(p.read_text(errors="replace").strip().splitlines()):
        line = line.strip()
        if line.startswith("{"):
            try:
                return json.loads(line)
            except json.JSONDecodeError:
                return None
    return None


def brief(d: dict) -> str:
    if "metric" in d and "stage_ms_per_step" in d:  # bench.py
        s = f"value {d['value']:.1f} stages {d['stage_ms_per_step']} frac {d.get('roofline', {}).get('frac')}"
        hd = d.get("path_a_1080p")
        if hd:
            s += f" | 1080p {hd.get('value')} {hd.get('stage_ms_per_step')}"
        return s
    if "mean_ms" in d:  # decode_latency.py
        return f"mean {d['mean_ms']} max {d.get('max_ms')} md5 {d.get('all_md5_ok')}"
    return json.dumps({k: v for k, v in d.items() if not isinstance(v, (list, dict))})[:300]


for p in sorted(Path(sys.argv[1]).glob("*.log")):
    d = last_json(p)
    if d is not None:
        print(f"{p.stem:24s} {brief(d)}")
