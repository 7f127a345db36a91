"""Throughput of the bit-exact HIP decoder (path B) on the shipped JVET class-E (1280x720;
CCMI_CLS=B: class-B 1920x1080) bitstreams: `reps` copies of the streams decoded per
ccmi_decode_batch call.
Prints one JSON line per batch size.  Wall clock around the whole call (host parse,
H2D, kernels, D2H of the YUV bytes)."""
import hashlib
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "cool-chic_amd"))

import torch  # noqa: E402

from ccmi import decode  # noqa: E402

MD5 = json.loads((ROOT / "tests/golden/ref_md5.json").read_text())
CLS = os.environ.get("CCMI_CLS", "E")
HH, WW = (720, 1280) if CLS == "E" else (1080, 1920)
files = sorted((ROOT / "tests/golden/cool").glob(f"{CLS}-*.cool"))
streams = [f.read_bytes() for f in files]
for reps in [int(x) for x in (sys.argv[1:] or ["1", "4"])]:
    batch = streams * reps
    decode.decode_batch(batch[:2])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    outs = decode.decode_batch(batch)
    dt = time.perf_counter() - t0
    ok = all(hashlib.md5(o).hexdigest() == MD5["jvet/" + f.name]["md5"] for f, o in zip(files * reps, outs))
    tm = decode.last_timing()
    kern = (tm["arm_cabac"] + tm["ups_syn_out"]) / 1e3
    print(json.dumps({"frames": len(batch), "seconds": round(dt, 4), "fps": round(len(batch) / dt, 2),
                      "mpix_s": round(len(batch) * WW * HH / dt / 1e6, 2),
                      "mpix_s_kernels": round(len(batch) * WW * HH / kern / 1e6, 2),
                      "stage_ms": {k: round(v, 2) for k, v in tm.items()}, "bit_exact": ok}), flush=True)
