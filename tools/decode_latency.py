"""Single-stream latency of the bit-exact decoder's drop-in entry point: ccmi_decode_file
(the cc_decode_cpu replacement, file in -> .yuv out) on each shipped class-E 1280x720
stream, one stream at a time, wall clock around the C call (parse, H2D, kernels, D2H,
file write), md5 of the output checked against the reference decoder's.  Also the
kernel stages of the same decode (ccmi_decode_last_timing).  Prints one JSON line.
Usage: python tools/decode_latency.py [reps]"""
import ctypes
import hashlib
import json
import statistics
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "cool-chic_amd"))

import ccmi  # noqa: E402

MD5 = json.loads((ROOT / "tests/golden/ref_md5.json").read_text())
files = sorted((ROOT / "tests/golden/cool").glob(sys.argv[2] if len(sys.argv) > 2 else "E-*.cool"))
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
L = ccmi.lib()
L.ccmi_decode_last_timing.argtypes = [ctypes.POINTER(ctypes.c_float)]
rows = []
with tempfile.TemporaryDirectory() as td:
    out = Path(td) / "o.yuv"
    assert L.ccmi_decode_file(str(files[0]).encode(), str(out).encode(), 0, 0, 0, 0) == 0, ccmi.last_error()
    for f in files:
        best, stages = None, None
        for _ in range(reps):
            t0 = time.perf_counter()
            rc = L.ccmi_decode_file(str(f).encode(), str(out).encode(), 0, 0, 0, 0)
            dt = time.perf_counter() - t0
            assert rc == 0, ccmi.last_error()
            if best is None or dt < best:
                best = dt
                ms = (ctypes.c_float * 4)()
                L.ccmi_decode_last_timing(ms)
                stages = [round(v, 2) for v in ms]
        ok = hashlib.md5(out.read_bytes()).hexdigest() == MD5["jvet/" + f.name]["md5"]
        rows.append({"stream": f.name.split("_")[0], "ms": round(best * 1e3, 2), "stages_ms": stages, "md5_ok": ok})
print(json.dumps({"metric": "ccmi_decode_file wall ms per stream (best of %d)" % reps,
                  "mean_ms": round(statistics.mean(r["ms"] for r in rows), 2),
                  "max_ms": max(r["ms"] for r in rows), "all_md5_ok": all(r["md5_ok"] for r in rows),
                  "stage_names": ["h2d+setup", "arm_cabac", "ups_syn_out", "d2h"], "rows": rows}))
