"""Bit-exact decode leg of bench.py on its own: python tools/ab_decode.py [reps ...]
(a -DCCMI_DIAG_NOSPEC build times the one-latent-per-pass ARM kernel)."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402

for reps in [int(x) for x in (sys.argv[1:] or ["1", "8"])]:
    print(json.dumps(bench.bench_bitexact_decode(reps)), flush=True)
