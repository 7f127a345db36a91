"""Decode one class-E stream (for counter profiling of the ARM/CABAC kernel)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "cool-chic_amd"))
from ccmi import decode  # noqa: E402

f = ROOT / "tests/golden/cool" / (sys.argv[1] if len(sys.argv) > 1 else "E-FourPeople-lmbda-00001_1280x720_60p_yuv420_8b.cool")
out = decode.decode_batch([f.read_bytes()])
print(decode.last_timing())
