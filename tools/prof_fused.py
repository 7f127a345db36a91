"""Per-phase cycles of the fused decode kernel (diagnostic stamps build):
CCMI_LIB=cool-chic_amd/lib/diag/libccmi_stamps.so python tools/prof_fused.py"""
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "cool-chic_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import ccmi  # noqa: E402

dev = torch.device("cuda:0")
B = 8
inp = bench.make_inputs(B, dev, seed=1)
pipe = bench.Pipeline(inp, B, dev)
L = ccmi.lib()
f = L.ccmi_debug_fused_stamps
f.argtypes = [ctypes.c_void_p, ctypes.c_int]
for _ in range(3):
    pipe.step()
torch.cuda.synchronize()
f(None, 1)
n = 10
for _ in range(n):
    pipe.step()
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 8)()
f(buf, 0)
tiles = (-(-1280 // 60)) * (-(-720 // 28)) * B
names = ["A raw tiles", "B h-pass", "C1 v-pass/gather", "C2 mlp", "D 3x3+store"]
tot = sum(buf[:5])
for i, nm in enumerate(names):
    print(f"{nm:18s} {buf[i] / (n * tiles):10.0f} cycles/WG  {100 * buf[i] / max(tot, 1):5.1f}%")
