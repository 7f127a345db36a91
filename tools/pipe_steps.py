"""Run N steps of bench.py's path-A decode pipeline (ARM + upsampling + fused synthesis) on
B synthetic 720p frames, no output checks -- a trace target for rocprofv3, also for the
diagnostic builds whose results are wrong by design (CCMI_DIAG_NOLOAD).
usage: python tools/pipe_steps.py [B=32] [N=20] [serial]  (serial: the ARM and the synthesis tail on
one stream, each kernel alone on the GPU)"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "cool-chic_amd"))
import torch  # noqa: E402

import bench  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
N = int(sys.argv[2]) if len(sys.argv) > 2 else 20
overlap = not (len(sys.argv) > 3 and sys.argv[3] == "serial")
dev = torch.device("cuda:0")
pipe = bench.Pipeline(bench.make_inputs(B, dev, seed=1), B, dev)
for _ in range(3):
    pipe.step(overlap=overlap)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(N):
    pipe.step(overlap=overlap)
e1.record()
torch.cuda.synchronize()
print(f"{B} frames: {e0.elapsed_time(e1) / N:.4f} ms per step", flush=True)
