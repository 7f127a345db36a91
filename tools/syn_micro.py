"""Synthesis-kernel micro-benchmark: time ccmi.forward.syn_forward on 720p frames for a
few layer stacks (head only, head + k 3x3 layers) to see where the fused kernel spends
its time.  Run on the GPU box: python tools/syn_micro.py"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "cool-chic_amd"))

import torch  # noqa: E402

from ccmi import forward as F  # noqa: E402

STACKS = {
    "head48": [(48, 1, False, True), (3, 1, False, False)],
    "head48+1x3": [(48, 1, False, True), (3, 1, False, False), (3, 3, False, True)],
    "head48+2x3": [(48, 1, False, True), (3, 1, False, False), (3, 3, False, True), (3, 3, True, True)],
    "hop": [(48, 1, False, True), (3, 1, False, False), (3, 3, False, True), (3, 3, True, True), (3, 3, True, False)],
    "head16+3x3": [(16, 1, False, True), (3, 1, False, False), (3, 3, False, True), (3, 3, True, True),
                   (3, 3, True, False)],
}


def main():
    B, C, H, W = 8, 7, 720, 1280
    dev = torch.device("cuda:0")
    x = torch.randn(B, C, H, W, device=dev)
    for name, layers in STACKS.items():
        P = F.syn_param_count(C, layers)
        p = (torch.randn(B, P, device=dev) * 0.2).contiguous()
        for _ in range(3):
            F.syn_forward(x, layers, p)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 20
        e0.record()
        for _ in range(n):
            F.syn_forward(x, layers, p)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / n
        print(f"{name:14s} {ms * 1e3:8.1f} us / {B} frames", flush=True)


if __name__ == "__main__":
    main()
