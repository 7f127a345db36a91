"""Synthetic workloads for bench.py: random-initialised Cool-chic frame parameters and seeded
latents / images, produced on the product side (no oracle import).

The draws follow the shapes and scales of a freshly initialised reference decoder
(arm.py:93-160 linear layers, upsampling.py:46-68 symmetric half-kernels around the bicubic
init, synthesis.py:50-120 conv layers).  The bench's CPU baseline converts the same tensors
into the oracle's ModelParams, so both legs time identical frames.
"""

from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Sequence

import torch

HOP = ((48, 1, False, True), (3, 1, False, False), (3, 3, True, True), (3, 3, True, False))
BICUBIC_HALF = (0.0351562, 0.1054687, -0.2617187, -0.8789063)   # upsampling.py:150 (8-tap, half)


def grid_sizes(H: int, W: int, n_grids: int = 7) -> list[tuple[int, int]]:
    """Latent grid sizes: level i is ceil(H / 2^i) x ceil(W / 2^i) (coolchic.py:208-214)."""
    out, h, w = [], H, W
    for _ in range(n_grids):
        out.append((h, w))
        h, w = (h + 1) // 2, (w + 1) // 2
    return out


def sym_full(half: torch.Tensor, k: int) -> torch.Tensor:
    """Full symmetric kernel from its stored half (upsampling.py:46-68)."""
    return torch.cat([half, torch.flip(half, [0])[k % 2:]])


@dataclass
class FrameWeights:
    """Float parameters of one frame's decoder (ARM MLP, upsampling halves, synthesis convs)."""
    H: int
    W: int
    dim_arm: int
    n_hidden: int
    layers: tuple
    n_grids: int
    gain: float
    arm: list = field(default_factory=list)        # [(W [out, in], b [out])] * (n_hidden + 1)
    ups_half: list = field(default_factory=list)   # n_grids - 1 tensors of 4 (8-tap kernels)
    pre_half: list = field(default_factory=list)   # n_grids - 1 tensors of 4 (7-tap kernels)
    syn: list = field(default_factory=list)        # [(W [out, in, k, k], b [out])]

    def ups_full(self, k: int = 8):
        return [sym_full(h, k) for h in self.ups_half]

    def pre_full(self, k: int = 7):
        return [sym_full(h, k) for h in self.pre_half]


def random_frame(H: int, W: int, dim_arm: int = 16, n_hidden: int = 2, layers: Sequence = HOP, n_grids: int = 7,
                 seed: int = 0, gain: float = 16.0) -> FrameWeights:
    """Seeded random decoder parameters of one frame (CPU tensors, float32)."""
    g = torch.Generator().manual_seed(seed)
    d = dim_arm
    arm = [(torch.randn(d, d, generator=g) / d, torch.randn(d, generator=g) * 0.1) for _ in range(n_hidden)]
    arm.append((torch.randn(2, d, generator=g) / d, torch.randn(2, generator=g) * 0.1))
    bic = torch.tensor(BICUBIC_HALF)
    ups = [bic + 0.02 * torch.randn(4, generator=g) for _ in range(n_grids - 1)]
    pre = [torch.tensor([0.0, 0.0, 0.0, 0.1]) + 0.02 * torch.randn(4, generator=g) for _ in range(n_grids - 1)]
    syn, c = [], n_grids
    for n_out, ks, _, _ in layers:
        syn.append((torch.randn(n_out, c, ks, ks, generator=g) / math.sqrt(c * ks * ks),
                    0.05 * torch.randn(n_out, generator=g)))
        c = n_out
    return FrameWeights(H, W, dim_arm, n_hidden, tuple(layers), n_grids, gain, arm, ups, pre, syn)


def random_latents(B: int, H: int, W: int, n_grids: int = 7, seed: int = 0, std: float = 0.5) -> torch.Tensor:
    """[B, sum_i h_i w_i] float latents, N(0, std^2), flat per frame (level 0 first)."""
    g = torch.Generator().manual_seed(seed)
    return std * torch.randn(B, sum(h * w for h, w in grid_sizes(H, W, n_grids)), generator=g)


def smooth_image(H: int, W: int, seed: int) -> torch.Tensor:
    """Seeded smooth RGB image in [0, 1], [3, H, W]: 2-D sinusoids + N(0, 0.02) noise."""
    g = torch.Generator().manual_seed(seed)
    yy, xx = torch.meshgrid(torch.linspace(0, 1, H), torch.linspace(0, 1, W), indexing="ij")
    f = 3 + seed % 5
    img = torch.stack([0.5 + 0.25 * torch.sin(f * 6.28 * xx) * torch.cos(2 * 6.28 * yy) + 0.1 * torch.sin(19 * xx * yy),
                       0.5 + 0.1 * torch.cos(3 * 6.28 * yy), 0.5 + 0.1 * torch.sin(2 * 6.28 * xx)])
    return (img + 0.02 * torch.randn(img.shape, generator=g)).clamp(0, 1)


__all__ = ["HOP", "grid_sizes", "sym_full", "FrameWeights", "random_frame", "random_latents", "smooth_image"]
