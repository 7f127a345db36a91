"""Synthetic .cool streams that drive the path-B ARM decode kernels into the integer forms
no shipped stream reaches (test data, not product code).

The reference's integer ARM (arm_cpu.cpp:65-95) multiplies in int32 everywhere.  The GPU
kernels pick cheaper forms when they are exact and switch at run time when they stop
being exact: 24-bit products while contexts (latent << 8) and weights fit 24 signed bits;
the chain kernel (d <= 16, >= 1 hidden layer) switches layer 0 to 32-bit products after a
decoded |q| > 16383 (CCMI_ARM_FLAG_Q32), its helper wave computes a chunk's preG in 32 bits
once a context leaves 22 bits (PRE32); every layer runs in 32 bits when an ARM weight is
>= 2^23 (W32); the nh = 0 speculative kernel and the one-latent kernel (d = 24 / 32) go to
32-bit layer 0 after a |q| >= 2^15 (BIG).  Every shipped stream decodes with |q| < 2^14 and
weights < 2^23, so these cases are built here: the networks of a committed JVET class-D
stream (upsampling, synthesis) with seeded ARM weights of the case's (dim_arm, n_hidden),
seeded N(0, 2) latents, and -- per case -- two layer-0 latents at +20,000 and -40,000 in the
middle of coded rows, and/or ARM weights of 2^23 + 20 in the last hidden layer and both
output rows.  The block-map header field is varied too (-16 adaptive flags, +8 bypass
flags, 0 no map).

The streams are written by the GPU writer (ccmi.encode.encode_frame), committed under
tests/golden/cool_synth/ (tools/gen_synth_streams.py), and the md5 of the REFERENCE
decoder's output for each (oracle/_ref/ccdec_ref, built from the reference sources) is in
tests/golden/synth_md5.json.
"""
from __future__ import annotations

from pathlib import Path

import numpy as np

GOLDEN = Path(__file__).resolve().parent / "golden"
BASE = GOLDEN / "cool" / "D-BQSquare-lmbda-0001_416x240_60p_yuv420_8b.cool"
SYNTH = GOLDEN / "cool_synth"

# name -> (dim_arm, n_hidden, big latents, big weights, hls_sig_blksize, expected flag bits)
Q32, W32, PRE32, BIG = 2, 4, 8, 16
CASES = {
    "d16h2_q32": (16, 2, True, False, -16, Q32 | PRE32),
    "d16h2_w32": (16, 2, False, True, -16, W32 | PRE32),  # the helper's 24-bit sums need 24-bit weights too
    "d16h2_w32_q32": (16, 2, True, True, -16, W32 | PRE32),
    "d8h1_q32_blk0": (8, 1, True, False, 0, Q32 | PRE32),
    "d16h3_q32_blk8": (16, 3, True, False, 8, Q32 | PRE32),
    "d16h0_q32": (16, 0, True, False, -16, BIG),
    "d8h0_blk8": (8, 0, False, False, 8, 0),
    "d24h2_q32": (24, 2, True, False, -16, BIG),
    "d32h1_w32": (32, 1, False, True, -16, W32),
    "d32h0_blk0": (32, 0, False, False, 0, 0),
}
BIG_AT = ((100, 200, 20000), (150, 301, -40000))  # (row, column, value) in latent grid 0


def kernel_of(name: str) -> str:
    d, nh = CASES[name][:2]
    return "chain" if d <= 16 and nh >= 1 else "spec" if d <= 16 else "one-latent"


def build(name: str, enc):
    """(CoolFrame, [int32 latent grid arrays]) of a case; enc = ccmi.encode."""
    import torch
    d, nh, big_lat, big_w, blk, _ = CASES[name]
    seed = sorted(CASES).index(name)
    fr = enc.parse(BASE.read_bytes())
    desc = fr.desc
    rng = np.random.default_rng(1000 + seed)
    n_w, n_b = nh * d * d + 2 * d, nh * d + 2
    w = rng.integers(-24, 25, n_w).astype(np.int64)
    b = rng.integers(-4, 5, n_b).astype(np.int64)
    if big_w:
        # decoder weight = coded integer << q_step_index[0] (cc-frame-decoder.cpp:201-258)
        sw = int(desc.q_step_index[0])
        big = ((1 << 23) + 20) >> sw
        assert big << sw >= 1 << 23
        last = (nh - 1) * d * d if nh else None
        if last is not None:
            w[last + 3 * d + 5] = big          # last hidden layer, neuron 3, input 5
        w[nh * d * d + 7] = big                # output row 0 (mu), input 7
        w[nh * d * d + d + 2] = -big           # output row 1 (log scale), input 2
    fr.nn["arm_w"], fr.nn["arm_b"] = w, b
    desc.dim_arm, desc.n_hidden_arm = d, nh
    desc.hls_sig_blksize = blk
    desc.ac_max_val_nn = min(65535, int(max(np.abs(v).max(initial=0) for v in fr.nn.values())) + 2)
    g = torch.Generator().manual_seed(seed)
    lat = [torch.round(2.0 * torch.randn(h * ww, generator=g)).to(torch.int32).numpy() for h, ww in fr.grid_sizes]
    lat[-1][:] = 0  # an all-zero grid -> empty substream
    if big_lat:
        W0 = fr.grid_sizes[0][1]
        for y, x, v in BIG_AT:
            lat[0][y * W0 + x] = v
    desc.ac_max_val_latent = min(65535, int(max(np.abs(a).max() for a in lat)) + 2)
    return fr, lat
