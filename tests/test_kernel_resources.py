"""Register / scratch budgets of the hot kernels, read from the gfx950 code-object metadata
of the built libccmi.so (no GPU needed).  A budget line here is a performance contract:
crossing a VGPR step halves or thirds the waves a SIMD can hold (512 VGPRs per lane slot:
<= 128 -> 4 waves, <= 168 -> 3, <= 256 -> 2), which the bench only shows at round end.
Round 2 lost 30 % of the headline this way (an opt-in MFMA head compiled into the default
fused kernel took it from 108 to 133 VGPRs)."""
import re
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
LIB = ROOT / "cool-chic_amd" / "lib" / "libccmi.so"
LLVM = Path("/opt/rocm/lib/llvm/bin")

# demangled-name prefix -> (max VGPRs, max VGPR spills, scratch bytes allowed)
BUDGET = {
    # path A fused decode, 7 grids: three workgroups per CU need <= 80 VGPRs (6 waves / SIMD)
    # (measured: 3 resident workgroups 0.79 ms vs 2 resident 0.85 ms per 32 frames,
    # tools/occ_probe.sh); no spills since the lane indices are re-derived after the head and
    # per 3x3 layer (round 2 held them across: 5 spilled VGPRs, ~190 MB of scratch writes
    # per 32-frame launch)
    "syn_fused_kernel<7, 3, true, false, 0, false>": (80, 0, 0),   # any head width
    "syn_fused_kernel<7, 3, true, false, 48, false>": (80, 0, 0),  # headline (hop): unrolled head
    "syn_fused_kernel<7, 3, true, false, 48, true>": (80, 0, 0),   # the same + the level-2 -> 1 fold (opt-in)
    "syn_fused_kernel<7, 4, true, false, 0, false>": (128, 0, 0),   # 4-channel tail: 2 workgroups
    "arm_fwd_kernel<16, 2>": (128, 0, 0),                   # path A ARM + rate (hop: 2 hidden layers)
    "arm_fwd_kernel<16, -1>": (128, 0, 0),                  # any hidden-layer count
    "ups_level_fixed<8, 7>": (64, 0, 0),                    # upsampling pyramid
    "dec_arm_kernel<16, 2>": (128, 0, 0),                   # path B ARM + CABAC
    "dec_arm_spec_kernel<16, 2>": (128, 0, 0),
    # path B chain kernel: one wave per stream, 4-5 streams per CU in a batch (LDS-bound); the
    # chunk precompute's 272 layer-0 weights are re-read per chunk (hoisted, they took the
    # kernel to 256 + 146 VGPRs at occupancy 1)
    "dec_arm_chain_kernel<16, 2>": (128, 0, 0),
    "dec_arm_chain_kernel<8, 2>": (128, 0, 0),
    "dec_ups_level_batch": (64, 0, 0),
    # training step (3 waves / SIMD).  t_arm16<2>: round 3 spilled 13 VGPRs across its tile
    # loop (their reloads' vmcnt(0) waited for the previous tile's gradient atomics); since
    # round 4 all weights sit in LDS, the ReLU masks in lane masks and the tile-invariant
    # indices are re-derived per tile: 4 waves / SIMD (<= 128 VGPRs) (477 -> 448 us per launch
    # against the 3-wave build, profiles/r4j_train_ab.txt).  Round 6: the prefetch's staging
    # indices too (two of them were spilled, reloaded with a vmcnt(0) inside the tile loop):
    # one spilled value left, live only in the prologue / epilogue
    "t_arm16<2>": (128, 1, 8),
    "t_head_bwd<7, 3, true>": (168, 0, 0),  # unit-pair packed form (output-ReLU architectures)
    # the tiled form (linear output layer, every reference architecture): 4 waves / SIMD
    "t_head_bwd_t<7, 3>": (128, 0, 0),
    # 3x3 backward, one launch (input + 4x4x1-MFMA weight gradients): 5 waves / SIMD (<= 96 VGPRs,
    # with the 31 KB of LDS five workgroups per CU; profiles/r5zf_*: with the border weights in
    # LDS, 74.6 -> 69.1 us per layer)
    "t_sp_bwd<3>": (96, 0, 0),
    "t_sp_bwd<11>": (96, 0, 0),   # the same + the previous layer's ReLU mask on the written gradient
    # persistent form with the next tile's ring in registers: 4 waves / SIMD (one spilled value in
    # the prologue); with the mask bit none
    "t_sp_bwd<7>": (128, 1, 8),
    "t_sp_bwd<15>": (128, 0, 0),
}


def _metadata(tmp_path):
    objdump, readelf = LLVM / "llvm-objdump", LLVM / "llvm-readelf"
    if not (LIB.exists() and objdump.exists() and readelf.exists()):
        pytest.skip("libccmi.so or the ROCm llvm tools are absent")
    lib = tmp_path / "libccmi.so"
    shutil.copy(LIB, lib)
    subprocess.run([str(objdump), "--offloading", str(lib)], cwd=tmp_path, check=True, capture_output=True)
    text = "".join(subprocess.run([str(readelf), "--notes", str(f)], capture_output=True, text=True).stdout
                   for f in sorted(tmp_path.glob("libccmi.so.*gfx950")))
    out, name = {}, None
    for line in text.splitlines():
        m = re.match(r"\s+\.name:\s+(\S+)", line)
        if m:
            name = m.group(1)
            out[name] = {}
            continue
        m = re.match(r"\s+\.(vgpr_count|vgpr_spill_count|private_segment_fixed_size):\s+(\d+)", line)
        if m and name:
            out[name][m.group(1)] = int(m.group(2))
    names = list(out)
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
    return {d: out[n] for n, d in zip(names, dem)}


def test_hot_kernel_register_budgets(tmp_path):
    meta = _metadata(tmp_path)
    assert len(meta) > 50
    lines = []
    for key, (vmax, spills, scratch) in BUDGET.items():
        hits = [(d, v) for d, v in meta.items() if key in d]
        assert hits, f"kernel {key} not found in libccmi.so"
        for d, v in hits:
            lines.append(f"{d[:100]}: {v}")
            assert v.get("vgpr_count", 0) <= vmax, lines[-1]
            assert v.get("vgpr_spill_count", 0) <= spills, lines[-1]
            assert v.get("private_segment_fixed_size", 0) <= scratch, lines[-1]
    print("\n".join(lines))
