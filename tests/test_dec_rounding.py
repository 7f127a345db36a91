"""Integer identities the path-B latency kernel relies on (dec_kernels.hip,
dec_arm_chain_kernel), checked on the CPU in int32 arithmetic with wraparound:

* the reference's symmetric rounding of a /256 (arm_cpu.cpp:94-97, cc-contexts.h:25-29),
  m < 0 ? -((-m + 128) >> 8) : (m + 128) >> 8, equals the branch-free (m + 128 + (m >> 31)) >> 8
  for |m| < 2^31 - 128;
* the scale index (cc-contexts.h:34-43): lsp < 0 ? 0 : min((5 lsp + 128) >> 8, 49) equals
  clamp((5 lsp + 128) >> 8, 0, 49), because (5 lsp + 128) >> 8 <= 0 for every lsp < 0.
Exhaustive on |m| < 2^24 (every value an ARM output of 24-bit operands reaches in practice)
plus 2^23 random int32 values over the whole range."""
import numpy as np


def _ref_round(m):
    m = m.astype(np.int64)
    return np.where(m < 0, -((-m + 128) >> 8), (m + 128) >> 8)


def _fast_round(m):
    m = m.astype(np.int32)
    with np.errstate(over="ignore"):
        return ((m + np.int32(128) + (m >> np.int32(31))) >> np.int32(8)).astype(np.int64)


def test_symmetric_rounding_branch_free():
    m = np.arange(-(1 << 24), 1 << 24, dtype=np.int64)
    assert np.array_equal(_ref_round(m), _fast_round(m))
    r = np.random.default_rng(0).integers(-(2**31) + 128, 2**31 - 128, size=1 << 23, dtype=np.int64)
    assert np.array_equal(_ref_round(r), _fast_round(r))


def test_scale_index_single_clamp():
    ls = np.arange(-(1 << 24), 1 << 24, dtype=np.int64)
    lsp = ls + 256
    ref = np.where(lsp < 0, 0, np.minimum((lsp * 5 + 128) >> 8, 49))
    fast = np.clip((lsp * 4 + lsp + 128) >> 8, 0, 49)
    assert np.array_equal(ref, fast)
