"""pytest configuration: markers, import paths, in-tree native builds.

`-m "not gpu"` tests run anywhere (oracle vs golden vectors, host logic, ABI checks);
`-m gpu` tests need an MI355X and call the HIP path through the C ABI (libccmi.so).
"""
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "cool-chic_amd", ROOT / "oracle"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); runs the libccmi kernels")


def _make(target_dir: Path, *args):
    subprocess.run(["make", "-s", "-C", str(target_dir), *args], check=True)


@pytest.fixture(scope="session")
def ccmi_lib():
    """libccmi.so, built in-tree if missing (hipcc cross-compiles for gfx950 without a GPU)."""
    so = ROOT / "cool-chic_amd" / "lib" / "libccmi.so"
    if not so.exists():
        _make(ROOT / "cool-chic_amd", "-j8")
    import ccmi
    return ccmi.lib()


@pytest.fixture(scope="session")
def oracle_c():
    """ctypes handle on the C restatement of the fixed-point decoder (oracle/)."""
    so = ROOT / "oracle" / "_build" / "libccoracle.so"
    if not so.exists():
        _make(ROOT / "oracle")
    import ctypes
    lib = ctypes.CDLL(str(so))
    lib.cco_decode_file.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    lib.cco_decode_frame_mem.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    lib.cco_frame_free.argtypes = [ctypes.c_void_p]
    lib.cco_arm_params.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    return lib


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but no HIP device is visible (run with -m 'not gpu' on CPU hosts)")
    return torch.device("cuda:0")
