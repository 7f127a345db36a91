"""The C-ABI library loads and exports every entry point include/ccmi.h declares.
No compute calls here (CPU hosts have no HIP device)."""
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _declared():
    text = (ROOT / "include" / "ccmi.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ccmi_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_expected_symbols():
    import ccmi
    assert _declared() == sorted(ccmi.EXPORTED)


def test_library_exports_every_declared_symbol(ccmi_lib):
    for name in _declared():
        assert hasattr(ccmi_lib, name), name


def test_library_is_built_for_gfx950():
    so = ROOT / "cool-chic_amd" / "lib" / "libccmi.so"
    data = so.read_bytes()
    assert b"amdgcn-amd-amdhsa--gfx950" in data  # offload bundle target id in .hip_fatbin


def test_errors_are_reported_not_fatal(ccmi_lib):
    import ccmi
    rc = ccmi_lib.ccmi_decode_file(b"/nonexistent.cool", b"/tmp/x.yuv", 0, 0, 0, 0)
    assert rc != 0
    assert ccmi.last_error()
    assert ccmi_lib.ccmi_version() >= 100
