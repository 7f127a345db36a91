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


def test_decode_batch_plan_is_host_only(ccmi_lib):
    """ccmi_decode_batch_plan sizes a batch from the streams' headers alone (no CABAC, no GPU):
    every committed stream's output size equals the reference decoder's output size
    (tests/golden/ref_md5.json), YUV and PPM; the workspace grows with the batch; truncated
    streams and null arguments are errors with a message, never a crash."""
    import ctypes as C
    import json
    import ccmi
    md5 = json.loads((ROOT / "tests" / "golden" / "ref_md5.json").read_text())
    files = sorted((ROOT / "tests" / "golden" / "cool").rglob("*.cool"))
    keys = [("clic20-pro-valid/" if f.parent.name == "clic" else "kodak/" if f.name.startswith("kodim") else "jvet/")
            + f.name for f in files]
    data = [f.read_bytes() for f in files]
    n = len(data)
    bufs = [C.create_string_buffer(d, len(d)) for d in data]
    sp = (C.c_void_p * n)(*[C.cast(b, C.c_void_p) for b in bufs])
    ln = (C.c_size_t * n)(*[len(d) for d in data])
    plan = ccmi_lib.ccmi_decode_batch_plan
    plan.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
    plan.restype = C.c_int
    sizes, need = (C.c_size_t * n)(), C.c_size_t(0)
    for as_yuv in (1, 0):
        checked = 0
        assert plan(sp, ln, n, 0, 0, as_yuv, sizes, C.byref(need)) == 0, ccmi.last_error()
        for k, s in zip(keys, sizes):
            ref = md5.get(k)
            if ref and (ref["ext"] == ".yuv") == bool(as_yuv):
                assert int(s) == ref["bytes"], k
                checked += 1
        assert checked > 0
    one, need1 = (C.c_size_t * 1)(), C.c_size_t(0)
    assert plan(sp, ln, 1, 0, 0, 1, one, C.byref(need1)) == 0
    assert 0 < need1.value < need.value
    short = C.create_string_buffer(data[0][:60], 60)
    sp1 = (C.c_void_p * 1)(C.cast(short, C.c_void_p))
    ln1 = (C.c_size_t * 1)(60)
    assert plan(sp1, ln1, 1, 0, 0, 1, one, C.byref(need1)) != 0 and ccmi.last_error()
    assert plan(None, ln1, 1, 0, 0, 1, one, C.byref(need1)) != 0 and "null" in ccmi.last_error()
