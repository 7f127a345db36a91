"""Register / scratch / LDS usage of the kernels in the built libccmi.so (gfx950 code-object
metadata): python tools/kres.py [name-substring ...]"""
import re
import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

LIB = Path(__file__).resolve().parents[1] / "cool-chic_amd" / "lib" / "libccmi.so"
LLVM = Path("/opt/rocm/lib/llvm/bin")

with tempfile.TemporaryDirectory() as td:
    lib = Path(td) / "libccmi.so"
    shutil.copy(LIB, lib)
    subprocess.run([str(LLVM / "llvm-objdump"), "--offloading", str(lib)], cwd=td, check=True, capture_output=True)
    text = "".join(subprocess.run([str(LLVM / "llvm-readelf"), "--notes", str(f)], capture_output=True, text=True).stdout
                   for f in sorted(Path(td).glob("libccmi.so.*gfx950")))
rows, rec = {}, None
KEYS = ("vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count", "private_segment_fixed_size",
        "group_segment_fixed_size")
for line in text.splitlines():
    # one kernel record per "  - ." list item; its own keys sit at 4 spaces (the args' deeper)
    m = re.match(r"^  - \.(\w+):\s*(\S*)", line) or re.match(r"^    \.(\w+):\s*(\S*)", line)
    if not m:
        continue
    if line.startswith("  - "):
        rec = {}
    if rec is None:
        continue
    key, val = m.groups()
    if key == "name":
        rows[val] = rec
    elif key in KEYS:
        rec[key] = int(val)
dem = subprocess.run(["c++filt"], input="\n".join(rows), capture_output=True, text=True).stdout.split("\n")
pats = sys.argv[1:]
for (k, v), d in zip(rows.items(), dem):
    if k.endswith(".kd"):
        continue
    if pats and not any(p in d for p in pats):
        continue
    print(f"{d[:90]:90s} v{v.get('vgpr_count')} a{v.get('agpr_count')} s{v.get('sgpr_count')} "
          f"vspill{v.get('vgpr_spill_count')} scratch{v.get('private_segment_fixed_size')} lds{v.get('group_segment_fixed_size')}")
