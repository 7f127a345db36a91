"""Record the reference decoder's output md5 for the shipped .cool bitstreams.

Runs oracle/_ref/ccdec_ref (the reference C++ decoder compiled from
/root/reference/coolchic/cpp by ``make -C oracle ref``) on every bitstream of the
chosen datasets and writes tests/golden/ref_md5.json:

    {"<dataset>/<file>.cool": {"md5": ..., "bytes": N, "ext": ".yuv"|".ppm",
                               "h": H, "w": W}}

It also copies a small subset of bitstreams into tests/golden/cool/ (data
fixtures; the GPU box has no /root/reference).  Build-container only.
"""

import hashlib
import json
import shutil
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
REF = ROOT / "oracle" / "_ref" / "ccdec_ref"
RESULTS = Path("/root/reference/results/image")
GOLDEN = ROOT / "tests" / "golden"

# fixtures copied into the repo: JVET class D (416x240) and class E (1280x720, the bench
# content) plus a few Kodak (RGB, PPM output) and class B (1080p) streams.
COPY_GLOBS = ["jvet/bitstreams/D-*.cool", "jvet/bitstreams/E-*.cool",
              "kodak/bitstreams/kodim0[1-3]-*.cool", "jvet/bitstreams/B-BQTerrace-*.cool"]


def header(path: Path):
    b = path.read_bytes()
    h, w = (b[2] << 8) | b[3], (b[4] << 8) | b[5]
    fdt = b[6] & 0xF
    return h, w, fdt


def run_one(path: Path):
    h, w, fdt = header(path)
    ext = ".yuv" if fdt != 0 else ".ppm"
    with tempfile.TemporaryDirectory() as td:
        out = Path(td) / ("o" + ext)
        subprocess.run([str(REF), f"--input={path}", f"--output={out}", "--avx2"], check=True,
                       stdout=subprocess.DEVNULL)
        data = out.read_bytes()
    return {"md5": hashlib.md5(data).hexdigest(), "bytes": len(data), "ext": ext, "h": h, "w": w}


def main(datasets):
    files = []
    for ds in datasets:
        files += sorted((RESULTS / ds / "bitstreams").glob("*.cool"))
    with ThreadPoolExecutor(8) as ex:
        res = list(ex.map(run_one, files))
    table = {f"{f.parent.parent.name}/{f.name}": r for f, r in zip(files, res)}
    out = GOLDEN / "ref_md5.json"
    old = json.loads(out.read_text()) if out.exists() else {}
    old.update(table)
    out.write_text(json.dumps(old, indent=1, sort_keys=True) + "\n")
    print(f"{len(table)} entries -> {out}")
    dst = GOLDEN / "cool"
    dst.mkdir(parents=True, exist_ok=True)
    for g in COPY_GLOBS:
        for f in sorted(RESULTS.glob(g)):
            shutil.copy(f, dst / f.name)


if __name__ == "__main__":
    main(sys.argv[1:] or ["jvet", "kodak"])
