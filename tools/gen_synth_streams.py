"""Write the synthetic .cool streams of tests/synth_streams.py with the GPU writer.

GPU box:    python tools/gen_synth_streams.py gpurun_out/synth     (ccmi.encode.encode_frame)
container:  python tools/gen_synth_streams.py --md5 DIR           (the reference decoder
            oracle/_ref/ccdec_ref on every DIR/*.cool -> tests/golden/synth_md5.json; copy the
            streams to tests/golden/cool_synth/ first)
"""
import hashlib
import json
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "cool-chic_amd"))
sys.path.insert(0, str(ROOT / "tests"))

import synth_streams as S  # noqa: E402


def write(out: Path) -> None:
    import numpy as np
    import torch
    from ccmi import encode as enc
    out.mkdir(parents=True, exist_ok=True)
    for name in S.CASES:
        fr, lat = S.build(name, enc)
        x = torch.from_numpy(np.concatenate(lat)).to("cuda:0")
        s = enc.encode_frame(fr, x, search_counts=True)
        (out / f"{name}.cool").write_bytes(s)
        print(name, len(s), "bytes", flush=True)


def md5(d: Path) -> None:
    ref = ROOT / "oracle" / "_ref" / "ccdec_ref"
    res = {}
    for f in sorted(d.glob("*.cool")):
        got = {}
        for mode in ("cpu", "avx2"):  # the reference's two decoders (ccdecapi_cpu / ccdecapi_avx2)
            with tempfile.TemporaryDirectory() as td:
                o = Path(td) / "o.yuv"
                subprocess.run([str(ref), f"--input={f}", f"--output={o}"] + (["--avx2"] if mode == "avx2" else []),
                               check=True, stdout=subprocess.DEVNULL)
                b = o.read_bytes()
            got[mode] = hashlib.md5(b).hexdigest()
        res[f.stem] = {"md5": got["cpu"], "md5_avx2": got["avx2"], "bytes": len(b), "ext": ".yuv"}
        print(f.stem, res[f.stem], flush=True)
    (ROOT / "tests" / "golden" / "synth_md5.json").write_text(json.dumps(
        {"source": "oracle/_ref/ccdec_ref (the reference decoder compiled from its own sources) on "
                   "tests/golden/cool_synth/*.cool", "streams": res}, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "--md5":
        md5(Path(sys.argv[2]))
    else:
        write(Path(sys.argv[1]))
