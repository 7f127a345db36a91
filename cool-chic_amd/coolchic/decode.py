"""Decode CLI, same flags as the reference coolchic/decode.py:20-53; the decoding runs
on the GPU (ccmi_decode_file).  --no_avx2 is accepted for compatibility (no effect)."""

import argparse
import sys

from ccmi.decode import decode_file


def main(argv=None) -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--input", "-i", type=str, default="./bitstream.cool", help="Bitstream path.")
    p.add_argument("--output", "-o", default="", help="output ppm (rgb) or yuv")
    p.add_argument("--no_avx2", action="store_true", help="accepted for compatibility")
    p.add_argument("--verbosity", type=int, default=0)
    p.add_argument("--output_chroma_format", type=int, default=0)
    p.add_argument("--output_bitdepth", type=int, default=0)
    p.add_argument("--device", type=int, default=0, help="HIP device")
    a = p.parse_args(argv)
    rc = decode_file(a.input, a.output, a.output_bitdepth, a.output_chroma_format, a.verbosity, a.device)
    if rc != 0:
        from ccmi import last_error
        print(f"decoding failed: {last_error()}", file=sys.stderr)
    elif a.output:
        print(f"{a.output} created")
    return rc


if __name__ == "__main__":
    sys.exit(main())
