"""``CCLIB.ccdecapi_cpu.cc_decode_cpu`` (reference ccdecapi_cpu.cpp:20-30), HIP-backed."""

from ccmi.decode import decode_file


def cc_decode_cpu(bitstream_filename: str, out_filename: str, output_bitdepth: int = 0,
                  output_chroma_format: int = 0, verbosity: int = 0) -> int:
    return decode_file(bitstream_filename, out_filename, output_bitdepth, output_chroma_format, verbosity)
