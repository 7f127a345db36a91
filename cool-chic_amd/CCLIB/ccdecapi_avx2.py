"""``CCLIB.ccdecapi_avx2.cc_decode_avx2`` (reference ccdecapi_avx2.cpp:27), HIP-backed."""

from ccmi.decode import decode_file


def cc_decode_avx2(bitstream_filename: str, out_filename: str, output_bitdepth: int = 0,
                   output_chroma_format: int = 0, verbosity: int = 0) -> int:
    return decode_file(bitstream_filename, out_filename, output_bitdepth, output_chroma_format, verbosity)
