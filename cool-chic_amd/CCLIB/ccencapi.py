"""``CCLIB.ccencapi`` (reference ccencapi.cpp:52-60, built by setup.py:27-40): the same
function / class names and argument meaning, backed by libccmi's host CABAC encoder."""

from pathlib import Path

from ccmi import encode as _enc


def cc_code_wb_bac(out_file: str, x: list, use_count: int) -> int:
    """Code weights / biases into out_file; returns the Exp-Golomb count used
    (use_count < 0: search 0..12 for the fewest bytes)."""
    b, used = _enc.code_wb(x, use_count)
    Path(out_file).write_bytes(b)
    return used


def cc_code_latent_layer_bac(out_file: str, x: list, mu: list, log_scale: list, layer_height: int,
                             layer_width: int, hls_sig_blksize: int) -> None:
    """Code one latent grid (integer values, mu / log_scale x256) into out_file."""
    Path(out_file).write_bytes(_enc.code_latent_layer(x, mu, log_scale, layer_height, layer_width,
                                                      hls_sig_blksize))


class cc_decode_wb:  # noqa: N801 -- reference class name
    """Sequential weight / bias decoder over one substream file (ccencapi.cpp:40-50, :412-454)."""

    def __init__(self, in_file: str):
        self._bytes = Path(in_file).read_bytes()
        self._runs = []

    def decode_wb_continue(self, n_weights: int, scale_index: int) -> list:
        self._runs.append((int(n_weights), int(scale_index)))
        return _enc.decode_wb(self._bytes, self._runs)[-1].tolist()
