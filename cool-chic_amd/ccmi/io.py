"""Frame files of the encoder, with the reference's conventions: PPM (coolchic/enc/io/format/
ppm.py), planar YUV 420 / 444 (yuv.py), PNG (png.py, which uses PIL -- absent here, so the
PNG reader below is zlib + the five row filters of the PNG specification), the frame loader
of enc/io/io.py, and the conversion to the flat target layout of ccmi.train.  Host-side
file I/O only: nothing here runs on the GPU.

Frames are float32 tensors in [0, 1]: RGB / YUV444 as [1, 3, H, W], YUV420 as a dict
{"y": [1, 1, H, W], "u": [1, 1, H/2, W/2], "v": [1, 1, H/2, W/2]} (DictTensorYUV,
yuv.py:22-39)."""

from __future__ import annotations

import math
import os
import struct
import zlib
from pathlib import Path

import numpy as np
import torch
import torch.nn.functional as F

_BLANKS = b"\t\n\x0b\x0c\r "  # C isspace() (ppm.py:56-60)


def _int_until_blank(data: bytes, pos: int) -> tuple[int, int]:
    """_read_int_until_blank (ppm.py:34-68): ASCII integer up to the next blank byte."""
    end = pos
    while data[end] not in _BLANKS:
        end += 1
    return int(data[pos:end].decode("utf-8")), end


def parse_ppm(data: bytes) -> tuple[torch.Tensor, int]:
    """read_ppm (ppm.py:95-157) on bytes: [1, 3, H, W] in [0, 1] and the bitdepth
    log2(max_val + 1).  Like the reference, header comments are not supported; 2-byte
    samples are big endian."""
    if data[:2] != b"P6":
        raise ValueError(f"Invalid file format. PPM file should start with P6. Found {data[:2]!r}.")
    w, p = _int_until_blank(data, 3)
    h, p = _int_until_blank(data, p + 1)
    max_val, p = _int_until_blank(data, p + 1)
    p += 1
    bitdepth = int(math.log2(max_val + 1))
    dt = np.dtype(np.uint8) if max_val <= 255 else np.dtype(">u2")
    raw = np.frombuffer(data, dtype=dt, count=3 * w * h, offset=p).astype(np.float32)
    img = torch.from_numpy(np.ascontiguousarray(raw.reshape(h, w, 3).transpose(2, 0, 1)))[None]
    return img / (2 ** bitdepth - 1), bitdepth


def read_ppm(file_path) -> tuple[torch.Tensor, int]:
    return parse_ppm(Path(file_path).read_bytes())


def ppm_bytes(data: torch.Tensor, bitdepth: int, norm: bool = True) -> bytes:
    """The bytes write_ppm (ppm.py:160-205) stores: "P6\\n{w} {h}\\n{max}\\n" then
    interleaved RGB, 1 byte per sample up to 255, else 2 bytes big endian."""
    c, h, w = data.shape[-3:]
    x = data.detach().reshape(c, h, w).float().cpu()
    max_val = 2 ** bitdepth - 1
    if norm:
        x = torch.round(x * max_val)
    arr = x.numpy().transpose(1, 2, 0)
    arr = arr.astype(np.uint8) if max_val <= 255 else arr.astype(">u2")
    return f"P6\n{w} {h}\n{max_val}\n".encode() + arr.tobytes()


def write_ppm(data: torch.Tensor, bitdepth: int, file_path, norm: bool = True) -> None:
    """write_ppm (ppm.py:160-205).  The reference takes the maximum value from
    `data.bitdepth`, an attribute a tensor does not have; the bitdepth argument is used."""
    Path(file_path).write_bytes(ppm_bytes(data, bitdepth, norm))


def _yuv_size(file_path) -> tuple[int, int]:
    """<name>_<W>x<H>_... (yuv.py:72-79)."""
    w, h = [int(t) for t in os.path.basename(str(file_path)).split(".")[0].split("_")[1].split("x")]
    return w, h


def read_yuv(file_path, frame_idx: int, frame_data_type: str, bit_depth: int):
    """read_yuv (yuv.py:42-125): frame frame_idx of a planar file, 1 byte per sample at 8
    bits, 2 bytes (little endian) otherwise; dict for yuv420, [1, 3, H, W] for yuv444."""
    w, h = _yuv_size(file_path)
    w_uv, h_uv = (int(w / 2), int(h / 2)) if frame_data_type == "yuv420" else (w, h)
    bpv = 1 if bit_depth == 8 else 2
    n_y, n_uv = h * w, h_uv * w_uv
    n = n_y + 2 * n_uv
    raw = np.memmap(file_path, mode="r", shape=n, offset=n * bpv * frame_idx,
                    dtype=np.uint8 if bpv == 1 else np.uint16).astype(np.float32)
    t = torch.from_numpy(raw)
    y = t[:n_y].view(1, 1, h, w)
    u = t[n_y:n_y + n_uv].view(1, 1, h_uv, w_uv)
    v = t[n_y + n_uv:].view(1, 1, h_uv, w_uv)
    norm = 2 ** bit_depth - 1
    if frame_data_type == "yuv420":
        return {"y": y / norm, "u": u / norm, "v": v / norm}
    return torch.cat([y, u, v], dim=1) / norm


def write_yuv(data, bitdepth: int, frame_data_type: str, file_path, norm: bool = True) -> None:
    """write_yuv (yuv.py:128-172): planes back to back, rounded, uint8 (uint16 at 10 bits)."""
    if frame_data_type not in ("yuv420", "yuv444"):
        raise ValueError(f"write_yuv: data type should be yuv420 or yuv444, found {frame_data_type}")
    raw = torch.cat([c.flatten() for c in data.values()]) if frame_data_type == "yuv420" else data.flatten()
    if norm:
        raw = raw * (2 ** bitdepth - 1)
    dt = np.uint16 if bitdepth == 10 else np.uint8
    torch.round(raw).cpu().numpy().astype(dt).tofile(str(file_path))


def rgb2yuv(rgb: torch.Tensor) -> torch.Tensor:
    """rgb2yuv (yuv.py:175-202): [B, 3, H, W] RGB in [0, 255] -> YUV444 in [0, 255]."""
    r, g, b = rgb.split(1, dim=1)
    y = torch.round(0.299 * r + 0.587 * g + 0.114 * b)
    u = torch.round(-0.1687 * r - 0.3313 * g + 0.5 * b + 128)
    v = torch.round(0.5 * r - 0.4187 * g - 0.0813 * b + 128)
    return torch.cat((y, u, v), dim=1)


def yuv2rgb(yuv: torch.Tensor) -> torch.Tensor:
    """yuv2rgb (yuv.py:205-237): the inverse matrix of rgb2yuv, [0, 255] in and out."""
    y, u, v = yuv.split(1, dim=1)
    r = 1.0 * y + -0.000007154783816076815 * u + 1.4019975662231445 * v - 179.45477266423404
    g = 1.0 * y + -0.3441331386566162 * u + -0.7141380310058594 * v + 135.45870971679688
    b = 1.0 * y + 1.7720025777816772 * u + 0.00001542569043522235 * v - 226.8183044444304
    return torch.cat((r, g, b), dim=1)


def convert_444_to_420(yuv444: torch.Tensor) -> dict:
    """convert_444_to_420 (yuv.py:275-299): U, V nearest-downsampled (even rows / cols)."""
    b, c, h, w = yuv444.shape
    uv = F.interpolate(yuv444[:, 1:3], scale_factor=(0.5, 0.5), mode="nearest")
    u, v = uv.split(1, dim=1)
    return {"y": yuv444[:, 0:1], "u": u, "v": v}


def convert_420_to_444(yuv420: dict) -> torch.Tensor:
    """convert_420_to_444 (yuv.py:302-315): U, V nearest-upsampled x2."""
    u = F.interpolate(yuv420["u"], scale_factor=(2, 2))
    v = F.interpolate(yuv420["v"], scale_factor=(2, 2))
    return torch.cat((yuv420["y"], u, v), dim=1)


_PNG_SIG = b"\x89PNG\r\n\x1a\n"


def _unfilter_row(f: int, line: np.ndarray, prev: np.ndarray, ch: int) -> np.ndarray:
    """PNG filter types 0-4 inverted on one row of bytes (ints); prev = the row above."""
    if f == 0:
        return line
    if f == 2:
        return (line + prev) & 255
    if f == 1:  # Sub: running sum per channel
        out = line.copy()
        for c in range(ch):
            out[c::ch] = np.cumsum(line[c::ch]) & 255
        return out
    cur = [0] * len(line)
    ln, pv = line.tolist(), prev.tolist()
    for i in range(len(ln)):
        a = cur[i - ch] if i >= ch else 0
        b = pv[i]
        if f == 3:
            pred = (a + b) >> 1
        elif f == 4:
            c = pv[i - ch] if i >= ch else 0
            p = a + b - c
            pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
            pred = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
        else:
            raise ValueError(f"PNG: bad filter type {f}")
        cur[i] = (ln[i] + pred) & 255
    return np.asarray(cur, dtype=np.int64)


def decode_png(data: bytes) -> tuple[torch.Tensor, int]:
    """read_png (png.py:22-39) without PIL: 8-bit non-interlaced grey / grey+alpha / RGB /
    RGBA (alpha dropped, grey replicated to 3 channels) -> [1, 3, H, W] in [0, 1], bitdepth 8."""
    if data[:8] != _PNG_SIG:
        raise ValueError("not a PNG file")
    pos, idat, hdr = 8, [], None
    while pos + 8 <= len(data):
        n, typ = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        pos += 12 + n
        if typ == b"IHDR":
            hdr = struct.unpack(">IIBBBBB", body)
        elif typ == b"IDAT":
            idat.append(body)
        elif typ == b"IEND":
            break
    if hdr is None:
        raise ValueError("PNG: no IHDR chunk")
    w, h, depth, ctype, _, _, interlace = hdr
    ch = {0: 1, 2: 3, 4: 2, 6: 4}.get(ctype)
    if depth != 8 or ch is None or interlace:
        raise ValueError(f"PNG: only 8-bit non-interlaced grey/RGB(A) is supported (depth {depth}, "
                         f"colour type {ctype}, interlace {interlace})")
    raw = np.frombuffer(zlib.decompress(b"".join(idat)), dtype=np.uint8)
    stride = w * ch
    if raw.size != h * (stride + 1):
        raise ValueError("PNG: image data size does not match the header")
    rows = raw.reshape(h, stride + 1)
    img = np.empty((h, stride), dtype=np.uint8)
    prev = np.zeros(stride, dtype=np.int64)
    for y in range(h):
        cur = _unfilter_row(int(rows[y, 0]), rows[y, 1:].astype(np.int64), prev, ch)
        img[y] = cur
        prev = cur
    px = img.reshape(h, w, ch)
    rgb = np.repeat(px[..., :1], 3, axis=2) if ch <= 2 else px[..., :3]
    t = torch.from_numpy(np.ascontiguousarray(rgb.transpose(2, 0, 1)).astype(np.float32) / 255.0)[None]
    return t, 8


def read_png(file_path) -> tuple[torch.Tensor, int]:
    return decode_png(Path(file_path).read_bytes())


def load_frame(file_path, idx_display_order: int = 0):
    """load_frame_data_from_file (enc/io/io.py:11-42): (data, bitdepth, frame_data_type).
    .yuv: 8 bits if "_8b" is in the name else 10, 420 if "420" is in the name else 444."""
    p = str(file_path)
    if p.endswith(".yuv"):
        bitdepth = 8 if "_8b" in p else 10
        fdt = "yuv420" if "420" in p else "yuv444"
        return read_yuv(p, idx_display_order, fdt, bitdepth), bitdepth, fdt
    if p.endswith(".png"):
        d, bd = read_png(p)
        return d, bd, "rgb"
    if p.endswith(".ppm"):
        d, bd = read_ppm(p)
        return d, bd, "rgb"
    raise ValueError(f"load_frame expects a .yuv, .png or .ppm file, found {p}")


def to_target(data, frame_data_type: str) -> torch.Tensor:
    """Frame data -> the flat float32 target of ccmi.train: Y, U, V (or R, G, B) planes back
    to back, chroma at half resolution for yuv420."""
    if frame_data_type == "yuv420":
        return torch.cat([data["y"].reshape(-1), data["u"].reshape(-1), data["v"].reshape(-1)]).float()
    return data.reshape(-1).float()


__all__ = ["parse_ppm", "read_ppm", "ppm_bytes", "write_ppm", "read_yuv", "write_yuv", "rgb2yuv", "yuv2rgb",
           "convert_444_to_420", "convert_420_to_444", "decode_png", "read_png", "load_frame", "to_target"]
