"""Frame files (ccmi.io, restating coolchic/enc/io/format/{ppm,yuv,png}.py and enc/io/io.py):
PPM / YUV round trips and header rules, the PNG reader on PNGs written here with each of the
five row filters, and on the reference's own test image (tests/golden/192x128_kodim15.png,
the input of test/sanity_check.py).  CPU only."""
import struct
import zlib
from pathlib import Path

import numpy as np
import pytest
import torch

GOLDEN = Path(__file__).resolve().parent / "golden"


def _png(img: np.ndarray, filters) -> bytes:
    """Minimal PNG writer (8-bit RGB, non-interlaced); row y filtered with filters[y % len]."""
    h, w, c = img.shape
    raw = bytearray()
    prev = np.zeros(w * c, dtype=np.int64)
    for y in range(h):
        cur = img[y].reshape(-1).astype(np.int64)
        f = filters[y % len(filters)]
        left = np.concatenate([np.zeros(c, np.int64), cur[:-c]])
        upleft = np.concatenate([np.zeros(c, np.int64), prev[:-c]])
        if f == 0:
            out = cur
        elif f == 1:
            out = cur - left
        elif f == 2:
            out = cur - prev
        elif f == 3:
            out = cur - (left + prev) // 2
        else:
            p = left + prev - upleft
            pa, pb, pc = np.abs(p - left), np.abs(p - prev), np.abs(p - upleft)
            out = cur - np.where((pa <= pb) & (pa <= pc), left, np.where(pb <= pc, prev, upleft))
        raw.append(f)
        raw += (out & 255).astype(np.uint8).tobytes()
        prev = cur

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)

    ihdr = struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0)
    return b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", ihdr) + chunk(b"IDAT", zlib.compress(bytes(raw))) + \
        chunk(b"IEND", b"")


@pytest.mark.parametrize("filters", [(0,), (1,), (2,), (3,), (4,), (0, 1, 2, 3, 4)])
def test_png_reader_every_filter(filters, tmp_path):
    from ccmi import io
    rng = np.random.default_rng(len(filters) * 7 + filters[0])
    img = rng.integers(0, 256, (9, 13, 3), dtype=np.uint8)
    p = tmp_path / "t.png"
    p.write_bytes(_png(img, filters))
    x, bd = io.read_png(p)
    assert bd == 8 and x.shape == (1, 3, 9, 13)
    got = np.round(x[0].numpy() * 255).astype(np.uint8).transpose(1, 2, 0)
    assert np.array_equal(got, img)


def test_png_reference_test_image():
    from ccmi import io
    x, bd = io.read_png(GOLDEN / "192x128_kodim15.png")
    assert bd == 8 and x.shape == (1, 3, 128, 192)
    assert 0.0 <= float(x.min()) and float(x.max()) <= 1.0 and float(x.std()) > 0.05
    # 8-bit content: every value on the 1/255 grid
    assert torch.equal(torch.round(x * 255) / 255, x)


def test_png_rejects_unsupported(tmp_path):
    from ccmi import io
    with pytest.raises(ValueError):
        io.decode_png(b"not a png")


@pytest.mark.parametrize("bd", [8, 10, 16])
def test_ppm_roundtrip(bd, tmp_path):
    from ccmi import io
    mx = 2 ** bd - 1
    g = torch.Generator().manual_seed(bd)
    img = torch.randint(0, mx + 1, (1, 3, 5, 7), generator=g).float() / mx
    io.write_ppm(img, bd, tmp_path / "a.ppm")
    data = (tmp_path / "a.ppm").read_bytes()
    assert data.startswith(f"P6\n7 5\n{mx}\n".encode())
    assert len(data) == len(f"P6\n7 5\n{mx}\n") + 3 * 5 * 7 * (1 if bd == 8 else 2)
    y, b2 = io.read_ppm(tmp_path / "a.ppm")
    assert b2 == bd and torch.equal(torch.round(y * mx), torch.round(img * mx))


def test_ppm_16bit_is_big_endian():
    from ccmi import io
    x, bd = io.parse_ppm(b"P6\n1 1\n65535\n" + bytes([0x01, 0x02, 0, 0, 0xFF, 0xFF]))
    assert bd == 16
    assert torch.allclose(x[0, :, 0, 0] * 65535, torch.tensor([258.0, 0.0, 65535.0]))


@pytest.mark.parametrize("fdt,bd", [("yuv420", 8), ("yuv420", 10), ("yuv444", 8)])
def test_yuv_roundtrip_and_loader(fdt, bd, tmp_path):
    from ccmi import io
    W, H = 16, 8
    mx = 2 ** bd - 1
    g = torch.Generator().manual_seed(3)
    if fdt == "yuv420":
        data = {k: torch.randint(0, mx + 1, s, generator=g).float() / mx
                for k, s in (("y", (1, 1, H, W)), ("u", (1, 1, H // 2, W // 2)), ("v", (1, 1, H // 2, W // 2)))}
    else:
        data = torch.randint(0, mx + 1, (1, 3, H, W), generator=g).float() / mx
    name = f"seq_{W}x{H}_{'420' if fdt == 'yuv420' else '444'}_{bd}b.yuv"
    p = tmp_path / name
    io.write_yuv(data, bd, fdt, p)
    n = H * W + 2 * (H // 2) * (W // 2) if fdt == "yuv420" else 3 * H * W
    assert p.stat().st_size == n * (1 if bd == 8 else 2)
    got, bd2, fdt2 = io.load_frame(p)
    assert (bd2, fdt2) == (bd, fdt)
    if fdt == "yuv420":
        for k in ("y", "u", "v"):
            assert torch.equal(torch.round(got[k] * mx), torch.round(data[k] * mx))
        assert io.to_target(got, fdt).numel() == n
    else:
        assert torch.equal(torch.round(got * mx), torch.round(data * mx))


def test_420_444_conversions():
    from ccmi import io
    x = torch.arange(2 * 3 * 4 * 6, dtype=torch.float32).reshape(2, 3, 4, 6)
    d = io.convert_444_to_420(x)
    assert torch.equal(d["u"][:, 0], x[:, 1, ::2, ::2]) and torch.equal(d["v"][:, 0], x[:, 2, ::2, ::2])
    back = io.convert_420_to_444(d)
    assert torch.equal(back[:, 1, ::2, ::2], x[:, 1, ::2, ::2]) and back.shape == x.shape
    rgb = torch.tensor([[[[255.0]], [[128.0]], [[0.0]]]])
    assert torch.allclose(io.yuv2rgb(io.rgb2yuv(rgb)), rgb, atol=1.5)
