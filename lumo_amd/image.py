"""Film output (film.rs:173-210, color/space.rs:6-33): tone-reproduction curve with lumo's
saturating `as u8` conversion, and an 8-bit RGB PNG writer (zlib from the standard library; the
reference uses the png crate).  Off the GPU path: the film itself is compared in f64."""
import struct
import zlib

import numpy as np

SRGB, DCI_P3, REC_2020 = 0, 1, 2  # lumo_camera_params.color_space


def _as_u8(x):
    """Rust `f64 as u8`: truncation toward zero, saturating at 0 / 255, NaN -> 0."""
    x = np.nan_to_num(np.asarray(x, dtype=np.float64), nan=0.0, posinf=255.0, neginf=0.0)
    return np.clip(np.trunc(x), 0, 255).astype(np.uint8)


def encode(rgb, color_space=DCI_P3):
    """ColorSpace::encode: sRGB curve for sRGB and DCI-P3, the Rec. 2020 curve otherwise."""
    c = np.asarray(rgb, dtype=np.float64)
    with np.errstate(invalid="ignore"):
        if color_space in (SRGB, DCI_P3):
            ec = np.where(c <= 0.0031308, 12.92 * c, 1.055 * np.power(c, 1.0 / 2.4) - 0.055)
        else:
            beta = 0.018053968510807
            alpha = 1.0 + 5.5 * beta
            ec = np.where(c <= beta, 4.5 * c, alpha * np.power(c, 0.45) - (alpha - 1.0))
    return _as_u8(ec * 255.0)


def write_png(path, img):
    """8-bit RGB PNG (ColorType::Rgb, BitDepth::Eight)."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w, _ = img.shape
    raw = b"".join(b"\x00" + img[y].tobytes() for y in range(h))

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)

    data = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0))
    data += chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b"")
    with open(path, "wb") as f:
        f.write(data)


def read_png(path):
    """Decoder for the files write_png produces (tests)."""
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, w, h = 8, b"", None, None
    while pos < len(data):
        n = struct.unpack(">I", data[pos:pos + 4])[0]
        t = data[pos + 4:pos + 8]
        d = data[pos + 8:pos + 8 + n]
        if t == b"IHDR":
            w, h = struct.unpack(">II", d[:8])
        elif t == b"IDAT":
            idat += d
        pos += 12 + n
    raw = zlib.decompress(idat)
    rows = [raw[y * (3 * w + 1) + 1:(y + 1) * (3 * w + 1)] for y in range(h)]
    return np.frombuffer(b"".join(rows), dtype=np.uint8).reshape(h, w, 3)
