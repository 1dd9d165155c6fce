"""Minimal PNG writer (stdlib zlib) for eyeballing renders: linear RGB -> sRGB-ish gamma."""
import struct
import sys
import zlib

import numpy as np


def save_png(path, rgb, exposure=1.0):
    a = np.nan_to_num(np.asarray(rgb, dtype=np.float64)) * exposure
    a = np.clip(a, 0, 1) ** (1 / 2.2)
    img = (a * 255 + 0.5).astype(np.uint8)
    h, w, _ = img.shape
    raw = b"".join(b"\x00" + img[y].tobytes() for y in range(h))

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)

    png = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0))
    png += chunk(b"IDAT", zlib.compress(raw, 9)) + chunk(b"IEND", b"")
    open(path, "wb").write(png)


if __name__ == "__main__":
    save_png(sys.argv[2], np.load(sys.argv[1]))
