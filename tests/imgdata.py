"""Image files written for the texture tests: a minimal PNG encoder (every row filter, every
colour type) that also returns the RGB triples lumo's Image::decode_png (image.rs:19-78) makes of
the image, and Radiance .hdr files (flat RGBE) with RGB::from_rgbe (rgb.rs:79-92)."""
import struct
import zlib

import numpy as np


def _chunk(tag, data):
    return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)


def _filter_row(f, raw, prev, bpp):
    out = bytearray(len(raw))
    for i in range(len(raw)):
        a = raw[i - bpp] if i >= bpp else 0
        b = prev[i]
        c = prev[i - bpp] if i >= bpp else 0
        if f == 0:
            p = 0
        elif f == 1:
            p = a
        elif f == 2:
            p = b
        elif f == 3:
            p = (a + b) // 2
        else:
            pa, pb, pc = abs(b - c), abs(a - c), abs(a + b - 2 * c)
            p = a if pa <= pb and pa <= pc else (b if pb <= pc else c)
        out[i] = (raw[i] - p) & 0xFF
    return bytes(out)


CHANNELS = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}


def png_bytes(w, h, ctype, bd, rows, palette=None, interlace=0):
    """rows: the raw (unfiltered) scanlines; row r uses filter r % 5."""
    bpp = max(1, CHANNELS[ctype] * bd // 8)
    prev = bytes(len(rows[0]))
    body = b""
    for r, raw in enumerate(rows):
        f = r % 5
        body += bytes([f]) + _filter_row(f, raw, prev, bpp)
        prev = raw
    out = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, bd, ctype, 0, 0, interlace))
    if palette is not None:
        out += _chunk(b"PLTE", bytes(palette))
    return out + _chunk(b"IDAT", zlib.compress(body)) + _chunk(b"IEND", b"")


def random_png(rng, w, h, ctype, bd):
    """A random image and the RGB triples lumo's decode_png makes of it."""
    line = (w * CHANNELS[ctype] * bd + 7) // 8
    rows = [bytes(rng.integers(0, 256, size=line, dtype=np.uint8)) for _ in range(h)]
    palette = None
    buf = b"".join(rows)
    if ctype == 3:
        palette = list(rng.integers(0, 256, size=3 * (1 << bd), dtype=np.uint8))
        px = []
        for idx in range(w * h):  # image.rs:29-50, verbatim arithmetic
            if bd == 8:
                bidx, rss, msk = idx, 0, 0xFF
            else:
                per = 8 // bd
                bidx, rss, msk = idx // per, bd * (idx % per), (1 << bd) - 1
            p = (buf[bidx] >> rss) & msk
            px.append((palette[3 * p], palette[3 * p + 1], palette[3 * p + 2]))
    else:
        step = CHANNELS[ctype]
        chunks = [buf[i:i + step] for i in range(0, len(buf), step)]
        px = [(c[0], c[0], c[0]) if ctype in (0, 4) else (c[0], c[1], c[2]) for c in chunks]
    return png_bytes(w, h, ctype, bd, rows, palette), px


def hdr_bytes(w, h, pixels, extra=b"FORMAT=32-bit_rle_rgbe\n\n"):
    return b"#?RADIANCE\n" + extra + f"-Y {h} +X {w}\n".encode() + bytes(np.asarray(pixels, np.uint8).ravel())


def from_rgbe(r, g, b, e):  # rgb.rs:79-92
    if e == 0:
        return (0.0, 0.0, 0.0)
    v = 2.0 ** (e - 128) / 256.0
    return (0.5 + v * r, 0.5 + v * g, 0.5 + v * b)
