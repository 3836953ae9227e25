"""Minimal PNG writer (zlib) for rendered float RGB images (row 0 = bottom)."""
import struct
import sys
import zlib

import numpy as np


def write_png(path, img):
    a = np.clip(np.asarray(img, dtype=np.float64), 0.0, 1.0)[::-1]
    a = np.round(a * 255.0).astype(np.uint8)
    h, w, _ = a.shape
    raw = b"".join(b"\x00" + a[y].tobytes() for y in range(h))

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)

    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n")
        f.write(chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0)))
        f.write(chunk(b"IDAT", zlib.compress(raw, 9)))
        f.write(chunk(b"IEND", b""))


if __name__ == "__main__":
    write_png(sys.argv[2], np.load(sys.argv[1]))
