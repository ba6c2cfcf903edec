"""Decode tests/golden/test/parse/test.png (the reference's test/parse/test.png, the image of
its SLM source test, test/photon/test_photon.f90:271-326) with a pure-Python PNG reader
(zlib + the five row filters) and store its first channel -- what stb_image hands the
reference, array = image(:,:,1) -- as image(x, y) in slm_test_png.npz.

Independent of the library's C++ reader (rsmcrt_amd/csrc/png.cpp), which the front-end test
checks against this fixture. Run: python tests/golden/make_png_fixture.py
"""
import os
import struct
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def decode(path):
    d = open(path, "rb").read()
    assert d[:8] == b"\x89PNG\r\n\x1a\n"
    i, idat = 8, b""
    while i < len(d):
        n, = struct.unpack(">I", d[i:i + 4])
        t = d[i + 4:i + 8]
        body = d[i + 8:i + 8 + n]
        if t == b"IHDR":
            w, h, depth, ctype, _, _, inter = struct.unpack(">IIBBBBB", body)
        elif t == b"IDAT":
            idat += body
        i += 12 + n
    assert depth == 8 and inter == 0
    ch = {0: 1, 2: 3, 4: 2, 6: 4}[ctype]
    raw = zlib.decompress(idat)
    stride = w * ch
    out = np.zeros((h, stride), dtype=np.int64)
    prev = np.zeros(stride, dtype=np.int64)
    for y in range(h):
        f = raw[y * (stride + 1)]
        row = np.frombuffer(raw, dtype=np.uint8, count=stride, offset=y * (stride + 1) + 1).astype(np.int64)
        cur = np.zeros(stride, dtype=np.int64)
        for x in range(stride):
            a = cur[x - ch] if x >= ch else 0
            b = prev[x]
            c = prev[x - ch] if x >= ch else 0
            v = row[x]
            if f == 1:
                v += a
            elif f == 2:
                v += b
            elif f == 3:
                v += (a + b) // 2
            elif f == 4:
                p = a + b - c
                pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
                v += a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
            cur[x] = v & 0xFF
        out[y] = cur
        prev = cur
    first = out[:, ::ch]          # [row y, column x]
    return first.T.astype(np.uint8)  # image(x, y)


if __name__ == "__main__":
    img = decode(os.path.join(HERE, "test", "parse", "test.png"))
    np.savez_compressed(os.path.join(HERE, "slm_test_png.npz"), first_channel=img)
    print(img.shape, img.dtype, int(img.max()), int((img > 0).sum()))
