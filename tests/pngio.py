"""Independent PNG writer/reader (zlib + struct) for the CLI tests: writes
every colour type / bit depth / row filter the CLI's decoder must handle, and
reads back the CLI's RGB output."""
import struct
import zlib

import numpy as np


def _chunk(t, data):
    return struct.pack(">I", len(data)) + t + data + struct.pack(">I", zlib.crc32(t + data) & 0xFFFFFFFF)


def _filter_row(f, row, prev, bpp):
    out = bytearray(len(row))
    for i in range(len(row)):
        a = row[i - bpp] if i >= bpp else 0
        b = prev[i] if prev is not None else 0
        c = prev[i - bpp] if (prev is not None and i >= bpp) else 0
        if f == 0:
            p = 0
        elif f == 1:
            p = a
        elif f == 2:
            p = b
        elif f == 3:
            p = (a + b) >> 1
        else:
            q = a + b - c
            pa, pb, pc = abs(q - a), abs(q - b), abs(q - c)
            p = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
        out[i] = (row[i] - p) & 0xFF
    return bytes(out)


def write_png(path, samples, ctype, depth, palette=None, filters=(0, 1, 2, 3, 4)):
    """samples: (H, W, ch) unsigned ints at `depth` bits (ch per colour type)."""
    H, W, ch = samples.shape
    rows = []
    for y in range(H):
        if depth < 8:
            per = 8 // depth
            r = bytearray((W * depth + 7) // 8)
            for x in range(W):
                r[x // per] |= int(samples[y, x, 0]) << (8 - depth * (x % per + 1))
            rows.append(bytes(r))
        elif depth == 8:
            rows.append(samples[y].astype(np.uint8).tobytes())
        else:
            rows.append(samples[y].astype(">u2").tobytes())
    bpp = max(1, ch * depth // 8)
    raw = b""
    prev = None
    for y, r in enumerate(rows):
        f = filters[y % len(filters)]
        raw += bytes([f]) + _filter_row(f, r, prev, bpp)
        prev = r
    ihdr = struct.pack(">IIBBBBB", W, H, depth, ctype, 0, 0, 0)
    data = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", ihdr)
    if palette is not None:
        data += _chunk(b"PLTE", bytes(np.asarray(palette, np.uint8).ravel()))
    data += _chunk(b"IDAT", zlib.compress(raw)) + _chunk(b"IEND", b"")
    with open(path, "wb") as fh:
        fh.write(data)


def write_gray8(path, img):
    write_png(path, img[..., None], 0, 8)


def read_rgb8(path):
    """Reader for the CLI's output (8-bit RGB, any filter) -> (H, W, 3) u8."""
    d = open(path, "rb").read()
    assert d[:8] == b"\x89PNG\r\n\x1a\n"
    p, idat, W = 8, b"", 0
    while True:
        n = struct.unpack(">I", d[p:p + 4])[0]
        t = d[p + 4:p + 8]
        body = d[p + 8:p + 8 + n]
        if t == b"IHDR":
            W, H, depth, ctype = struct.unpack(">IIBB", body[:10])
            assert depth == 8 and ctype == 2
        elif t == b"IDAT":
            idat += body
        elif t == b"IEND":
            break
        p += 12 + n
    raw = zlib.decompress(idat)
    stride = 3 * W + 1
    out = np.zeros((H, W * 3), np.uint8)
    prev = np.zeros(W * 3, np.int64)
    for y in range(H):
        f = raw[y * stride]
        row = np.frombuffer(raw[y * stride + 1:(y + 1) * stride], np.uint8).astype(np.int64)
        cur = np.zeros(W * 3, np.int64)
        for i in range(W * 3):
            a = cur[i - 3] if i >= 3 else 0
            b = prev[i]
            c = prev[i - 3] if i >= 3 else 0
            pr = [0, a, b, (a + b) >> 1, None][f]
            if f == 4:
                q = a + b - c
                pa, pb, pc = abs(q - a), abs(q - b), abs(q - c)
                pr = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
            cur[i] = (row[i] + pr) & 0xFF
        out[y] = cur
        prev = cur
    return out.reshape(H, W, 3)


def luma(r, g, b):
    """cvtColor RGB->GRAY fixed point (what the CLI's decoder applies)."""
    return ((r.astype(np.int64) * 4899 + g.astype(np.int64) * 9617 + b.astype(np.int64) * 1868 + (1 << 13)) >> 14
            ).astype(np.uint8)
