"""Generates the texture-decoder fixtures (run here, where /root/reference
exists; the outputs are committed):

  tests/golden/images/*.png|*.jpg   small synthetic inputs covering the PNG and
                                    JPEG features Texture2D's stb_image path meets
  tests/golden/images.json          for each synthetic input and each texture
                                    file of the reference's Data/*/textures:
                                    width, height, channels and the sha256 of
                                    the pixels the REFERENCE's stb_image
                                    (oracle/_ref/ref_stb_decode, compiled from
                                    /root/reference/external/stb/stb_image.h)
                                    returns with flip_vertically_on_load(true)

    make -C oracle ref && python tests/golden/make_texture_golden.py
"""
import glob
import hashlib
import json
import os
import struct
import subprocess
import tempfile
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
IMG = os.path.join(HERE, "images")
STB = os.path.join(ROOT, "oracle", "_ref", "ref_stb_decode")
REF = "/root/reference/RayTracing/Data"


# --- a small PNG encoder: every colour type / depth, tRNS, Adam7, all filters ---
def _chunk(t, data):
    c = struct.pack(">I", len(data)) + t + data
    return c + struct.pack(">I", zlib.crc32(t + data) & 0xffffffff)


def _pack_row(samples, depth):
    """samples: 1-D int array of one row (already interleaved)."""
    if depth == 8:
        return bytes(np.asarray(samples, np.uint8))
    if depth == 16:
        return b"".join(struct.pack(">H", int(v)) for v in samples)
    out, acc, nb = bytearray(), 0, 0
    for v in samples:
        acc = (acc << depth) | int(v)
        nb += depth
        if nb == 8:
            out.append(acc)
            acc, nb = 0, 0
    if nb:
        out.append(acc << (8 - nb))
    return bytes(out)


def _filter(raw, prev, bpp, ftype):
    out = bytearray(len(raw))
    for i in range(len(raw)):
        a = raw[i - bpp] if i >= bpp else 0
        b = prev[i] if prev is not None else 0
        c = prev[i - bpp] if (prev is not None and i >= bpp) else 0
        if ftype == 0:
            p = 0
        elif ftype == 1:
            p = a
        elif ftype == 2:
            p = b
        elif ftype == 3:
            p = (a + b) >> 1
        else:
            pp = a + b - c
            pa, pb, pc = abs(pp - a), abs(pp - b), abs(pp - c)
            p = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
        out[i] = (raw[i] - p) & 255
    return bytes(out)


def write_png(path, img, depth, color, palette=None, trns=None, interlace=False):
    """img: (h, w, channels) ints at `depth` (palette: indices)."""
    h, w, ch = img.shape
    bpp = max(1, ch * depth // 8)
    passes = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)] \
        if interlace else [(0, 0, 1, 1)]
    data = bytearray()
    k = 0
    for x0, y0, dx, dy in passes:
        sub = img[y0::dy, x0::dx]
        if sub.shape[0] == 0 or sub.shape[1] == 0:
            continue
        prev = None
        for row in sub:
            raw = _pack_row(row.reshape(-1), depth)
            ftype = k % 5
            k += 1
            data += bytes([ftype]) + _filter(raw, prev, bpp, ftype)
            prev = raw
    out = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, color, 0, 0, int(interlace)))
    if palette is not None:
        out += _chunk(b"PLTE", bytes(np.asarray(palette, np.uint8).reshape(-1)))
    if trns is not None:
        out += _chunk(b"tRNS", trns)
    out += _chunk(b"tEXt", b"Comment\x00ancillary chunk, ignored")
    comp = zlib.compress(bytes(data), 9)  # split over two IDAT chunks
    out += _chunk(b"IDAT", comp[:len(comp) // 2]) + _chunk(b"IDAT", comp[len(comp) // 2:])
    out += _chunk(b"IEND", b"")
    with open(path, "wb") as f:
        f.write(out)


def synth_pngs(rng):
    cases = []

    def pat(h, w, ch, maxv):
        y, x = np.mgrid[0:h, 0:w]
        base = np.stack([(x * 37 + y * 11 + c * 57) for c in range(ch)], -1)
        noise = rng.integers(0, maxv + 1, (h, w, ch))
        return np.where(((x + y) % 3 == 0)[..., None], noise, base % (maxv + 1))

    for depth in (1, 2, 4, 8, 16):
        cases.append((f"gray{depth}", pat(7, 13, 1, (1 << depth) - 1), depth, 0, {}))
    for depth in (8, 16):
        cases.append((f"graya{depth}", pat(9, 11, 2, (1 << depth) - 1), depth, 4, {}))
        cases.append((f"rgb{depth}", pat(9, 11, 3, (1 << depth) - 1), depth, 2, {}))
        cases.append((f"rgba{depth}", pat(9, 11, 4, (1 << depth) - 1), depth, 6, {}))
    pal = rng.integers(0, 256, (256, 3))
    for depth in (1, 2, 4, 8):
        cases.append((f"pal{depth}", pat(10, 17, 1, (1 << depth) - 1), depth, 3, {"palette": pal[:1 << depth]}))
    cases.append(("pal8_trns", pat(10, 17, 1, 255), 8, 3, {"palette": pal, "trns": bytes(range(0, 250, 3))}))
    g = pat(8, 12, 1, 255)
    g[2:5, 3:7] = 77
    cases.append(("gray8_trns", g, 8, 0, {"trns": struct.pack(">H", 77)}))
    g2 = pat(8, 12, 1, 3)
    cases.append(("gray2_trns", g2, 2, 0, {"trns": struct.pack(">H", 2)}))
    c = pat(8, 12, 3, 255)
    c[1:3, :] = (10, 20, 30)
    cases.append(("rgb8_trns", c, 8, 2, {"trns": struct.pack(">HHH", 10, 20, 30)}))
    c16 = pat(8, 12, 3, 65535)
    c16[4, :] = (1000, 2000, 3000)
    cases.append(("rgb16_trns", c16, 16, 2, {"trns": struct.pack(">HHH", 1000, 2000, 3000)}))
    for name, (h, w) in (("a", (11, 9)), ("b", (1, 1)), ("c", (17, 3))):
        cases.append((f"adam7_rgb8_{name}", pat(h, w, 3, 255), 8, 2, {"interlace": True}))
    cases.append(("adam7_gray1", pat(13, 21, 1, 1), 1, 0, {"interlace": True}))
    cases.append(("adam7_pal4", pat(13, 21, 1, 15), 4, 3, {"palette": pal[:16], "interlace": True}))
    cases.append(("adam7_rgba16", pat(10, 10, 4, 65535), 16, 6, {"interlace": True}))
    cases.append(("rgb8_wide_odd", pat(5, 33, 3, 255), 8, 2, {}))  # 99-byte rows: GL unpack alignment
    out = []
    for name, img, depth, color, kw in cases:
        path = os.path.join(IMG, name + ".png")
        write_png(path, np.asarray(img), depth, color, **kw)
        out.append(name + ".png")
    return out


def synth_jpegs(rng):
    from PIL import Image
    out = []

    def picture(h, w):
        y, x = np.mgrid[0:h, 0:w]
        r = (128 + 100 * np.sin(x / 5.0) * np.cos(y / 7.0)).astype(np.uint8)
        g = ((x * 7 + y * 3) % 256).astype(np.uint8)
        b = np.clip(rng.normal(128, 60, (h, w)), 0, 255).astype(np.uint8)
        return np.stack([r, g, b], -1)

    specs = [
        ("rgb444_q90", (37, 29), dict(quality=90, subsampling=0)),
        ("rgb422_q75", (37, 29), dict(quality=75, subsampling=1)),
        ("rgb420_q60", (37, 29), dict(quality=60, subsampling=2)),
        ("rgb420_q95_opt", (64, 48), dict(quality=95, subsampling=2, optimize=True)),
        ("rgb444_q100", (16, 16), dict(quality=100, subsampling=0)),
        ("rgb420_1x1", (1, 1), dict(quality=85, subsampling=2)),
        ("rgb420_odd", (17, 9), dict(quality=85, subsampling=2)),
        ("rgb444_q10", (40, 24), dict(quality=10, subsampling=0)),
    ]
    for name, (w, h), kw in specs:
        Image.fromarray(picture(h, w)).save(os.path.join(IMG, name + ".jpg"), "JPEG", **kw)
        out.append(name + ".jpg")
    Image.fromarray(picture(23, 31)[..., 0]).save(os.path.join(IMG, "gray_q80.jpg"), "JPEG", quality=80)
    out.append("gray_q80.jpg")
    try:  # restart intervals (Pillow option), every 2 MCUs
        Image.fromarray(picture(40, 56)).save(os.path.join(IMG, "rgb420_restart.jpg"), "JPEG", quality=80,
                                              subsampling=2, restart_marker_blocks=2)
        out.append("rgb420_restart.jpg")
    except (TypeError, ValueError, OSError):
        pass
    Image.fromarray(picture(24, 32)).save(os.path.join(IMG, "progressive.jpg"), "JPEG", quality=80,
                                          progressive=True)
    out.append("progressive.jpg")
    return out


def stb_decode(path):
    with tempfile.NamedTemporaryFile(suffix=".raw") as t:
        r = subprocess.run([STB, path, t.name], capture_output=True, text=True)
        if r.returncode != 0:
            return None
        w, h, n = map(int, r.stdout.split())
        data = open(t.name, "rb").read()
    assert len(data) == w * h * n
    return dict(width=w, height=h, channels=n, sha256=hashlib.sha256(data).hexdigest())


def main():
    os.makedirs(IMG, exist_ok=True)
    rng = np.random.default_rng(7)
    res = {"synthetic": {}, "reference": {}}
    for name in synth_pngs(rng) + synth_jpegs(rng):
        res["synthetic"][name] = stb_decode(os.path.join(IMG, name))
    for path in sorted(glob.glob(os.path.join(REF, "*", "textures", "*"))):
        res["reference"][os.path.relpath(path, REF)] = stb_decode(path)
    with open(os.path.join(HERE, "images.json"), "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(len(res["synthetic"]), "synthetic,", len(res["reference"]), "reference textures")


if __name__ == "__main__":
    main()
