"""RGBA8 image codec for the three on-disk forms the labs use.

* ``.data`` — little-endian int32 w, int32 h, then w*h RGBA8 pixels, row-major
  (reference lab2/src/main.c:73-91, utils/converter.py:77-79);
* ``.txt``  — hex of those bytes in 8-hex-digit groups (one pixel per group);
  ground-truth files put the header on one line and one image row per line
  (reference lab2/data_out_gt/test_01.txt); comparison ignores whitespace/case;
* ``.png``  — decoded with PIL, **alpha forced to 255** exactly as the reference
  harness does (reference utils/converter.py:97-115); palette/gray PNGs are
  converted to RGB first instead of crashing.

Differences from the reference ``ImgData`` (utils/converter.py:16-60):
  - numpy-vectorised instead of per-pixel Python loops (the reference's hot loop);
  - sidecar files are written to a cache directory, never next to the inputs
    (SURVEY Appendix B #8); ``ImgData(path, cache_dir=None)`` writes nothing;
  - ``size_kb`` keeps the reference's ``sys.getsizeof(bytes)/1024`` definition
    because it is part of the CSV ``filename`` column.
"""

from __future__ import annotations

import binascii
import os
import struct
import sys
from typing import Optional

import numpy as np

HEADER = struct.Struct("<ii")


def decode_data(raw: bytes) -> np.ndarray:
    """bytes of a .data file -> (h, w, 4) uint8 array."""
    if len(raw) < 8:
        raise ValueError("truncated .data header")
    w, h = HEADER.unpack_from(raw, 0)
    if w < 0 or h < 0 or len(raw) < 8 + 4 * w * h:
        raise ValueError(f"bad .data payload for {w}x{h}")
    return np.frombuffer(raw, dtype=np.uint8, count=4 * w * h, offset=8).reshape(h, w, 4).copy()


def encode_data(img: np.ndarray) -> bytes:
    img = np.ascontiguousarray(img, dtype=np.uint8)
    if img.ndim != 3 or img.shape[2] != 4:
        raise ValueError("expected (h, w, 4) uint8")
    h, w = img.shape[:2]
    return HEADER.pack(w, h) + img.tobytes()


def hex_groups(raw: bytes, row_pixels: Optional[int] = None) -> str:
    """Hex text: 8-digit groups separated by spaces (reference _to_hex), optionally
    one line for the header and one line per image row (ground-truth layout)."""
    hx = binascii.hexlify(raw).decode()
    groups = [hx[i:i + 8] for i in range(0, len(hx), 8)]
    if row_pixels is None:
        return " ".join(groups)
    lines = [" ".join(groups[:2])]
    body = groups[2:]
    for i in range(0, len(body), row_pixels):
        lines.append(" ".join(body[i:i + row_pixels]))
    return "\n".join(lines)


def parse_hex(text: str) -> bytes:
    return binascii.unhexlify("".join(text.split()))


def normalize_hex(text: str) -> str:
    """The reference's comparison key: whitespace removed, upper case
    (reference lab2/lab2_processor.py:142-144)."""
    return "".join(text.split()).upper()


def png_to_rgba(path: str) -> np.ndarray:
    from PIL import Image

    with Image.open(path) as im:
        rgb = np.asarray(im.convert("RGB"), dtype=np.uint8)
    a = np.full(rgb.shape[:2] + (1,), 255, dtype=np.uint8)
    return np.concatenate([rgb, a], axis=2)


def rgba_to_png(img: np.ndarray, path: str) -> None:
    from PIL import Image

    Image.fromarray(np.ascontiguousarray(img, dtype=np.uint8), "RGBA").save(path)


class ImgData:
    """One image in any of the three forms; exposes ``pixels`` (h, w, 4 uint8),
    ``raw`` (.data bytes), ``hex`` and a ``data_path`` a lab binary can read."""

    def __init__(self, path: str, idx: Optional[int] = None, cache_dir: Optional[str] = None):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        self.idx = idx
        self.src_path = path
        base = os.path.basename(path)
        self.data_name, self.data_ext = os.path.splitext(base)
        ext = self.data_ext.lower()
        if ext == ".data":
            with open(path, "rb") as f:
                self.raw = f.read()
            self.pixels = decode_data(self.raw)
        elif ext == ".png":
            self.pixels = png_to_rgba(path)
            self.raw = encode_data(self.pixels)
        elif ext == ".txt":
            with open(path) as f:
                self.raw = parse_hex(f.read())
            self.pixels = decode_data(self.raw)
        else:
            raise ValueError(f"expected .data, .png or .txt, got {path}")
        self.cache_dir = cache_dir
        self.data_path = path if ext == ".data" else None
        if self.data_path is None and cache_dir is not None:
            os.makedirs(cache_dir, exist_ok=True)
            self.data_path = os.path.join(cache_dir, f"{self.data_name}.data")
            with open(self.data_path, "wb") as f:
                f.write(self.raw)

    @property
    def width(self) -> int:
        return int(self.pixels.shape[1])

    @property
    def height(self) -> int:
        return int(self.pixels.shape[0])

    @property
    def hex(self) -> str:
        return hex_groups(self.raw)

    @property
    def size_kb(self) -> float:
        return sys.getsizeof(self.raw) / 1024

    def write_sidecars(self, out_dir: str, keep: Optional[str] = None) -> None:
        """The reference's .txt/.png side files, but into ``out_dir``. ``keep``:
        a source file that must not be overwritten by its own sidecar (a .txt or
        .png input converted in place, as the reference does)."""
        os.makedirs(out_dir, exist_ok=True)
        keep = os.path.abspath(keep) if keep else None
        txt = os.path.join(out_dir, f"{self.data_name}.txt")
        if os.path.abspath(txt) != keep:
            with open(txt, "w") as f:
                f.write(self.hex)
        png = os.path.join(out_dir, f"{self.data_name}.png")
        if os.path.abspath(png) != keep:
            rgba_to_png(self.pixels, png)
