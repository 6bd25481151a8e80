"""Shared test helpers: fixture locations and the .data / hex GT codecs."""

import binascii
import os
import struct

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LAB2_DATA = os.path.join(ROOT, "labs", "lab2", "data")
LAB2_GT = os.path.join(ROOT, "labs", "lab2", "data_out_gt")
LAB3_DATA = os.path.join(ROOT, "labs", "lab3", "data")
LAB3_GT = os.path.join(ROOT, "labs", "lab3", "data_out_gt")

# the reference's hard-coded lab3 classes (lab3/lab3_processor.py:42-51)
LAB3_CLASSES = [np.array([[1, 2], [1, 0], [2, 2], [2, 1]]), np.array([[0, 0], [0, 1], [1, 1], [2, 0]])]


def hex_bytes(path):
    return binascii.unhexlify(open(path).read().replace("\n", "").replace(" ", ""))


def bytes_to_img(b: bytes) -> torch.Tensor:
    w, h = struct.unpack("<ii", b[:8])
    return torch.frombuffer(bytearray(b[8:8 + 4 * w * h]), dtype=torch.uint8).reshape(h, w, 4).clone()


def img_to_bytes(img: torch.Tensor) -> bytes:
    h, w = img.shape[:2]
    return struct.pack("<ii", w, h) + img.cpu().contiguous().numpy().tobytes()


def rand_img(h, w, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, 256, (h, w, 4), dtype=torch.uint8, generator=g)


def smooth_img(h, w, seed=0):
    """Natural-image-like data: smooth gradients + noise (exercises non-saturated outputs)."""
    g = torch.Generator().manual_seed(seed)
    yy, xx = torch.meshgrid(torch.arange(h, dtype=torch.float32), torch.arange(w, dtype=torch.float32), indexing="ij")
    base = torch.stack([128 + 100 * torch.sin(xx / 17.0 + c) * torch.cos(yy / 23.0 - c) for c in range(3)], -1)
    noise = torch.randn((h, w, 3), generator=g) * 6
    rgb = torch.clamp(base + noise, 0, 255).to(torch.uint8)
    a = torch.randint(0, 256, (h, w, 1), dtype=torch.uint8, generator=g)
    return torch.cat([rgb, a], -1).contiguous()
