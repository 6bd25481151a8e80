"""Fetch an extra input image over HTTP(S) in 8 KiB chunks (reference
utils/download_files.py:5-35). Offline environments get a clear error instead
of a hang: a short connect timeout, and ``file://`` URLs are copied locally."""

from __future__ import annotations

import os
import shutil
import uuid
from typing import Optional


def download_file(url: str, save_dir: str, filename: Optional[str] = None, timeout: float = 10.0) -> str:
    os.makedirs(save_dir, exist_ok=True)
    if not filename:
        filename = os.path.basename(url.split("?")[0]) or f"{uuid.uuid4()}.png"
    dst = os.path.join(save_dir, filename)
    if url.startswith("file://"):
        shutil.copyfile(url[len("file://"):], dst)
        return dst
    import requests

    with requests.get(url, stream=True, timeout=timeout) as resp:
        resp.raise_for_status()
        with open(dst, "wb") as f:
            for chunk in resp.iter_content(chunk_size=8192):
                f.write(chunk)
    return dst
