"""Utilities: RGBA8 image codec, offline-safe downloader."""

from .download import download_file
from .imgdata import ImgData, decode_data, encode_data, hex_groups, normalize_hex, parse_hex

__all__ = ["download_file", "ImgData", "decode_data", "encode_data", "hex_groups", "normalize_hex", "parse_hex"]
