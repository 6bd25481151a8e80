#!/usr/bin/env python3
"""Ground truth for the lab2 metric_calc buckets from the CPU reference.

The reference ships GT for two 3x3 images only (lab2/data_out_gt/test_0{1,2});
every other image passes its harness unconditionally
(/root/reference/lab2/lab2_processor.py:139-144). This
writes <bucket>_out_gt/<stem>.{txt,png} next to each bucket, computed by the
serial C reference program (labs/lab2/src/cpu_exe, the reference's
lab2/src/main.c behaviour with contraction off): hex .txt (the reference's GT
format) for the small .data images, lossless RGBA .png for the medium/large
PNG inputs (their alpha is 255, so PNG round-trips exactly; hex would be
~9 bytes per pixel of text). The harness picks them up as GT automatically.

  python tools/make_metric_gt.py [--check]   (--check: verify existing GT, write nothing)
"""
import argparse
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from cuda_mpi_openmp_amd.utils.imgdata import ImgData, decode_data, hex_groups, rgba_to_png  # noqa: E402

BUCKETS = os.path.join(ROOT, "labs", "lab2", "metric_calc")
CPU = os.path.join(ROOT, "labs", "lab2", "src", "cpu_exe")


def reference_output(path: str, tmp: str) -> bytes:
    item = ImgData(path, cache_dir=tmp)
    out = os.path.join(tmp, item.data_name + ".out.data")
    r = subprocess.run([CPU], input=f"{item.data_path}\n{out}", capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        raise RuntimeError(r.stderr)
    return open(out, "rb").read()


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--check", action="store_true")
    a = p.parse_args()
    bad = 0
    with tempfile.TemporaryDirectory() as tmp:
        for bucket in ("small", "medium", "large"):
            src = os.path.join(BUCKETS, bucket)
            gt_dir = os.path.join(BUCKETS, f"{bucket}_out_gt")
            os.makedirs(gt_dir, exist_ok=True)
            for name in sorted(os.listdir(src)):
                stem, ext = os.path.splitext(name)
                raw = reference_output(os.path.join(src, name), tmp)
                img = decode_data(raw)
                if ext == ".png":
                    if not (img[..., 3] == 255).all():
                        raise ValueError(f"{name}: alpha not 255, PNG GT would not round-trip")
                    dst = os.path.join(gt_dir, stem + ".png")
                else:
                    dst = os.path.join(gt_dir, stem + ".txt")
                if a.check:
                    ok = os.path.exists(dst) and ImgData(dst).raw == raw
                    bad += not ok
                    print(f"{'ok  ' if ok else 'BAD '} {dst}")
                    continue
                if ext == ".png":
                    rgba_to_png(img, dst)
                else:
                    w, h = img.shape[1], img.shape[0]
                    with open(dst, "w") as f:
                        f.write(hex_groups(raw, row_pixels=w if w else None).upper() + "\n")
                assert ImgData(dst).raw == raw, dst
                print(f"wrote {dst} ({img.shape[1]}x{img.shape[0]})")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
