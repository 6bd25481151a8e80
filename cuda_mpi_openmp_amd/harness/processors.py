"""Lab processors: input generation, stdin construction, output parsing and
ground-truth verification for lab1/lab2/lab3 (reference lab*/lab*_processor.py).

Behaviour kept from the reference: seeded numpy RNG (42), the fixed image
candidate list and its order, round-robin over available inputs, output path
``<data>_out/<bin>_<k1>_<k2>/<name>.data``, byte-exact uppercase-hex GT compare,
lab3's hard-coded two-class definition by default.

Defects fixed: lab1 pre_process accepts the runner's kwargs
(#1); lab1 vectors are printed in full round-trip precision instead of
np.array2string's 1000-element summary (#2) and verification is re-enabled
with the lab's 1e-10 relative precision (#3); list kwargs work (#5); sidecar
files go to a cache directory, not the input directory (#8); lab3's
``count_classes`` / ``count_pts`` opt into random classes (#12). New:
``synthetic="WxH"`` generates a seeded random image as an extra input.

``compat=True`` (``run_test.py --compat``, VERDICT r4 Next #7) switches the
output-changing fixes back for a literal replay of the reference harness —
every deviation in one place, :data:`COMPAT_DEVIATIONS`:
lab1 stdin is ``np.array2string`` text (summarised beyond 1000 elements:
the binaries then read 3 values and garbage), lab1 verification always
passes, and the image labs write their ``.data`` / ``.txt`` / ``.png`` sidecars
next to the inputs, the ground truth and the outputs.
"""

from __future__ import annotations

import os
import shutil
import subprocess
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..utils.imgdata import ImgData, encode_data, hex_groups, normalize_hex

REPO_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

LAB_IMAGE_FILES = [
    "stalker2.png", "98.data", "AoE.png", "doom.png", "hf2.png", "starcraft.png", "warcraft.png",
    "test_01.txt", "test_02.txt", "lenna.png", "57.data", "95.data", "99.data", "02.data", "96.data", "97.data",
]
LAB3_EXTRA_FILES = ["04.data", "09.data", "test_01_lab3.txt", "test_02_lab3.txt"]
MAX_CLASSES = 32
MAX_NUM_POINTS = 2 ** 19
# reference lab3/lab3_processor.py:42-51: the class set used for every image
DEFAULT_LAB3_CLASSES = [
    np.array([[1, 2], [1, 0], [2, 2], [2, 1]]),
    np.array([[0, 0], [0, 1], [1, 1], [2, 0]]),
]


# Appendix B items switched back by compat=True (processors) and by the
# Tester's compat mode (CSV schema / file names). Everything else — the
# kwargs fix (#1), list kwargs (#5), PNG conversion (#9), the native
# programs' fixes (#10, #11, #16) — cannot change a result the reference
# could produce, so it stays on.
COMPAT_DEVIATIONS = {
    2: "lab1 stdin: np.array2string(separator=' ', max_line_width=inf, precision=precision_array)[1:-1] "
       "(lab1_processor.py:37-48), summarised with '...' beyond 1000 elements — the reference programs then "
       "read 3 values and garbage, ours refuse the short input (checked I/O, #11 stays fixed), so such runs "
       "are recorded as failed instead of passing on garbage",
    3: "lab1 verification always True (lab1_processor.py:60-67)",
    6: "the CPU binary's CSV is stats_<bin>.csv even when it shares the GPU binary's name (tester.py:267-269)",
    8: "sidecar .data/.txt/.png written next to every input, ground truth and output (utils/converter.py:32-53)",
    "csv": "CSV columns exactly the reference's: no device / wall_ms / n_gpus / throughput / pixels columns and "
           "no speedup_<bin>.csv (tester.py:224-285)",
}


def compat_vector_text(v: np.ndarray, precision: int) -> str:
    """The reference's lab1 vector text (lab1_processor.py:37-48)."""
    return np.array2string(v, separator=" ", max_line_width=np.inf, precision=precision)[1:-1].strip()


class LabProcessor:
    """Hooks used by the runner: pre_process -> (stdin, verify_kwargs, debug cols),
    get_task_result(payload) and verify_result(result) -> bool."""

    def __init__(self, seed: int = 42):
        self.seed = seed
        self.rng = np.random.RandomState(seed)

    def get_attr(self) -> Dict[str, Any]:
        return {}

    def pre_process(self, **kwargs) -> Tuple[str, Dict[str, Any], Dict[str, Any]]:
        raise NotImplementedError

    def get_task_result(self, payload: str, **kwargs):
        return payload

    def verify_result(self, result, **kwargs) -> bool:
        return True


def fmt_vector(v: np.ndarray) -> str:
    """Exact round-trip decimal text (17 significant digits)."""
    return " ".join(np.char.mod("%.17g", v))


class Lab1Processor(LabProcessor):
    def __init__(self, seed: int = 42, min_vector_size: int = 1024, max_vector_size: int = 3072, atol: float = 1e-10,
                 precision_array: int = 10, rtol: float = 1e-10, lo: float = -1e100, hi: float = 1e100,
                 compat: bool = False, **_):
        super().__init__(seed)
        self.compat = bool(compat)
        self.min_vector_size, self.max_vector_size = int(min_vector_size), int(max_vector_size)
        self.atol, self.rtol, self.precision_array = atol, rtol, precision_array
        self.lo, self.hi = lo, hi

    def get_attr(self):
        return {"min_vector_size": self.min_vector_size, "max_vector_size": self.max_vector_size, "atol": self.atol}

    def pre_process(self, **kwargs):
        # reference draw: randint(min, max) (upper bound exclusive); a fixed
        # size (min == max) is that size instead of numpy's ValueError
        lo, hi = self.min_vector_size, self.max_vector_size
        n = int(self.rng.randint(lo, hi)) if hi > lo else int(lo)
        a = self.rng.uniform(self.lo, self.hi, n)
        b = self.rng.uniform(self.lo, self.hi, n)
        fmt = (lambda v: compat_vector_text(v, self.precision_array)) if self.compat else fmt_vector
        return f"{n}\n{fmt(a)}\n{fmt(b)}", {"first_vector": a, "second_vector": b}, {"vector_size": n}

    def get_task_result(self, payload: str, **kwargs):
        payload = payload.strip()
        return np.array(payload.split(), dtype=np.float64) if payload else np.zeros(0)

    def verify_result(self, result, **kwargs) -> bool:
        if self.compat:
            return True  # reference lab1_processor.py:60-67 (allclose commented out)
        expect = kwargs["first_vector"] - kwargs["second_vector"]
        if result.shape != expect.shape:
            print(f"[verify_result] lab1: expected {expect.size} values, got {result.size}")
            return False
        # the binaries print %.10e: 11 significant digits, relative error <= 5e-11
        ok = bool(np.allclose(result, expect, rtol=self.rtol, atol=0.0))
        if not ok:
            bad = int(np.argmax(np.abs(result - expect) / np.maximum(np.abs(expect), 1e-300)))
            print(f"[verify_result] lab1 mismatch at {bad}: {result[bad]!r} vs {expect[bad]!r}")
        return ok


class _ImageLabProcessor(LabProcessor):
    files: Sequence[str] = LAB_IMAGE_FILES

    def __init__(self, seed: int = 42, atol: float = 1e-10, precision_array: int = 10,
                 extra_links_to_png: Optional[List[str]] = None, dir_to_data: Optional[str] = None,
                 dir_to_data_out: Optional[str] = None, dir_to_data_out_gt: Optional[str] = None,
                 lab_dir: Optional[str] = None, synthetic: Optional[str] = None, verify: str = "auto",
                 compat: bool = False, **_):
        super().__init__(seed)
        self.atol, self.precision_array = atol, precision_array
        self.compat = bool(compat)
        # verify: "gt" = ground truth where it exists, other images pass (the
        # reference, lab2_processor.py:139-144); "cpu" = every image without GT
        # is compared byte for byte with the OpenMP CPU reference program's
        # output (labs/<lab>/src/cpu_omp_exe, run once per image); "auto" =
        # "cpu" when that program is built, else "gt" with a warning.
        if verify not in ("auto", "gt", "cpu"):
            raise ValueError("verify must be auto, gt or cpu")
        self.cpu_oracle = os.path.join(REPO_ROOT, "labs", self.lab, "src", "cpu_omp_exe")
        if verify == "cpu" and not os.path.exists(self.cpu_oracle):
            raise FileNotFoundError(f"--verify cpu needs {self.cpu_oracle} (make apps)")
        self.verify = "cpu" if verify == "cpu" or (verify == "auto" and os.path.exists(self.cpu_oracle)) else "gt"
        self._expected: Dict[int, bytes] = {}
        if dir_to_data is None:
            dir_to_data = os.path.join(lab_dir, "data") if lab_dir else f"./{self.lab}/data"
        dir_to_data = os.path.normpath(dir_to_data)
        parent, base = os.path.dirname(dir_to_data), os.path.basename(dir_to_data)
        self.dir_to_data = dir_to_data
        self.dir_to_data_out = dir_to_data_out or os.path.join(parent, f"{base}_out")
        gt_dir = dir_to_data_out_gt or os.path.join(parent, f"{base}_out_gt")
        # outputs and converted inputs live under the output dir, never next to the inputs
        if os.path.isdir(self.dir_to_data_out):
            shutil.rmtree(self.dir_to_data_out)
        os.makedirs(self.dir_to_data_out, exist_ok=True)
        cache = os.path.join(self.dir_to_data_out, "_inputs")
        paths = [os.path.join(dir_to_data, f) for f in self.files if os.path.exists(os.path.join(dir_to_data, f))]
        for link in extra_links_to_png or []:
            if isinstance(link, str) and os.path.exists(link):
                paths.append(link)
            else:
                from ..utils.download import download_file

                paths.append(download_file(link, cache))
        if synthetic:
            paths.append(self._make_synthetic(str(synthetic), cache))
        if not paths:
            raise FileNotFoundError(f"no input images in {dir_to_data}")
        self.inputs: Dict[int, ImgData] = {}
        self.ground_truth: Dict[int, ImgData] = {}
        for i, p in enumerate(paths):
            # compat: the converted .data and the .txt / .png sidecars next to the
            # input (reference utils/converter.py:32-53), else in the cache dir
            side = os.path.dirname(os.path.abspath(p)) if self.compat else None
            self.inputs[i] = ImgData(p, idx=i, cache_dir=side or cache)
            if side:
                self.inputs[i].write_sidecars(side, keep=p)
            stem = self.inputs[i].data_name
            for ext in ("txt", "data", "png"):
                g = os.path.join(gt_dir, f"{stem}.{ext}")
                if os.path.exists(g):
                    gside = os.path.dirname(os.path.abspath(g)) if self.compat else None
                    self.ground_truth[i] = ImgData(g, idx=i, cache_dir=gside)
                    if gside:
                        self.ground_truth[i].write_sidecars(gside, keep=g)
                    break
        self.cursor = 0

    def _make_synthetic(self, spec: str, cache: str) -> str:
        w, h = (int(v) for v in spec.lower().split("x"))
        img = np.random.RandomState(self.seed).randint(0, 256, size=(h, w, 4), dtype=np.uint8)
        os.makedirs(cache, exist_ok=True)
        path = os.path.join(cache, f"synthetic_{w}x{h}.data")
        with open(path, "wb") as f:
            f.write(encode_data(img))
        return path

    def get_attr(self):
        return {"precision_array": self.precision_array, "atol": self.atol}

    def next_item(self) -> ImgData:
        item = self.inputs[self.cursor]
        self.cursor = (self.cursor + 1) % len(self.inputs)
        return item

    def _out_path(self, device_info: str, item: ImgData) -> str:
        d = os.path.join(self.dir_to_data_out, device_info)
        os.makedirs(d, exist_ok=True)
        return os.path.join(d, f"{item.data_name}.data")

    def _debug(self, item: ImgData) -> Dict[str, Any]:
        return {"filename": f"{item.data_name}{item.data_ext} ({item.size_kb:.5f} KB)",
                "pixels": item.width * item.height}

    def get_task_result(self, payload: str, **kwargs):
        res = ImgData(kwargs["out_path_res"])
        if self.compat:  # the reference converts every output, writing .txt / .png beside it
            res.write_sidecars(os.path.dirname(os.path.abspath(kwargs["out_path_res"])), keep=kwargs["out_path_res"])
        return res

    def task_stdin(self, item: ImgData, out_path: str) -> str:
        """The CPU program's stdin for ``item`` (the task without launch geometry)."""
        return f"{item.data_path}\n{out_path}"

    def cpu_expected(self, idx: int) -> bytes:
        """The OpenMP CPU reference program's output bytes for input ``idx``
        (computed once, kept under the output directory)."""
        if idx not in self._expected:
            item = self.inputs[idx]
            d = os.path.join(self.dir_to_data_out, "_cpu_reference")
            os.makedirs(d, exist_ok=True)
            out = os.path.join(d, f"{item.data_name}.data")
            r = subprocess.run([self.cpu_oracle], input=self.task_stdin(item, out), capture_output=True, text=True,
                               timeout=600)
            if r.returncode != 0:
                raise RuntimeError(f"CPU reference failed on {item.data_name}: {r.stderr[-500:]}")
            with open(out, "rb") as f:
                self._expected[idx] = f.read()
        return self._expected[idx]

    def verify_result(self, result: ImgData, **kwargs) -> bool:
        idx = kwargs["idx_data"]
        result.idx = idx
        gt = self.ground_truth.get(idx)
        if gt is None:
            if self.verify != "cpu":
                return True  # reference behaviour (lab2_processor.py:139-144): no GT, no check
            want = self.cpu_expected(idx)
            ok = result.raw == want
            if not ok:
                a = np.frombuffer(result.raw, dtype=np.uint8)
                b = np.frombuffer(want, dtype=np.uint8)
                n = min(a.size, b.size)
                bad = np.flatnonzero(a[:n] != b[:n])
                first = int(bad[0]) if bad.size else n
                print(f"[verify_result] FAILED `verify_result` vs CPU reference: `{result.data_name}`: "
                      f"{bad.size + abs(a.size - b.size)} bytes differ, first at byte {first} "
                      f"(pixel {(first - 8) // 4 if first >= 8 else 'header'})")
            return ok
        ok = normalize_hex(result.hex) == normalize_hex(gt.hex)
        if not ok:
            src = self.inputs[idx]
            print(f"[verify_result] FAILED `verify_result`: `{result.data_name}`!")
            print(f"[verify_result] [input_data.hex] {hex_groups(src.raw).upper()}")
            print(f"[verify_result] [task_result.hex] {hex_groups(result.raw).upper()}")
            print(f"[verify_result] [ground_truth.hex] {hex_groups(gt.raw).upper()}")
        return ok


class Lab2Processor(_ImageLabProcessor):
    lab = "lab2"

    def pre_process(self, **kwargs):
        item = self.next_item()
        out = self._out_path(kwargs["device_info"], item)
        return self.task_stdin(item, out), {"idx_data": item.idx, "out_path_res": out}, self._debug(item)


def random_class_points(w: int, h: int, count_pts: Optional[int], rng: np.random.RandomState) -> np.ndarray:
    """Opt-in random training points (the reference's commented-out path,
    lab3/img_data_classifier.py:16-24): ``count_pts`` points in a random
    top-left sub-rectangle; at least 2 points so the covariance is defined."""
    n = int(count_pts) if count_pts else int(rng.randint(2, MAX_CLASSES + 1))
    n = max(2, min(n, MAX_NUM_POINTS))
    xt, yt = rng.randint(1, w + 1), rng.randint(1, h + 1)
    return np.stack([rng.randint(xt, size=n), rng.randint(yt, size=n)], axis=1)


class Lab3Processor(_ImageLabProcessor):
    lab = "lab3"
    files = LAB_IMAGE_FILES + LAB3_EXTRA_FILES

    def __init__(self, count_classes: Optional[int] = None, count_pts: Optional[int] = None, **kw):
        super().__init__(**kw)
        self.count_classes, self.count_pts = count_classes, count_pts
        self.classes: Dict[int, List[np.ndarray]] = {}
        for i, item in self.inputs.items():
            if count_classes:
                nc = max(1, min(int(count_classes), MAX_CLASSES))
                self.classes[i] = [random_class_points(item.width, item.height, count_pts, self.rng)
                                   for _ in range(nc)]
            else:
                self.classes[i] = DEFAULT_LAB3_CLASSES
            if not 0 < len(self.classes[i]) <= MAX_CLASSES:
                raise ValueError(f"need 0 < classes <= {MAX_CLASSES}")

    def task_stdin(self, item: ImgData, out_path: str) -> str:
        cls = self.classes[item.idx]
        rows = "\n".join(f"{len(c)} " + " ".join(str(int(v)) for v in np.asarray(c).reshape(-1)) for c in cls)
        return f"{item.data_path}\n{out_path}\n{len(cls)}\n{rows}"

    def pre_process(self, **kwargs):
        item = self.next_item()
        out = self._out_path(kwargs["device_info"], item)
        cls = self.classes[item.idx]
        dbg = self._debug(item)
        dbg["stat_init_pts"] = f"Count Classes: {len(cls)}, Count Points: {set(len(c) for c in cls)}"
        return self.task_stdin(item, out), {"idx_data": item.idx, "out_path_res": out}, dbg


LAB5_TYPES = {"int": np.int32, "float": np.float32, "uchar": np.uint8}


def lab5_sorted(a: np.ndarray) -> np.ndarray:
    """Expected lab5 order: numeric for int32/uint8, the IEEE total order for
    float32 (-NaN < -inf < ... < -0 < +0 < ... < +inf < +NaN), matching the
    order-preserving uint32 keys of native/src/kernels/sort.hip."""
    if a.dtype != np.float32:
        return np.sort(a, kind="stable")
    u = a.view(np.uint32)
    key = np.where(u >> 31 == 1, ~u, u | np.uint32(0x80000000))
    return a[np.argsort(key, kind="stable")]


class Lab5Processor(LabProcessor):
    """lab5 (sort). The reference ships only the binary fixtures
    ``lab5/data/{int10,float10,uchar10}`` (int32 n + n elements) and no
    processor, so this one is ours: it round-robins over the fixtures of the
    chosen ``elem_type`` (plus ``n_random`` seeded random arrays of
    ``min_size..max_size`` elements), feeds them as binary stdin, and verifies
    the binary stdout byte-exactly against numpy's sort. The element type
    reaches the program through ``MPX_LAB5_TYPE``; lab5 programs take no
    launch geometry, so none is prepended."""

    lab = "lab5"
    binary_io = True
    takes_geometry = False

    def __init__(self, seed: int = 42, elem_type: str = "int", n_random: int = 2, min_size: int = 1024,
                 max_size: int = 1 << 20, dir_to_data: Optional[str] = None, lab_dir: Optional[str] = None, **_):
        super().__init__(seed)
        if elem_type not in LAB5_TYPES:
            raise ValueError(f"elem_type must be one of {sorted(LAB5_TYPES)}")
        self.elem_type, self.dtype = elem_type, LAB5_TYPES[elem_type]
        self.env = {"MPX_LAB5_TYPE": elem_type}
        if dir_to_data is None:
            dir_to_data = os.path.join(lab_dir, "data") if lab_dir else "./lab5/data"
        self.items: List[Tuple[str, np.ndarray]] = []
        fixture = os.path.join(dir_to_data, f"{elem_type}10")
        if os.path.exists(fixture):
            raw = open(fixture, "rb").read()
            n = int(np.frombuffer(raw[:4], dtype="<i4")[0])
            self.items.append((os.path.basename(fixture), np.frombuffer(raw[4:], dtype=self.dtype, count=n).copy()))
        for i in range(int(n_random)):
            n = int(self.rng.randint(int(min_size), int(max_size) + 1))
            if elem_type == "float":
                a = (self.rng.standard_normal(n) * 10.0 ** self.rng.randint(-30, 30, n)).astype(np.float32)
            else:
                info = np.iinfo(self.dtype)
                a = self.rng.randint(int(info.min), int(info.max) + 1, n, dtype=np.int64).astype(self.dtype)
            self.items.append((f"random_{i}_{n}", a))
        if not self.items:
            raise FileNotFoundError(f"no lab5 inputs for {elem_type}")
        self.cursor = 0

    def get_attr(self):
        return {"elem_type": self.elem_type}

    def pre_process(self, **kwargs):
        name, a = self.items[self.cursor]
        idx = self.cursor
        self.cursor = (self.cursor + 1) % len(self.items)
        stdin = np.int32(a.size).astype("<i4").tobytes() + a.astype(self.dtype).tobytes()
        return stdin, {"idx_data": idx}, {"filename": name, "n": int(a.size)}

    def get_task_result(self, payload: bytes, **kwargs):
        return np.frombuffer(payload, dtype=self.dtype)

    def verify_result(self, result, **kwargs) -> bool:
        expect = lab5_sorted(self.items[kwargs["idx_data"]][1])
        ok = result.size == expect.size and result.tobytes() == expect.tobytes()
        if not ok:
            print(f"[verify_result] lab5 {self.elem_type} mismatch: got {result.size} elements, want {expect.size}")
        return ok


PROCESSORS = {"lab1": Lab1Processor, "lab2": Lab2Processor, "lab3": Lab3Processor, "lab5": Lab5Processor}
