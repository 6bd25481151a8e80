"""``run_test.py`` command line (reference run_test.py:19-83, same flags).

    python run_test.py --binary_path_cuda ./labs/lab2/src/to_plot_hip_exe \
        --binary_path_cpu ./labs/lab2/src/cpu_exe --k_times 12 \
        --kernel_sizes "[[[32,32],[16,16]]]" --metadata_columns2plot '["filename"]'

The lab is the grandparent directory name of the GPU binary (reference
run_test.py:58-60). Unknown ``--key value`` options go to the lab processor.
New flags: ``--binary_path_hip`` (alias), ``--timeout`` per run, ``--timing``
(cold | cold-lazy | warm | median:N — exported as MPX_TIMING to the GPU binary), and the
default ``--metadata_columns2plot`` is ``[]`` (the reference default raised a
KeyError in the plot); ``--compat`` restores the
reference's output-changing behaviour for a literal replay
(processors.COMPAT_DEVIATIONS).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
from typing import List, Optional

from .args import passthrough_kwargs
from .processors import PROCESSORS
from .tester import Tester


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="Run kernel testing with subprocess.")
    p.add_argument("--binary_path_cuda", "--binary_path_hip", dest="binary_path_cuda", type=str,
                   help="Path to the GPU (HIP) binary (benchmark personality).")
    p.add_argument("--binary_path_cpu", type=str, default=None, help="Path to the CPU binary.")
    p.add_argument("--k_times", type=int, default=20, help="Number of times to run the kernel.")
    p.add_argument("--return_inp", action="store_true", help="Keep the stdin of every run in the CSV.")
    p.add_argument("--return_task_res", action="store_true", help="Keep the task result in the CSV.")
    p.add_argument("--kernel_sizes", type=str, default="[[512, 512]]",
                   help="JSON list of [k1, k2] launch geometries, e.g. '[[1, 32], [512, 512]]'")
    p.add_argument("--metadata_columns2plot", type=str, default="[]",
                   help='JSON list of CSV columns listed in the plot legend, e.g. ["filename"]')
    p.add_argument("--timeout", type=float, default=None, help="Per-run timeout in seconds.")
    p.add_argument("--timing", type=str, default=None, help="GPU timing policy: cold | cold-lazy | warm | median:N")
    p.add_argument("--warmup", type=int, default=None,
                   help="untimed launches before the timed one(s) in the GPU binary (MPX_WARMUP)")
    p.add_argument("--compat", action="store_true",
                   help="literal replay of the reference harness: lab1 array2string stdin and no lab1 check, "
                        "sidecars next to the inputs, the reference CSV schema (processors.COMPAT_DEVIATIONS)")
    p.add_argument("--n_gpus", type=int, default=1,
                   help="split each run over N GPUs inside the GPU binary (MPX_NGPUS); reported time is the "
                        "slowest device's kernel time")
    return p


def main(argv: Optional[List[str]] = None) -> int:
    args, unknown = build_parser().parse_known_args(argv)
    if not args.binary_path_cuda:
        print("--binary_path_cuda is required", file=sys.stderr)
        return 2
    kwargs = passthrough_kwargs(unknown)
    kernel_sizes = json.loads(args.kernel_sizes) if args.kernel_sizes else None
    meta = json.loads(args.metadata_columns2plot) if args.metadata_columns2plot else []
    lab_dir = os.path.dirname(os.path.dirname(os.path.abspath(args.binary_path_cuda)))
    lab_name = os.path.basename(lab_dir)
    if lab_name not in PROCESSORS:
        print(f"cannot infer the lab from {args.binary_path_cuda} (grandparent dir '{lab_name}')", file=sys.stderr)
        return 2
    print("Params:")
    print(f"return_inp=<{args.return_inp}>")
    print(f"return_task_res=<{args.return_task_res}>")
    print(f"lab_name=<{lab_name}>")
    print(f"binary_path_cuda=<{args.binary_path_cuda}>")
    print(f"binary_path_cpu=<{args.binary_path_cpu}>")
    print(f"k_times=<{args.k_times}>")
    print(f"kernel_sizes=<{kernel_sizes}>")
    print(f"kwargs=<{json.dumps(kwargs, indent=2)}>")
    print(f"metadata_columns2plot=<{json.dumps(meta, indent=2)}>")
    print(f"n_gpus=<{args.n_gpus}>")
    if args.compat:
        from .processors import COMPAT_DEVIATIONS

        print("compat=<True>: reference behaviour restored for " + "; ".join(f"#{k}" for k in COMPAT_DEVIATIONS))
        kwargs["compat"] = True
    if lab_name in ("lab2", "lab3", "lab5") and "dir_to_data" not in kwargs:
        kwargs["lab_dir"] = lab_dir
    env = {}
    if args.timing:
        env["MPX_TIMING"] = args.timing
    if args.warmup is not None:
        env["MPX_WARMUP"] = str(max(0, args.warmup))
    if args.n_gpus and args.n_gpus > 1:
        # an N-GPU row must come from N GPUs: refuse when fewer are visible,
        # unless explicitly rehearsing on shared devices (then the CSV records
        # devices_used)
        from ..parallel.launch import visible_devices

        ndev = visible_devices()
        shared = os.environ.get("MPX_ALLOW_SHARED") == "1"
        if ndev < args.n_gpus and not shared:
            print(f"[harness] --n_gpus {args.n_gpus} requested but {ndev} GPU(s) are visible; refusing to record "
                  f"an N-GPU result (MPX_ALLOW_SHARED=1 rehearses on shared devices)", file=sys.stderr)
            return 2
        env["MPX_NGPUS"] = str(args.n_gpus)
        env["MPX_DEVICES_USED"] = str(max(1, min(args.n_gpus, ndev)))
        if shared:
            env["MPX_ALLOW_SHARED"] = "1"
    env = env or None
    tester = Tester(binary_path_gpu=args.binary_path_cuda, k_times=args.k_times, kernel_sizes=kernel_sizes,
                    metadata_columns2plot=meta, binary_path_cpu=args.binary_path_cpu, return_inp=args.return_inp,
                    return_task_res=args.return_task_res, timeout=args.timeout, gpu_env=env, compat=args.compat)
    processor = PROCESSORS[lab_name](**kwargs)
    df = tester.run_experiments(processor)
    return 0 if len(df) else 1
