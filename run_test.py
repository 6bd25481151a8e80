#!/usr/bin/env python3
"""Drop-in replacement of the reference harness entry point (run_test.py).
See cuda_mpi_openmp_amd/harness/cli.py for the flags."""

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from cuda_mpi_openmp_amd.harness.cli import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
