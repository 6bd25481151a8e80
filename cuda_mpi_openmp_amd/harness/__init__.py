"""Benchmark + verification harness compatible with the reference's
run_test.py / tester.py / lab processors (see cli.py)."""

from .core import RunRecord, parse_timing, run_binary, time_stats
from .processors import PROCESSORS, Lab1Processor, Lab2Processor, Lab3Processor, Lab5Processor
from .tester import Tester

__all__ = ["RunRecord", "parse_timing", "run_binary", "time_stats", "PROCESSORS", "Lab1Processor",
           "Lab2Processor", "Lab3Processor", "Lab5Processor", "Tester"]
