#!/usr/bin/env python3
"""How often the two-stage selection leaves |S| > 1 over one bench step (diagnostics)."""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "admm-quantization_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from admmq import _lib  # noqa: E402
import bench  # noqa: E402

lib = _lib.load()
buf = (ctypes.c_ulonglong * 3)()
work, _, _ = bench.build_workload("resnet18", 0, 1, "replica", torch.device("cuda:0"))
lib.admmq_debug_sel_stats(buf, 1)
bench.run_step(work, int(sys.argv[1]) if len(sys.argv) > 1 else 1000)
torch.cuda.synchronize()
lib.admmq_debug_sel_stats(buf, 0)
tot = sum(buf)
print(f"selections {tot}: |S|=1 {buf[0]} ({100*buf[0]/max(tot,1):.3f}%), 2..64 {buf[1]}, exhaustive {buf[2]}")
