#!/usr/bin/env python3
"""F9: per-channel quantizer KATs generated from the reference (survey container only).

Run:  python3 -B tests/golden/gen_f9_channel.py [--reference /root/reference]

Imports ``source.quantization`` from the read-only reference (no bytecode written) and
stores, per case of ``golden_cases.f9_cases()`` (inputs regenerated from numpy seeds),
the reference's output of ``quantize_tensor(x, bits, qscheme, dim=dim)`` (array + SHA-256
+ shape) or the exception type it raises. Only data is written: ``f9_channel.npz`` and
``f9_channel.json`` next to this script.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.dont_write_bytecode = True
import numpy as np  # noqa: E402
import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import golden_cases as gc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    a = ap.parse_args()
    sys.path.insert(0, a.reference)
    from source import quantization as ref_quant  # noqa: E402
    torch.set_num_threads(1)
    meta, arrays = [], {}
    for case in gc.f9_cases():
        x = gc.f9_input(case)
        try:
            y = ref_quant.quantize_tensor(torch.from_numpy(x.copy()), bits=case["bits"], qscheme=case["qscheme"],
                                          dim=case["dim"])
            y = y.numpy().astype(np.float32)
            arrays[case["id"]] = y
            rec = dict(case, error=None, sha=gc.canonical_sha(y), out_shape=list(y.shape))
        except Exception as e:  # error behaviour is part of the contract
            rec = dict(case, error=type(e).__name__, message=str(e)[:200], sha=None)
        meta.append(rec)
    np.savez_compressed(os.path.join(HERE, "f9_channel.npz"), **arrays)
    with open(os.path.join(HERE, "f9_channel.json"), "w") as f:
        json.dump({"torch": torch.__version__, "threads": 1, "cases": meta}, f, indent=1)
    print(f"F9: {len(meta)} cases, {len(arrays)} outputs, {sum(1 for m in meta if m['error'])} errors")


if __name__ == "__main__":
    main()
