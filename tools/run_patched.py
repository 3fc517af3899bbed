#!/usr/bin/env python3
"""Run a script with module-level constants patched first -- the A/B arm of the "A/B by patching" toggles
(e.g. ``ops.norm._TAIL_OFF``, ``ops.activation._FUSED_OFF``, ``ops.linear._HIP_TAIL``) without an
environment switch in the product code.

    python tools/run_patched.py finetune_controller_amd.ops.norm._TAIL_OFF=True -- bench.py --steps 10
"""
import ast
import importlib
import os
import runpy
import sys


def main():
    argv = sys.argv[1:]
    if "--" not in argv:
        raise SystemExit(__doc__)
    cut = argv.index("--")
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    for spec in argv[:cut]:
        target, value = spec.split("=", 1)
        mod, attr = target.rsplit(".", 1)
        setattr(importlib.import_module(mod), attr, ast.literal_eval(value))
        print(f"[patched] {target} = {value}", flush=True)
    script, rest = argv[cut + 1], argv[cut + 2:]
    sys.argv = [script] + rest
    runpy.run_path(script, run_name="__main__")


if __name__ == "__main__":
    main()
