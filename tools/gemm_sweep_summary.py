#!/usr/bin/env python3
"""Prints one line per (shape, config) of a tools/bench_gemm_nt.py log: shape, config, ours / library
TF/s, speed-up, max rel error vs the library."""
import json
import sys

for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        print(d["gemm"], d["config"], d["ours_tf"], d["lib_tf"], d["speedup"], d["max_rel_err_vs_lib"])
    elif line.strip():
        print(line.rstrip())
