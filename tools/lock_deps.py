#!/usr/bin/env python3
"""Write the pinned dependency locks the images install from (``deploy/lock/*.lock.txt``).

The reference pins its environment with ``uv.lock`` + ``.python-version`` (/root/reference/uv.lock,
/root/reference/.python-version); this is the pip equivalent: the transitive closure of the control
plane's and the worker's runtime dependencies, resolved from the environment the test suite ran in,
every entry an exact ``==`` pin, with the interpreter version in the header.  Regenerate after a
dependency change:

    python tools/lock_deps.py            # rewrite the locks
    python tools/lock_deps.py --check    # exit 1 if they are stale (tests/test_packaging.py)

torch (the ROCm build) is NOT locked: it comes with the ROCm base image of the worker.
"""
from __future__ import annotations

import argparse
import importlib.metadata as md
import re
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
LOCKS = {
    "controlplane": ["fastapi", "uvicorn", "pydantic", "httpx", "pyyaml", "pymongo", "prometheus-client"],
    "worker": ["numpy", "safetensors", "pyyaml", "pybind11", "ninja"],
}
SKIP = {"torch"}  # from the base image


def _norm(name: str) -> str:
    return re.sub(r"[-_.]+", "-", name).lower()


def _requires(dist: md.Distribution) -> list[str]:
    """Names of the unconditional requirements (no extras, markers true for this interpreter)."""
    out = []
    for req in dist.requires or []:
        body, _, marker = req.partition(";")
        if "extra" in marker:
            continue
        if marker.strip():
            try:
                from packaging.markers import Marker

                if not Marker(marker.strip()).evaluate():
                    continue
            except Exception:
                pass
        name = re.match(r"\s*([A-Za-z0-9_.\-]+)", body).group(1)
        out.append(name)
    return out


def closure(roots: list[str]) -> dict[str, str]:
    pins: dict[str, str] = {}
    todo = list(roots)
    while todo:
        name = todo.pop()
        key = _norm(name)
        if key in pins or key in SKIP:
            continue
        dist = md.distribution(name)
        pins[key] = dist.version
        todo.extend(_requires(dist))
    return dict(sorted(pins.items()))


def render(lock: str, pins: dict[str, str]) -> str:
    v = sys.version_info
    head = (f"# {lock} runtime lock: exact pins of the transitive closure of {', '.join(LOCKS[lock])}\n"
            f"# resolved from the tested environment (python {v.major}.{v.minor}); regenerate with\n"
            f"# `python tools/lock_deps.py` -- checked by tests/test_packaging.py\n"
            f"# python_version == {v.major}.{v.minor}\n")
    return head + "".join(f"{k}=={ver}\n" for k, ver in pins.items())


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--check", action="store_true")
    a = ap.parse_args()
    out = ROOT / "deploy" / "lock"
    stale = []
    for lock, roots in LOCKS.items():
        text = render(lock, closure(roots))
        path = out / f"{lock}.lock.txt"
        if a.check:
            if not path.exists() or path.read_text() != text:
                stale.append(str(path))
        else:
            out.mkdir(parents=True, exist_ok=True)
            path.write_text(text)
            print(f"wrote {path.relative_to(ROOT)}")
    if stale:
        print("stale locks: " + ", ".join(stale), file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
