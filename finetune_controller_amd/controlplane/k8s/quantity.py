"""Kubernetes resource quantity parsing ("500m", "32Gi", "2", "1e3")."""
from __future__ import annotations

_BIN = {"Ki": 2**10, "Mi": 2**20, "Gi": 2**30, "Ti": 2**40, "Pi": 2**50, "Ei": 2**60}
_DEC = {"n": 1e-9, "u": 1e-6, "m": 1e-3, "": 1.0, "k": 1e3, "K": 1e3, "M": 1e6, "G": 1e9, "T": 1e12, "P": 1e15,
        "E": 1e18}


def parse_quantity(v) -> float:
    if isinstance(v, (int, float)):
        return float(v)
    s = str(v).strip()
    for suf, mul in _BIN.items():
        if s.endswith(suf):
            return float(s[: -len(suf)]) * mul
    if s and s[-1] in _DEC and not s[-1].isdigit():
        return float(s[:-1]) * _DEC[s[-1]]
    return float(s)
