"""Packaging metadata (pyproject.toml): the console scripts resolve, the control-plane requirements
file the images install from matches the declared dependencies, and the package list covers the code.
(The offline image ships setuptools 59, too old to build a PEP 621 wheel without build isolation, so
the metadata is checked directly.)"""
import importlib
import os
import re

import pytest

tomli = pytest.importorskip("tomli")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _pyproject():
    with open(os.path.join(ROOT, "pyproject.toml"), "rb") as f:
        return tomli.load(f)


def test_console_scripts_resolve():
    for name, target in _pyproject()["project"]["scripts"].items():
        mod, fn = target.split(":")
        assert callable(getattr(importlib.import_module(mod), fn)), name


def test_requirements_file_matches_dependencies():
    declared = {re.split(r"[<>=\[ ]", d)[0].lower() for d in _pyproject()["project"]["dependencies"]}
    with open(os.path.join(ROOT, "deploy", "requirements-controlplane.txt")) as f:
        pinned = {re.split(r"[<>=\[ ]", ln.split("#")[0].strip())[0].lower() for ln in f if ln.split("#")[0].strip()}
    assert declared == pinned


def test_packages_cover_the_code():
    from setuptools import find_packages

    pkgs = set(find_packages(ROOT, include=["finetune_controller_amd*"]))
    for d, _, files in os.walk(os.path.join(ROOT, "finetune_controller_amd")):
        if "__pycache__" in d or not any(f.endswith(".py") for f in files):
            continue
        rel = os.path.relpath(d, ROOT).replace(os.sep, ".")
        if rel.endswith("spec.custom"):  # user model specs: data files, imported by path
            continue
        assert rel in pkgs, f"{rel} has .py files but no __init__.py (not packaged)"


def test_dockerfile_copy_sources_survive_dockerignore():
    """Every COPY source of deploy/docker/* exists and is not excluded from the build context."""
    import fnmatch
    import glob

    ignore = [ln.strip().rstrip("/") for ln in open(os.path.join(ROOT, ".dockerignore"))
              if ln.strip() and not ln.startswith("#")]
    for df in glob.glob(os.path.join(ROOT, "deploy", "docker", "Dockerfile.*")):
        for ln in open(df):
            if not ln.startswith("COPY "):
                continue
            for src in ln.split()[1:-1]:
                assert os.path.exists(os.path.join(ROOT, src)), (df, src)
                assert not any(fnmatch.fnmatch(src, pat) or src.split("/")[0] == pat for pat in ignore), (df, src)
