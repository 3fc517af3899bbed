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


def test_dependency_locks_are_current_and_cover_the_requirements():
    """deploy/lock/*.lock.txt (the uv.lock equivalent the images install with ``-c``) are exact pins of
    the tested environment, up to date with tools/lock_deps.py, and every requirement's lower bound holds
    for its pinned version."""
    import subprocess
    import sys

    from packaging.requirements import Requirement
    from packaging.version import Version

    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "lock_deps.py"), "--check"], capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stderr
    for lock, req_file in (("controlplane", "requirements-controlplane.txt"), ("worker", "requirements-worker.txt")):
        pins = {}
        with open(os.path.join(ROOT, "deploy", "lock", f"{lock}.lock.txt")) as f:
            for ln in f:
                ln = ln.split("#")[0].strip()
                if ln:
                    name, ver = ln.split("==")
                    pins[re.sub(r"[-_.]+", "-", name).lower()] = Version(ver)
        with open(os.path.join(ROOT, "deploy", req_file)) as f:
            for ln in f:
                ln = ln.split("#")[0].strip()
                if not ln:
                    continue
                req = Requirement(ln)
                key = re.sub(r"[-_.]+", "-", req.name).lower()
                assert key in pins, f"{req.name} not pinned in {lock}.lock.txt"
                assert pins[key] in req.specifier, f"{req.name}=={pins[key]} violates {req.specifier}"
    for df in ("Dockerfile.controlplane", "Dockerfile.monitor", "Dockerfile.worker"):
        with open(os.path.join(ROOT, "deploy", "docker", df)) as f:
            assert "-c /tmp/lock.txt" in f.read(), df


def test_in_cluster_build_path(tmp_path):
    """deploy/scripts/publish_cluster.sh (OpenShift binary builds, the reference's publish_git.sh flow)
    applies the BuildConfigs and starts one build per image whose Dockerfile exists."""
    import subprocess

    import yaml

    with open(os.path.join(ROOT, "deploy", "openshift", "buildconfigs.yaml")) as f:
        items = [d for d in yaml.safe_load_all(f) if d]
    bcs = {i["metadata"]["name"]: i for i in items if i["kind"] == "BuildConfig"}
    assert set(bcs) == {"ftc-controlplane", "ftc-monitor", "ftc-worker-rocm"}
    for bc in bcs.values():
        assert os.path.exists(os.path.join(ROOT, bc["spec"]["strategy"]["dockerStrategy"]["dockerfilePath"]))
    env = dict(os.environ, DRY_RUN="1", DIRTY_OK="1", NAMESPACE="ml")
    r = subprocess.run(["bash", os.path.join(ROOT, "deploy", "scripts", "publish_cluster.sh")], capture_output=True,
                       text=True, env=env, timeout=60)
    assert r.returncode == 0, r.stderr
    starts = [ln for ln in r.stdout.splitlines() if ln.startswith("oc start-build")]
    assert len(starts) == 3 and all("--from-archive=" in s and "--namespace=ml" in s for s in starts)
