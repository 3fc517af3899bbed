"""In-tree build of the native parts of finetune_controller_amd (no JIT cache, no pip install).

Produces, next to the Python sources (so they travel with the repo snapshot to the GPU box):

* ``finetune_controller_amd/_C.so``    -- gfx950 HIP kernels (``csrc/kernels/*.hip``) + the
  torch binding (``csrc/binding.cpp``);
* ``finetune_controller_amd/_comm.so`` -- the RCCL communicator / bucketed all-reduce engine
  (``csrc/comm/*.cpp``);
* ``finetune_controller_amd/_rt.so``   -- native runtime pieces: the token data loader
  (``csrc/runtime/*.cpp``).

Device code is compiled with ``hipcc --offload-arch=gfx950`` only (CDNA4 is the single target);
host-only translation units that include torch headers are compiled with g++ against the ROCm
headers.  Objects are rebuilt only when a source or header is newer.

Usage: ``python -m finetune_controller_amd.tools.build [--force] [-j N]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
PKG = ROOT / "finetune_controller_amd"
CSRC = ROOT / "csrc"
BUILD = ROOT / "build" / "native"
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("FTC_OFFLOAD_ARCH", "gfx950")


def _torch_paths():
    import torch
    from torch.utils import cpp_extension as ce

    inc = ce.include_paths(device_type="cuda") if "device_type" in ce.include_paths.__code__.co_varnames else ce.include_paths(cuda=True)
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    pyb = []
    for name, flag in (("_PYBIND11_COMPILER_TYPE", "PYBIND11_COMPILER_TYPE"), ("_PYBIND11_STDLIB", "PYBIND11_STDLIB"),
                       ("_PYBIND11_BUILD_ABI", "PYBIND11_BUILD_ABI")):
        val = getattr(torch._C, name, None)
        if val is not None:
            pyb.append(f'-D{flag}="{val}"')
    return inc, lib, abi, pyb


def _newer(out: Path, deps: list[Path]) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps if d.exists())


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build step failed ({r.returncode}):\n{' '.join(cmd)}\n{r.stdout}")


# per-source compiler flags (the kernel's header says why):
#   flash_attn_fwd.hip -- MFMAs in VGPR form (the softmax reads S with no v_accvgpr copies) and no SLP packing
#   of the softmax's f32 adds into v_pk_add_f32 (an anti-lever beside MFMAs: MI355X_MICROARCH.md cycle
#   constants); the shipped 32-row kernel was measured with them in round 6, and the lab W64 build
#   (tools/w64_lab/build.sh, which depends on them) uses the same
EXTRA_FLAGS = {"flash_attn_fwd.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form", "-fno-slp-vectorize"]}


def _hip_obj(src: Path, headers: list[Path], force: bool) -> Path:
    out = BUILD / (src.stem + ".hip.o")
    if force or _newer(out, [src, *headers, Path(__file__)]):
        _run(["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", str(src), "-o", str(out),
              "-I", str(CSRC / "kernels"), "-Wno-unused-result", "-ffp-contract=fast", *EXTRA_FLAGS.get(src.name, [])])
    return out


def _host_obj(src: Path, extra_inc: list[str], defines: list[str], force: bool, torch_headers: bool) -> Path:
    out = BUILD / (src.stem + ".cpp.o")
    if force or _newer(out, [src, *sorted(src.parent.glob("*.h"))]):  # + headers next to the source
        cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-c", str(src), "-o", str(out), "-D__HIP_PLATFORM_AMD__=1",
               "-DUSE_ROCM=1", f"-I{ROCM}/include", f"-I{sysconfig.get_paths()['include']}"]
        cmd += [f"-I{p}" for p in extra_inc] + defines
        if torch_headers:
            cmd += ["-DTORCH_API_INCLUDE_EXTENSION_H", "-Wno-deprecated-declarations"]
        _run(cmd)
    return out


def _check_kernel_stubs(so: Path) -> None:
    """A kernel whose host-side instantiation fails is dropped SILENTLY by hipcc (its launch then
    references an undefined ``__device_stub__``): the .so links but cannot be loaded.  Fail here."""
    r = subprocess.run(["nm", "-C", "-u", str(so)], stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
    missing = [ln.strip() for ln in r.stdout.splitlines() if "__device_stub__" in ln]
    if missing:
        so.unlink()
        raise RuntimeError("kernels without host stubs (host pass rejected their bodies):\n  " + "\n  ".join(missing))


def build(force: bool = False, jobs: int | None = None, verbose: bool = True) -> dict[str, Path]:
    BUILD.mkdir(parents=True, exist_ok=True)
    inc, tlib, abi, pyb = _torch_paths()
    jobs = jobs or min(16, os.cpu_count() or 4)
    abi_def = [f"-D_GLIBCXX_USE_CXX11_ABI={abi}"]
    headers = sorted((CSRC / "kernels").glob("*.h"))
    hip_srcs = sorted((CSRC / "kernels").glob("*.hip"))
    products: dict[str, Path] = {}
    link_torch = [f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
                  f"-Wl,-rpath,{tlib}", f"-L{ROCM}/lib", "-lamdhip64", f"-Wl,-rpath,{ROCM}/lib"]

    with cf.ThreadPoolExecutor(jobs) as ex:
        hip_futs = [ex.submit(_hip_obj, s, headers, force) for s in hip_srcs]
        bind_fut = ex.submit(_host_obj, CSRC / "binding.cpp", inc, abi_def + pyb + ["-DTORCH_EXTENSION_NAME=_C"], force, True)
        comm_srcs = sorted((CSRC / "comm").glob("*.cpp"))
        comm_futs = [ex.submit(_host_obj, s, inc, abi_def + pyb + ["-DTORCH_EXTENSION_NAME=_comm"], force, True)
                     for s in comm_srcs]
        rt_srcs = sorted((CSRC / "runtime").glob("*.cpp"))
        rt_futs = [ex.submit(_host_obj, s, [str(Path(p)) for p in _pybind_inc()], abi_def, force, False) for s in rt_srcs]
        hip_objs = [f.result() for f in hip_futs]
        bind_obj = bind_fut.result()
        comm_objs = [f.result() for f in comm_futs]
        rt_objs = [f.result() for f in rt_futs]

    so = PKG / "_C.so"
    if force or _newer(so, hip_objs + [bind_obj]):
        _run(["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(so), *map(str, hip_objs), str(bind_obj),
              *link_torch])
        _check_kernel_stubs(so)
    products["_C"] = so

    if comm_objs:
        so = PKG / "_comm.so"
        if force or _newer(so, comm_objs):
            rccl = os.path.join(tlib, "librccl.so")
            rccl_link = [rccl] if os.path.exists(rccl) else [f"-L{ROCM}/lib", "-lrccl"]
            _run(["g++", "-shared", "-fPIC", "-o", str(so), *map(str, comm_objs), *link_torch, *rccl_link])
        products["_comm"] = so

    if rt_objs:
        so = PKG / "_rt.so"
        if force or _newer(so, rt_objs):
            _run(["g++", "-shared", "-fPIC", "-o", str(so), *map(str, rt_objs), "-lpthread"])
        products["_rt"] = so
    if verbose:
        for k, v in products.items():
            print(f"[ftc-build] {k}: {v.relative_to(ROOT)} ({v.stat().st_size // 1024} KiB)")
    return products


def _pybind_inc() -> list[str]:
    import pybind11

    return [pybind11.get_include()]


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    a = ap.parse_args(argv)
    build(force=a.force, jobs=a.j)
    return 0


if __name__ == "__main__":
    sys.exit(main())
