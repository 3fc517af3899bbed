"""The shipped extension: built for gfx950 only, and free of diagnostic code (timing-only modes with wrong
results and cycle stamps exist only in the tools' diagnostic builds: FTC_EXPERIMENTS, FTC_GEMM_STAMP,
FTC_STAMPS -- never set by finetune_controller_amd/tools/build.py)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "finetune_controller_amd", "_C.so")


def _strings(path):
    r = subprocess.run(["strings", "-n", "6", path], capture_output=True, text=True, check=True)
    return r.stdout


@pytest.mark.skipif(not os.path.exists(SO), reason="extension not built (python -m finetune_controller_amd.tools.build)")
def test_extension_has_no_diagnostic_hooks():
    text = _strings(SO)
    for name in ("FTC_GEMM_TN_MODE", "FTC_GEMM_NT_MODE", "FTC_GEMM_NT_V5_MODE", "FTC_GEMM_NT_V7_MODE",
                 "FTC_GEMM_NT_PB_MODE", "FTC_FLASH_FWD_PIPE", "FTC_FLASH_FWD_PP", "FTC_FLASH_DKDV_PP2",
                 "g_gemm_stamps", "g_stamps", "ftc_gemm_nt_stamps"):
        assert name not in text, name
    syms = subprocess.run(["nm", "-C", SO], capture_output=True, text=True, check=True).stdout
    # one production projection-GEMM kernel template (bf16 / fp32 C x epilogue x store policy x beta)
    assert "gemm_nt_kernel<" in syms
    for old in ("gemm_nt_v5_kernel", "gemm_nt_w4d_kernel", "gemm_nt_pb_kernel", "gemm_nt_pp_kernel",
                "flash_fwd_pipe_kernel", "flash_fwd_qb2_kernel"):
        assert old not in syms, old


def test_build_script_sets_no_diagnostic_define():
    src = open(os.path.join(ROOT, "finetune_controller_amd", "tools", "build.py")).read()
    for d in ("FTC_EXPERIMENTS", "FTC_GEMM_STAMP", "FTC_STAMPS"):
        assert d not in src
