"""HBM planner (utils/memplan.py): calibration against the measured MI355X peaks, the 90 % budget, and the
``auto`` values flowing from the job spec into the pod command and from the CLI into the trainer."""
import json
import subprocess
import sys

import pytest

from finetune_controller_amd.models.config import get_config
from finetune_controller_amd.utils import memplan

L8 = memplan.Dims.of(get_config("llama3-8b"))
L70 = memplan.Dims.of(get_config("llama3-70b"))
M7 = memplan.Dims.of(get_config("mistral-7b"))

# (model, method, micro-batch, seq_len, kwargs, measured peak GB) -- BASELINE.md round-1 table,
# profiles/configs/ (torch.cuda.max_memory_allocated on MI355X)
MEASURED = [
    (L8, "lora", 4, 4096, {}, 107.7),
    (L8, "full", 4, 4096, {}, 218.0),
    (L8, "lora", 1, 32768, {}, 183.0),
    (L8, "lora", 2, 16384, {}, 183.0),
    (L8, "lora", 1, 65536, {"checkpoint_layers": True}, 100.0),
    (L70, "lora", 1, 4096, {}, 240.0),
    (L70, "qlora", 2, 4096, {}, 233.0),
    (M7, "qlora", 4, 4096, {}, 81.0),
]


@pytest.mark.parametrize("dims,method,b,s,kw,meas", MEASURED)
def test_estimate_matches_measured_peaks(dims, method, b, s, kw, meas):
    e = memplan.estimate(dims, method, b, s, 288.0, **kw)
    assert abs(e["total"] / meas - 1) < 0.10, (e["total"], meas, e)


def test_tn_copy_policy_follows_the_trainer():
    """The transposed backward copies are kept for 8B (2 x 16 GB <= 45 % of 288 GB), dropped for 70B."""
    assert memplan.estimate(L8, "lora", 4, 4096)["tn_copies_on"]
    assert not memplan.estimate(L70, "lora", 1, 4096)["tn_copies_on"]


@pytest.mark.parametrize("dims", [L8, L70, M7, memplan.Dims.of(get_config("llama3.2-1b"))])
@pytest.mark.parametrize("method", ["lora", "qlora", "full"])
@pytest.mark.parametrize("seq_len", [512, 4096, 16384, 65536])
@pytest.mark.parametrize("world", [1, 8])
def test_plan_stays_within_ninety_percent(dims, method, seq_len, world):
    try:
        p = memplan.plan(dims, method, seq_len, 288.0, world=world)
    except ValueError as e:  # does not fit even checkpointed: only for configurations that truly cannot
        assert dims is L70 and method in ("full", "lora") or seq_len >= 65536, str(e)
        return
    assert p.peak_gb <= 0.9 * 288.0 + 1e-6
    assert p.batch_size >= 1 and p.batch_size * seq_len <= max(memplan.TARGET_TOKENS, seq_len)
    again = memplan.estimate(dims, method, p.batch_size, seq_len, 288.0, world=world,
                             checkpoint_layers=p.checkpoint_layers)
    assert abs(again["total"] - p.peak_gb) < 0.1


def test_plan_choices_on_the_baseline_configs():
    assert memplan.plan(L8, "lora", 4096).as_args() == {"batch_size": 4, "checkpoint_layers": False}
    assert memplan.plan(L8, "full", 4096).batch_size == 4
    assert memplan.plan(L70, "qlora", 4096).batch_size == 2  # the 288 GB showcase: 2 x 4096 fits, 3 does not
    assert memplan.plan(L8, "lora", 32768).as_args() == {"batch_size": 1, "checkpoint_layers": False}
    assert memplan.plan(L8, "lora", 131072).checkpoint_layers  # 128k tokens only fit checkpointed
    with pytest.raises(ValueError, match="sequence parallelism"):
        memplan.plan(L70, "full", 4096)  # 70B full FT needs ZeRO over many GPUs: 1.1 TB of optimizer state
    # ZeRO-1 over 8 GPUs shards the optimizer: 8B full FT then leaves room for the same 4 x 4096
    assert memplan.plan(L8, "full", 4096, world=8).peak_gb < memplan.plan(L8, "full", 4096).peak_gb


def test_spec_passes_auto_to_the_worker_and_validates_it():
    """"auto" reaches the pod (the worker plans against the real total_memory); the control plane
    only checks that some plan fits the spec's accelerator, and rejects 0 / negative micro-batches."""
    from pydantic import ValidationError

    from finetune_controller_amd.controlplane.spec.models.builtin import Llama3_8B_LoRA
    from finetune_controller_amd.train.cli import build_parser

    spec = Llama3_8B_LoRA(training_arguments={"batch_size": "auto", "seq_len": 32768, "checkpoint_layers": "auto"})
    cmd = spec.run_cmd()[-1].split()
    assert "--batch-size=auto" in cmd and "--checkpoint-layers=auto" in cmd
    # the rendered flags parse in the worker CLI
    flags = [t for t in cmd if t.startswith("--") and not t.startswith(("--standalone", "--nproc"))]
    a = build_parser().parse_args(flags)
    assert a.batch_size == 0 and a.checkpoint_layers == "auto"
    spec = Llama3_8B_LoRA(training_arguments={"batch_size": 2})  # explicit values pass through untouched
    assert "--batch-size=2" in spec.run_cmd()[-1].split()
    for bad in (0, -1):
        with pytest.raises(ValidationError):
            Llama3_8B_LoRA(training_arguments={"batch_size": bad})
    # a job no plan can fit is refused when the command is rendered (submission), not in the pod
    huge = Llama3_8B_LoRA(training_arguments={"batch_size": "auto", "seq_len": 1 << 22, "checkpoint_layers": "auto"})
    with pytest.raises(ValueError):
        huge.run_cmd()


def test_control_plane_plans_without_torch():
    code = ("import sys; from finetune_controller_amd.controlplane.spec.models.builtin import Llama3_8B_LoRA; "
            "s = Llama3_8B_LoRA(training_arguments={'batch_size': 'auto'}); print(s.memory_plan().batch_size); "
            "print('torch' in sys.modules)")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == ["4", "False"]


def test_cli_auto_flags_reach_the_trainer(tmp_path):
    from finetune_controller_amd.train.cli import build_parser, config_from_args
    from finetune_controller_amd.train.trainer import Trainer

    a = build_parser().parse_args(["--model", "llama-tiny", "--batch-size", "auto", "--checkpoint-layers", "auto",
                                   "--seq-len", "32", "--device", "cpu", "--synthetic", "--max-steps", "1",
                                   "--checkpoint_path", str(tmp_path)])
    tc = config_from_args(a)
    assert tc.batch_size == 0 and tc.checkpoint_layers == "auto"
    tr = Trainer(tc)
    try:
        assert tr.tc.batch_size >= 1 and tr.tc.checkpoint_layers is False
        assert tr.mem_plan is not None and json.dumps(tr.mem_plan.parts_gb)
        tr.train_step(1e-4)
    finally:
        tr.close()
    with pytest.raises(SystemExit):
        build_parser().parse_args(["--batch-size", "0"])
