"""Identifier helpers (C20; ``/root/reference/app/utils/naming.py:4-6``)."""
import re
import uuid


def generate_short_uuid() -> str:
    """8 lowercase hex characters of a uuid4 (job-id suffix, fallback file names)."""
    return uuid.uuid4().hex[:8]


def safe_filename(name: str | None) -> str:
    """A dataset object name that is safe in an S3 key and in the worker's shell command lines: the
    basename, with anything outside ``[A-Za-z0-9._-]`` replaced by ``_`` (user uploads and
    ``Content-Disposition`` headers are untrusted), no leading dots, at most 200 characters."""
    base = (name or "").replace("\\", "/").rsplit("/", 1)[-1]
    base = re.sub(r"[^A-Za-z0-9._-]", "_", base).lstrip(".")[:200]
    return base or f"dataset-{generate_short_uuid()}"


def make_job_id(model_name: str) -> str:
    """``{model-name-lowercased, '_'->'-'}-{uuid8}`` (``/root/reference/app/main.py:422``), made RFC-1123 safe
    because it becomes the PyTorchJob / pod name."""
    base = model_name.strip().lower().replace("_", "-")
    base = re.sub(r"[^a-z0-9-]", "-", base).strip("-") or "job"
    if not base[0].isalpha():  # PyTorchJob names must be DNS-1035 labels
        base = "j" + base
    return f"{base[:50]}-{generate_short_uuid()}"
