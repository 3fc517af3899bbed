"""API-side schemas (C11): job submission input and the frontend table payloads.

Shapes follow ``/root/reference/app/schemas/jobs_schemas.py:11-132``.  ``JobInput.device`` is validated
against the configured workers by the caller (the worker list is injected, not read at import).
"""
from __future__ import annotations

from datetime import datetime
from typing import Any

from urllib.parse import urlparse

from pydantic import BaseModel, ConfigDict, field_validator

from ..spec.finetuning import BaseFineTuneModel


class UploadedFile(BaseModel):
    """A multipart upload held in a spooled temp file (``fastapi.UploadFile`` stand-in)."""

    model_config = ConfigDict(arbitrary_types_allowed=True)
    filename: str
    content_type: str = "application/octet-stream"
    path: str  # local temp path
    size: int = 0


def validate_http_url(v: str | None) -> str | None:
    """An absolute http(s) URL with a host (the reference types the field ``HttpUrl``,
    ``/root/reference/app/schemas/jobs_schemas.py:13``): anything else is a 422, not a 500 in the
    streaming download."""
    if v is None:
        return v
    v = v.strip()
    u = urlparse(v)
    if u.scheme not in ("http", "https") or not u.hostname or any(c in v for c in " \t\r\n"):
        raise ValueError("dataset_url must be an absolute http(s) URL")
    return v


class DatasetInput(BaseModel):
    dataset_id: str | None = None
    dataset_url: str | None = None
    dataset_file: UploadedFile | None = None
    dataset_description: str = ""

    _url = field_validator("dataset_url")(classmethod(lambda cls, v: validate_http_url(v)))


class JobInput(BaseModel):
    model_config = ConfigDict(arbitrary_types_allowed=True, protected_namespaces=())
    user_id: str
    job_name: str
    model_name: str
    model: BaseFineTuneModel
    device: str
    arguments: dict[str, Any] | None
    s3_uri: str = ""
    s3_artifacts_uri: str = ""
    dataset_url: str = ""
    job_id: str = ""


class JobIdsRequest(BaseModel):
    job_ids: list[str]


# -------- frontend --------
class JobMetaData(BaseModel):
    job_name: str | None = None
    job_id: str | None = None
    model_name: str | None = None
    promotion_path: str | None = None
    dataset_name: str | None = None
    device: str | None = None
    task: str | None = None
    framework: str | None = None
    arguments: dict | str | None = None


class JobMeta(BaseModel):
    error: str | None = None
    note: str | None = None
    data: JobMetaData = JobMetaData()


class Job(BaseModel):
    index_: int
    job_id: str
    job_name: str
    status: str
    status_merged: str
    promoted: str
    model_name: str
    queue_pos: int | None
    start_time: datetime | None
    end_time: datetime | None
    duration: int | None
    dataset_id: str | None
    meta_: JobMeta = JobMeta()


class DatasetMeta(BaseModel):
    error: str | None = None
    note: str | None = None
    data: dict | None = None


class Dataset(BaseModel):
    index_: int
    id: str
    dataset_name: str
    created_at: datetime
    job_ref_names: list[str] | None = None
    meta_: DatasetMeta = DatasetMeta()


class PaginatedTableResponse(BaseModel):
    total: int
    totalPages: int
    resultIndices: list[int]
    page: int
    pageSize: int
    items: list[Job | Dataset]
