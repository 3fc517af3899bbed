"""Orchestration services (C5 task builder, C14 dataset ingest, C15 promotion).

* ``task_builder`` -- resolve the dataset (reuse by id / stream from URL / uploaded file), compute the
  artifacts URI, render and submit the PyTorchJob, insert the job document
  (``/root/reference/app/jobs/task_builder.py:19-81``);
* ``upload_dataset_file`` / ``stream_dataset_url`` -- into ``finetune_jobs/{user}/{job}/dataset/`` plus
  a dataset document (``/root/reference/app/utils/dataset_helpers.py:20-145``); the URL path streams
  chunks straight to object storage (never buffered whole);
* ``PromotionTask`` -- IN_PROGRESS -> copy -> COMPLETED / FAILED, and DELETING -> cleanup ->
  NOT_PROMOTED (revert to COMPLETED on error) (``/root/reference/app/tasks/promotion.py:11-62``).
"""
from __future__ import annotations

import asyncio
import ipaddress
import logging
import os
import socket
from urllib.parse import urlparse

import httpx

from ..context import AppContext
from ..core.naming import generate_short_uuid, safe_filename
from ..k8s.manifest import build_pytorchjob_manifest
from ..schemas.db import DatasetModel, DatasetTypes, PromotionStatus
from ..schemas.jobs import DatasetInput, JobInput

logger = logging.getLogger("ftc.tasks")


class NotFound(Exception):
    pass


class BlockedURL(ValueError):
    pass


def _blocked_ip(ip: str) -> bool:
    """Anything that is not a globally routable unicast address: private, loopback, link-local, reserved,
    multicast, unspecified, and the shared / carrier-grade NAT space 100.64.0.0/10 (``is_global`` is
    False there; it holds some clouds' metadata endpoints and the pod / service CIDRs of several CNIs)."""
    a = ipaddress.ip_address(ip)
    if isinstance(a, ipaddress.IPv6Address) and a.ipv4_mapped is not None:
        a = a.ipv4_mapped
    return (not a.is_global) or a.is_multicast or a.is_unspecified


def _resolve(host: str) -> list[str]:
    return [ai[4][0] for ai in socket.getaddrinfo(host, None, proto=socket.IPPROTO_TCP)]


def _check_host(host: str, resolve=_resolve) -> list[str]:
    """The addresses ``host`` stands for, after refusing any non-public one (BlockedURL)."""
    if not host:
        raise BlockedURL("dataset_url has no host")
    if host.lower() in ("localhost", "localhost.localdomain") or host.lower().endswith(".localhost"):
        raise BlockedURL(f"dataset_url host {host!r} is not allowed")
    try:
        ipaddress.ip_address(host)
        addrs = [host]
    except ValueError:
        try:
            addrs = resolve(host)
        except OSError as e:
            raise BlockedURL(f"dataset_url host {host!r} does not resolve") from e
    if not addrs:
        raise BlockedURL(f"dataset_url host {host!r} does not resolve")
    bad = [ip for ip in addrs if _blocked_ip(ip)]
    if bad:
        raise BlockedURL(f"dataset_url host {host!r} resolves to a non-public address ({bad[0]})")
    return addrs


def guard_url(request: httpx.Request) -> None:
    """Refuse a request whose host is, or resolves to, a non-public address -- the API server must not
    become a proxy into the cluster network or the cloud metadata endpoint."""
    _check_host(request.url.host)


class PinnedTransport(httpx.BaseTransport):
    """Connects to the address that was CHECKED, not to whatever the name resolves to at connect time.

    Checking a name and then letting the HTTP stack resolve it again is open to DNS rebinding (a low-TTL
    name answers a public address to the check and 169.254.169.254 to the connection).  Here every hop
    (redirects included: the client re-enters the transport) resolves once, refuses non-public answers,
    and sends the request to that IP literal; the original name stays in the ``Host`` header and is the
    TLS SNI / certificate name (httpcore's ``sni_hostname`` extension)."""

    def __init__(self, inner: httpx.BaseTransport | None = None, resolve=None):
        self._inner = inner or httpx.HTTPTransport()
        self._resolve = resolve or _resolve

    def handle_request(self, request: httpx.Request) -> httpx.Response:
        host = request.url.host
        ip = _check_host(host, self._resolve)[0]
        if ip != host:
            request.extensions = {**request.extensions, "sni_hostname": host}
            request.url = request.url.copy_with(host=ip)  # the Host header keeps the name
        return self._inner.handle_request(request)

    def close(self) -> None:
        self._inner.close()


def _http_client(allow_private: bool = False, transport: httpx.BaseTransport | None = None,
                 resolve=None) -> httpx.Client:
    """HTTP client used to stream dataset URLs (patched in tests).  No bound on the whole transfer (a
    dataset may take long), but a server that stops answering fails the submission instead of holding its
    worker thread forever: 30 s to connect, 300 s per read.  Every hop goes through ``PinnedTransport``
    unless ``DATASET_URL_ALLOW_PRIVATE``."""
    if not allow_private:
        transport = PinnedTransport(transport, resolve)
    return httpx.Client(timeout=httpx.Timeout(None, connect=30.0, read=300.0), follow_redirects=True,
                        transport=transport)


async def upload_dataset_file(ctx: AppContext, job: JobInput, upload, description: str) -> DatasetModel:
    try:
        name = safe_filename(upload.filename)
        s3_uri = await ctx.s3.upload_dataset(upload.path, job.user_id, job.job_id, name=name)
        doc = await ctx.store.insert_dataset(job.user_id, job.job_id, DatasetTypes(s3_uri=s3_uri), name, description)
        job.s3_uri = doc.dataset.s3_uri
        job.model.dataset_info.dataset_name = doc.dataset_name
        return doc
    finally:
        if os.path.exists(upload.path):
            os.remove(upload.path)


def filename_from_response(headers, url: str) -> str:
    """Dataset name from ``Content-Disposition`` or the URL path, sanitised (both are untrusted and
    end up in the worker pod's shell command: ``k8s.manifest``)."""
    cd = headers.get("Content-Disposition") or headers.get("content-disposition")
    if cd and "filename=" in cd:
        return safe_filename(cd.split("filename=")[-1].strip().strip('"'))
    return safe_filename(os.path.basename(urlparse(url).path) or "default_filename-" + generate_short_uuid())


async def stream_dataset_url(ctx: AppContext, job: JobInput, url: str, description: str,
                             http_client: httpx.Client | None = None) -> DatasetModel:
    def run():
        client = http_client or _http_client(bool(getattr(ctx.settings, "DATASET_URL_ALLOW_PRIVATE", False)))
        try:
            with client.stream("GET", url) as r:
                r.raise_for_status()
                name = filename_from_response(r.headers, url)
                key = f"{ctx.s3.get_dataset_uri_string(ctx.s3.bucket, job.user_id, job.job_id, True)}/{os.path.basename(name)}"
                ctx.objects.put_stream(ctx.s3.bucket, key, r.iter_bytes(1 << 20))
                return name, f"s3://{ctx.s3.bucket}/{key}"
        finally:
            if http_client is None:
                client.close()

    name, s3_uri = await asyncio.to_thread(run)
    doc = await ctx.store.insert_dataset(job.user_id, job.job_id, DatasetTypes(s3_uri=s3_uri, http_url=url), name,
                                         description)
    job.s3_uri = doc.dataset.s3_uri
    job.model.dataset_info.dataset_name = doc.dataset_name
    return doc


async def task_builder(ctx: AppContext, job: JobInput, dataset_input: DatasetInput, http_client=None) -> dict:
    dataset_doc = None
    if dataset_input.dataset_id:
        dataset_doc = await ctx.store.update_dataset(job.user_id, dataset_input.dataset_id, job.job_id)
        if dataset_doc is None:
            raise NotFound("Selected dataset not available")
        job.s3_uri = dataset_doc.dataset.s3_uri
        job.model.dataset_info.dataset_name = dataset_doc.dataset_name
    elif dataset_input.dataset_url:
        dataset_doc = await stream_dataset_url(ctx, job, str(dataset_input.dataset_url),
                                               dataset_input.dataset_description, http_client)
    elif dataset_input.dataset_file:
        dataset_doc = await upload_dataset_file(ctx, job, dataset_input.dataset_file, dataset_input.dataset_description)

    job.s3_artifacts_uri = ctx.s3.get_artifacts_uri_string(ctx.settings.S3_BUCKET_NAME, job.user_id, job.job_id)
    worker = ctx.devices.get_worker(job.device)
    if worker is None:
        raise ValueError(f"Invalid device '{job.device}'. Must be one of {ctx.devices.list_workers()}.")
    manifest = build_pytorchjob_manifest(job, worker, ctx.settings, ctx.namespace)
    result = await asyncio.to_thread(ctx.kube.create_pytorchjob, ctx.namespace, manifest)
    k8s_name = (result.get("metadata") or {}).get("name")
    try:
        await ctx.store.create_job(
            user_id=job.user_id, job_id=job.job_id, job_name=job.job_name, model_name=job.model_name, device=job.device,
            task=job.model.task.value, framework=job.model.framework.value, arguments=job.arguments,
            dataset_id=dataset_doc.id if dataset_doc else None, atrifacts_uri=job.s3_artifacts_uri,
            dataset_name=job.model.dataset_info.dataset_name or None,
            metadata={"kubernetes_job_name": k8s_name})
    except Exception:
        # no job document: the monitor would treat the PyTorchJob as another controller's and leave it
        # holding its GPUs -- take it back before reporting the failure
        try:
            await asyncio.to_thread(ctx.kube.delete_pytorchjob, ctx.namespace, k8s_name or job.job_id)
        except Exception as e:
            logger.error("could not delete PyTorchJob %s after the job insert failed: %s", k8s_name, e)
        raise
    return result


class PromotionTask:
    @staticmethod
    async def promote_job_task(ctx: AppContext, job_id: str, atrifacts_uri: str, destination_uri: str) -> None:
        try:
            await ctx.store.update_job_promotion(job_id, PromotionStatus.IN_PROGRESS, destination_uri)
            await ctx.s3.copy_s3_object(atrifacts_uri, destination_uri)
            await ctx.store.update_job_promotion(job_id, PromotionStatus.COMPLETED, destination_uri)
            logger.info("promotion complete for job %s", job_id)
        except Exception as e:
            logger.error("promotion failed for job %s: %s", job_id, e)
            await ctx.store.update_job_promotion(job_id, PromotionStatus.FAILED, destination_uri)

    @staticmethod
    async def unpromote_job_task(ctx: AppContext, job_id: str, destination_uri: str) -> None:
        try:
            await ctx.store.update_job_promotion(job_id, PromotionStatus.DELETING, destination_uri)
            await ctx.s3.cleanup_uri_items(destination_uri)
            await ctx.store.update_job_promotion(job_id, PromotionStatus.NOT_PROMOTED, None)
            logger.info("unpromotion complete for job %s", job_id)
        except Exception as e:
            logger.error("unpromotion failed for job %s: %s", job_id, e)
            await ctx.store.update_job_promotion(job_id, PromotionStatus.COMPLETED, destination_uri)
