"""FastAPI application factory (C1/C2/C4): the REST + WebSocket surface of the controller.

Routes, status codes and payloads follow ``/root/reference/app/main.py``:

=======  ============================================  ==========
method   path                                          rate limit
=======  ============================================  ==========
GET      /auth/cookie, /auth/generate, /auth/verify    10/min (non-production only)
GET      /health, /api/v1/health                       20/min
GET      /api/v1/models                                20/min
GET      /api/v1/models/{model}                        50/min
WS       /api/v1/logs/{job_id}                         (now authenticated)
POST     /api/v1/jobs  (multipart form)                10/min
GET      /api/v1/jobs                                  50/min
GET      /api/v1/jobs/{job_id}                         50/min
GET      /api/v1/jobs/{job_id}/metrics                 50/min
POST     /api/v1/jobs/{job_id}/promote                 2/min
POST     /api/v1/jobs/{job_id}/unpromote               2/min
POST     /api/v1/jobs/{job_id}/cancel
DELETE   /api/v1/jobs/delete  {"job_ids": [...]}
GET      /api/v1/datasets/all                          30/min
GET      /api/v1/datasets                              30/min
DELETE   /api/v1/datasets/{dataset_id}
GET      /api/v1/admin/artifacts/{job_id}  (zip)       5/min
GET      /api/v1/admin/artifacts/presigned_urls/{id}   10/min
GET      /api/v1/admin/job/poll/{job_id}
GET      /api/v1/admin/jobs/list
DELETE   /api/v1/admin/jobs/{user_id}
GET      /api/v1/sample-data.csv
=======  ============================================  ==========

Error envelope ``{"detail", "status_code"}``; the reference's quirks that clients depend on are kept
(promote answers 200/202 *errors* for running / in-progress jobs, the delete response uses the literal
key ``"job_id"``); ``DELETE /admin/jobs/{user_id}`` is fixed (the reference calls ``delete_job`` with
the wrong signature and crashes).
"""
from __future__ import annotations

import asyncio
import json
import logging
import shutil
from contextlib import asynccontextmanager
from datetime import datetime, timezone
from typing import Any

from fastapi import APIRouter, BackgroundTasks, FastAPI, HTTPException, Query, Request, Response, WebSocket
from fastapi.encoders import jsonable_encoder
from fastapi.middleware.cors import CORSMiddleware
from fastapi.openapi.utils import get_openapi
from fastapi.responses import JSONResponse, StreamingResponse
from pydantic import ValidationError

from ..auth.security import (HTTPAuthError, OpenBridgeAuthMiddleware, TokenValidator, auth_enabled,
                             dev_generate_token, verify_token)
from ..context import AppContext
from ..core.naming import make_job_id
from ..k8s.client import KubeError
from ..k8s.queue import pod_events, pod_status
from ..logs.stream import LogStreamManager
from ..monitor.reconciler import JobMonitor
from ..observability import PrometheusMiddleware, get_metrics
from ..schemas.db import DatabaseStatusEnum, PromotionStatus
from ..schemas.jobs import (Dataset, DatasetInput, DatasetMeta, Job, JobIdsRequest, JobInput, JobMetaData,
                            PaginatedTableResponse)
from ..schemas.kubeflow import TrainingJobStatus
from ..spec.finetuning import TrainingTask
from ..tasks.services import BlockedURL, NotFound, PromotionTask, task_builder
from .forms import FormError, discard_uploads, parse_form
from .ratelimit import Limiter, RateLimitExceeded, remote_address

logger = logging.getLogger("ftc.api")
DEFAULT_USER = "default_user"
USER_ID_RE = r"^[a-zA-Z0-9._@]+$"

HIDDEN_DETAIL_FIELDS = {"name", "image", "image_pull_secret", "command", "framework", "description",
                        "checkpoint_mount", "dataset_mount", "task", "dataset_name"}


def custom_openapi_jwt_auth(app: FastAPI, api_prefix: str):
    """OpenAPI with a BearerAuth (JWT) scheme applied to every /api/v1 path (C4)."""

    def build():
        if app.openapi_schema:
            return app.openapi_schema
        schema = get_openapi(title="Finetune Controller API (MI355X)", version="1.0.0",
                             description="Fine-tune job control plane with JWT authentication", routes=app.routes)
        schema.setdefault("components", {})["securitySchemes"] = {
            "BearerAuth": {"type": "http", "scheme": "bearer", "bearerFormat": "JWT"}}
        for path, methods in schema.get("paths", {}).items():
            if path.startswith(api_prefix):
                for m in methods.values():
                    m["security"] = [{"BearerAuth": []}]
        app.openapi_schema = schema
        return schema

    return build


def create_app(ctx: AppContext, run_monitor: bool | None = None, validator_factory=None,
               force_auth: bool | None = None, limiter: Limiter | None = None) -> FastAPI:
    s = ctx.settings
    limiter = limiter or Limiter()
    monitor = JobMonitor(ctx)
    run_monitor = s.DEV_LOCAL_JOB_MONITOR if run_monitor is None else run_monitor

    @asynccontextmanager
    async def lifespan(app: FastAPI):
        logger.info("running in %s environment", s.ENVIRONMENT)
        await ctx.store.connect()
        if run_monitor:
            logger.warning("local job monitor enabled (single leader enforced by a Mongo lease)")
            await monitor.start()
        yield
        if monitor.monitoring_task:
            await monitor.stop()
        await ctx.store.close()

    app = FastAPI(lifespan=lifespan, title="Finetune Controller (MI355X)")
    metrics = get_metrics(ctx)
    app.state.ctx = ctx
    app.state.limiter = limiter
    app.state.monitor = monitor

    # ---- middleware: auth (pure ASGI, HTTP + WS), CORS ----
    use_auth = auth_enabled(s) if force_auth is None else force_auth
    if use_auth:
        factory = validator_factory or (lambda: TokenValidator(
            s.OPENBRIDGE_JWK_URL, s.OPENBRIDGE_INTROSPECTION_URL, s.OPENBRIDGE_CLIENT_ID,
            s.OPENBRIDGE_CLIENT_SECRET.get_secret_value() if s.OPENBRIDGE_CLIENT_SECRET else None))
        app.add_middleware(OpenBridgeAuthMiddleware, settings=s, validator_factory=factory)
    app.add_middleware(CORSMiddleware, allow_origins=s.FRONTEND_URL_CORS, allow_credentials=True,
                       allow_methods=["*"], allow_headers=["*"])
    app.add_middleware(PrometheusMiddleware, metrics=metrics)  # outermost: sees auth rejections too

    @app.get("/metrics", include_in_schema=False)
    async def prometheus_metrics():
        body, ctype = metrics.exposition()
        return Response(content=body, media_type=ctype)
    app.openapi = custom_openapi_jwt_auth(app, s.API_V1_STR)

    @app.exception_handler(HTTPException)
    async def http_exc(request: Request, exc: HTTPException):
        if request.method == "POST" and request.url.path == f"{s.API_V1_STR}/jobs":
            metrics.submit_failures.labels(str(exc.status_code)).inc()
        return JSONResponse(status_code=exc.status_code, content={"detail": exc.detail, "status_code": exc.status_code})

    @app.exception_handler(RateLimitExceeded)
    async def rate_exc(request: Request, exc: RateLimitExceeded):
        logger.debug("rate limit hit by %s", remote_address(request))
        return JSONResponse(status_code=429, content={"detail": "Rate limit exceeded", "status_code": 429})

    @app.exception_handler(HTTPAuthError)
    async def auth_exc(request: Request, exc: HTTPAuthError):
        return JSONResponse(status_code=exc.status_code, content={"detail": exc.detail, "status_code": exc.status_code})

    api = APIRouter(prefix=s.API_V1_STR)

    # ---------------------------------------------------------------- helpers
    def decode_request(request):
        st = request.scope.get("state", {})
        return st.get("jwt_data"), st.get("decoded_jwt")

    def validate_user_access(jwt, record):
        if jwt and record and jwt.user_id != record.user_id:
            logger.warning("user %s tried to access restricted resource %s", jwt.user_id, record.job_id)
            raise HTTPException(status_code=400, detail="Cannot access resource")

    def is_admin(jwt) -> bool:
        return bool(jwt) and (s.ADMIN_SCOPE in (jwt.available_models or []) or jwt.user_id in (s.ADMIN_USERS or []))

    def require_admin(jwt, action: str, owner: str | None = None):
        """Admin routes: with auth on, only an admin (scope / user list) -- or, for per-user routes,
        that user -- may act.  Without auth (dev / local) the reference's open behaviour is kept."""
        if not jwt or is_admin(jwt) or (owner is not None and jwt.user_id == owner):
            return
        logger.warning("user %s denied admin action %s", jwt.user_id, action)
        raise HTTPException(status_code=403, detail="Admin privileges required")

    def parse_limit(limit: str | None) -> list[int] | None:
        """``limit``: comma-separated row indices of the table view; anything else is the client's error."""
        if not limit:
            return None
        try:
            return [int(x) for x in limit.split(",")]
        except ValueError as e:
            raise HTTPException(status_code=422, detail="limit: comma-separated integers expected") from e

    def available_models(jwt=None) -> list[str]:
        return ctx.registry.available_for(jwt.available_models if jwt else None)

    def device_names():
        return ctx.devices.list_workers()

    # ---------------------------------------------------------------- dev auth
    if s.ENVIRONMENT != "production":
        @app.get("/auth/cookie", tags=["Auth"])
        @limiter.limit("10/minute")
        async def get_dev_bridge_user_cookie(request: Request, response: Response, user: str = Query("default_user")):
            token = dev_generate_token(s.JWT_SECRET_KEY, s.JWT_ALGORITHM, user, ctx.registry.all_inference_names())
            cookie = json.dumps({"config": None, "resources": [], "subject": "foobar", "user_type": "group",
                                 "token": token})
            response.set_cookie(key="bridge-user", value=cookie, httponly=True, samesite="strict")
            return token

        @app.get("/auth/generate", tags=["Auth"])
        @limiter.limit("10/minute")
        async def generate_token_auth(request: Request, user: str = Query("default_user"),
                                      include_models: str = Query("", description="Comma separated models")):
            models = [m.strip() for m in include_models.split(",") if m.strip()] or ctx.registry.all_inference_names()
            return {"token": dev_generate_token(s.JWT_SECRET_KEY, s.JWT_ALGORITHM, user, models)}

        @app.get("/auth/verify", tags=["Auth"])
        @limiter.limit("10/minute")
        async def verify_token_auth(request: Request, token: str):
            return verify_token(s.JWT_SECRET_KEY, s.JWT_ALGORITHM, token)

    # ---------------------------------------------------------------- general
    @app.get("/health")
    @limiter.limit("20/minute")
    async def health_root(request: Request):
        return {"status": "ok"}

    @api.get("/health")
    @limiter.limit("20/minute")
    async def health(request: Request):
        return {"status": "ok"}

    @api.get("/models", tags=["Models"])
    @limiter.limit("20/minute")
    async def list_available_models(request: Request) -> dict[str, Any]:
        jwt_data, jwt = decode_request(request)
        names = available_models(jwt if (jwt_data and jwt) else None)
        out = {}
        for name in names:
            try:
                m = ctx.registry.instance(name)
                out[name] = {"description": m.description, "url": m.project_url,
                             "arguments": m.training_arguments.model_json_schema().get("properties", {}),
                             "task": m.task, "devices": device_names(),
                             "dataset_required": m.dataset_info.dataset_required,
                             "dataset_description": m.dataset_info.description}
            except Exception as e:
                logger.error("could not get form data for model %s: %s", name, e)
        return out

    @api.get("/models/{model}", tags=["Models"])
    @limiter.limit("50/minute")
    async def get_model_details(model: str, request: Request):
        jwt_data, jwt = decode_request(request)
        if jwt_data and model not in available_models(jwt):
            raise HTTPException(status_code=404, detail=f"Model '{model}' not found")
        cls = ctx.registry.get(model)
        if not cls:
            raise HTTPException(status_code=404, detail=f"Model '{model}' not found")
        try:
            inst = cls()
            schema = inst.model_json_schema()
            required = set(schema.get("required", []))
            args, detail = {}, {}
            for fname in schema.get("properties", {}):
                if fname not in required and fname not in HIDDEN_DETAIL_FIELDS:
                    args[fname] = getattr(inst, fname)
                elif fname in ("framework", "description", "task"):
                    detail[fname] = getattr(inst, fname)
            return jsonable_encoder({"arguments": args} | detail)
        except Exception as e:
            raise HTTPException(status_code=500, detail=f"Error getting model options: {e}") from e

    @api.websocket("/logs/{job_id}")
    async def stream_job(websocket: WebSocket, job_id: str, full_log: bool = True, follow: bool = True,
                         last_lines: int = 100):
        await websocket.accept()
        jwt_data = websocket.scope.get("state", {}).get("decoded_jwt")
        if jwt_data is not None:
            rec = await ctx.store.get_job(job_id)
            if rec and rec.user_id != jwt_data.user_id:
                await websocket.send_text("Error: Cannot access resource")
                await websocket.close(code=1008)
                return
        mgr = LogStreamManager(ctx, websocket, job_id, full_log, follow, last_lines, s.LOG_STREAM_SEARCH_STRING)
        try:
            await mgr.run()
        except Exception as e:
            logger.error("unexpected error in stream_job: %s", e)

    # ---------------------------------------------------------------- jobs
    @api.post("/jobs", tags=["Jobs"], openapi_extra={"requestBody": {"content": {"multipart/form-data": {"schema": {
        "type": "object", "required": ["job_name", "model", "device", "task"],
        "properties": {"user_id": {"type": "string", "default": DEFAULT_USER}, "job_name": {"type": "string"},
                       "model": {"type": "string"}, "device": {"type": "string"}, "task": {"type": "string"},
                       "arguments": {"type": "string", "default": "{}"},
                       "dataset_description": {"type": "string"}, "dataset_id": {"type": "string"},
                       "dataset_url": {"type": "string"}, "dataset": {"type": "string", "format": "binary"}}}}}}})
    @limiter.limit("10/minute")
    async def start_job(request: Request):
        try:
            fields, files = await parse_form(request)
        except FormError as e:
            raise HTTPException(status_code=422, detail=str(e)) from e
        try:
            return await submit_job(request, fields, files)
        finally:
            discard_uploads(files)  # a rejected request leaves no spooled upload behind

    async def submit_job(request: Request, fields: dict, files: dict):
        user_id = fields.get("user_id") or DEFAULT_USER
        import re

        if len(user_id) < 4 or not re.match(USER_ID_RE, user_id):
            raise HTTPException(status_code=422, detail="user_id: must be >= 4 characters of [a-zA-Z0-9._@]")
        missing = [k for k in ("job_name", "model", "device", "task") if not fields.get(k)]
        if missing:
            raise HTTPException(status_code=422, detail=f"missing form fields: {', '.join(missing)}")
        job_name, model, device, task_s = fields["job_name"], fields["model"], fields["device"], fields["task"]
        if device not in device_names():
            raise HTTPException(status_code=422, detail=f"device: must be one of {device_names()}")
        try:
            task = TrainingTask(task_s)
        except ValueError:
            try:
                task = TrainingTask[task_s]
            except KeyError:
                raise HTTPException(status_code=422, detail=f"task: must be one of {[t.value for t in TrainingTask]}")
        jwt_data, jwt = decode_request(request)
        if jwt_data and jwt:
            user_id = jwt.user_id
            if model not in available_models(jwt):
                raise HTTPException(status_code=404, detail=f"Model '{model}' not found")
        try:
            model_arguments = json.loads(fields.get("arguments") or "{}")
        except json.JSONDecodeError as e:
            raise HTTPException(status_code=400, detail="Invalid JSON for arguments") from e
        if not isinstance(model_arguments, dict):
            raise HTTPException(status_code=400, detail="Invalid JSON for arguments: expected an object")
        job_id = make_job_id(model)
        if fields.get("dataset_id"):
            ds = DatasetInput(dataset_id=fields["dataset_id"])
        elif fields.get("dataset_url"):
            try:
                ds = DatasetInput(dataset_url=fields["dataset_url"])
            except ValidationError as e:
                raise HTTPException(status_code=422, detail="dataset_url: must be an absolute http(s) URL") from e
        elif files.get("dataset"):
            ds = DatasetInput(dataset_file=files["dataset"])
        else:
            ds = DatasetInput()
        ds.dataset_description = fields.get("dataset_description") or ""
        try:
            cls = ctx.registry.get(model)
            if not cls:
                raise HTTPException(status_code=404, detail=f"Model '{model}' not found")
            # user arguments override the SPEC's default arguments (the reference rebuilds the arguments
            # class from its field defaults, silently dropping per-spec defaults such as GPT-2's seq_len)
            base = cls.model_fields["training_arguments"].get_default()
            merged = {**(base.model_dump() if base is not None else {}), **model_arguments}
            inst = cls.model_validate(cls(training_arguments=merged))
            model_arguments = inst.training_arguments.model_dump()
            if task != inst.task:
                raise HTTPException(status_code=400, detail=f"Invalid task ({task.name}) for model ({inst.task.name})")
            # a spec that declares dataset_required is refused without one here, not as a failed pod later
            if inst.dataset_info.dataset_required and not (ds.dataset_id or ds.dataset_url or ds.dataset_file):
                raise HTTPException(status_code=400, detail=f"Model '{model}': dataset is required "
                                                            "(dataset, dataset_url or dataset_id)")
        except ValidationError as e:
            msgs = [f"{(err['loc'][-1] if err['loc'] else 'unknown field')}: {err['msg']}" for err in e.errors()]
            raise HTTPException(status_code=400, detail="<b class='regular'>Invalid model parameters:</b><br>• "
                                                        + "<br>• ".join(msgs)) from e
        job = JobInput(user_id=user_id, job_name=job_name, model_name=model, model=inst, device=device,
                       arguments=model_arguments or None, job_id=job_id)
        try:
            await task_builder(ctx, job, ds)
            logger.info("job started successfully: %s", job_id)
            metrics.jobs_submitted.labels(model, str(getattr(device, "value", device))).inc()
            return {"message": "Job started successfully", "job_id": job_id}
        except NotFound as e:
            raise HTTPException(status_code=404, detail=str(e)) from e
        except BlockedURL as e:
            raise HTTPException(status_code=422, detail=f"dataset_url: {e}") from e
        except KubeError as e:
            raise HTTPException(status_code=e.status, detail=f"Failed to start job {job_name} / {job_id}<br>{e}") from e
        except Exception as e:
            logger.error("job submission failed: %s", e, exc_info=True)
            info = "<br>".join(f"{k}: {v}" for k, v in {"dataset_id": ds.dataset_id, "dataset_url": ds.dataset_url}.items() if v)
            raise HTTPException(status_code=500, detail=f"Failed to start job {job_name} / {job_id}<br>{e}<br>{info}") from e

    @api.get("/jobs", tags=["Jobs"])
    @limiter.limit("50/minute")
    async def get_user_jobs_page(request: Request, user_id: str = Query(DEFAULT_USER), page: int = Query(1),
                                 page_size: int = Query(10), sort: str | None = Query(None),
                                 query: str | None = Query(None), limit: str | None = Query(None),
                                 status: str | None = Query(None), model_name: str | None = Query(None)):
        jwt_data, jwt = decode_request(request)
        if jwt_data and jwt:
            user_id = jwt.user_id
        lim = parse_limit(limit)
        try:
            data = await ctx.store.get_user_jobs(user_id, page, page_size, sort, query, lim, status, model_name)
            items = []
            for j in data.items:
                m = ctx.registry.instance(j.model_name)
                promo = m.promotion_path.strip("/") if m and m.promotion_path else "Not available"
                extra = j.model_extra or {}
                items.append(Job(
                    index_=extra.get("index_", 0), job_id=j.job_id, job_name=j.job_name, promoted=j.promoted.value,
                    model_name=j.model_name, queue_pos=j.metadata.queue_pos if j.metadata else None,
                    status=j.status.value, status_merged=extra.get("status_merged") or j.status.value,
                    start_time=extra.get("start_time"), end_time=extra.get("end_time"), duration=extra.get("duration"),
                    dataset_id=j.dataset_id,
                    meta_={"error": None, "note": None, "data": JobMetaData(
                        job_name=j.job_name, job_id=j.job_id, model_name=j.model_name, promotion_path=promo,
                        device=j.device, task=j.task, framework=j.framework, arguments=j.arguments or "-",
                        dataset_name=j.dataset_name or "-")}))
            return PaginatedTableResponse(total=data.total, totalPages=data.total_pages, resultIndices=[], page=page,
                                          pageSize=page_size, items=items)
        except Exception as e:
            logger.error("get jobs failed: %s", e, exc_info=True)
            raise HTTPException(status_code=500, detail=f"Failed to get job status: {e}") from e

    @api.get("/jobs/{job_id}", tags=["Jobs"])
    @limiter.limit("50/minute")
    async def get_job(request: Request, job_id: str):
        jwt_data, jwt = decode_request(request)
        info = await ctx.store.get_job(job_id)
        validate_user_access(jwt, info)
        if not info:
            raise HTTPException(status_code=404, detail=f"Job '{job_id}' not found")
        return jsonable_encoder(info)

    @api.get("/jobs/{job_id}/metrics", tags=["Jobs"])
    @limiter.limit("50/minute")
    async def get_job_metrics(request: Request, job_id: str):
        jwt_data, jwt = decode_request(request)
        info = await ctx.store.get_job(job_id)
        validate_user_access(jwt, info)
        if not info:
            raise HTTPException(status_code=404, detail=f"Job '{job_id}' not found")
        m = await ctx.store.get_job_metrics(job_id)
        if not m and TrainingJobStatus.is_running(info.status):
            raise HTTPException(status_code=202, detail="Job is still running. no metrics found")
        if not m:
            raise HTTPException(status_code=404, detail=f"no metrics available for job {job_id}")
        rows = list(m.metrics or [])
        rows.reverse()
        data = m.model_dump()
        data["metrics"] = rows[:100]
        try:
            urls = await ctx.s3.get_presigned_urls(m.user_id, job_id)
            data["metrics_url"] = next((u["url"] for u in urls if u["key"] == "metrics.csv"), None)
        except Exception as e:
            logger.error("presigned urls failed for %s: %s", job_id, e)
            data["metrics_url"] = None
        return jsonable_encoder(data)

    @api.post("/jobs/{job_id}/promote", tags=["Jobs"])
    @limiter.limit("2/minute")
    async def promote_job(request: Request, job_id: str, background_tasks: BackgroundTasks):
        jwt_data, jwt = decode_request(request)
        info = await ctx.store.get_job(job_id)
        validate_user_access(jwt, info)
        bucket = s.S3_DEFAULT_DEPLOY_BUCKET.strip()
        if not info:
            raise HTTPException(status_code=404, detail=f"Job '{job_id}' not found")
        if info.promoted == PromotionStatus.IN_PROGRESS:
            raise HTTPException(status_code=202, detail="Job is being promoted already")
        if info.promoted == PromotionStatus.DELETING:
            # a copy started now would race the running delete of the same prefix
            raise HTTPException(status_code=409, detail="Job is being unpromoted; promote it again when that is done")
        if TrainingJobStatus.is_running(info.status):
            raise HTTPException(status_code=200, detail="Cannot promote running job")
        if not info.atrifacts_uri or not bucket:
            raise HTTPException(status_code=404, detail="Cannot promote this job")
        m = ctx.registry.instance(info.model_name)
        if info.promoted == PromotionStatus.COMPLETED:
            return {"status": PromotionStatus.COMPLETED.value, "model": m.promotion_path.strip("/") if m else None,
                    "version": job_id}
        if not m or not m.promotion_path:
            raise HTTPException(status_code=400, detail="Model cannot be promoted")
        dest = "s3://" + "/".join([bucket, m.promotion_path.strip("/"), job_id])
        busy = [PromotionStatus.IN_PROGRESS, PromotionStatus.DELETING, PromotionStatus.COMPLETED]
        if not await ctx.store.claim_job_promotion(job_id, PromotionStatus.IN_PROGRESS, dest, unless=busy):
            raise HTTPException(status_code=409, detail="Job promotion state changed concurrently")
        background_tasks.add_task(PromotionTask.promote_job_task, ctx, job_id, info.atrifacts_uri, dest)
        return {"status": "promotion_initiated", "job_id": job_id, "message": "Job promotion started in background"}

    @api.post("/jobs/{job_id}/unpromote", tags=["Jobs"])
    @limiter.limit("2/minute")
    async def unpromote_job(request: Request, background_tasks: BackgroundTasks, job_id: str):
        jwt_data, jwt = decode_request(request)
        info = await ctx.store.get_job(job_id)
        validate_user_access(jwt, info)
        if not info:
            raise HTTPException(status_code=400, detail="Job not found")
        if info.promoted != PromotionStatus.COMPLETED:
            raise HTTPException(status_code=400, detail="Model not promoted. cannot unpromote")
        if not info.destination_uri:
            raise HTTPException(status_code=400, detail="Cannot unpromote model")
        if not await ctx.store.claim_job_promotion(job_id, PromotionStatus.DELETING, info.destination_uri,
                                                   when=[PromotionStatus.COMPLETED]):
            raise HTTPException(status_code=400, detail="Model not promoted. cannot unpromote")
        background_tasks.add_task(PromotionTask.unpromote_job_task, ctx, job_id, info.destination_uri)
        return {"status": "unpromotion_initiated", "job_id": job_id, "message": "Job unpromotion started in background"}

    @api.post("/jobs/{job_id}/cancel", tags=["Jobs"])
    async def cancel_job(request: Request, job_id: str):
        jwt_data, jwt = decode_request(request)
        info = await ctx.store.get_job(job_id)
        validate_user_access(jwt, info)
        if not info:
            raise HTTPException(status_code=404, detail=f"Job '{job_id}' not found")
        if TrainingJobStatus.is_stopped(info.status):
            raise HTTPException(status_code=409, detail="Item already cancelled")
        try:
            await asyncio.to_thread(ctx.kube.delete_pytorchjob, ctx.namespace, job_id)
        except KubeError as e:
            if e.status != 404:
                raise HTTPException(status_code=e.status, detail=f"Failed to cancel job {job_id}: {e}") from e
        await ctx.store.update_job_status(job_id, DatabaseStatusEnum.canceled.value, metadata={
            "cancellation_time": datetime.now(timezone.utc), "message": "Job canceled by user"})
        info = await ctx.store.get_job(job_id)
        extra = info.model_extra or {}
        return jsonable_encoder({"status": info.status, "start_time": extra.get("start_time"),
                                 "end_time": extra.get("end_time"), "duration": extra.get("duration")})

    async def _delete_one(job_id: str, jwt):
        info = await ctx.store.get_job(job_id)
        validate_user_access(jwt, info)
        if not info:
            raise HTTPException(status_code=404, detail=f"Job '{job_id}' not found")
        if TrainingJobStatus.is_running(info.status):
            raise HTTPException(status_code=400, detail="Job is still running")
        # a failed job's PyTorchJob stays on the cluster (only succeeded ones are removed by the monitor):
        # deleting the job takes it along, or it would outlive every record of it
        try:
            await asyncio.to_thread(ctx.kube.delete_pytorchjob, ctx.namespace, job_id)
        except KubeError as e:
            if e.status != 404:
                logger.warning("job %s: PyTorchJob delete failed: %s", job_id, e)
        except Exception as e:  # noqa: BLE001 -- cleanup must not block the record deletion
            logger.warning("job %s: PyTorchJob delete failed: %s", job_id, e)
        if info.promoted == PromotionStatus.COMPLETED and info.destination_uri:
            await ctx.s3.cleanup_uri_items(info.destination_uri)
        if info.atrifacts_uri:
            await ctx.s3.cleanup_uri_items(info.atrifacts_uri)
        await ctx.store.delete_metrics(job_id)
        await ctx.store.delete_job(job_id)

    @api.delete("/jobs/delete", tags=["Jobs"])
    async def delete_job(request: Request, body: JobIdsRequest):
        jwt_data, jwt = decode_request(request)
        out = {}
        for job_id in body.job_ids:
            await _delete_one(job_id, jwt)
            out["job_id"] = {"message": "Jobs deleted successfully"}  # literal key: reference response shape
        return out

    # ---------------------------------------------------------------- datasets
    @api.get("/datasets/all", tags=["Datasets"])
    @limiter.limit("30/minute")
    async def get_user_datasets_all(request: Request, user_id: str = Query(DEFAULT_USER)):
        jwt_data, jwt = decode_request(request)
        if jwt and jwt_data:
            user_id = jwt.user_id
        return jsonable_encoder([d.model_dump(exclude={"dataset": {"s3_uri"}}) for d in
                                 await ctx.store.get_user_datasets_all(user_id)])

    @api.get("/datasets", tags=["Datasets"])
    @limiter.limit("30/minute")
    async def get_user_datasets_page(request: Request, user_id: str = Query(DEFAULT_USER), page: int = Query(1),
                                     page_size: int = Query(10), sort: str | None = Query(None),
                                     query: str | None = Query(None), limit: str | None = Query(None)):
        jwt_data, jwt = decode_request(request)
        if jwt:
            user_id = jwt.user_id
        lim = parse_limit(limit)
        try:
            data = await ctx.store.get_user_datasets_page(user_id, page, page_size, sort, query, lim)
            items = []
            for d in data.items:
                extra = d.model_extra or {}
                names = extra.get("job_ref_names") or []
                meta = {"Id": d.id, "Related jobs": ", ".join(names) if names else "-"}
                if d.dataset.http_url:
                    meta["Source"] = d.dataset.http_url
                items.append(Dataset(index_=extra.get("index_", 0), id=d.id, dataset_name=d.dataset_name,
                                     created_at=d.created_at, job_ref_names=names,
                                     meta_=DatasetMeta(error=None, note=d.description, data=meta)))
            return PaginatedTableResponse(total=data.total, totalPages=data.total_pages, resultIndices=[], page=page,
                                          pageSize=page_size, items=items)
        except Exception as e:
            raise HTTPException(status_code=500, detail=f"Failed to get datasets: {e}") from e

    @api.delete("/datasets/{dataset_id}", tags=["Datasets"])
    async def delete_datasets(request: Request, dataset_id: str, user_id: str = Query(DEFAULT_USER)):
        jwt_data, jwt = decode_request(request)
        if jwt:
            user_id = jwt.user_id
        d = await ctx.store.get_user_dataset(user_id, dataset_id)
        if not d:
            raise HTTPException(status_code=404, detail=f"Dataset '{dataset_id}' not found")
        if d.dataset.s3_uri:
            await ctx.s3.cleanup_uri_items(d.dataset.s3_uri)
        await ctx.store.delete_dataset(user_id, dataset_id)
        return {"message": "Dataset deleted successfully"}

    # ---------------------------------------------------------------- admin
    async def _owned_finished_job(job_id, user_id, jwt):
        info = await ctx.store.get_job(job_id)
        if not info:
            raise HTTPException(status_code=404, detail=f"Job '{job_id}' not found")
        if jwt and info.user_id != jwt.user_id:
            raise HTTPException(status_code=400, detail="Cannot access resource")
        if TrainingJobStatus.is_running(info.status):
            raise HTTPException(status_code=400, detail="Job is still running or has not completed successfully")
        return info

    @api.get("/admin/artifacts/{job_id}", tags=["Admin"])
    @limiter.limit("5/minute")
    async def get_artifacts(request: Request, job_id: str, user_id: str = Query(DEFAULT_USER)):
        jwt_data, jwt = decode_request(request)
        if jwt:
            user_id = jwt.user_id
        info = await _owned_finished_job(job_id, user_id, jwt)
        try:
            zip_path, temp_dir = await ctx.s3.download_artifacts(info.user_id if not jwt else user_id, job_id)
        except Exception as e:
            raise HTTPException(status_code=404, detail=str(e)) from e

        def stream():
            try:
                with open(zip_path, "rb") as f:
                    while chunk := f.read(1 << 16):
                        yield chunk
            finally:
                shutil.rmtree(temp_dir, ignore_errors=True)

        return StreamingResponse(stream(), media_type="application/zip",
                                 headers={"Content-Disposition": f"attachment; filename=artifacts_{job_id}.zip"})

    @api.get("/admin/artifacts/presigned_urls/{job_id}", tags=["Admin"])
    @limiter.limit("10/minute")
    async def get_artifact_urls(request: Request, job_id: str, user_id: str = Query(DEFAULT_USER)):
        jwt_data, jwt = decode_request(request)
        if jwt:
            user_id = jwt.user_id
        info = await _owned_finished_job(job_id, user_id, jwt)
        try:
            return {"artifacts": await ctx.s3.get_presigned_urls(info.user_id if not jwt else user_id, job_id)}
        except Exception as e:
            raise HTTPException(status_code=404, detail=str(e)) from e

    @api.get("/admin/job/poll/{job_id}", tags=["Admin"])
    async def poll_admin_job(request: Request, job_id: str):
        jwt_data, jwt = decode_request(request)
        if jwt and not is_admin(jwt):
            info = await ctx.store.get_job(job_id)
            require_admin(jwt, f"poll {job_id}", owner=info.user_id if info else None)
        try:
            job = await asyncio.to_thread(ctx.kube.get_pytorchjob, ctx.namespace, job_id)
            st = job.get("status") or {}
            selector = st["replicaStatuses"]["Master"]["selector"]
            events = await asyncio.to_thread(pod_events, ctx.kube, ctx.namespace, selector)
            pstat = await asyncio.to_thread(pod_status, ctx.kube, ctx.namespace, selector)
            cond = dict(st["conditions"][-1])
            cond["events"] = [{"type": e.get("type"), "message": e.get("message"), "reason": e.get("reason")}
                              for e in events]
            if pstat:
                cond.update(pstat)
            return {"status": cond}
        except KubeError as e:
            if e.status == 404:
                raise HTTPException(status_code=404, detail=f"Job '{job_id}' not found") from e
            raise HTTPException(status_code=500, detail=f"Failed to get job status: '{job_id}'") from e
        except Exception as e:
            raise HTTPException(status_code=404, detail=str(e)) from e

    @api.get("/admin/jobs/list", tags=["Admin"])
    async def list_jobs(request: Request):
        require_admin(decode_request(request)[1], "list cluster jobs")
        try:
            jobs = await asyncio.to_thread(ctx.kube.list_pytorchjobs, ctx.namespace)
            return {"jobs": [j["metadata"]["name"] for j in jobs]}
        except KubeError as e:
            raise HTTPException(status_code=500, detail=f"Failed to list jobs: {e}") from e

    @api.delete("/admin/jobs/{user_id}", tags=["Admin"])
    async def clean_user_jobs(request: Request, user_id: str):
        # fixed route (the reference calls delete_job with the wrong signature and never deletes):
        # with auth on, only that user or an admin may wipe a user's jobs
        require_admin(decode_request(request)[1], f"delete jobs of {user_id}", owner=user_id)
        jobs = await ctx.store.get_all_user_jobs(user_id)
        deleted, skipped = [], []
        for j in jobs:
            try:
                await _delete_one(j.job_id, None)
                deleted.append(j.job_id)
            except HTTPException as e:
                skipped.append({"job_id": j.job_id, "reason": e.detail})
        if not deleted:
            return {"message": "No jobs deleted", "jobs": [], "skipped": skipped}
        return {"message": "Jobs deleted successfully", "jobs": deleted, "skipped": skipped}

    @api.get("/sample-data.csv")
    async def csv_sample():
        data = "Id,SMILES,esol\naaa,CCC(=O)C=C(N)C(C)(C)c1nccs1,2.1\nbbb,CCOC(=O)CC(=O)C(C)(C)c1ccccn1,9.2\n" \
               "ccc,CCOC(=O)CC(N)C(C)(C)c1ccccn1,6.5"
        return Response(content=data, media_type="text/csv")

    app.include_router(api)
    return app


def app_from_env() -> FastAPI:
    """uvicorn entry: ``uvicorn finetune_controller_amd.controlplane.api.app:app_from_env --factory``."""
    from ..core.config import get_settings
    from ..core.logging_config import setup_logging

    setup_logging()
    return create_app(AppContext.from_settings(get_settings()))
