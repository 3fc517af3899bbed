"""Job / dataset / metrics persistence (C9).

Same collections (``jobs``, ``metrics``, ``datasets``, ``archived_jobs``), indexes, document shapes and
aggregation-derived fields as ``/root/reference/app/database/db.py:24-706``, written once against a
Motor-style async collection API and backed by either

* MongoDB through pymongo's native ``AsyncMongoClient`` (``tz_aware=True``), or
* the in-memory engine of ``store/memory.py`` (tests, single-process dev, the e2e FakeCluster run).

Changes vs the reference:
* ``update_job_status`` merges metadata with atomic ``$set`` on ``metadata.<field>`` paths instead of a
  read-modify-write of the whole sub-document (concurrent monitor + API cancel were racy);
* ``update_dataset`` appends the job reference with ``$addToSet``;
* the datasets page reports the number of ITEMS as ``total`` (the reference returns the page count);
* ``acquire_lock`` -- a TTL lease document used to keep a single active job monitor;
* the name search of the jobs / datasets pages matches the user's text literally (``re.escape``): the
  reference hands it to ``$regex`` as a pattern, so ``(`` or ``[`` fail the request and a crafted pattern
  can make the server backtrack for a long time.
"""
from __future__ import annotations

import datetime as _dt
import inspect
import logging
import re
from typing import Any

from bson import ObjectId

from ..schemas.db import (DatabaseStatusEnum, DatasetModel, DatasetPage, DatasetTypes, JobsPage, JobStatus,
                          MetricsDocument, PromotionStatus)
from .memory import DuplicateKeyError, MemoryClient

logger = logging.getLogger("ftc.store")


def _utcnow():
    return _dt.datetime.now(tz=_dt.timezone.utc)


async def _maybe_await(x):
    return await x if inspect.isawaitable(x) else x


def _enum_values(d):
    """Plain values for storage (str Enums -> str) so both backends hold identical documents."""
    if isinstance(d, dict):
        return {k: _enum_values(v) for k, v in d.items()}
    if isinstance(d, list):
        return [_enum_values(v) for v in d]
    if hasattr(d, "value") and isinstance(getattr(d, "value"), str) and d.__class__.__module__ != "builtins":
        return d.value
    return d


class JobStore:
    def __init__(self, client=None, database: str = "default", url: str | None = None, username=None,
                 password=None):
        self._client = client
        self.database = database
        self.url, self.username, self.password = url, username, password
        self.db = None
        self.jobs_collection = self.metrics_collection = self.datasets_collection = None
        self.archived_jobs_collection = self.locks_collection = None

    @classmethod
    def memory(cls, database: str = "default") -> "JobStore":
        return cls(client=MemoryClient(), database=database)

    @classmethod
    def from_settings(cls, settings) -> "JobStore":
        if settings.STORE_BACKEND == "memory":
            return cls.memory(settings.MONGODB_DATABASE)
        return cls(url=settings.MONGODB_URL, database=settings.MONGODB_DATABASE,
                   username=settings.MONGODB_USERNAME.get_secret_value() if settings.MONGODB_USERNAME else None,
                   password=settings.MONGODB_PASSWORD.get_secret_value() if settings.MONGODB_PASSWORD else None)

    async def connect(self):
        if self._client is None:
            from pymongo import AsyncMongoClient

            kw: dict[str, Any] = {"tz_aware": True}
            if self.username and self.password:
                kw.update(username=self.username, password=self.password)
            self._client = AsyncMongoClient(self.url, **kw)
        self.db = self._client[self.database]
        self.jobs_collection = self.db["jobs"]
        self.metrics_collection = self.db["metrics"]
        self.datasets_collection = self.db["datasets"]
        self.archived_jobs_collection = self.db["archived_jobs"]
        self.locks_collection = self.db["locks"]
        await self._ensure_indexes()

    async def close(self):
        if self._client is not None:
            await _maybe_await(self._client.close())

    async def _ensure_indexes(self):
        j = self.jobs_collection
        await j.create_index("user_id")
        await j.create_index("job_id", unique=True)
        await j.create_index([("job_name", "text"), ("model_name", "text")])
        await j.create_index([("user_id", 1), ("status", 1)])
        await j.create_index([("user_id", 1), ("job_id", 1)])
        await self.archived_jobs_collection.create_index("user_id")
        await self.archived_jobs_collection.create_index("job_id", unique=True)
        await self.metrics_collection.create_index("user_id")
        await self.metrics_collection.create_index("job_id", unique=True)
        await self.metrics_collection.create_index([("user_id", 1), ("job_id", 1)])
        await self.datasets_collection.create_index([("_id", 1), ("user_id", 1)])
        await self.datasets_collection.create_index("user_id")

    # ------------------------------------------------------------------ jobs
    async def create_job(self, user_id, job_id, job_name, model_name, device, task, framework, arguments=None,
                         dataset_id=None, atrifacts_uri=None, dataset_name=None, metadata=None) -> JobStatus:
        now = _utcnow()
        job = JobStatus(user_id=user_id, job_id=job_id, job_name=job_name, status=DatabaseStatusEnum.queued,
                        promoted=PromotionStatus.NOT_PROMOTED, created_at=now, updated_at=now,
                        model_name=model_name, device=device, task=task, framework=framework, arguments=arguments,
                        dataset_id=dataset_id, atrifacts_uri=atrifacts_uri, dataset_name=dataset_name,
                        metadata=metadata or {})  # always a sub-document: metadata.<k> $set needs one
        await self.jobs_collection.insert_one(_enum_values(job.model_dump()))
        return job

    async def update_job_status(self, job_id: str, status: str, metadata: dict | None = None) -> JobStatus | None:
        upd: dict[str, Any] = {"status": _enum_values(status), "updated_at": _utcnow()}
        for k, v in (metadata or {}).items():
            upd[f"metadata.{k}"] = _enum_values(v)
        res = await self.jobs_collection.update_one({"job_id": job_id}, {"$set": upd})
        if res.modified_count > 0:
            return await self.get_job(job_id)
        return None

    async def update_job_promotion(self, job_id: str, value: PromotionStatus, destination_uri: str | None = None):
        res = await self.jobs_collection.update_one(
            {"job_id": job_id}, {"$set": {"promoted": _enum_values(value), "destination_uri": destination_uri}})
        if res.modified_count > 0:
            return await self.get_job(job_id)
        return None

    async def claim_job_promotion(self, job_id: str, value: PromotionStatus, destination_uri: str | None,
                                  *, when: list[PromotionStatus] | None = None,
                                  unless: list[PromotionStatus] | None = None) -> bool:
        """Set the promotion state only if the current one is in ``when`` / not in ``unless``, in one
        conditional update: of two concurrent promote (or unpromote) requests exactly one wins."""
        cur = {"$in": _enum_values(list(when))} if when is not None else {"$nin": _enum_values(list(unless or []))}
        res = await self.jobs_collection.update_one(
            {"job_id": job_id, "promoted": cur},
            {"$set": {"promoted": _enum_values(value), "destination_uri": destination_uri}})
        return res.matched_count > 0

    async def get_job(self, job_id: str) -> JobStatus | None:
        pipeline = [{"$match": {"job_id": job_id}}] + self._job_pipeline_add_fields() + [{"$unset": "_id"}]
        cur = await _maybe_await(self.jobs_collection.aggregate(pipeline))
        docs = await cur.to_list(length=1)
        return JobStatus(**docs[0]) if docs else None

    async def get_active_jobs(self) -> list[JobStatus]:
        """Jobs in a running state (queued / starting / restarting / running), any user."""
        states = [DatabaseStatusEnum.queued.value, DatabaseStatusEnum.starting.value,
                  DatabaseStatusEnum.restarting.value, DatabaseStatusEnum.running.value]
        out = []
        async for d in self.jobs_collection.find({"status": {"$in": states}}):
            d.pop("_id", None)
            out.append(JobStatus(**d))
        return out

    async def get_all_user_jobs(self, user_id: str) -> list[JobStatus]:
        out = []
        async for d in self.jobs_collection.find({"user_id": user_id}):
            d.pop("_id", None)
            out.append(JobStatus(**d))
        return out

    async def get_user_jobs(self, user_id, page=1, page_size=10, sort=None, query=None, limit=None, status=None,
                            model_name=None) -> JobsPage:
        page, page_size = max(1, int(page)), max(1, int(page_size))
        skip = (page - 1) * page_size
        q: dict[str, Any] = {"user_id": user_id}
        if status:
            if status == "promoted":  # a UI filter backed by the promotion flag
                q["promoted"] = PromotionStatus.COMPLETED.value
            else:
                q["status"] = status
        if model_name:
            q["model_name"] = model_name
        if query:
            q["job_name"] = {"$regex": re.escape(query), "$options": "i"}
        key, order = _sort_spec(sort or "-start_time")
        pipeline = [{"$match": q}] + self._job_pipeline_add_fields() + [
            {"$setWindowFields": {"sortBy": {key: order}, "output": {"index_": {"$documentNumber": {}}}}},
            {"$sort": {key: order}},
        ]
        if limit is not None:
            pipeline.append({"$match": {"index_": {"$in": list(limit)}}})
        pipeline += [{"$skip": skip}, {"$limit": page_size}]
        cur = await _maybe_await(self.jobs_collection.aggregate(pipeline))
        total = await self.jobs_collection.count_documents(q)
        items = []
        async for d in cur:
            d.pop("_id", None)
            items.append(JobStatus(**d))
        return JobsPage(items=items, total=total, total_pages=(total + page_size - 1) // page_size)

    def _job_pipeline_add_fields(self) -> list[dict]:
        """start_time / end_time / status_merged, then duration (milliseconds) -- UI table fields."""
        P = PromotionStatus
        start = {"$cond": {"if": {"$and": [{"$eq": ["$status", DatabaseStatusEnum.queued.value]},
                                           {"$eq": [{"$ifNull": ["$metadata.start_time", None]}, None]}]},
                           "then": "$created_at", "else": "$metadata.start_time"}}
        end = {"$cond": {"if": {"$eq": ["$status", "completed"]}, "then": "$metadata.completion_time",
                         "else": {"$cond": {"if": {"$eq": ["$status", "canceled"]},
                                            "then": "$metadata.cancellation_time", "else": None}}}}
        ended = {"$and": [{"$eq": ["$status", DatabaseStatusEnum.canceled.value]},
                          {"$ne": [{"$ifNull": ["$metadata.training_duration", "__MISSING__"]}, "__MISSING__"]}]}
        merged = {"$cond": {"if": {"$eq": ["$promoted", P.COMPLETED.value]}, "then": "deployed",
                            "else": {"$cond": {"if": {"$eq": ["$promoted", P.IN_PROGRESS.value]}, "then": "deploying",
                                               "else": {"$cond": {"if": {"$eq": ["$promoted", P.DELETING.value]},
                                                                  "then": "retracting",
                                                                  "else": {"$cond": {"if": ended, "then": "ended",
                                                                                     "else": "$status"}}}}}}}}
        duration = {"$cond": {"if": {"$and": ["$start_time", "$end_time"]},
                              "then": {"$subtract": ["$end_time", "$start_time"]},
                              "else": {"$cond": {"if": {"$and": ["$start_time", {"$eq": ["$status", "running"]}]},
                                                 "then": {"$subtract": [_utcnow(), "$start_time"]},
                                                 "else": None}}}}
        return [{"$addFields": {"start_time": start, "end_time": end, "status_merged": merged}},
                {"$addFields": {"duration": duration}}]

    async def delete_job(self, job_id: str) -> bool:
        doc = await self.get_job(job_id)
        if doc:
            try:
                await self.archived_jobs_collection.insert_one(_enum_values(doc.model_dump()))
            except Exception as e:  # already archived (re-submitted id): keep going
                if not isinstance(e, DuplicateKeyError) and "duplicate" not in str(e).lower():
                    raise
        res = await self.jobs_collection.delete_one({"job_id": job_id})
        return res.deleted_count > 0

    # ------------------------------------------------------------------ metrics
    async def create_job_metrics(self, user_id, job_id, job_name, data) -> MetricsDocument:
        doc = {"user_id": user_id, "job_id": job_id, "job_name": job_name, "metrics": data}
        await self.metrics_collection.insert_one(dict(doc))
        return MetricsDocument(**doc)

    async def job_metrics_update(self, user_id, job_id, data) -> bool:
        res = await self.metrics_collection.update_one({"job_id": job_id, "user_id": user_id},
                                                       {"$set": {"metrics": data}})
        return res.matched_count > 0

    async def upsert_job_metrics(self, user_id, job_id, job_name, data) -> None:
        await self.metrics_collection.update_one(
            {"job_id": job_id}, {"$set": {"user_id": user_id, "job_name": job_name, "metrics": data}}, upsert=True)

    async def get_job_metrics(self, job_id: str) -> MetricsDocument | None:
        d = await self.metrics_collection.find_one({"job_id": job_id})
        return MetricsDocument(**d) if d else None

    async def delete_metrics(self, job_id: str) -> bool:
        return (await self.metrics_collection.delete_one({"job_id": job_id})).deleted_count > 0

    # ------------------------------------------------------------------ datasets
    async def insert_dataset(self, user_id, job_id, dataset: DatasetTypes, dataset_name, description) -> DatasetModel:
        doc = {"user_id": user_id, "dataset": dataset.model_dump(), "dataset_name": dataset_name,
               "job_ref": [job_id], "description": description, "created_at": _utcnow()}
        r = await self.datasets_collection.insert_one(doc)
        doc["_id"] = r.inserted_id
        return DatasetModel(**doc)

    async def get_user_datasets_all(self, user_id: str) -> list[DatasetModel]:
        docs = await self.datasets_collection.find({"user_id": user_id}).to_list(length=None)
        return [DatasetModel(**d) for d in docs]

    async def get_user_dataset(self, user_id: str, dataset_id: str) -> DatasetModel | None:
        try:
            d = await self.datasets_collection.find_one({"_id": ObjectId(dataset_id), "user_id": user_id})
        except Exception as e:
            logger.error("get_user_dataset: %s", e)
            return None
        return DatasetModel(**d) if d else None

    async def get_user_datasets_page(self, user_id, page=1, page_size=10, sort=None, query=None,
                                     limit=None) -> DatasetPage:
        page, page_size = max(1, int(page)), max(1, int(page_size))
        q: dict[str, Any] = {"user_id": user_id}
        if query:
            q["dataset_name"] = {"$regex": re.escape(query), "$options": "i"}
        key, order = _sort_spec(sort or "-created_at")
        if key == "start_time":  # the reference's default key does not exist on datasets
            key = "created_at"
        pipeline = [{"$match": q},
                    {"$setWindowFields": {"sortBy": {key: order}, "output": {"index_": {"$documentNumber": {}}}}},
                    {"$sort": {key: order}},
                    {"$lookup": {"from": "jobs", "localField": "job_ref", "foreignField": "job_id",
                                 "as": "job_ref_details"}},
                    {"$addFields": {"job_ref_names": {"$map": {"input": "$job_ref_details", "as": "job",
                                                               "in": "$$job.job_name"}}}},
                    {"$unset": "job_ref_details"}]
        if limit is not None:
            pipeline.append({"$match": {"index_": {"$in": list(limit)}}})
        pipeline += [{"$skip": (page - 1) * page_size}, {"$limit": page_size}]
        cur = await _maybe_await(self.datasets_collection.aggregate(pipeline))
        total = await self.datasets_collection.count_documents(q)
        items = [DatasetModel(**d) async for d in cur]
        return DatasetPage(items=items, total=total, total_pages=(total + page_size - 1) // page_size)

    async def update_dataset(self, user_id: str, dataset_id: str, job_id: str) -> DatasetModel | None:
        try:
            flt = {"user_id": user_id, "_id": ObjectId(dataset_id)}
        except Exception:
            return None
        res = await self.datasets_collection.update_one(flt, {"$addToSet": {"job_ref": job_id}})
        if res.matched_count == 0:
            return None
        d = await self.datasets_collection.find_one(flt)
        return DatasetModel(**d) if d else None

    async def delete_dataset(self, user_id: str, dataset_id: str) -> bool:
        try:
            flt = {"_id": ObjectId(dataset_id), "user_id": user_id}
        except Exception:
            return False
        return (await self.datasets_collection.delete_one(flt)).deleted_count > 0

    # ------------------------------------------------------------------ leader lease
    async def acquire_lock(self, name: str, owner: str, ttl_s: float) -> bool:
        now = _utcnow()
        exp = now + _dt.timedelta(seconds=ttl_s)
        try:
            await self.locks_collection.insert_one({"_id": name, "owner": owner, "expires_at": exp})
            return True
        except Exception as e:
            if not isinstance(e, DuplicateKeyError) and "duplicate" not in str(e).lower():
                raise
        res = await self.locks_collection.update_one(
            {"_id": name, "$or": [{"owner": owner}, {"expires_at": {"$lt": now}}]},
            {"$set": {"owner": owner, "expires_at": exp}})
        return res.matched_count > 0

    async def release_lock(self, name: str, owner: str) -> None:
        await self.locks_collection.delete_one({"_id": name, "owner": owner})


def _sort_spec(sort: str) -> tuple[str, int]:
    if sort.startswith("-"):
        return sort[1:], -1
    return sort, 1
