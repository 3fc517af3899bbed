"""The JobStore's production path: pymongo's ``AsyncMongoClient`` over the MongoDB wire protocol
(store/jobstore.py ``connect``), against tests/mongo_wire.py -- a wire endpoint whose storage is the
in-memory engine.  The same job / dataset / metrics / lease scenario runs on the in-memory backend
and over the wire, and the two transcripts must be identical: BSON round trips (tz-aware datetimes,
ObjectIds, str enums), command shapes (insert / update with $set paths and $addToSet / aggregate
with $lookup and $setWindowFields / count_documents / find / delete), unique-index violations
surfacing as pymongo's DuplicateKeyError, and the lease's upsert path.

What this cannot pin is the server's own semantics -- the wire endpoint executes the same engine
the memory backend uses (no mongod in this image; parity with a real server stays unpinned).
"""
import asyncio
import datetime as dt

import pytest

pytest.importorskip("pymongo")

from mongo_wire import MongoWireServer  # noqa: E402

from finetune_controller_amd.controlplane.schemas.db import DatasetTypes, PromotionStatus  # noqa: E402
from finetune_controller_amd.controlplane.store.jobstore import JobStore  # noqa: E402


def _norm(x):
    """Transcript values comparable across backends (ObjectIds differ; times are checked separately)."""
    if isinstance(x, dict):
        return {k: _norm(v) for k, v in sorted(x.items()) if k not in ("_id", "id", "created_at", "updated_at")}
    if isinstance(x, (list, tuple)):
        return [_norm(v) for v in x]
    if isinstance(x, dt.datetime):
        assert x.tzinfo is not None, "naive datetime came back"
        return "<datetime>"
    if hasattr(x, "model_dump"):
        return _norm(x.model_dump())
    if hasattr(x, "value") and isinstance(x.value, str):
        return x.value
    if type(x).__name__ == "ObjectId":
        return "<oid>"
    return x


async def _scenario(store: JobStore) -> list:
    t = []
    await store.connect()
    for i, (jid, user) in enumerate([("llama-a", "alice"), ("llama-b", "alice"), ("mnist-c", "bob")]):
        await store.create_job(user, jid, f"job {i}", "Llama3-8B-LoRA" if "llama" in jid else "MNIST", "mi355x",
                               "causal_lm", "pytorch", arguments={"lr": 1e-4, "steps": i},
                               atrifacts_uri=f"s3://b/{jid}")
    t.append(("dup", await _raises_duplicate(store)))
    now = dt.datetime.now(dt.timezone.utc)
    await store.update_job_status("llama-a", "running", {"start_time": now - dt.timedelta(seconds=90),
                                                         "queue_pos": None})
    await store.update_job_status("llama-a", "completed", {"completion_time": now, "message": "done"})
    await store.update_job_status("llama-b", "queued", {"queue_pos": 2})
    await store.update_job_promotion("llama-a", PromotionStatus.COMPLETED, "s3://deploy/x/llama-a")
    j = await store.get_job("llama-a")
    t.append(("job", j))
    t.append(("duration_s", round(j.model_extra.get("duration", 0) / 1000) if j.model_extra.get("duration") else None))
    t.append(("all", await store.get_all_user_jobs("alice")))
    page = await store.get_user_jobs("alice", page=1, page_size=1, sort="-created_at")
    t.append(("page", page.total, page.total_pages, [x.job_id for x in page.items]))
    page = await store.get_user_jobs("alice", page=1, page_size=10, status="completed")
    t.append(("filtered", [x.job_id for x in page.items]))
    await store.upsert_job_metrics("alice", "llama-a", "job 0", [{"step": 1, "loss": 2.5}])
    await store.upsert_job_metrics("alice", "llama-a", "job 0", [{"step": 1, "loss": 2.5}, {"step": 2, "loss": 2.0}])
    t.append(("metrics", await store.get_job_metrics("llama-a")))
    d = await store.insert_dataset("alice", "llama-a", DatasetTypes(s3_uri="s3://b/d.csv"), "d.csv", "desc")
    await store.update_dataset("alice", str(d.id), "llama-b")
    await store.update_dataset("alice", str(d.id), "llama-b")  # $addToSet: no duplicate ref
    t.append(("dataset", await store.get_user_dataset("alice", str(d.id))))
    dp = await store.get_user_datasets_page("alice", page=1, page_size=5)
    t.append(("datasets_page", dp.total, [x.model_extra.get("job_ref_names") for x in dp.items]))
    t.append(("lease", await store.acquire_lock("monitor", "pod-1", 30), await store.acquire_lock("monitor", "pod-2", 30)))
    await store.release_lock("monitor", "pod-1")
    t.append(("lease2", await store.acquire_lock("monitor", "pod-2", 30)))
    t.append(("delete", await store.delete_metrics("llama-a"), await store.delete_job("llama-a"),
              await store.get_job("llama-a") is None, await store.delete_dataset("alice", str(d.id))))
    t.append(("archived", await store.archived_jobs_collection.find_one({"job_id": "llama-a"}) is not None))
    await store.close()
    return _norm(t)


async def _raises_duplicate(store) -> bool:
    try:
        await store.create_job("alice", "llama-a", "again", "M", "cpu", "causal_lm", "pytorch")
    except Exception as e:  # memory: store.memory.DuplicateKeyError; wire: pymongo.errors.DuplicateKeyError
        return "duplicate" in type(e).__name__.lower() or "E11000" in str(e)
    return False


def test_pymongo_wire_path_matches_memory_backend():
    srv = MongoWireServer()
    try:
        wire = asyncio.run(_scenario(JobStore(url=srv.url, database="ftc")))
        mem = asyncio.run(_scenario(JobStore.memory("ftc")))
        assert wire == mem
        tr = {row[0]: row[1:] for row in wire}
        assert tr["dup"] == [True] and tr["lease"] == [True, False] and tr["lease2"] == [True]
        seen = set(srv.commands)
        assert {"insert", "update", "aggregate", "find", "delete", "createIndexes"} <= seen, seen
    finally:
        srv.close()
