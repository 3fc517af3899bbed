"""Job store on the in-memory Mongo engine: aggregation-derived fields, pagination, datasets $lookup,
atomic metadata merge, archive-on-delete, leader lease (SURVEY.md §7.4 "in-memory Mongo must reproduce
the aggregation-derived fields")."""
import asyncio
import datetime as dt

import pytest

from finetune_controller_amd.controlplane.schemas.db import DatasetTypes, PromotionStatus
from finetune_controller_amd.controlplane.store.jobstore import JobStore
from finetune_controller_amd.controlplane.store.memory import MemoryDatabase, evaluate, match


def run(coro):
    return asyncio.run(coro)


@pytest.fixture
def store():
    s = JobStore.memory()
    run(s.connect())
    return s


async def _mk(store, jid, user="u1", name=None, **kw):
    return await store.create_job(user, jid, name or jid, "M", "cpu", "causal_lm", "pytorch", **kw)


def test_matcher_and_expressions():
    d = {"a": {"b": 3}, "s": "Hello", "l": ["x", "y"], "t": dt.datetime(2024, 1, 1, tzinfo=dt.timezone.utc)}
    assert match(d, {"a.b": 3, "s": {"$regex": "^hel", "$options": "i"}, "l": "y"})
    assert not match(d, {"a.b": {"$in": [1, 2]}})
    assert match(d, {"$or": [{"a.b": 1}, {"s": "Hello"}], "missing": {"$exists": False}})
    assert match(d, {"t": {"$lt": dt.datetime(2025, 1, 1, tzinfo=dt.timezone.utc)}})
    e = {"$cond": {"if": {"$and": ["$a.b", {"$eq": ["$s", "Hello"]}]}, "then": {"$subtract": [
        dt.datetime(2024, 1, 1, 0, 0, 2, tzinfo=dt.timezone.utc), "$t"]}, "else": None}}
    assert evaluate(e, d) == 2000  # milliseconds, like MongoDB
    assert evaluate({"$ifNull": ["$nope", "dflt"]}, d) == "dflt"
    assert evaluate({"$map": {"input": "$l", "as": "v", "in": "$$v"}}, d) == ["x", "y"]


def test_unique_index_and_updates():
    db = MemoryDatabase()
    c = db["c"]
    run(c.create_index("k", unique=True))
    run(c.insert_one({"k": 1, "m": {"a": 1}}))
    with pytest.raises(Exception):
        run(c.insert_one({"k": 1}))
    r = run(c.update_one({"k": 1}, {"$set": {"m.b": 2}, "$addToSet": {"refs": "j1"}}))
    assert r.modified_count == 1
    run(c.update_one({"k": 1}, {"$addToSet": {"refs": "j1"}}))
    d = run(c.find_one({"k": 1}))
    assert d["m"] == {"a": 1, "b": 2} and d["refs"] == ["j1"]


def test_job_pipeline_fields(store):
    async def go():
        await _mk(store, "j-queued")
        await _mk(store, "j-run")
        t0 = dt.datetime.now(dt.timezone.utc) - dt.timedelta(seconds=30)
        await store.update_job_status("j-run", "running", {"start_time": t0})
        await _mk(store, "j-done")
        await store.update_job_status("j-done", "completed", {"start_time": t0,
                                                             "completion_time": t0 + dt.timedelta(seconds=10)})
        await _mk(store, "j-canc")
        await store.update_job_status("j-canc", "canceled", {"start_time": t0, "training_duration": 5.0,
                                                             "cancellation_time": t0 + dt.timedelta(seconds=3)})
        await _mk(store, "j-prom")
        await store.update_job_status("j-prom", "completed", {})
        await store.update_job_promotion("j-prom", PromotionStatus.COMPLETED, "s3://d/x")
        q = await store.get_job("j-queued")
        assert q.model_extra["start_time"] == q.created_at and q.model_extra["end_time"] is None
        assert q.model_extra["status_merged"] == "queued" and q.model_extra["duration"] is None
        r = await store.get_job("j-run")
        assert 29_000 <= r.model_extra["duration"] <= 40_000 and r.model_extra["end_time"] is None
        d = await store.get_job("j-done")
        assert d.model_extra["duration"] == 10_000
        c = await store.get_job("j-canc")
        assert c.model_extra["status_merged"] == "ended" and c.model_extra["duration"] == 3000
        p = await store.get_job("j-prom")
        assert p.model_extra["status_merged"] == "deployed"
        assert await store.get_job("nope") is None

    run(go())


def test_metadata_merge_is_atomic_per_field(store):
    async def go():
        await _mk(store, "j1", metadata={"kubernetes_job_name": "j1"})
        await store.update_job_status("j1", "running", {"queue_pos": 3})
        await store.update_job_status("j1", "running", {"message": "hi"})
        j = await store.get_job("j1")
        md = j.metadata.model_dump()
        assert md["kubernetes_job_name"] == "j1" and md["queue_pos"] == 3 and md["message"] == "hi"

    run(go())


def test_user_jobs_pagination_sort_filter(store):
    async def go():
        for i in range(7):
            await _mk(store, f"job-{i}", name=f"run {i}")
        await _mk(store, "other", user="u2")
        await store.update_job_status("job-3", "failed", {})
        page = await store.get_user_jobs("u1", page=1, page_size=3, sort="job_name")
        assert page.total == 7 and page.total_pages == 3
        assert [j.job_id for j in page.items] == ["job-0", "job-1", "job-2"]
        assert [j.model_extra["index_"] for j in page.items] == [1, 2, 3]
        p2 = await store.get_user_jobs("u1", page=3, page_size=3, sort="-job_name")
        assert [j.job_id for j in p2.items] == ["job-0"]
        f = await store.get_user_jobs("u1", status="failed")
        assert [j.job_id for j in f.items] == ["job-3"]
        s = await store.get_user_jobs("u1", query="RUN 5")
        assert [j.job_id for j in s.items] == ["job-5"]
        lim = await store.get_user_jobs("u1", sort="job_name", limit=[2, 4], page_size=10)
        assert [j.job_id for j in lim.items] == ["job-1", "job-3"]
        # the search text is literal: regex metacharacters neither fail the query nor act as a pattern
        await _mk(store, "job-x", name="run (v2) [final]")
        s = await store.get_user_jobs("u1", query="(V2) [")
        assert [j.job_id for j in s.items] == ["job-x"]
        assert (await store.get_user_jobs("u1", query="run .")).total == 0
        assert (await store.get_user_jobs("u1", query="(a+)+$")).total == 0

    run(go())


def test_datasets_lookup_and_total(store):
    async def go():
        await _mk(store, "ja", name="Alpha")
        d = await store.insert_dataset("u1", "ja", DatasetTypes(s3_uri="s3://b/k"), "data.csv", "desc")
        await _mk(store, "jb", name="Beta")
        d2 = await store.update_dataset("u1", d.id, "jb")
        assert d2.job_ref == ["ja", "jb"]
        await store.update_dataset("u1", d.id, "jb")
        for i in range(3):
            await store.insert_dataset("u1", f"x{i}", DatasetTypes(), f"d{i}", "")
        page = await store.get_user_datasets_page("u1", page=1, page_size=2, sort="created_at")
        assert page.total == 4 and page.total_pages == 2
        first = page.items[0]
        assert first.dataset_name == "data.csv" and first.model_extra["job_ref_names"] == ["Alpha", "Beta"]
        assert await store.get_user_dataset("u2", d.id) is None
        assert await store.get_user_dataset("u1", "not-an-oid") is None
        assert await store.delete_dataset("u1", d.id)
        assert len(await store.get_user_datasets_all("u1")) == 3

    run(go())


def test_metrics_and_archive(store):
    async def go():
        await _mk(store, "j1")
        await store.upsert_job_metrics("u1", "j1", "j1", [{"step": 1}])
        await store.upsert_job_metrics("u1", "j1", "j1", [{"step": 1}, {"step": 2}])
        m = await store.get_job_metrics("j1")
        assert len(m.metrics) == 2
        assert await store.delete_metrics("j1")
        assert await store.delete_job("j1")
        assert await store.get_job("j1") is None
        archived = await store.archived_jobs_collection.find_one({"job_id": "j1"})
        assert archived is not None

    run(go())


def test_leader_lease(store):
    async def go():
        assert await store.acquire_lock("mon", "a", 10)
        assert not await store.acquire_lock("mon", "b", 10)
        assert await store.acquire_lock("mon", "a", 10)  # renewal
        await store.locks_collection.update_one({"_id": "mon"}, {"$set": {
            "expires_at": dt.datetime.now(dt.timezone.utc) - dt.timedelta(seconds=1)}})
        assert await store.acquire_lock("mon", "b", 10)  # expired lease taken over
        await store.release_lock("mon", "b")
        assert await store.acquire_lock("mon", "c", 10)

    run(go())
