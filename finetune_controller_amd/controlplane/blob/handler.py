"""S3Handler (C10): the job-oriented object-storage operations of the control plane.

Path scheme and semantics follow ``/root/reference/app/utils/S3Handler.py``:
``finetune_jobs/{user}/{job}/{dataset,artifacts}``; metrics = newest object whose key contains
``metrics`` and ends ``.csv``, parsed to records with NaN -> 0; presigned URLs and the artifact zip use
``basename(key)``; promotion copies a single object or a whole prefix.  Improvements: prefix copy and
presigned listing are paginated (the reference stops at 1000 keys), the metrics CSV is parsed with the
stdlib (no pandas needed), and the zip is built in a worker thread.
"""
from __future__ import annotations

import asyncio
import csv
import io
import math
import os
import shutil
import tempfile
import zipfile

from .store import ObjectStore, split_s3_uri

BASE_PATH = "finetune_jobs"


def parse_metrics_csv(content: bytes) -> list[dict]:
    rows = []
    for r in csv.DictReader(io.StringIO(content.decode("utf-8"))):
        rec = {}
        for k, v in r.items():
            if k is None:
                continue
            if v is None or v == "":
                rec[k] = 0
                continue
            try:
                x = float(v)
                rec[k] = 0 if math.isnan(x) else (int(x) if x.is_integer() and "." not in v and "e" not in v.lower() else x)
            except ValueError:
                rec[k] = v
        rows.append(rec)
    return rows


class S3Handler:
    def __init__(self, store: ObjectStore, bucket: str):
        self.store = store
        self.bucket = bucket
        self.base_path = BASE_PATH

    # ---- URIs ----
    def get_base_uri_path(self, user_id: str, job_id: str) -> str:
        return f"{self.base_path}/{user_id}/{job_id}"

    def get_dataset_uri_string(self, bucket, user_id, job_id, path_only=False) -> str:
        p = f"{self.get_base_uri_path(user_id, job_id)}/dataset"
        return p if path_only else f"s3://{bucket}/{p}"

    def get_artifacts_uri_string(self, bucket, user_id, job_id, path_only=False) -> str:
        p = f"{self.get_base_uri_path(user_id, job_id)}/artifacts"
        return p if path_only else f"s3://{bucket}/{p}"

    # ---- datasets ----
    async def upload_dataset(self, file_path: str, user_id: str, job_id: str, name: str | None = None) -> str:
        fname = os.path.basename(name or file_path)
        key = f"{self.get_dataset_uri_string(self.bucket, user_id, job_id, True)}/{fname}"
        await asyncio.to_thread(self.store.put_file, self.bucket, key, file_path)
        return f"s3://{self.bucket}/{key}"

    async def upload_dataset_bytes(self, data: bytes, dataset_name: str, user_id: str, job_id: str) -> str:
        key = f"{self.get_dataset_uri_string(self.bucket, user_id, job_id, True)}/{os.path.basename(dataset_name)}"
        await asyncio.to_thread(self.store.put_bytes, self.bucket, key, data)
        return f"s3://{self.bucket}/{key}"

    async def stream_dataset_bytes(self, chunks, dataset_name: str, user_id: str, job_id: str) -> str:
        """``chunks``: a sync iterator of bytes (consumed in a worker thread, never fully in memory)."""
        key = f"{self.get_dataset_uri_string(self.bucket, user_id, job_id, True)}/{os.path.basename(dataset_name)}"
        await asyncio.to_thread(self.store.put_stream, self.bucket, key, chunks)
        return f"s3://{self.bucket}/{key}"

    async def validate_s3_uri(self, s3_uri: str) -> bool:
        try:
            b, k = split_s3_uri(s3_uri)
        except ValueError:
            return False
        return await asyncio.to_thread(self.store.head, b, k) is not None

    # ---- artifacts ----
    async def _list_artifacts(self, user_id, job_id):
        prefix = self.get_artifacts_uri_string(self.bucket, user_id, job_id, True)
        return await asyncio.to_thread(self.store.list, self.bucket, prefix)

    async def get_presigned_urls(self, user_id: str, job_id: str, expiration: int = 3600) -> list[dict]:
        urls = []
        for o in await self._list_artifacts(user_id, job_id):
            if o.Key.endswith("/"):
                continue
            urls.append({"key": os.path.basename(o.Key), "url": self.store.presign(self.bucket, o.Key, expiration)})
        return urls

    async def cleanup_uri_items(self, s3_uri: str) -> int:
        """Delete the object ``s3_uri`` names, or everything under it as a directory.  A plain key-prefix
        delete (the reference's) would also take sibling keys that merely start with the same text --
        ``.../job-1`` sweeping ``.../job-1-retry/...``, ``data.csv`` taking ``data.csv.bak``."""
        bucket, prefix = split_s3_uri(s3_uri)
        objs = await asyncio.to_thread(self.store.list, bucket, prefix)
        root = prefix.rstrip("/")
        keys = [o.Key for o in objs if o.Key == prefix or o.Key == root or o.Key.startswith(root + "/")]
        if keys:
            await asyncio.to_thread(self.store.delete, bucket, keys)
        return len(keys)

    async def cleanup_job_data(self, user_id: str, job_id: str) -> int:
        return await self.cleanup_uri_items(f"s3://{self.bucket}/{self.get_base_uri_path(user_id, job_id)}")

    async def get_metrics(self, user_id: str, job_id: str) -> list[dict]:
        objs = await self._list_artifacts(user_id, job_id)
        if not objs:
            raise FileNotFoundError(f"No data found for job {job_id}")
        files = [o for o in objs if "metrics" in o.Key and o.Key.endswith(".csv")]
        if not files:
            raise FileNotFoundError(f"No metrics file found for job {job_id}")
        newest = sorted(files, key=lambda o: o.LastModified, reverse=True)[0]
        content = await asyncio.to_thread(self.store.get_bytes, self.bucket, newest.Key)
        try:
            return parse_metrics_csv(content)
        except Exception as e:
            raise ValueError("Could not read file content. corrupted?") from e

    async def download_artifacts(self, user_id: str, job_id: str) -> tuple[str, str]:
        objs = await self._list_artifacts(user_id, job_id)
        if not objs:
            raise FileNotFoundError(f"No artifacts found for job {job_id}")
        temp_dir = tempfile.mkdtemp(prefix="ftc-artifacts-")
        try:
            art = os.path.join(temp_dir, "artifacts")
            os.makedirs(art)

            def fetch(o):
                name = os.path.basename(o.Key)
                if name:
                    self.store.get_file(self.bucket, o.Key, os.path.join(art, name))

            await asyncio.gather(*(asyncio.to_thread(fetch, o) for o in objs))
            zip_path = os.path.join(temp_dir, f"artifacts_{job_id}.zip")

            def make_zip():
                with zipfile.ZipFile(zip_path, "w", zipfile.ZIP_DEFLATED) as z:
                    for fn in sorted(os.listdir(art)):
                        z.write(os.path.join(art, fn), arcname=fn)

            await asyncio.to_thread(make_zip)
            return zip_path, temp_dir
        except Exception:
            shutil.rmtree(temp_dir, ignore_errors=True)
            raise

    async def copy_s3_object(self, source_s3_uri: str, destination_s3_uri: str) -> int:
        sb, sk = split_s3_uri(source_s3_uri)
        db, dk = split_s3_uri(destination_s3_uri)
        if not sk or not dk:
            raise ValueError("Invalid S3 URI format")
        if await asyncio.to_thread(self.store.head, sb, sk) is not None:
            await asyncio.to_thread(self.store.copy, sb, sk, db, dk)
            return 1
        objs = await asyncio.to_thread(self.store.list, sb, sk)
        if not objs:
            raise FileNotFoundError(f"No objects found at {source_s3_uri}")
        src_root, dst_root = sk.rstrip("/"), dk.rstrip("/")
        await asyncio.gather(*(asyncio.to_thread(self.store.copy, sb, o.Key, db, o.Key.replace(src_root, dst_root, 1))
                               for o in objs))
        return len(objs)
