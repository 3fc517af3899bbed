"""S3Handler (controlplane/blob/handler.py) over the local object store: deletion scope and key
containment."""
import asyncio

import pytest

from finetune_controller_amd.controlplane.blob.handler import S3Handler
from finetune_controller_amd.controlplane.blob.store import LocalObjectStore


def test_cleanup_deletes_the_object_or_its_directory_not_siblings_by_prefix(tmp_path):
    st = LocalObjectStore(str(tmp_path))
    h = S3Handler(st, "ftc")
    keys = ["promo/llama/job-1/adapter.safetensors", "promo/llama/job-1/cfg/a.json",
            "promo/llama/job-1-retry/adapter.safetensors",  # another job whose id starts with "job-1"
            "finetune_jobs/u/j/dataset/data.csv", "finetune_jobs/u/j/dataset/data.csv.bak"]
    for k in keys:
        st.put_bytes("ftc", k, b"x")
    assert asyncio.run(h.cleanup_uri_items("s3://ftc/promo/llama/job-1")) == 2
    assert asyncio.run(h.cleanup_uri_items("s3://ftc/finetune_jobs/u/j/dataset/data.csv")) == 1
    left = [o.Key for o in st.list("ftc", "")]
    assert left == ["finetune_jobs/u/j/dataset/data.csv.bak", "promo/llama/job-1-retry/adapter.safetensors"]
    # a trailing slash means the directory too
    assert asyncio.run(h.cleanup_uri_items("s3://ftc/promo/llama/job-1-retry/")) == 1


def test_local_store_keys_cannot_reach_a_sibling_bucket(tmp_path):
    st = LocalObjectStore(str(tmp_path))
    st.put_bytes("ftc-other", "secret.txt", b"s")
    with pytest.raises(ValueError, match="escapes"):
        st.get_bytes("ftc", "../ftc-other/secret.txt")
    with pytest.raises(ValueError, match="escapes"):
        st.put_bytes("ftc", "../../outside.txt", b"x")
    st.put_bytes("ftc", "a/../b.txt", b"ok")  # normalised, still inside the bucket
    assert st.get_bytes("ftc", "b.txt") == b"ok"
