"""Object storage behind one protocol (C10 transport layer).

The reference binds S3 through aioboto3 (``/root/reference/app/utils/S3Handler.py:22-44``).  Neither
boto nor aioboto3 is required here:

* ``S3ObjectStore`` -- S3 REST with AWS Signature V4 written against ``httpx`` (ListObjectsV2 with
  continuation, Get/Put/Head/Copy/DeleteObjects, multipart upload for large files, presigned GETs);
  works with AWS, MinIO, Ceph RGW (``S3_ENDPOINT_URL``);
* ``LocalObjectStore`` -- ``s3://bucket/key`` mapped onto ``<root>/bucket/key`` (tests, single-node
  deployments, the FakeCluster's dataset init container and sync sidecar).

All methods are synchronous and thread-safe; the async ``S3Handler`` runs them in worker threads.
"""
from __future__ import annotations

import datetime as _dt
import hashlib
import hmac
import logging
import os
import shutil
import threading
import urllib.parse
import xml.etree.ElementTree as ET
from dataclasses import dataclass

import httpx


def split_s3_uri(uri: str) -> tuple[str, str]:
    if not uri.startswith("s3://"):
        raise ValueError(f"not an s3 uri: {uri!r}")
    rest = uri[5:]
    bucket, _, key = rest.partition("/")
    return bucket, key


@dataclass
class ObjectInfo:
    Key: str
    Size: int
    LastModified: _dt.datetime

    def as_dict(self):
        return {"Key": self.Key, "Size": self.Size, "LastModified": self.LastModified}


class ObjectNotFound(Exception):
    pass


class ObjectStore:
    def put_bytes(self, bucket: str, key: str, data: bytes) -> None: raise NotImplementedError
    def put_file(self, bucket: str, key: str, path: str) -> None: raise NotImplementedError
    def put_stream(self, bucket: str, key: str, chunks) -> None: raise NotImplementedError
    def get_bytes(self, bucket: str, key: str) -> bytes: raise NotImplementedError
    def get_file(self, bucket: str, key: str, path: str) -> None: raise NotImplementedError
    def head(self, bucket: str, key: str) -> ObjectInfo | None: raise NotImplementedError
    def list(self, bucket: str, prefix: str) -> list[ObjectInfo]: raise NotImplementedError
    def delete(self, bucket: str, keys: list[str]) -> None: raise NotImplementedError
    def copy(self, src_bucket: str, src_key: str, dst_bucket: str, dst_key: str) -> None: raise NotImplementedError
    def presign(self, bucket: str, key: str, expires: int = 3600) -> str: raise NotImplementedError


# ---------------------------------------------------------------- local directory store
class LocalObjectStore(ObjectStore):
    def __init__(self, root: str, url_base: str | None = None):
        self.root = os.path.abspath(root)
        os.makedirs(self.root, exist_ok=True)
        self.url_base = url_base  # e.g. "http://host:8000/files" when served; default file://
        self._lock = threading.Lock()

    def _p(self, bucket, key):
        base = os.path.abspath(os.path.join(self.root, bucket))
        p = os.path.abspath(os.path.join(base, key))
        # (a bare startswith(base) would let "../<bucket>-other/..." into a sibling bucket)
        if not (p == base or p.startswith(base + os.sep)) or not base.startswith(self.root + os.sep):
            raise ValueError("key escapes bucket")
        return p

    def put_bytes(self, bucket, key, data):
        p = self._p(bucket, key)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        tmp = p + ".part"
        with open(tmp, "wb") as f:
            f.write(data)
        os.replace(tmp, p)

    def put_file(self, bucket, key, path):
        p = self._p(bucket, key)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        shutil.copyfile(path, p + ".part")
        os.replace(p + ".part", p)

    def put_stream(self, bucket, key, chunks):
        p = self._p(bucket, key)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p + ".part", "wb") as f:
            for c in chunks:
                f.write(c)
        os.replace(p + ".part", p)

    def get_bytes(self, bucket, key):
        p = self._p(bucket, key)
        if not os.path.isfile(p):
            raise ObjectNotFound(f"s3://{bucket}/{key}")
        with open(p, "rb") as f:
            return f.read()

    def get_file(self, bucket, key, path):
        p = self._p(bucket, key)
        if not os.path.isfile(p):
            raise ObjectNotFound(f"s3://{bucket}/{key}")
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        shutil.copyfile(p, path)

    def head(self, bucket, key):
        p = self._p(bucket, key)
        if not os.path.isfile(p):
            return None
        st = os.stat(p)
        return ObjectInfo(key, st.st_size, _dt.datetime.fromtimestamp(st.st_mtime, _dt.timezone.utc))

    def list(self, bucket, prefix):
        base = os.path.join(self.root, bucket)
        out = []
        if not os.path.isdir(base):
            return out
        for dp, _, files in os.walk(base):
            for fn in files:
                if fn.endswith(".part"):
                    continue
                full = os.path.join(dp, fn)
                key = os.path.relpath(full, base).replace(os.sep, "/")
                if key.startswith(prefix):
                    st = os.stat(full)
                    out.append(ObjectInfo(key, st.st_size, _dt.datetime.fromtimestamp(st.st_mtime, _dt.timezone.utc)))
        return sorted(out, key=lambda o: o.Key)

    def delete(self, bucket, keys):
        for k in keys:
            p = self._p(bucket, k)
            if os.path.isfile(p):
                os.remove(p)

    def copy(self, src_bucket, src_key, dst_bucket, dst_key):
        self.put_file(dst_bucket, dst_key, self._p(src_bucket, src_key))

    def presign(self, bucket, key, expires=3600):
        if self.url_base:
            return f"{self.url_base.rstrip('/')}/{bucket}/{urllib.parse.quote(key)}"
        return "file://" + self._p(bucket, key)


# ---------------------------------------------------------------- S3 (SigV4) store
def _sha256(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def _sign(key: bytes, msg: str) -> bytes:
    return hmac.new(key, msg.encode(), hashlib.sha256).digest()


def _uri_encode(s: str, keep_slash: bool) -> str:
    return urllib.parse.quote(s, safe="/-_.~" if keep_slash else "-_.~")


def _canonical_query(query: dict) -> str:
    return "&".join(f"{_uri_encode(str(k), False)}={_uri_encode(str(v), False)}"
                    for k, v in sorted((str(k), str(v)) for k, v in query.items()))


def sigv4_signature(secret_key: str, region: str, amz_date: str, method: str, path: str, query: dict,
                    headers: dict, payload_hash: str, service: str = "s3") -> tuple[str, str]:
    """AWS Signature Version 4 over one request: returns (signed_headers, hex signature).

    ``headers`` are the headers to sign (names lower-cased here, values trimmed); ``path`` is the
    un-encoded absolute path; ``amz_date`` is ``YYYYMMDDTHHMMSSZ``.  Pure function of its inputs, so
    AWS's published examples are known answers for it (tests/test_adapters_transport.py)."""
    h = {k.lower(): " ".join(str(v).strip().split()) for k, v in headers.items()}
    signed = ";".join(sorted(h))
    canon_h = "".join(f"{k}:{h[k]}\n" for k in sorted(h))
    creq = "\n".join([method, _uri_encode(path, True), _canonical_query(query), canon_h, signed, payload_hash])
    date = amz_date[:8]
    scope = f"{date}/{region}/{service}/aws4_request"
    sts = "\n".join(["AWS4-HMAC-SHA256", amz_date, scope, _sha256(creq.encode())])
    k = _sign(_sign(_sign(_sign(("AWS4" + secret_key).encode(), date), region), service), "aws4_request")
    return signed, hmac.new(k, sts.encode(), hashlib.sha256).hexdigest()


def sigv4_presign_query(access_key: str, secret_key: str, region: str, amz_date: str, host: str, path: str,
                        expires: int, session_token: str | None = None, method: str = "GET") -> dict:
    """Query-string authentication (presigned URL): the X-Amz-* parameters including the signature."""
    scope = f"{amz_date[:8]}/{region}/s3/aws4_request"
    q = {"X-Amz-Algorithm": "AWS4-HMAC-SHA256", "X-Amz-Credential": f"{access_key}/{scope}", "X-Amz-Date": amz_date,
         "X-Amz-Expires": str(int(expires)), "X-Amz-SignedHeaders": "host"}
    if session_token:
        q["X-Amz-Security-Token"] = session_token
    _, sig = sigv4_signature(secret_key, region, amz_date, method, path, q, {"host": host}, "UNSIGNED-PAYLOAD")
    q["X-Amz-Signature"] = sig
    return q


class S3ObjectStore(ObjectStore):
    """Minimal S3 client: AWS Signature Version 4; path-style (``/{bucket}/{key}`` on the endpoint,
    the default: works with MinIO / Ceph / any custom ``S3_ENDPOINT_URL``) or virtual-hosted
    (``{bucket}.{endpoint host}/{key}``, what AWS recommends for new buckets)."""

    MULTIPART_THRESHOLD = 64 * 1024 * 1024
    PART_SIZE = 32 * 1024 * 1024

    def __init__(self, access_key: str | None, secret_key: str | None, region: str = "us-east-1",
                 endpoint: str | None = None, session_token: str | None = None, timeout: float = 120.0,
                 addressing: str = "path", transport: httpx.BaseTransport | None = None, clock=None):
        if addressing not in ("path", "virtual"):
            raise ValueError("addressing must be 'path' or 'virtual'")
        self.ak, self.sk, self.region, self.token = access_key, secret_key, region, session_token
        self.endpoint = (endpoint or f"https://s3.{region}.amazonaws.com").rstrip("/")
        u = urllib.parse.urlparse(self.endpoint)
        self.scheme, self.host = u.scheme, u.netloc
        self.addressing = addressing
        self.http = httpx.Client(timeout=timeout, transport=transport)
        self._clock = clock or (lambda: _dt.datetime.now(_dt.timezone.utc))

    def _target(self, bucket: str, key: str = "") -> tuple[str, str]:
        """(host, un-encoded path) of an object or bucket request."""
        if self.addressing == "virtual":
            return f"{bucket}.{self.host}", "/" + key
        return self.host, f"/{bucket}" + (f"/{key}" if key else "")

    # ---- signing ----
    def _headers(self, method, host, path, query: dict, payload_hash: str, extra: dict | None = None):
        amz = self._clock().strftime("%Y%m%dT%H%M%SZ")
        h = {"host": host, "x-amz-date": amz, "x-amz-content-sha256": payload_hash}
        if self.token:
            h["x-amz-security-token"] = self.token
        if extra:
            h.update({k.lower(): v for k, v in extra.items()})
        if not (self.ak and self.sk):
            return h
        signed, sig = sigv4_signature(self.sk, self.region, amz, method, path, query, h, payload_hash)
        scope = f"{amz[:8]}/{self.region}/s3/aws4_request"
        h["authorization"] = f"AWS4-HMAC-SHA256 Credential={self.ak}/{scope}, SignedHeaders={signed}, Signature={sig}"
        return h

    def _req(self, method, bucket, key="", query=None, body: bytes = b"", extra=None, ok=(200, 204, 206)):
        host, path = self._target(bucket, key)
        query = query or {}
        h = self._headers(method, host, path, query, _sha256(body), extra)
        # the query string is sent exactly as it was signed (httpx's own encoding could differ)
        qs = _canonical_query(query)
        url = f"{self.scheme}://{host}{_uri_encode(path, True)}" + (f"?{qs}" if qs else "")
        r = self.http.request(method, url, content=body or None, headers=h)
        if r.status_code == 404 and 404 not in ok:
            raise ObjectNotFound(f"s3://{bucket}/{key}")
        if r.status_code not in ok:
            raise RuntimeError(f"S3 {method} {path} failed: {r.status_code} {r.text[:300]}")
        return r

    # ---- operations ----
    def put_bytes(self, bucket, key, data):
        self._req("PUT", bucket, key, body=data)

    def put_file(self, bucket, key, path):
        size = os.path.getsize(path)
        if size <= self.MULTIPART_THRESHOLD:
            with open(path, "rb") as f:
                self.put_bytes(bucket, key, f.read())
            return
        with open(path, "rb") as f:
            self.put_stream(bucket, key, iter(lambda: f.read(self.PART_SIZE), b""))

    def put_stream(self, bucket, key, chunks):
        r = self._req("POST", bucket, key, query={"uploads": ""})
        upload_id = ET.fromstring(r.text).find("{*}UploadId").text
        parts, buf, n = [], bytearray(), 1  # (a bytearray: appending chunks does not re-copy the part)
        try:
            for c in chunks:
                buf += c
                while len(buf) >= self.PART_SIZE:
                    part = bytes(buf[: self.PART_SIZE])
                    del buf[: self.PART_SIZE]
                    rr = self._req("PUT", bucket, key, query={"partNumber": n, "uploadId": upload_id}, body=part)
                    parts.append((n, rr.headers["ETag"]))
                    n += 1
            if buf or not parts:
                rr = self._req("PUT", bucket, key, query={"partNumber": n, "uploadId": upload_id}, body=bytes(buf))
                parts.append((n, rr.headers["ETag"]))
            xml = "<CompleteMultipartUpload>" + "".join(
                f"<Part><PartNumber>{i}</PartNumber><ETag>{e}</ETag></Part>" for i, e in parts) + \
                "</CompleteMultipartUpload>"
            self._req("POST", bucket, key, query={"uploadId": upload_id}, body=xml.encode())
        except Exception:
            try:  # AbortMultipartUpload; never let a failing abort mask the original error
                self._req("DELETE", bucket, key, query={"uploadId": upload_id}, ok=(200, 204, 404))
            except Exception as abort_err:  # noqa: BLE001
                logging.getLogger("ftc.s3").warning("abort of multipart upload %s failed: %s", upload_id, abort_err)
            raise

    def get_bytes(self, bucket, key):
        return self._req("GET", bucket, key).content

    def get_file(self, bucket, key, path):
        """Streamed to disk: a multi-GB checkpoint shard never sits whole in the API server's memory."""
        host, upath = self._target(bucket, key)
        h = self._headers("GET", host, upath, {}, _sha256(b""))
        url = f"{self.scheme}://{host}{_uri_encode(upath, True)}"
        tmp = path + ".part"
        with self.http.stream("GET", url, headers=h) as r:
            if r.status_code == 404:
                raise ObjectNotFound(f"s3://{bucket}/{key}")
            if r.status_code not in (200, 206):
                raise RuntimeError(f"S3 GET {upath} failed: {r.status_code} {r.read()[:300]!r}")
            with open(tmp, "wb") as f:
                for chunk in r.iter_bytes(1 << 20):
                    f.write(chunk)
        os.replace(tmp, path)

    def head(self, bucket, key):
        try:
            r = self._req("HEAD", bucket, key)
        except ObjectNotFound:
            return None
        lm = r.headers.get("Last-Modified")
        ts = _dt.datetime.strptime(lm, "%a, %d %b %Y %H:%M:%S %Z").replace(tzinfo=_dt.timezone.utc) if lm else None
        return ObjectInfo(key, int(r.headers.get("Content-Length", 0)), ts)

    def list(self, bucket, prefix):
        out, token = [], None
        while True:
            q = {"list-type": "2", "prefix": prefix}
            if token:
                q["continuation-token"] = token
            root = ET.fromstring(self._req("GET", bucket, query=q).text)
            for c in root.findall("{*}Contents"):
                lm = c.find("{*}LastModified").text
                out.append(ObjectInfo(c.find("{*}Key").text, int(c.find("{*}Size").text),
                                      _dt.datetime.fromisoformat(lm.replace("Z", "+00:00"))))
            trunc = root.find("{*}IsTruncated")
            if trunc is not None and trunc.text == "true":
                token = root.find("{*}NextContinuationToken").text
            else:
                return out

    def delete(self, bucket, keys):
        for i in range(0, len(keys), 1000):
            xml = "<Delete><Quiet>true</Quiet>" + "".join(
                f"<Object><Key>{_xml_escape(k)}</Key></Object>" for k in keys[i:i + 1000]) + "</Delete>"
            body = xml.encode()
            md5 = __import__("base64").b64encode(hashlib.md5(body).digest()).decode()
            r = self._req("POST", bucket, query={"delete": ""}, body=body, extra={"Content-MD5": md5})
            # DeleteObjects answers 200 even when some keys were not deleted: they are listed as <Error>
            errs = ET.fromstring(r.text).findall("{*}Error") if r.text.strip() else []
            if errs:
                first = errs[0]
                raise RuntimeError(f"S3 delete: {len(errs)} of {len(keys[i:i + 1000])} keys not deleted "
                                   f"(e.g. {first.findtext('{*}Key')}: {first.findtext('{*}Code')})")

    def copy(self, src_bucket, src_key, dst_bucket, dst_key):
        self._req("PUT", dst_bucket, dst_key,
                  extra={"x-amz-copy-source": urllib.parse.quote(f"/{src_bucket}/{src_key}", safe="/-_.~")})

    def presign(self, bucket, key, expires=3600):
        host, path = self._target(bucket, key)
        q = sigv4_presign_query(self.ak or "", self.sk or "", self.region, self._clock().strftime("%Y%m%dT%H%M%SZ"),
                                host, path, expires, self.token)
        return f"{self.scheme}://{host}{_uri_encode(path, True)}?{_canonical_query(q)}"


def _xml_escape(s: str) -> str:
    return s.replace("&", "&amp;").replace("<", "&lt;").replace(">", "&gt;")


def make_object_store(spec: str, settings=None) -> ObjectStore:
    """``"s3"`` -> S3ObjectStore from settings; ``"local:<dir>"`` -> LocalObjectStore."""
    if spec.startswith("local:"):
        return LocalObjectStore(spec[len("local:"):])
    if spec == "s3":
        ak = settings.aws_access_key.get_secret_value() if settings and settings.aws_access_key else None
        sk = settings.aws_secret_key.get_secret_value() if settings and settings.aws_secret_key else None
        return S3ObjectStore(ak, sk, settings.AWS_REGION if settings else "us-east-1",
                             getattr(settings, "S3_ENDPOINT_URL", None) if settings else None,
                             os.environ.get("AWS_SESSION_TOKEN"))
    raise ValueError(f"unknown object store {spec!r}")
