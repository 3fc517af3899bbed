"""Kubernetes access (C18) behind a small protocol, with a REST implementation.

The reference loads kubeconfig at IMPORT time and talks through the ``kubernetes`` + ``kubeflow``
SDK singletons (``/root/reference/app/utils/kube_config.py:9-23``, ``kf_config.py:12``) -- which makes
every module untestable without a cluster.  Here the control plane depends on the
``KubeClient`` protocol only:

* ``HttpKubeClient`` -- direct REST calls to the API server (in-cluster service-account token, or a
  kubeconfig file: token / client-certificate / CA data), no SDK dependency;
* ``FakeCluster`` (``fake.py``) -- an in-process cluster that reconciles PyTorchJobs like the Kubeflow
  training operator and admits them like Kueue, used by the tests and the local e2e path.

Objects are plain dicts in the API server's JSON form.
"""
from __future__ import annotations

import base64
import os
import tempfile
from typing import Iterator

import httpx

PT_GROUP, PT_VERSION, PT_PLURAL = "kubeflow.org", "v1", "pytorchjobs"
KUEUE_GROUP, KUEUE_VERSION = "kueue.x-k8s.io", "v1beta1"
JOB_NAME_LABEL = "training.kubeflow.org/job-name"
REPLICA_TYPE_LABEL = "training.kubeflow.org/replica-type"
JOB_ROLE_LABEL = "training.kubeflow.org/job-role"


class KubeError(Exception):
    def __init__(self, status: int, reason: str = "", body: str = ""):
        super().__init__(f"({status}) {reason}: {body[:500]}")
        self.status, self.reason, self.body = status, reason, body


class KubeClient:
    """Protocol (duck-typed); every method is synchronous -- async callers use ``asyncio.to_thread``."""

    def create_custom(self, group, version, namespace, plural, body) -> dict: raise NotImplementedError
    def get_custom(self, group, version, namespace, plural, name) -> dict: raise NotImplementedError
    def delete_custom(self, group, version, namespace, plural, name) -> dict: raise NotImplementedError
    def list_custom(self, group, version, namespace, plural, label_selector=None) -> dict: raise NotImplementedError
    def list_pods(self, namespace, label_selector=None) -> list[dict]: raise NotImplementedError
    def read_pod(self, namespace, name) -> dict: raise NotImplementedError
    def read_pod_log(self, namespace, name, container=None, tail_lines=None) -> str: raise NotImplementedError
    def stream_pod_log(self, namespace, name, container=None, tail_lines=None) -> Iterator[bytes]: raise NotImplementedError
    def list_events(self, namespace) -> list[dict]: raise NotImplementedError
    def read_secret(self, name, namespace) -> dict: raise NotImplementedError

    # ---- conveniences shared by implementations ----
    def list_pytorchjobs(self, namespace) -> list[dict]:
        return self.list_custom(PT_GROUP, PT_VERSION, namespace, PT_PLURAL).get("items", [])

    def get_pytorchjob(self, namespace, name) -> dict:
        return self.get_custom(PT_GROUP, PT_VERSION, namespace, PT_PLURAL, name)

    def create_pytorchjob(self, namespace, body) -> dict:
        return self.create_custom(PT_GROUP, PT_VERSION, namespace, PT_PLURAL, body)

    def delete_pytorchjob(self, namespace, name) -> dict:
        return self.delete_custom(PT_GROUP, PT_VERSION, namespace, PT_PLURAL, name)

    def list_workloads(self, namespace) -> list[dict]:
        return self.list_custom(KUEUE_GROUP, KUEUE_VERSION, namespace, "workloads").get("items", [])

    def get_job_pod_names(self, job_name, namespace, is_master=True) -> list[str]:
        sel = f"{JOB_NAME_LABEL}={job_name}"
        if is_master:
            sel += f",{REPLICA_TYPE_LABEL}=master"
        return [p["metadata"]["name"] for p in self.list_pods(namespace, sel)]


class _TokenFileAuth(httpx.Auth):
    """Bearer token read from a projected service-account token file.  The kubelet rotates bound
    tokens (about hourly), so a controller that read the file once at start-up would begin failing
    with 401 after the first rotation.  The file is re-read when its mtime changes, and once more
    (then the request retried) on a 401."""

    def __init__(self, path: str):
        self.path, self._token, self._mtime = path, "", None

    def _load(self, force: bool = False) -> str:
        try:
            m = os.stat(self.path).st_mtime_ns
        except OSError:
            return self._token
        if force or m != self._mtime:
            with open(self.path) as f:
                self._token = f.read().strip()
            self._mtime = m
        return self._token

    def auth_flow(self, request):
        request.headers["Authorization"] = f"Bearer {self._load()}"
        response = yield request
        if response.status_code == 401:
            request.headers["Authorization"] = f"Bearer {self._load(force=True)}"
            yield request


class HttpKubeClient(KubeClient):
    SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"

    def __init__(self, server: str | None = None, token: str | None = None, verify=True, cert=None,
                 kubeconfig: str | None = None, timeout: float = 30.0, transport: httpx.BaseTransport | None = None,
                 token_file: str | None = None):
        if server is None:
            server, token, verify, cert, token_file = self._discover(kubeconfig)
        self.server = server.rstrip("/")
        self.verify, self.cert = verify, cert
        auth = _TokenFileAuth(token_file) if token_file else None
        headers = {"Authorization": f"Bearer {token}"} if token and not token_file else {}
        if transport is not None:  # injected transport (tests replay API-server responses): no TLS setup
            self.http = httpx.Client(base_url=self.server, headers=headers, timeout=timeout, transport=transport,
                                     auth=auth)
        else:
            self.http = httpx.Client(base_url=self.server, headers=headers, verify=verify, cert=cert, timeout=timeout,
                                     auth=auth)

    # ---- configuration discovery (in-cluster first, then kubeconfig) ----
    @classmethod
    def _discover(cls, kubeconfig: str | None):
        host, port = os.environ.get("KUBERNETES_SERVICE_HOST"), os.environ.get("KUBERNETES_SERVICE_PORT")
        if host and port and os.path.exists(os.path.join(cls.SA_DIR, "token")):
            # in-cluster: the token is read per request from the rotating file (_TokenFileAuth)
            return f"https://{host}:{port}", None, os.path.join(cls.SA_DIR, "ca.crt"), None, \
                os.path.join(cls.SA_DIR, "token")
        path = kubeconfig or os.environ.get("KUBECONFIG", os.path.expanduser("~/.kube/config"))
        import yaml

        with open(path) as f:
            kc = yaml.safe_load(f)
        ctx_name = kc.get("current-context")
        ctx = next(c["context"] for c in kc["contexts"] if c["name"] == ctx_name)
        cluster = next(c["cluster"] for c in kc["clusters"] if c["name"] == ctx["cluster"])
        user = next(u["user"] for u in kc["users"] if u["name"] == ctx["user"])
        verify = True
        if cluster.get("insecure-skip-tls-verify"):
            verify = False
        elif "certificate-authority-data" in cluster:
            verify = cls._tmpfile(base64.b64decode(cluster["certificate-authority-data"]))
        elif "certificate-authority" in cluster:
            verify = cluster["certificate-authority"]
        cert = None
        if "client-certificate-data" in user:
            cert = (cls._tmpfile(base64.b64decode(user["client-certificate-data"])),
                    cls._tmpfile(base64.b64decode(user["client-key-data"])))
        elif "client-certificate" in user:
            cert = (user["client-certificate"], user["client-key"])
        return cluster["server"], user.get("token"), verify, cert, None

    @staticmethod
    def _tmpfile(data: bytes) -> str:
        fd, p = tempfile.mkstemp(prefix="ftc-kube-")
        with os.fdopen(fd, "wb") as f:
            f.write(data)
        return p

    # ---- REST ----
    def _req(self, method, path, **kw):
        r = self.http.request(method, path, **kw)
        if r.status_code >= 400:
            raise KubeError(r.status_code, r.reason_phrase, r.text)
        return r

    @staticmethod
    def _cpath(group, version, namespace, plural, name=None):
        p = f"/apis/{group}/{version}/namespaces/{namespace}/{plural}"
        return p + (f"/{name}" if name else "")

    def create_custom(self, group, version, namespace, plural, body):
        return self._req("POST", self._cpath(group, version, namespace, plural), json=body).json()

    def get_custom(self, group, version, namespace, plural, name):
        return self._req("GET", self._cpath(group, version, namespace, plural, name)).json()

    def delete_custom(self, group, version, namespace, plural, name):
        return self._req("DELETE", self._cpath(group, version, namespace, plural, name),
                         json={"propagationPolicy": "Foreground"}).json()

    def list_custom(self, group, version, namespace, plural, label_selector=None):
        params = {"labelSelector": label_selector} if label_selector else None
        return self._req("GET", self._cpath(group, version, namespace, plural), params=params).json()

    def list_pods(self, namespace, label_selector=None):
        params = {"labelSelector": label_selector} if label_selector else None
        return self._req("GET", f"/api/v1/namespaces/{namespace}/pods", params=params).json().get("items", [])

    def read_pod(self, namespace, name):
        return self._req("GET", f"/api/v1/namespaces/{namespace}/pods/{name}/status").json()

    def read_pod_log(self, namespace, name, container=None, tail_lines=None):
        params = {}
        if container:
            params["container"] = container
        if tail_lines:
            params["tailLines"] = int(tail_lines)
        return self._req("GET", f"/api/v1/namespaces/{namespace}/pods/{name}/log", params=params).text

    def stream_pod_log(self, namespace, name, container=None, tail_lines=None):
        params = {"follow": "true"}
        if container:
            params["container"] = container
        if tail_lines:
            params["tailLines"] = int(tail_lines)
        with self.http.stream("GET", f"/api/v1/namespaces/{namespace}/pods/{name}/log", params=params,
                              timeout=None) as r:
            if r.status_code >= 400:
                raise KubeError(r.status_code, r.reason_phrase, r.read().decode(errors="replace"))
            for line in r.iter_lines():
                yield (line + "\n").encode()

    def list_events(self, namespace):
        return self._req("GET", f"/api/v1/namespaces/{namespace}/events").json().get("items", [])

    def read_secret(self, name, namespace):
        return self._req("GET", f"/api/v1/namespaces/{namespace}/secrets/{name}").json().get("data", {})
