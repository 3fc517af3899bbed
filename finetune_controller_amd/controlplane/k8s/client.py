"""Kubernetes access (C18) behind a small protocol, with a REST implementation.

The reference loads kubeconfig at IMPORT time and talks through the ``kubernetes`` + ``kubeflow``
SDK singletons (``/root/reference/app/utils/kube_config.py:9-23``, ``kf_config.py:12``) -- which makes
every module untestable without a cluster.  Here the control plane depends on the
``KubeClient`` protocol only:

* ``HttpKubeClient`` -- direct REST calls to the API server (in-cluster service-account token, or a
  kubeconfig file: token, token file, client certificate, CA, ``exec`` credential plugins,
  ``auth-provider`` tokens, the context's namespace), no SDK dependency;
* ``FakeCluster`` (``fake.py``) -- an in-process cluster that reconciles PyTorchJobs like the Kubeflow
  training operator and admits them like Kueue, used by the tests and the local e2e path.

Objects are plain dicts in the API server's JSON form.
"""
from __future__ import annotations

import base64
import os
import tempfile
import threading
import time
from dataclasses import dataclass
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


class _ExecCredentialAuth(httpx.Auth):
    """A kubeconfig ``exec`` user (client.authentication.k8s.io ExecCredential plugins: aws-iam-authenticator,
    ``gke-gcloud-auth-plugin``, kubelogin / OIDC, ...).  The plugin is run when there is no token yet or
    the cached one is past its ``status.expirationTimestamp``, and once more (then the request retried) on
    a 401.  The plugin's stdout is the ExecCredential JSON; only ``status.token`` credentials are
    supported (a client-certificate credential raises: it would need the TLS session rebuilt)."""

    requires_response_body = False

    def __init__(self, spec: dict, cwd: str | None = None):
        self.cmd = [spec["command"], *[str(a) for a in (spec.get("args") or [])]]
        self.env = {e["name"]: str(e["value"]) for e in (spec.get("env") or [])}
        self.api_version = spec.get("apiVersion", "client.authentication.k8s.io/v1")
        self.cwd = cwd
        self._token: str | None = None
        self._expires: float | None = None  # epoch seconds
        self.runs = 0
        self._lock = threading.Lock()

    def _run(self) -> str:
        import json
        import subprocess

        info = {"apiVersion": self.api_version, "kind": "ExecCredential", "spec": {"interactive": False}}
        env = dict(os.environ, **self.env, KUBERNETES_EXEC_INFO=json.dumps(info))
        cmd = self.cmd
        if self.cwd and os.sep in cmd[0] and not os.path.isabs(cmd[0]):  # relative to the kubeconfig's dir
            cmd = [os.path.join(self.cwd, cmd[0]), *cmd[1:]]
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=60, stdin=subprocess.DEVNULL)
        self.runs += 1
        if r.returncode != 0:
            raise KubeError(401, "exec credential plugin failed", f"{cmd[0]}: exit {r.returncode}: {r.stderr[-300:]}")
        status = (json.loads(r.stdout) or {}).get("status") or {}
        tok = status.get("token")
        if not tok:
            raise KubeError(401, "exec credential plugin returned no token",
                            "client-certificate ExecCredentials are not supported")
        exp = status.get("expirationTimestamp")
        self._expires = _parse_rfc3339(exp) if exp else None
        self._token = tok
        return tok

    def token(self, force: bool = False) -> str:
        with self._lock:
            stale = self._token is None or (self._expires is not None and time.time() >= self._expires - 10)
            if force or stale:
                return self._run()
            return self._token

    def auth_flow(self, request):
        request.headers["Authorization"] = f"Bearer {self.token()}"
        response = yield request
        if response.status_code == 401:
            request.headers["Authorization"] = f"Bearer {self.token(force=True)}"
            yield request


def _parse_rfc3339(ts: str) -> float:
    import datetime as _dt

    return _dt.datetime.fromisoformat(ts.replace("Z", "+00:00")).timestamp()


@dataclass
class KubeConfig:
    """What ``HttpKubeClient._discover`` resolved: server, TLS (an in-memory ``ssl.SSLContext`` built from
    the *-data fields, so no CA / certificate / private key is ever left on disk, or a CA path / False),
    the request auth (static token, rotating token file, exec plugin or auth-provider token) and the
    context's namespace."""
    server: str
    verify: object = True
    token: str | None = None
    token_file: str | None = None
    auth: httpx.Auth | None = None
    namespace: str | None = None


def _ssl_context(cluster: dict, user: dict, base_dir: str):
    """TLS settings of a kubeconfig (cluster, user) pair: False (insecure-skip-tls-verify), True (system
    CAs, no client certificate) or an ``ssl.SSLContext``.  CA data is loaded from memory (``cadata``);
    client certificate / key data must pass through ``load_cert_chain``, which reads files only: they are
    written 0600 into a private temporary directory and removed before this returns."""
    import ssl

    def path(p):
        return p if os.path.isabs(p) else os.path.join(base_dir, p)

    has_cert = any(k in user for k in ("client-certificate-data", "client-certificate"))
    ca_data = cluster.get("certificate-authority-data")
    ca_file = cluster.get("certificate-authority")
    if cluster.get("insecure-skip-tls-verify") and not has_cert:
        return False
    if not (ca_data or ca_file or has_cert):
        return True
    ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_CLIENT)  # verifies peer + hostname by default
    if not (ca_data or ca_file):
        ctx.load_default_certs()  # a cluster CA, when named, is the ONLY trust anchor (kubeconfig semantics)
    if cluster.get("insecure-skip-tls-verify"):
        ctx.check_hostname = False
        ctx.verify_mode = ssl.CERT_NONE
    elif ca_data:
        ctx.load_verify_locations(cadata=base64.b64decode(ca_data).decode())
    elif ca_file:
        ctx.load_verify_locations(cafile=path(ca_file))
    if "client-certificate-data" in user:
        with tempfile.TemporaryDirectory(prefix="ftc-kube-") as d:
            crt, key = os.path.join(d, "c"), os.path.join(d, "k")
            for fn, field in ((crt, "client-certificate-data"), (key, "client-key-data")):
                fd = os.open(fn, os.O_WRONLY | os.O_CREAT | os.O_EXCL, 0o600)
                with os.fdopen(fd, "wb") as f:
                    f.write(base64.b64decode(user[field]))
            ctx.load_cert_chain(crt, key)
    elif "client-certificate" in user:
        ctx.load_cert_chain(path(user["client-certificate"]), path(user["client-key"]))
    return ctx


class HttpKubeClient(KubeClient):
    SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"

    def __init__(self, server: str | None = None, token: str | None = None, verify=True, cert=None,
                 kubeconfig: str | None = None, timeout: float = 30.0, transport: httpx.BaseTransport | None = None,
                 token_file: str | None = None, auth: httpx.Auth | None = None, namespace: str | None = None):
        if server is None:
            kc = self._discover(kubeconfig)
            server, token, verify, token_file, auth, namespace = (kc.server, kc.token, kc.verify, kc.token_file,
                                                                  kc.auth, kc.namespace)
        self.server = server.rstrip("/")
        self.verify, self.cert = verify, cert
        self.namespace = namespace  # the kubeconfig context's / service account's namespace (None: unset)
        if auth is None and token_file:
            auth = _TokenFileAuth(token_file)
        headers = {"Authorization": f"Bearer {token}"} if token and auth is None else {}
        if transport is not None:  # injected transport (tests replay API-server responses): no TLS setup
            self.http = httpx.Client(base_url=self.server, headers=headers, timeout=timeout, transport=transport,
                                     auth=auth)
        else:
            self.http = httpx.Client(base_url=self.server, headers=headers, verify=verify, cert=cert, timeout=timeout,
                                     auth=auth)

    def close(self):
        self.http.close()

    # ---- configuration discovery (in-cluster first, then kubeconfig) ----
    @classmethod
    def _discover(cls, kubeconfig: str | None) -> KubeConfig:
        """In-cluster service account, else the kubeconfig's current context (``KUBECONFIG`` / ``~/.kube/config``)
        -- the reference's ``config.load_incluster_config()`` / ``load_kube_config()``
        (``/root/reference/app/utils/kube_config.py:9-16``): token, token-file, client certificate (inline
        or path), ``exec`` credential plugins and ``auth-provider`` tokens (oidc ``id-token``, gcp / azure
        ``access-token``), the context's ``namespace``."""
        host, port = os.environ.get("KUBERNETES_SERVICE_HOST"), os.environ.get("KUBERNETES_SERVICE_PORT")
        if host and port and os.path.exists(os.path.join(cls.SA_DIR, "token")):
            # in-cluster: the token is read per request from the rotating file (_TokenFileAuth)
            ns = None
            try:
                with open(os.path.join(cls.SA_DIR, "namespace")) as f:
                    ns = f.read().strip() or None
            except OSError:
                pass
            return KubeConfig(f"https://{host}:{port}", verify=os.path.join(cls.SA_DIR, "ca.crt"),
                              token_file=os.path.join(cls.SA_DIR, "token"), namespace=ns)
        path = kubeconfig or (os.environ.get("KUBECONFIG") or os.path.expanduser("~/.kube/config")).split(os.pathsep)[0]
        import yaml

        with open(path) as f:
            kc = yaml.safe_load(f) or {}
        base = os.path.dirname(os.path.abspath(path))
        ctx_name = kc.get("current-context")
        ctxs = {c["name"]: c.get("context") or {} for c in kc.get("contexts") or []}
        if ctx_name not in ctxs:
            raise KubeError(0, "kubeconfig", f"{path}: current-context {ctx_name!r} is not among its contexts")
        ctx = ctxs[ctx_name]
        clusters = {c["name"]: c.get("cluster") or {} for c in kc.get("clusters") or []}
        users = {u["name"]: u.get("user") or {} for u in kc.get("users") or []}
        if ctx.get("cluster") not in clusters:
            raise KubeError(0, "kubeconfig", f"{path}: context {ctx_name!r} names unknown cluster {ctx.get('cluster')!r}")
        cluster = clusters[ctx["cluster"]]
        user = users.get(ctx.get("user"), {})
        out = KubeConfig(cluster["server"], verify=_ssl_context(cluster, user, base), namespace=ctx.get("namespace"))
        if user.get("token"):
            out.token = user["token"]
        elif user.get("tokenFile"):
            tf = user["tokenFile"]
            out.token_file = tf if os.path.isabs(tf) else os.path.join(base, tf)
        elif user.get("exec"):
            out.auth = _ExecCredentialAuth(user["exec"], cwd=base)
        elif user.get("auth-provider"):
            conf = (user["auth-provider"] or {}).get("config") or {}
            tok = conf.get("id-token") or conf.get("access-token")
            if not tok:
                raise KubeError(0, "kubeconfig", f"{path}: auth-provider {user['auth-provider'].get('name')!r} "
                                                 "holds no id-token / access-token (log in with its CLI first)")
            out.token = tok
        elif user.get("username") and user.get("password"):
            out.auth = httpx.BasicAuth(user["username"], user["password"])
        return out

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
