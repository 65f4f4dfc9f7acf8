"""Model-weight store: resolve a weights URI to a local file and load it safely.

Reference parity: the reference's Triton server image pulls its model
from MinIO with an OIDC token from Keycloak exchanged for temporary S3 credentials
(``docker/server/utils/download_model_s3_keycloak.py:68-238``: token request →
STS ``AssumeRoleWithWebIdentity`` → boto3 ``download_file``), with the credentials
written in plain text into the Dockerfile (``docker/server/Dockerfile:9-17``).

Here the same flow is plain ``urllib`` (no boto3 / keycloak dependency) and no
credential ever lives in a file of this repo — everything secret comes from the
environment:

=========================  ====================================================
URI                        how it is fetched
=========================  ====================================================
``/path`` / ``file://``    used in place
``http(s)://…``            GET; ``Authorization: Bearer $TCA_MODEL_STORE_TOKEN``
                           only to hosts listed in ``$TCA_MODEL_STORE_TOKEN_HOSTS``
                           (comma-separated ``host[:port]``) and only over https
``s3://bucket/key``        SigV4-signed GET against ``$TCA_S3_ENDPOINT``
                           (path-style, MinIO-compatible; https).  Credentials:
                           ``AWS_ACCESS_KEY_ID`` / ``AWS_SECRET_ACCESS_KEY`` /
                           ``AWS_SESSION_TOKEN``, or — when ``TCA_OIDC_TOKEN_URL``
                           is set — an OIDC token (client-credentials grant, or
                           password grant when ``TCA_OIDC_USERNAME`` is set)
                           exchanged at the endpoint's STS for temporary keys.
=========================  ====================================================

Credentials never follow a redirect: every fetch goes through an opener whose
redirect handler drops ``Authorization`` and ``x-amz-*`` headers and refuses an
https → http downgrade.  Plain-http token / SigV4 traffic (a MinIO on a private
network) needs ``TCA_MODEL_STORE_ALLOW_HTTP=1``.

Downloads land in a content cache (``$TCA_MODEL_CACHE`` or
``~/.cache/triton_client_amd/models``) via write-to-temp + atomic rename, with
a ``.sha256`` sidecar written at download time.  A cached copy is reused only
if it still matches the expected sha256 (when one is given — the model
repository carries it as the ``weights_sha256`` parameter) or its sidecar;
``refresh=True`` always fetches again.  ``load_state_dict`` only ever calls
``torch.load(..., weights_only=True)``.
"""
from __future__ import annotations

import datetime as _dt
import hashlib
import hmac
import json
import os
import tempfile
import urllib.parse
import urllib.request
import xml.etree.ElementTree as ET
from dataclasses import dataclass
from pathlib import Path
from typing import Optional

__all__ = ["S3Credentials", "resolve", "load_state_dict", "sigv4_headers", "oidc_token", "sts_web_identity"]


class ModelStoreError(RuntimeError):
    pass


@dataclass
class S3Credentials:
    access_key: str
    secret_key: str
    session_token: Optional[str] = None


def _cache_dir() -> Path:
    d = os.environ.get("TCA_MODEL_CACHE") or os.path.join(os.path.expanduser("~"), ".cache", "triton_client_amd", "models")
    p = Path(d)
    p.mkdir(parents=True, exist_ok=True)
    return p


def _sha256_file(path: Path) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


_SECRET_HEADERS = ("authorization", "x-amz-")


class _NoCredentialRedirect(urllib.request.HTTPRedirectHandler):
    """urllib copies every header but Content-Length/-Type onto a redirected
    request; this one strips credentials and refuses an https → http hop."""

    def redirect_request(self, req, fp, code, msg, headers, newurl):
        new = super().redirect_request(req, fp, code, msg, headers, newurl)
        if new is None:
            return None
        if urllib.parse.urlsplit(req.full_url).scheme == "https" and urllib.parse.urlsplit(newurl).scheme != "https":
            raise ModelStoreError(f"refusing https -> {urllib.parse.urlsplit(newurl).scheme} redirect to {newurl}")
        for k in list(new.headers):
            if k.lower().startswith(_SECRET_HEADERS):
                del new.headers[k]
        for k in list(new.unredirected_hdrs):
            if k.lower().startswith(_SECRET_HEADERS):
                del new.unredirected_hdrs[k]
        return new


_OPENER = urllib.request.build_opener(_NoCredentialRedirect)


def _open(req: urllib.request.Request, timeout: float):
    return _OPENER.open(req, timeout=timeout)


def _allow_plain_http() -> bool:
    return os.environ.get("TCA_MODEL_STORE_ALLOW_HTTP", "") == "1"


def _token_for(parts: urllib.parse.SplitResult) -> Optional[str]:
    """The bearer token, if this URL may receive it (allow-listed host, https)."""
    tok = os.environ.get("TCA_MODEL_STORE_TOKEN")
    if not tok:
        return None
    hosts = {h.strip().lower() for h in os.environ.get("TCA_MODEL_STORE_TOKEN_HOSTS", "").split(",") if h.strip()}
    if parts.netloc.lower() not in hosts and (parts.hostname or "").lower() not in hosts:
        return None
    if parts.scheme != "https" and not _allow_plain_http():
        raise ModelStoreError(f"refusing to send TCA_MODEL_STORE_TOKEN over {parts.scheme}:// "
                              "(set TCA_MODEL_STORE_ALLOW_HTTP=1 for a private-network store)")
    return tok


def _download(req: urllib.request.Request, dest: Path, timeout: float) -> str:
    """Stream ``req`` into ``dest`` (atomic rename); returns the sha256."""
    fd, tmp = tempfile.mkstemp(dir=dest.parent, prefix=".part-")
    h = hashlib.sha256()
    try:
        with os.fdopen(fd, "wb") as out, _open(req, timeout) as r:
            while True:
                blk = r.read(1 << 20)
                if not blk:
                    break
                h.update(blk)
                out.write(blk)
        os.replace(tmp, dest)
        return h.hexdigest()
    except BaseException:
        try:
            os.unlink(tmp)
        except FileNotFoundError:
            pass
        raise


# ---------------------------------------------------------------- SigV4 (S3)
def _hmac(key: bytes, msg: str) -> bytes:
    return hmac.new(key, msg.encode(), hashlib.sha256).digest()


def sigv4_headers(method: str, url: str, creds: S3Credentials, region: str = "us-east-1",
                  now: Optional[_dt.datetime] = None, payload_sha256: str = "UNSIGNED-PAYLOAD") -> dict:
    """AWS Signature V4 headers for one S3 request (path-style URL)."""
    u = urllib.parse.urlsplit(url)
    now = now or _dt.datetime.now(_dt.timezone.utc)
    amz_date, date = now.strftime("%Y%m%dT%H%M%SZ"), now.strftime("%Y%m%d")
    hdrs = {"host": u.netloc, "x-amz-content-sha256": payload_sha256, "x-amz-date": amz_date}
    if creds.session_token:
        hdrs["x-amz-security-token"] = creds.session_token
    names = sorted(hdrs)
    canon_q = "&".join(f"{urllib.parse.quote(k, safe='-_.~')}={urllib.parse.quote(v, safe='-_.~')}"
                       for k, v in sorted(urllib.parse.parse_qsl(u.query, keep_blank_values=True)))
    canonical = "\n".join([
        method, urllib.parse.quote(u.path or "/", safe="/-_.~"), canon_q,
        "".join(f"{k}:{hdrs[k].strip()}\n" for k in names), ";".join(names), payload_sha256])
    scope = f"{date}/{region}/s3/aws4_request"
    to_sign = "\n".join(["AWS4-HMAC-SHA256", amz_date, scope, hashlib.sha256(canonical.encode()).hexdigest()])
    key = _hmac(_hmac(_hmac(_hmac(("AWS4" + creds.secret_key).encode(), date), region), "s3"), "aws4_request")
    sig = hmac.new(key, to_sign.encode(), hashlib.sha256).hexdigest()
    out = {k: v for k, v in hdrs.items() if k != "host"}
    out["Authorization"] = (f"AWS4-HMAC-SHA256 Credential={creds.access_key}/{scope}, "
                            f"SignedHeaders={';'.join(names)}, Signature={sig}")
    return out


# ------------------------------------------------------- OIDC → STS exchange
def oidc_token(token_url: str, client_id: str, client_secret: Optional[str] = None,
               username: Optional[str] = None, password: Optional[str] = None, timeout: float = 30.0) -> str:
    """Fetch an OIDC token (Keycloak-style token endpoint); returns the access token."""
    form = {"client_id": client_id}
    if client_secret:
        form["client_secret"] = client_secret
    if username:
        form.update(grant_type="password", username=username, password=password or "")
    else:
        form["grant_type"] = "client_credentials"
    req = urllib.request.Request(token_url, data=urllib.parse.urlencode(form).encode(), method="POST",
                                 headers={"Content-Type": "application/x-www-form-urlencoded"})
    with _open(req, timeout) as r:
        body = json.loads(r.read())
    tok = body.get("access_token") or body.get("id_token")
    if not tok:
        raise ModelStoreError(f"OIDC endpoint returned no token (keys: {sorted(body)})")
    return tok


def sts_web_identity(endpoint: str, token: str, duration_s: int = 3600, timeout: float = 30.0) -> S3Credentials:
    """STS AssumeRoleWithWebIdentity (MinIO / AWS form) → temporary S3 credentials."""
    form = {"Action": "AssumeRoleWithWebIdentity", "Version": "2011-06-15",
            "WebIdentityToken": token, "DurationSeconds": str(duration_s)}
    req = urllib.request.Request(endpoint, data=urllib.parse.urlencode(form).encode(), method="POST",
                                 headers={"Content-Type": "application/x-www-form-urlencoded"})
    with _open(req, timeout) as r:
        root = ET.fromstring(r.read())
    found = {el.tag.rsplit("}", 1)[-1]: (el.text or "") for el in root.iter()}
    try:
        return S3Credentials(found["AccessKeyId"], found["SecretAccessKey"], found.get("SessionToken") or None)
    except KeyError as e:
        raise ModelStoreError(f"STS response has no {e.args[0]}") from None


def _s3_credentials(endpoint: str) -> S3Credentials:
    env = os.environ
    if env.get("TCA_OIDC_TOKEN_URL"):
        tok = oidc_token(env["TCA_OIDC_TOKEN_URL"], env.get("TCA_OIDC_CLIENT_ID", "minio"),
                         env.get("TCA_OIDC_CLIENT_SECRET"), env.get("TCA_OIDC_USERNAME"), env.get("TCA_OIDC_PASSWORD"))
        return sts_web_identity(env.get("TCA_STS_ENDPOINT", endpoint), tok)
    if env.get("AWS_ACCESS_KEY_ID") and env.get("AWS_SECRET_ACCESS_KEY"):
        return S3Credentials(env["AWS_ACCESS_KEY_ID"], env["AWS_SECRET_ACCESS_KEY"], env.get("AWS_SESSION_TOKEN"))
    raise ModelStoreError("s3:// URI needs AWS_ACCESS_KEY_ID/AWS_SECRET_ACCESS_KEY or TCA_OIDC_TOKEN_URL in the environment")


# ------------------------------------------------------------------ public
def _cached_ok(path: Path, sha256: Optional[str]) -> bool:
    if not path.is_file():
        return False
    want = sha256.lower() if sha256 else None
    if want is None:
        side = path.with_name(path.name + ".sha256")
        want = side.read_text().strip() if side.is_file() else None
    return want is not None and _sha256_file(path) == want


def resolve(uri: str, sha256: Optional[str] = None, timeout: float = 120.0, refresh: bool = False) -> Path:
    """Return a local path holding the object named by ``uri`` (downloading it if remote)."""
    parts = urllib.parse.urlsplit(uri)
    if parts.scheme in ("", "file"):
        path = Path(urllib.parse.unquote(parts.path) if parts.scheme == "file" else uri)
        if not path.is_file():
            raise ModelStoreError(f"weights file not found: {path}")
    else:
        name = hashlib.sha256(uri.encode()).hexdigest()[:16] + "-" + (Path(parts.path).name or "object")
        path = _cache_dir() / name
        if refresh or not _cached_ok(path, sha256):
            if parts.scheme in ("http", "https"):
                tok = _token_for(parts)
                req = urllib.request.Request(uri, headers={"Authorization": "Bearer " + tok} if tok else {})
            elif parts.scheme == "s3":
                endpoint = os.environ.get("TCA_S3_ENDPOINT")
                if not endpoint:
                    raise ModelStoreError("s3:// URI needs TCA_S3_ENDPOINT (e.g. https://minio:9000)")
                if urllib.parse.urlsplit(endpoint).scheme != "https" and not _allow_plain_http():
                    raise ModelStoreError(f"TCA_S3_ENDPOINT {endpoint} is not https "
                                          "(set TCA_MODEL_STORE_ALLOW_HTTP=1 for a private-network MinIO)")
                url = endpoint.rstrip("/") + "/" + parts.netloc + "/" + parts.path.lstrip("/")
                hdrs = sigv4_headers("GET", url, _s3_credentials(endpoint), os.environ.get("TCA_S3_REGION", "us-east-1"))
                req = urllib.request.Request(url, headers=hdrs)
            else:
                raise ModelStoreError(f"unsupported weights URI scheme: {parts.scheme!r}")
            digest = _download(req, path, timeout)
            path.with_name(path.name + ".sha256").write_text(digest + "\n")
            if sha256 and digest != sha256.lower():
                raise ModelStoreError(f"sha256 mismatch for {uri}")
            return path
    if sha256 and _sha256_file(path) != sha256.lower():
        raise ModelStoreError(f"sha256 mismatch for {uri}")
    return path


def load_state_dict(uri: str, sha256: Optional[str] = None):
    """Resolve ``uri`` and load it as a tensor-only state_dict (``weights_only=True``)."""
    import torch

    return torch.load(resolve(uri, sha256), map_location="cpu", weights_only=True)
