"""Streaming ``multipart/form-data`` / urlencoded form parsing.

FastAPI's ``Form``/``File`` parameters need the python-multipart package; this control plane parses
the job-submission form itself: text fields are collected in memory (bounded), file parts are
streamed to a temp file in ``/tmp/ftjobs`` (the reference spools uploads there too,
``/root/reference/app/utils/dataset_helpers.py:27``) so a multi-GB dataset upload never sits in RAM.
"""
from __future__ import annotations

import os
import tempfile
from urllib.parse import parse_qs

from ..schemas.jobs import UploadedFile

MAX_FIELD_BYTES = 1 << 20
MAX_URLENCODED_BYTES = 8 * MAX_FIELD_BYTES
UPLOAD_DIR = "/tmp/ftjobs"


class FormError(ValueError):
    pass


def discard_uploads(files: dict[str, UploadedFile]) -> None:
    """Remove the spooled temp files of ``files`` that nothing consumed (the dataset ingest removes its
    own after the upload to object storage)."""
    for f in files.values():
        try:
            os.remove(f.path)
        except FileNotFoundError:
            pass


def _boundary(ctype: str) -> bytes:
    for part in ctype.split(";"):
        part = part.strip()
        if part.lower().startswith("boundary="):
            b = part.split("=", 1)[1].strip().strip('"')
            return b.encode()
    raise FormError("multipart boundary missing")


def _parse_disposition(value: str) -> dict:
    out = {}
    for item in value.split(";")[1:]:
        if "=" in item:
            k, v = item.strip().split("=", 1)
            out[k.lower()] = v.strip().strip('"')
    return out


async def parse_form(request) -> tuple[dict[str, str], dict[str, UploadedFile]]:
    """Fields and spooled files of the request body.  On any failure (a bad part, an oversized field,
    the client going away mid-upload) every temp file written so far is removed before re-raising."""
    spooled: list[str] = []
    try:
        return await _parse_form(request, spooled)
    except BaseException:
        for path in spooled:
            try:
                os.remove(path)
            except FileNotFoundError:
                pass
        raise


async def _parse_form(request, spooled: list[str]) -> tuple[dict[str, str], dict[str, UploadedFile]]:
    ctype = request.headers.get("content-type", "")
    if ctype.startswith("application/x-www-form-urlencoded"):
        body = bytearray()
        async for chunk in request.stream():  # bounded: an urlencoded form carries no file
            body += chunk
            if len(body) > MAX_URLENCODED_BYTES:
                raise FormError("form too large")
        q = parse_qs(body.decode("utf-8", errors="replace"), keep_blank_values=True)
        return {k: v[-1] for k, v in q.items()}, {}
    if not ctype.startswith("multipart/form-data"):
        raise FormError("expected multipart/form-data or application/x-www-form-urlencoded")
    delim = b"--" + _boundary(ctype)
    fields: dict[str, str] = {}
    files: dict[str, UploadedFile] = {}
    buf = b""
    state = "preamble"
    headers: dict[str, str] = {}
    cur_name = None
    cur_file = None
    cur_fh = None
    cur_val = bytearray()
    os.makedirs(UPLOAD_DIR, exist_ok=True)

    def finish_part():
        nonlocal cur_fh, cur_file, cur_val
        if cur_file is not None:
            cur_fh.close()
            cur_file.size = os.path.getsize(cur_file.path)
            if cur_file.filename:
                if cur_name in files:  # a repeated file field: the last one wins, the earlier is dropped
                    os.remove(files[cur_name].path)
                files[cur_name] = cur_file
            else:
                os.remove(cur_file.path)
        elif cur_name is not None:
            fields[cur_name] = cur_val.decode("utf-8", errors="replace")
        cur_fh = cur_file = None
        cur_val = bytearray()

    async for chunk in request.stream():
        buf += chunk
        while True:
            if state == "preamble":
                i = buf.find(delim)
                if i < 0:
                    buf = buf[-len(delim):]
                    break
                buf = buf[i + len(delim):]
                state = "after_delim"
            if state == "after_delim":
                if len(buf) < 2:
                    break
                if buf.startswith(b"--"):
                    return fields, files
                if buf.startswith(b"\r\n"):
                    buf = buf[2:]
                state = "headers"
                headers = {}
            if state == "headers":
                j = buf.find(b"\r\n\r\n")
                if j < 0:
                    if len(buf) > 64 * 1024:
                        raise FormError("part headers too large")
                    break
                for line in buf[:j].decode("utf-8", errors="replace").split("\r\n"):
                    if ":" in line:
                        k, v = line.split(":", 1)
                        headers[k.strip().lower()] = v.strip()
                buf = buf[j + 4:]
                disp = _parse_disposition(headers.get("content-disposition", ""))
                cur_name = disp.get("name")
                if "filename" in disp:
                    fname = os.path.basename(disp["filename"])
                    fd, path = tempfile.mkstemp(prefix="upload-", dir=UPLOAD_DIR)
                    spooled.append(path)
                    cur_fh = os.fdopen(fd, "wb")
                    cur_file = UploadedFile(filename=fname, path=path,
                                            content_type=headers.get("content-type", "application/octet-stream"))
                state = "body"
            if state == "body":
                k = buf.find(b"\r\n" + delim)
                if k < 0:
                    keep = len(delim) + 2
                    if len(buf) > keep:
                        data, buf = buf[:-keep], buf[-keep:]
                        if cur_fh is not None:
                            cur_fh.write(data)
                        else:
                            cur_val.extend(data)
                            if len(cur_val) > MAX_FIELD_BYTES:
                                raise FormError("form field too large")
                    break
                data, buf = buf[:k], buf[k + 2 + len(delim):]
                if cur_fh is not None:
                    cur_fh.write(data)
                else:
                    cur_val.extend(data)
                    if len(cur_val) > MAX_FIELD_BYTES:  # (also when the whole field came in one chunk)
                        raise FormError("form field too large")
                finish_part()
                state = "after_delim"
    if state in ("headers", "body"):
        # the body ended inside a part (no closing delimiter): a cut-off upload must not become a
        # dataset of whatever bytes arrived
        raise FormError("multipart body ended inside a part (truncated upload?)")
    return fields, files
