"""multipart/form-data parsing without python-multipart (not installed offline).

FastAPI's ``UploadFile = File(...)`` parameters require python-multipart at route
definition time, so the upload route reads the raw body and parses it here into
Starlette ``UploadFile`` objects (spooled to disk above 1 MiB, like Starlette).
Missing fields reproduce FastAPI's RequestValidationError body for
``file: UploadFile = File(...)`` (reference app/main.py:205-209).
"""
from __future__ import annotations

import re
import tempfile

from starlette.datastructures import Headers, UploadFile

_BOUNDARY = re.compile(r'boundary="?([^";]+)"?', re.I)
_DISP = re.compile(r'(\w+)\*?=(?:"((?:[^"\\]|\\.)*)"|([^;]*))')


class MultipartError(ValueError):
    pass


def _parse_disposition(value: str) -> dict:
    out = {}
    for m in _DISP.finditer(value):
        k = m.group(1).lower()
        v = m.group(2) if m.group(2) is not None else (m.group(3) or "").strip()
        out[k] = v.replace('\\"', '"')
    return out


def parse_form(body: bytes, content_type: str) -> dict[str, list]:
    """-> {field_name: [str | UploadFile, ...]}"""
    m = _BOUNDARY.search(content_type or "")
    if not content_type.lower().startswith("multipart/form-data") or not m:
        raise MultipartError("not multipart/form-data")
    delim = b"--" + m.group(1).encode("latin-1")
    fields: dict[str, list] = {}
    parts = body.split(delim)
    for part in parts[1:]:
        if part.startswith(b"--"):
            break
        if part.startswith(b"\r\n"):
            part = part[2:]
        elif part.startswith(b"\n"):
            part = part[1:]
        sep = part.find(b"\r\n\r\n")
        skip = 4
        if sep < 0:
            sep, skip = part.find(b"\n\n"), 2
        if sep < 0:
            continue
        raw_headers = part[:sep].decode("latin-1")
        data = part[sep + skip:]
        if data.endswith(b"\r\n"):
            data = data[:-2]
        elif data.endswith(b"\n"):
            data = data[:-1]
        hdrs = {}
        for line in raw_headers.splitlines():
            if ":" in line:
                k, v = line.split(":", 1)
                hdrs[k.strip().lower()] = v.strip()
        disp = _parse_disposition(hdrs.get("content-disposition", ""))
        name = disp.get("name")
        if name is None:
            continue
        if "filename" in disp:
            spool = tempfile.SpooledTemporaryFile(max_size=1024 * 1024)
            spool.write(data)
            spool.seek(0)
            fname = disp["filename"]
            try:
                fname = fname.encode("latin-1").decode("utf-8")
            except (UnicodeDecodeError, UnicodeEncodeError):
                pass
            value = UploadFile(file=spool, size=len(data), filename=fname,
                               headers=Headers({k: v for k, v in hdrs.items()}))
        else:
            value = data.decode("utf-8", "replace")
        fields.setdefault(name, []).append(value)
    return fields


def missing_field_detail(name: str) -> list:
    """FastAPI's validation error entry for a missing required body field."""
    return [{"type": "missing", "loc": ["body", name], "msg": "Field required", "input": None}]
