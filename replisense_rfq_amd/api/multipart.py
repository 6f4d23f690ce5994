"""Streaming multipart/form-data parsing without python-multipart (not installed
offline).

FastAPI's ``UploadFile = File(...)`` parameters require python-multipart at route
definition time, so the upload route streams the raw body through
:class:`MultipartStream` into Starlette ``UploadFile`` objects (spooled to disk
above 1 MiB, like Starlette).  The body is never held in memory as a whole, and a
file part is stored only up to ``max_file_bytes + 1`` bytes: past that the
response is decided already (400 for a missing name / unsupported type, else 413,
in the reference's order, app/main.py:214-227), so the rest is counted, not kept.
Only the first file part of each field name is stored at all (the route reads
``files[0]``); later ones are counted.  Starlette's limits hold for the rest:
non-file parts up to 1 MiB, at most 1,000 fields and 1,000 files
(:class:`MultipartLimitError`, answered 400 "There was an error parsing the body"
as FastAPI does for a form Starlette refuses).
Missing fields reproduce FastAPI's RequestValidationError body for
``file: UploadFile = File(...)`` (reference app/main.py:205-209).
"""
from __future__ import annotations

import re
import tempfile

from starlette.datastructures import Headers, UploadFile

_BOUNDARY = re.compile(r'boundary="?([^";]+)"?', re.I)
_DISP = re.compile(r'(\w+)\*?=(?:"((?:[^"\\]|\\.)*)"|([^;]*))')
SPOOL_BYTES = 1024 * 1024
MAX_HEADER_BYTES = 16 * 1024
MAX_PART_BYTES = 1024 * 1024       # Starlette's max_part_size for non-file parts
MAX_FIELDS = 1000                  # Starlette's max_fields / max_files
MAX_FILES = 1000


class MultipartError(ValueError):
    pass


class MultipartLimitError(MultipartError):
    """The body breaks a size / count limit (answered 400, not treated as 'no form')."""


def _parse_disposition(value: str) -> dict:
    out = {}
    for m in _DISP.finditer(value):
        k = m.group(1).lower()
        v = m.group(2) if m.group(2) is not None else (m.group(3) or "").strip()
        out[k] = v.replace('\\"', '"')
    return out


class _Part:
    def __init__(self, headers: dict, limit: int | None):
        self.headers = headers
        disp = _parse_disposition(headers.get("content-disposition", ""))
        self.name = disp.get("name")
        self.filename = disp.get("filename")
        self.is_file = "filename" in disp
        self.size = 0
        self.limit = limit
        self.sink = tempfile.SpooledTemporaryFile(max_size=SPOOL_BYTES) if self.is_file \
            else bytearray()

    def write(self, data) -> None:
        if not data:
            return
        n = len(data)
        if self.is_file:
            keep = n if self.limit is None else max(0, min(n, self.limit + 1 - self.size))
            if keep:
                self.sink.write(bytes(data[:keep]))
        else:
            if self.size + n > MAX_PART_BYTES:
                raise MultipartLimitError(
                    f"Part exceeded maximum size of {MAX_PART_BYTES // 1024}KB.")
            self.sink += data
        self.size += n

    def value(self):
        if not self.is_file:
            return bytes(self.sink).decode("utf-8", "replace")
        self.sink.seek(0)
        fname = self.filename or ""
        try:
            fname = fname.encode("latin-1").decode("utf-8")
        except (UnicodeDecodeError, UnicodeEncodeError):
            pass
        return UploadFile(file=self.sink, size=self.size, filename=fname,
                          headers=Headers(dict(self.headers)))


class MultipartStream:
    """Incremental multipart/form-data parser: ``feed(chunk)`` as the body
    arrives, ``close()`` -> {field_name: [str | UploadFile, ...]}.  Tolerates bare
    LF line endings like the reference's parser stack."""

    def __init__(self, content_type: str, max_file_bytes: int | None = None):
        m = _BOUNDARY.search(content_type or "")
        if not (content_type or "").lower().startswith("multipart/form-data") or not m:
            raise MultipartError("not multipart/form-data")
        self.delim = b"--" + m.group(1).encode("latin-1")
        self.body_delim = b"\n" + self.delim          # "\r" before it is stripped
        self.limit = max_file_bytes
        self.buf = bytearray()
        self.state = "preamble"
        self.part: _Part | None = None
        self.fields: dict[str, list] = {}
        self.nfields = self.nfiles = 0

    def _finish_part(self) -> None:
        p = self.part
        self.part = None
        if p is not None and p.name is not None:
            # a repeated field name keeps the LAST part (what Starlette's form.get()
            # hands a single-valued FastAPI parameter); the earlier part's spool is
            # closed, so repeated parts never hold more than one file's bytes
            for old in self.fields.get(p.name, []):
                if not isinstance(old, str):
                    old.file.close()
            self.fields[p.name] = [p.value()]

    def feed(self, chunk: bytes) -> None:
        self.buf += chunk
        while True:
            if self.state == "preamble":
                i = self.buf.find(self.delim)
                if i < 0:
                    keep = len(self.delim) - 1
                    if len(self.buf) > keep:
                        del self.buf[:len(self.buf) - keep]
                    return
                del self.buf[:i + len(self.delim)]
                self.state = "after_delim"
            elif self.state == "after_delim":
                if len(self.buf) < 2:
                    return
                if self.buf[:2] == b"--":
                    self.state = "done"
                    self.buf.clear()
                    return
                if self.buf[:2] == b"\r\n":
                    del self.buf[:2]
                elif self.buf[:1] == b"\n":
                    del self.buf[:1]
                self.state = "headers"
            elif self.state == "headers":
                i, skip = self.buf.find(b"\r\n\r\n"), 4
                j = self.buf.find(b"\n\n")
                if j >= 0 and (i < 0 or j < i):
                    i, skip = j, 2
                if i < 0:
                    if len(self.buf) > MAX_HEADER_BYTES:
                        raise MultipartError("part headers too large")
                    return
                hdrs = {}
                for line in bytes(self.buf[:i]).decode("latin-1").splitlines():
                    if ":" in line:
                        k, v = line.split(":", 1)
                        hdrs[k.strip().lower()] = v.strip()
                del self.buf[:i + skip]
                part = _Part(hdrs, self.limit)
                if part.is_file:
                    self.nfiles += 1
                    if self.nfiles > MAX_FILES:
                        raise MultipartLimitError(
                            f"Too many files. Maximum number of files is {MAX_FILES}.")
                else:
                    self.nfields += 1
                    if self.nfields > MAX_FIELDS:
                        raise MultipartLimitError(
                            f"Too many fields. Maximum number of fields is {MAX_FIELDS}.")
                self.part = part
                self.state = "body"
            elif self.state == "body":
                i = self.buf.find(self.body_delim)
                if i < 0:
                    safe = len(self.buf) - len(self.body_delim)
                    if safe > 0:
                        self.part.write(self.buf[:safe])
                        del self.buf[:safe]
                    return
                end = i - 1 if i > 0 and self.buf[i - 1:i] == b"\r" else i
                self.part.write(self.buf[:end])
                del self.buf[:i + len(self.body_delim)]
                self._finish_part()
                self.state = "after_delim"
            else:  # done / epilogue
                self.buf.clear()
                return

    def close(self) -> dict[str, list]:
        if self.state == "body" and self.part is not None:
            # unterminated final part: keep what arrived (lenient, like the old parser)
            self.part.write(self.buf)
            self.buf.clear()
            self._finish_part()
        return self.fields


def parse_form(body: bytes, content_type: str, max_file_bytes: int | None = None) -> dict:
    """-> {field_name: [str | UploadFile, ...]} for a complete body."""
    mp = MultipartStream(content_type, max_file_bytes)
    mp.feed(body)
    return mp.close()


def missing_field_detail(name: str) -> list:
    """FastAPI's validation error entry for a missing required body field."""
    return [{"type": "missing", "loc": ["body", name], "msg": "Field required", "input": None}]
