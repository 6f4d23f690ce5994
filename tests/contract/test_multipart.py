"""Streaming multipart parser (api/multipart.py): chunk-boundary independence,
bounded storage of oversized file parts, and the reference's 400-before-413 order
through the API."""
import random

import pytest
from fastapi.testclient import TestClient

from replisense_rfq_amd.api.multipart import MultipartStream, parse_form

CT = "multipart/form-data; boundary=XyZ123"


def _body(parts, eol=b"\r\n"):
    out = b"preamble" + eol
    for name, filename, data in parts:
        out += b"--XyZ123" + eol
        disp = f'Content-Disposition: form-data; name="{name}"'
        if filename is not None:
            disp += f'; filename="{filename}"'
        out += disp.encode() + eol
        if filename is not None:
            out += b"Content-Type: application/octet-stream" + eol
        out += eol + data + eol
    return out + b"--XyZ123--" + eol


def _dump(form):
    out = {}
    for k, vs in form.items():
        out[k] = []
        for v in vs:
            if isinstance(v, str):
                out[k].append(v)
            else:
                v.file.seek(0)
                out[k].append((v.filename, v.size, v.file.read()))
    return out


@pytest.mark.parametrize("eol", [b"\r\n", b"\n"])
def test_chunking_does_not_change_the_result(eol):
    rng = random.Random(0)
    blob = bytes(rng.randrange(256) for _ in range(50_000)) + b"\r\n--XyZ12 not a delimiter"
    body = _body([("note", None, b"hello"), ("file", "réq.pdf", blob),
                  ("file", "b.txt", b"")], eol)
    body2 = _body([("note", None, b"hello"), ("file", "réq.pdf", blob)], eol)
    whole = _dump(parse_form(body, CT))
    assert whole["note"] == ["hello"]
    assert whole["file"] == [("b.txt", 0, b"")]         # the last part of a repeated name
    assert _dump(parse_form(body2, CT))["file"] == [("réq.pdf", len(blob), blob)]
    for trial in range(20):
        mp = MultipartStream(CT)
        i = 0
        while i < len(body):
            n = rng.choice([1, 2, 7, 64, 1000, 8192])
            mp.feed(body[i:i + n])
            i += n
        assert _dump(mp.close()) == whole


def test_oversized_part_is_counted_not_stored():
    data = b"x" * 5000
    form = parse_form(_body([("file", "a.pdf", data)]), CT, max_file_bytes=1000)
    f = form["file"][0]
    assert f.size == 5000                       # the 413 check sees the real size
    f.file.seek(0, 2)
    assert f.file.tell() == 1001                # but only limit + 1 bytes were kept


def test_api_order_400_before_413(monkeypatch):
    from replisense_rfq_amd.api import main

    from replisense_rfq_amd.service.extract import ExtractService, MockBackend
    from replisense_rfq_amd.service.parser import FileParser

    monkeypatch.setattr(main, "MAX_FILE_SIZE_MB", 1)
    # the services without running the app's startup (as test_api.py does); neither
    # is reached before the 400 / 413 checks
    monkeypatch.setitem(main.app.dependency_overrides, main.get_parser, lambda: FileParser())
    monkeypatch.setitem(main.app.dependency_overrides, main.get_field_generator,
                        lambda: ExtractService(MockBackend()))
    client = TestClient(main.app)
    big = b"a" * (1024 * 1024 + 10)
    r = client.post("/upload/", files={"file": ("doc.exe", big, "application/octet-stream")})
    assert r.status_code == 400 and r.json()["error"].startswith("Unsupported file type")
    r = client.post("/upload/", files={"file": ("doc.txt", big, "text/plain")})
    assert r.status_code == 413
    assert r.json()["error"] == "File too large. Maximum size: 1MB"


def test_limits_text_part_field_and_file_counts():
    """non-file parts are capped at 1 MiB and the field / file
    counts at 1,000 (Starlette's limits); a repeated file part replaces the earlier one
    (whose spool is closed), as Starlette's form.get() returns the last value."""
    from replisense_rfq_amd.api.multipart import MultipartLimitError

    with pytest.raises(MultipartLimitError):
        parse_form(_body([("note", None, b"y" * (1024 * 1024 + 1))]), CT)
    with pytest.raises(MultipartLimitError):
        parse_form(_body([(f"f{i}", None, b"v") for i in range(1001)]), CT)
    with pytest.raises(MultipartLimitError):
        parse_form(_body([("file", f"{i}.txt", b"v") for i in range(1001)]), CT)
    mp = MultipartStream(CT)
    mp.feed(_body([("file", "a.txt", b"first"), ("file", "b.txt", b"x" * 4096)]))
    form = mp.close()
    (last,) = form["file"]
    assert _dump({"f": [last]})["f"][0] == ("b.txt", 4096, b"x" * 4096)


def test_api_two_file_parts_uses_the_last(monkeypatch):
    """a body with two 'file' parts is processed with the LAST one (FastAPI's
    single UploadFile parameter); a text field named 'file' followed by the real upload
    no longer 422s."""
    from replisense_rfq_amd.api import main
    from replisense_rfq_amd.service.extract import ExtractService, MockBackend
    from replisense_rfq_amd.service.parser import FileParser

    monkeypatch.setitem(main.app.dependency_overrides, main.get_parser, lambda: FileParser())
    monkeypatch.setitem(main.app.dependency_overrides, main.get_field_generator,
                        lambda: ExtractService(MockBackend()))
    client = TestClient(main.app)
    body = _body([("file", "a.exe", b"nope"), ("file", "b.txt", b"Need 5 bolts")])
    r = client.post("/upload/", content=body, headers={"content-type": CT})
    assert r.status_code == 200, r.text
    assert r.json()["data"]["parsing_info"]["original_filename"] == "b.txt"
    body = _body([("file", None, b"just text"), ("file", "c.txt", b"Need 7 nuts")])
    r = client.post("/upload/", content=body, headers={"content-type": CT})
    assert r.status_code == 200, r.text
    assert r.json()["data"]["parsing_info"]["original_filename"] == "c.txt"


def test_api_oversized_text_field_is_400(monkeypatch):
    from replisense_rfq_amd.api import main
    from replisense_rfq_amd.service.extract import ExtractService, MockBackend
    from replisense_rfq_amd.service.parser import FileParser

    monkeypatch.setitem(main.app.dependency_overrides, main.get_parser, lambda: FileParser())
    monkeypatch.setitem(main.app.dependency_overrides, main.get_field_generator,
                        lambda: ExtractService(MockBackend()))
    client = TestClient(main.app)
    r = client.post("/upload/", files={"file": ("a.txt", b"hello", "text/plain")},
                    data={"note": "z" * (1024 * 1024 + 10)})
    assert r.status_code == 400
    assert r.json()["error"] == "There was an error parsing the body"
