"""API contract tests (reference tests/test_main.py scenarios + the endpoints the
reference never tested).  The generator is mocked exactly like the reference does
(AsyncMock on generate_async); no GPU, no network."""
import io
import json
import os
from unittest.mock import AsyncMock

import pytest
from fastapi.testclient import TestClient

os.environ.setdefault("RFQ_BACKEND", "mock")

from replisense_rfq_amd.api import main as api  # noqa: E402
from replisense_rfq_amd.api.main import app, get_field_generator, get_parser  # noqa: E402
from replisense_rfq_amd.service.extract import ExtractService, MockBackend  # noqa: E402
from replisense_rfq_amd.service.parser import FileParser  # noqa: E402
from replisense_rfq_amd.utils import docgen, synth  # noqa: E402

client = TestClient(app)


def mock_generator(success=True, result=None):
    gen = ExtractService(MockBackend())
    if success:
        gen.generate_async = AsyncMock(return_value=result or {
            "title": "Mock RFQ", "confidence_score": 0.9, "success": True,
            "requires_review": False, "message": "Mock success"})
    else:
        gen.generate_async = AsyncMock(side_effect=Exception("Mock LLM failure"))
    return gen


@pytest.fixture(autouse=True)
def _overrides():
    app.dependency_overrides[get_parser] = lambda: FileParser()
    yield
    app.dependency_overrides.clear()


def test_parse_text_success():
    app.dependency_overrides[get_field_generator] = lambda: mock_generator()
    r = client.post("/parse-text/", json={"text": "Mock input"})
    assert r.status_code == 200
    body = r.json()
    assert body["success"] is True and "confidence_score" in body["data"]
    assert list(body) == ["success", "data", "message", "timestamp"]
    assert body["message"] == "Successfully processed text input"
    assert body["data"]["parsing_info"] == {"input_type": "direct_text", "text_length": 10,
                                            "source_file": "direct_text_input"}
    assert "x-process-time" in r.headers
    float(r.headers["x-process-time"])


def test_parse_text_invalid_json():
    app.dependency_overrides[get_field_generator] = lambda: mock_generator()
    r = client.post("/parse-text/", content="not-json")
    assert r.status_code == 400
    body = r.json()
    assert body["success"] is False
    assert body["error"] == "Invalid JSON payload: Expecting value: line 1 column 1 (char 0)"
    assert body["details"] == "POST /parse-text/"
    assert list(body) == ["success", "error", "details", "timestamp"]


def test_parse_text_empty_text_and_non_object():
    app.dependency_overrides[get_field_generator] = lambda: mock_generator()
    r = client.post("/parse-text/", json={"text": "   "})
    assert r.status_code == 400 and "Text field is required" in r.json()["error"]
    r = client.post("/parse-text/", json=[1, 2])
    assert r.status_code == 400 and r.json()["error"] == "Payload must be a JSON object"


def test_parse_text_llm_failure():
    app.dependency_overrides[get_field_generator] = lambda: mock_generator(success=False)
    r = client.post("/parse-text/", json={"text": "Trigger failure"})
    assert r.status_code == 500
    assert r.json()["error"] == "RFQ processing failed: Mock LLM failure"


def test_generation_error_dict_is_http_200():
    # errors swallowed inside generation -> 200 with the error dict (rfq_agent.py:178-182)
    class Boom(MockBackend):
        async def acomplete(self, messages):
            raise RuntimeError("engine down")
    app.dependency_overrides[get_field_generator] = lambda: ExtractService(Boom())
    r = client.post("/parse-text/", json={"text": "hello"})
    assert r.status_code == 200
    d = r.json()["data"]
    assert list(d) == ["success", "error", "confidence_score", "requires_review",
                       "missing_fields", "source_file", "parsing_info"]
    assert d["success"] is False and d["error"] == "engine down"


def test_root_health_formats_and_defaults():
    r = client.get("/")
    assert r.status_code == 200
    assert r.json()["data"] == {"status": "healthy", "version": "2.0.0"}
    r = client.get("/supported-formats/")
    d = r.json()["data"]
    assert sorted(d["supported_extensions"]) == sorted(api.ALLOWED_EXTENSIONS)
    assert d["max_file_size_mb"] == 10 and len(d["recommendations"]) == 4
    # services not initialised (no lifespan) -> 503 with a *success* envelope
    r = client.get("/health")
    assert r.status_code == 503 and r.json()["success"] is True
    assert r.json()["data"]["field_generator"] == "unhealthy"
    # Starlette-level errors keep FastAPI's default bodies
    assert client.get("/nope").json() == {"detail": "Not Found"}
    assert client.get("/parse-text/").json() == {"detail": "Method Not Allowed"}


def test_dependency_guard_503():
    r = client.post("/parse-text/", json={"text": "x"})
    assert r.status_code == 503
    assert r.json()["error"] == "RFQ field generator service not initialized"


def test_upload_pdf_end_to_end(tmp_path):
    app.dependency_overrides[get_field_generator] = lambda: ExtractService(MockBackend())
    doc = synth.make_rfq(7, style="formal")
    data = docgen.rfq_attachment(doc, "pdf")
    r = client.post("/upload/", files={"file": ("rfq.pdf", io.BytesIO(data), "application/pdf")})
    assert r.status_code == 200, r.text
    body = r.json()
    assert body["message"] == "Successfully processed rfq.pdf"
    d = body["data"]
    assert d["source_file"] == "rfq.pdf" and d["message"] == "RFQ processed from rfq.pdf"
    pi = d["parsing_info"]
    assert pi["original_filename"] == "rfq.pdf" and pi["parsing_method"] == "async_pdf"
    assert pi["file_size_bytes"] == len(data) and pi["text_length"] > 100
    keys = list(d)
    assert keys[:3] == ["title", "client_name", "client_email"] and keys[-1] == "parsing_info"
    assert not list(api.TEMP_DIR.glob("*.pdf")), "temp file must be cleaned up"


@pytest.mark.parametrize("fmt", ["xlsx", "xls", "docx", "csv", "json", "txt"])
def test_upload_other_formats(fmt):
    app.dependency_overrides[get_field_generator] = lambda: ExtractService(MockBackend())
    data = docgen.rfq_attachment(synth.make_rfq(11), fmt)
    r = client.post("/upload/", files={"file": (f"a.{fmt}", io.BytesIO(data), "x/y")})
    assert r.status_code == 200, r.text
    assert r.json()["data"]["parsing_info"]["parsing_method"] == f"async_{fmt}"


def test_upload_errors():
    app.dependency_overrides[get_field_generator] = lambda: ExtractService(MockBackend())
    r = client.post("/upload/", files={"file": ("a.exe", io.BytesIO(b"x"), "x/y")})
    assert r.status_code == 400 and r.json()["error"].startswith("Unsupported file type. Allowed: ")
    big = b"x" * (10 * 1024 * 1024 + 1)
    r = client.post("/upload/", files={"file": ("a.txt", io.BytesIO(big), "text/plain")})
    assert r.status_code == 413 and r.json()["error"] == "File too large. Maximum size: 10MB"
    r = client.post("/upload/", files={"file": ("bad.json", io.BytesIO(b"{nope"), "x/y")})
    assert r.status_code == 422
    assert r.json()["error"].startswith("File parsing failed: Failed to parse ")
    assert "Invalid JSON format" in r.json()["error"]
    r = client.post("/upload/", data={"other": "1"})
    assert r.status_code == 422
    assert r.json()["detail"][0]["loc"] == ["body", "file"]
    app.dependency_overrides[get_field_generator] = lambda: mock_generator(success=False)
    r = client.post("/upload/", files={"file": ("a.txt", io.BytesIO(b"hello"), "text/plain")})
    assert r.status_code == 500 and r.json()["error"] == "RFQ processing failed: Mock LLM failure"


def test_cors_headers():
    r = client.options("/parse-text/", headers={"Origin": "http://x.example",
                                                 "Access-Control-Request-Method": "POST"})
    assert r.status_code == 200
    assert r.headers["access-control-allow-origin"] in ("*", "http://x.example")


def test_lifespan_with_mock_backend():
    with TestClient(app) as c:
        r = c.get("/health")
        assert r.status_code == 200
        r = c.post("/parse-text/", json={"text": "RFQ for 10 pcs of ABC-123"})
        assert r.status_code == 200 and r.json()["data"]["success"] is True
        assert c.get("/metrics").json()["data"]["backend"] == "MockBackend"


def test_server_config_env(monkeypatch):
    from replisense_rfq_amd.api.serve import server_config

    monkeypatch.setenv("PORT", "9123")
    monkeypatch.setenv("LOG_LEVEL", "DEBUG")
    monkeypatch.setenv("RFQ_BACKEND", "engine")
    c = server_config()
    assert c["port"] == 9123 and c["log_level"] == "debug" and c["reload"] is False
    monkeypatch.setenv("RFQ_BACKEND", "mock")
    assert server_config()["reload"] is True


def test_process_time_header_and_http_exception_envelope():
    r = client.get("/")
    assert float(r.headers["X-Process-Time"]) >= 0.0
    app.dependency_overrides[get_field_generator] = lambda: mock_generator()
    r = client.post("/parse-text/", json={"text": "  "})  # HTTPException -> error envelope
    assert r.status_code == 400
    body = r.json()
    assert set(body) == {"success", "error", "details", "timestamp"}
    assert body["details"] == "POST /parse-text/"


def test_prometheus_metrics():
    client.get("/")
    r = client.get("/metrics/prometheus")
    assert r.status_code == 200 and r.headers["content-type"].startswith("text/plain")
    assert 'rfq_http_requests_total{path="/",status="200"}' in r.text
    assert "rfq_http_request_seconds_bucket" in r.text
