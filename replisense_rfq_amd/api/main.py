"""FastAPI surface — byte-compatible with the reference app/main.py.

Routes, envelopes, status codes, detail strings and headers follow
SURVEY.md §2.1 A1-A15 / §7.4:

  GET  /                     success envelope {"status": "healthy", "version": "2.0.0"}
  GET  /health               per-service health; 503 (with a *success* envelope) if
                             a service is missing
  POST /upload/              multipart "file": 400 no filename / unsupported type,
                             413 too large, 422 parse failure, 500 generation failure;
                             data = RFQ dict + parsing_info
  POST /parse-text/          JSON {"text", "source_file"?}: 400 invalid JSON / not an
                             object / empty text, 500 generation failure
  GET  /supported-formats/   static format table
  GET  /metrics              (additive) engine counters and per-request span summary

Middleware order (outermost first): log_requests (X-Process-Time header) -> CORS ->
TrustedHost, exception handlers for HTTPException / FileParsingError / Exception
as in the reference.  The generator behind ``get_field_generator`` is the
ExtractService over the on-node engine (RFQ_BACKEND=engine, default on a GPU
host), a deterministic mock (RFQ_BACKEND=mock, BASELINE config 1) or the
recorded-completion replay (RFQ_BACKEND=replay).
"""
from __future__ import annotations

import json
import logging
import os
import tempfile
import time
import uuid
from contextlib import asynccontextmanager
from pathlib import Path
from typing import Any, Optional

from fastapi import Depends, FastAPI, HTTPException, Request
from fastapi.exceptions import RequestValidationError
from fastapi.middleware.cors import CORSMiddleware
from fastapi.middleware.trustedhost import TrustedHostMiddleware
from fastapi.responses import JSONResponse

from ..service.extract import ExtractService
from ..service.parser import FileParser, FileParsingError
from ..utils.dotenv import load_dotenv
from .multipart import (MultipartError, MultipartLimitError, MultipartStream,
                        missing_field_detail)

load_dotenv()                              # app/main.py:23 (before the constants below)
logging.basicConfig(level=logging.INFO,
                    format="%(asctime)s - %(name)s - %(levelname)s - %(message)s")
logger = logging.getLogger("replisense_rfq_amd.api")

MAX_FILE_SIZE_MB = int(os.getenv("MAX_FILE_SIZE_MB", "10"))
ALLOWED_EXTENSIONS = {".txt", ".pdf", ".xlsx", ".xls", ".docx", ".csv", ".json"}
UPLOAD_DIR = Path("./uploads")
TEMP_DIR = Path(tempfile.gettempdir()) / "rfq_processing"
TEMP_DIR.mkdir(exist_ok=True)

parser: Optional[FileParser] = None
field_generator: Optional[ExtractService] = None
_engine_handles: dict = {}
# An ExtractService built by the embedding process (bench.py's in-process HTTP phase
# serves the engine it already owns); the lifespan then builds no backend of its own.
_provided_generator: Optional[ExtractService] = None


def provide_generator(svc: Optional[ExtractService]) -> None:
    global _provided_generator
    _provided_generator = svc


def build_generator() -> ExtractService:
    """Select the inference backend (RFQ_BACKEND = engine | mock | replay), optionally
    behind the exact-request response cache (RFQ_RESPONSE_CACHE)."""
    backend = os.getenv("RFQ_BACKEND", "")
    if not backend:
        import torch

        backend = "engine" if torch.cuda.is_available() else "mock"
    svc = _build_backend(backend)
    cache_path = os.getenv("RFQ_RESPONSE_CACHE")
    if cache_path:                        # reference: ag2 diskcache, cache_seed 42
        from ..service.cache import CachedBackend, ResponseCache
        from ..utils.config import EngineConfig

        cfg = EngineConfig.from_env()
        svc.backend = CachedBackend(svc.backend, ResponseCache(cache_path), cfg.model,
                                    cfg.temperature, cfg.max_tokens)
    return svc


def _build_backend(backend: str) -> ExtractService:
    from ..service.extract import EngineBackend, MockBackend, ReplayBackend

    if backend == "mock":
        return ExtractService(MockBackend())
    if backend == "replay":
        path = os.getenv("RFQ_REPLAY_FILE",
                         str(Path(__file__).resolve().parents[2] / "tests" / "assets" / "golden"
                             / "cache_rows.json"))
        with open(path) as f:
            return ExtractService(ReplayBackend(json.load(f), MockBackend()))
    from ..engine.engine import AsyncEngine, LLMEngine
    from ..engine.router import maybe_router
    from ..utils.config import EngineConfig

    cfg = EngineConfig.from_env()
    router = maybe_router(cfg)
    if router is not None:                  # DP replicas in worker processes
        _engine_handles["router"] = router
        return ExtractService(router.backend())
    engine = LLMEngine(cfg)
    aeng = AsyncEngine(engine)
    _engine_handles.update(engine=engine, async_engine=aeng)
    return ExtractService(EngineBackend(engine, aeng))


@asynccontextmanager
async def lifespan(app: FastAPI):
    global parser, field_generator
    logger.info("Starting RFQ Processing API...")
    try:
        parser = FileParser(max_file_size_mb=MAX_FILE_SIZE_MB,
                            processes=int(os.getenv("RFQ_PARSER_PROCS", "0")))
        field_generator = _provided_generator or build_generator()
        logger.info("Services initialized successfully")
    except Exception as e:
        logger.error("Failed to initialize services: %s", e)
        raise
    yield
    logger.info("Shutting down RFQ Processing API...")
    if parser is not None:
        parser.close()
    if "async_engine" in _engine_handles:
        _engine_handles["async_engine"].shutdown()
    if "router" in _engine_handles:
        _engine_handles["router"].shutdown()
    _engine_handles.clear()


app = FastAPI(title="RFQ Processing API",
              description="API for processing RFQ documents and extracting structured data",
              version="2.0.0", lifespan=lifespan)
app.add_middleware(TrustedHostMiddleware, allowed_hosts=["*"])
app.add_middleware(CORSMiddleware, allow_origins=os.getenv("ALLOWED_ORIGINS", "*").split(","),
                   allow_credentials=True, allow_methods=["GET", "POST"], allow_headers=["*"])


# Prometheus exposition (additive: GET /metrics/prometheus).  A private registry
# keeps repeated app imports (tests) from colliding in the global one.
from prometheus_client import CollectorRegistry, Counter, Histogram  # noqa: E402
from prometheus_client import generate_latest, CONTENT_TYPE_LATEST  # noqa: E402

PROM = CollectorRegistry()
_REQS = Counter("rfq_http_requests_total", "HTTP requests", ["path", "status"], registry=PROM)
_LAT = Histogram("rfq_http_request_seconds", "HTTP request latency", ["path"], registry=PROM,
                 buckets=(0.05, 0.1, 0.2, 0.3, 0.5, 0.75, 1.0, 1.5, 2.5, 5, 10, 30))


@app.middleware("http")
async def log_requests(request: Request, call_next):
    start = time.time()
    logger.info("%s %s - Client: %s", request.method, request.url.path,
                request.client.host if request.client else "-")
    try:
        response = await call_next(request)
        dt = time.time() - start
        logger.info("%s %s - Status: %s - Duration: %.2fs", request.method, request.url.path,
                    response.status_code, dt)
        response.headers["X-Process-Time"] = str(dt)
        path = request.url.path if request.url.path in _KNOWN_PATHS else "other"
        _REQS.labels(path, str(response.status_code)).inc()
        _LAT.labels(path).observe(dt)
        return response
    except Exception as e:
        logger.error("%s %s - Error: %s - Duration: %.2fs", request.method, request.url.path,
                     e, time.time() - start)
        raise


async def get_parser() -> FileParser:
    if parser is None:
        raise HTTPException(status_code=503, detail="File parser service not initialized")
    return parser


async def get_field_generator() -> ExtractService:
    if field_generator is None:
        raise HTTPException(status_code=503, detail="RFQ field generator service not initialized")
    return field_generator


class StandardResponse:
    @staticmethod
    def success(data: Any, message: str = "Operation successful") -> dict[str, Any]:
        return {"success": True, "data": data, "message": message, "timestamp": time.time()}

    @staticmethod
    def error(error: str, details: Optional[str] = None) -> dict[str, Any]:
        return {"success": False, "error": error, "details": details, "timestamp": time.time()}


def validate_file_type(filename: str) -> bool:
    return Path(filename).suffix.lower() in ALLOWED_EXTENSIONS


def validate_file_size(file) -> bool:
    if getattr(file, "size", None):
        return file.size <= MAX_FILE_SIZE_MB * 1024 * 1024
    return True


def _copy_to(src, destination: Path) -> None:
    src.seek(0)
    with open(destination, "wb") as f:
        while chunk := src.read(1 << 20):
            f.write(chunk)


async def save_upload_file(file, destination: Path) -> None:
    """Write the upload to `destination` off the event loop (the reference streams
    8 KiB chunks through aiofiles, app/main.py:157-167); a partial file is removed."""
    import asyncio

    try:
        await asyncio.get_running_loop().run_in_executor(None, _copy_to, file.file, destination)
    except Exception:
        if destination.exists():
            destination.unlink()
        raise


async def cleanup_file(filepath: Path) -> None:
    try:
        if filepath.exists():
            filepath.unlink()
    except Exception as e:
        logger.warning("Failed to cleanup file %s: %s", filepath, e)


# ------------------------------------------------------------------ routes
@app.get("/")
async def root():
    return StandardResponse.success(data={"status": "healthy", "version": "2.0.0"},
                                    message="RFQ Processing API is running")


@app.get("/health")
async def health_check():
    status = {
        "api": "healthy",
        "file_parser": "healthy" if parser else "unhealthy",
        "field_generator": "healthy" if field_generator and field_generator.healthy
        else "unhealthy",
        "temp_dir": str(TEMP_DIR),
        "max_file_size_mb": MAX_FILE_SIZE_MB,
        "supported_extensions": list(ALLOWED_EXTENSIONS),
    }
    ok = all(status[k] == "healthy" for k in ("api", "file_parser", "field_generator"))
    return JSONResponse(status_code=200 if ok else 503,
                        content=StandardResponse.success(status, "Health check completed"))


async def _upload_file_param(request: Request):
    """Stream the request body through the incremental multipart parser: the body
    is never buffered whole and a file part is stored only up to the size limit
    (the 400/413 checks in upload_file still run in the reference's order)."""
    form = {}
    try:
        mp = MultipartStream(request.headers.get("content-type", ""),
                             max_file_bytes=MAX_FILE_SIZE_MB * 1024 * 1024)
        async for chunk in request.stream():
            mp.feed(chunk)
        form = mp.close()
    except MultipartLimitError as e:
        # FastAPI's answer to a form Starlette refuses (field / file / part limits)
        raise HTTPException(status_code=400, detail="There was an error parsing the body") from e
    except MultipartError:
        form = {}
    files = form.get("file")
    if not files:
        raise RequestValidationError(missing_field_detail("file"))
    f = files[-1]                  # the last part of that name, as Starlette's form.get()
    if isinstance(f, str):
        raise RequestValidationError([{"type": "value_error", "loc": ["body", "file"],
                                       "msg": "Value error, Expected UploadFile, received: "
                                              "<class 'str'>", "input": f, "ctx": {"error": {}}}])
    return f


@app.post("/upload/")
async def upload_file(file=Depends(_upload_file_param),
                      file_parser: FileParser = Depends(get_parser),
                      rfq_generator: ExtractService = Depends(get_field_generator)):
    if not file.filename:
        raise HTTPException(status_code=400, detail="No filename provided")
    if not validate_file_type(file.filename):
        raise HTTPException(status_code=400,
                            detail=f"Unsupported file type. Allowed: {', '.join(ALLOWED_EXTENSIONS)}")
    if not validate_file_size(file):
        raise HTTPException(status_code=413,
                            detail=f"File too large. Maximum size: {MAX_FILE_SIZE_MB}MB")
    temp_path = TEMP_DIR / f"{uuid.uuid4()}{Path(file.filename).suffix}"
    try:
        await save_upload_file(file, temp_path)
        logger.info("Saved uploaded file: %s", temp_path)
        try:
            parsed = await file_parser.parse_file_async(str(temp_path))
        except FileParsingError as e:
            logger.warning("File parsing failed for %s: %s", file.filename, e)
            raise HTTPException(status_code=422, detail=f"File parsing failed: {str(e)}")
        try:
            if hasattr(rfq_generator, "generate_async"):
                result = await rfq_generator.generate_async(raw_text=parsed["raw_text"],
                                                            source_file=file.filename)
            else:
                result = rfq_generator.generate(raw_text=parsed["raw_text"],
                                                source_file=file.filename)
        except Exception as e:
            logger.error("RFQ generation failed for %s: %s", file.filename, e)
            raise HTTPException(status_code=500, detail=f"RFQ processing failed: {str(e)}")
        result.update({"parsing_info": {
            "original_filename": file.filename,
            "file_size_bytes": parsed.get("file_size", 0),
            "parsing_method": parsed.get("parsing_method", "unknown"),
            "text_length": len(parsed["raw_text"]),
        }})
        return StandardResponse.success(data=result,
                                        message=f"Successfully processed {file.filename}")
    except HTTPException:
        raise
    except Exception as e:
        logger.error("Unexpected error processing %s: %s", file.filename, e)
        raise HTTPException(status_code=500, detail=f"Internal server error: {str(e)}")
    finally:
        await cleanup_file(temp_path)


@app.post("/parse-text/")
async def parse_text(request: Request,
                     rfq_generator: ExtractService = Depends(get_field_generator)):
    try:
        try:
            payload = await request.json()
        except Exception as e:
            raise HTTPException(status_code=400, detail=f"Invalid JSON payload: {str(e)}")
        if not isinstance(payload, dict):
            raise HTTPException(status_code=400, detail="Payload must be a JSON object")
        raw_text = payload.get("text", "")
        if not raw_text or not raw_text.strip():
            raise HTTPException(status_code=400, detail="Text field is required and cannot be empty")
        source_file = payload.get("source_file", "direct_text_input")
        try:
            if hasattr(rfq_generator, "generate_async"):
                result = await rfq_generator.generate_async(raw_text, source_file)
            else:
                result = rfq_generator.generate(raw_text, source_file)
        except Exception as e:
            logger.error("RFQ generation failed for text input: %s", e)
            raise HTTPException(status_code=500, detail=f"RFQ processing failed: {str(e)}")
        result.update({"parsing_info": {"input_type": "direct_text", "text_length": len(raw_text),
                                        "source_file": source_file}})
        return StandardResponse.success(data=result, message="Successfully processed text input")
    except HTTPException:
        raise
    except Exception as e:
        logger.error("Unexpected error processing text input: %s", e)
        raise HTTPException(status_code=500, detail=f"Internal server error: {str(e)}")


@app.get("/supported-formats/")
async def get_supported_formats():
    formats = {
        ".txt": "Plain text files",
        ".pdf": "PDF documents (with table support)",
        ".xlsx": "Excel spreadsheets (newer format)",
        ".xls": "Excel spreadsheets (legacy format)",
        ".docx": "Microsoft Word documents (with table support)",
        ".csv": "Comma-separated values",
        ".json": "JSON data files",
    }
    return StandardResponse.success(data={
        "supported_extensions": list(ALLOWED_EXTENSIONS),
        "format_descriptions": formats,
        "max_file_size_mb": MAX_FILE_SIZE_MB,
        "recommendations": [
            "For best results with PDFs, ensure text is selectable (not scanned images)",
            "Excel files will be limited to first 1000 rows per sheet",
            "Word documents will extract both text and table content",
            "Large files may take longer to process",
        ],
    }, message="Supported file formats retrieved")


@app.get("/metrics")
async def metrics():
    """Engine counters (additive route)."""
    eng = _engine_handles.get("engine")
    router = _engine_handles.get("router")
    data: dict[str, Any] = {"backend": type(getattr(field_generator, "backend", None)).__name__}
    if eng is not None:
        data["engine"] = eng.stats()
    if router is not None:
        data["router"] = router.stats()
    return StandardResponse.success(data=data, message="Metrics")


@app.get("/metrics/prometheus")
async def metrics_prometheus():
    """Prometheus text format: HTTP counters/latency + engine gauges."""
    from fastapi.responses import Response

    lines = [generate_latest(PROM).decode()]
    eng = _engine_handles.get("engine")
    stats = eng.stats() if eng is not None else {}
    router = _engine_handles.get("router")
    if router is not None:
        stats.update({f"router_{k}": v for k, v in router.stats().items()})
    for k, v in sorted(stats.items()):
        if isinstance(v, (int, float)) and not isinstance(v, bool):
            name = "rfq_engine_" + "".join(c if c.isalnum() else "_" for c in k)
            lines.append(f"# TYPE {name} gauge\n{name} {float(v)}\n")
    return Response("".join(lines), media_type=CONTENT_TYPE_LATEST)


_KNOWN_PATHS = {"/", "/health", "/upload/", "/parse-text/", "/supported-formats/", "/metrics",
                "/metrics/prometheus"}


# --------------------------------------------------------- exception handlers
@app.exception_handler(HTTPException)
async def http_exception_handler(request: Request, exc: HTTPException):
    return JSONResponse(status_code=exc.status_code,
                        content=StandardResponse.error(error=exc.detail,
                                                       details=f"{request.method} {request.url.path}"))


@app.exception_handler(FileParsingError)
async def file_parsing_exception_handler(request: Request, exc: FileParsingError):
    logger.warning("File parsing error on %s: %s", request.url.path, exc)
    return JSONResponse(status_code=422,
                        content=StandardResponse.error(error="File parsing failed", details=str(exc)))


@app.exception_handler(Exception)
async def general_exception_handler(request: Request, exc: Exception):
    logger.error("Unexpected error on %s: %s", request.url.path, exc, exc_info=True)
    return JSONResponse(status_code=500, content=StandardResponse.error(
        error="Internal server error",
        details="An unexpected error occurred. Please check the logs."))


def main():  # pragma: no cover - dev server entry (reference main.py:410-422)
    import uvicorn

    cfg = {"host": "0.0.0.0", "port": int(os.getenv("PORT", 8000)),
           "reload": os.getenv("ENVIRONMENT", "development") == "development",
           "log_level": os.getenv("LOG_LEVEL", "info").lower(), "access_log": True}
    logger.info("Starting server with config: %s", cfg)
    uvicorn.run("replisense_rfq_amd.api.main:app", **cfg)


if __name__ == "__main__":  # pragma: no cover
    main()
