"""CPU document ingestion — the reference's FileParser (app/file_parser.py) rebuilt
on in-tree readers (service/docs/*: PDF, XLSX, XLS, DOCX; pandas for CSV).

Observable contract kept:
  * ``parse_file_async(path)`` -> ``{"raw_text", "source_file", "file_size",
    "file_hash" (md5), "parsing_method": "async_<ext>"}``;
  * missing file -> ``FileNotFoundError`` (not wrapped: the API answers 500);
    too large / unsupported / unreadable -> ``FileParsingError`` with the same
    messages; any error inside a format parser -> ``FileParsingError("Failed to
    parse {name}: {e}")``;
  * text formats are byte-identical to the reference's: page / sheet / table
    headers, ``"\\n\\n"`` joins, pandas ``to_string`` layouts, sentinels for
    empty documents (verified against the parses recorded in cache.db rows
    11-13 for the reference fixtures);
  * format parsers run in a 4-thread pool (file_parser.py:33) off the event loop.
The result cache stays a stub, as in the reference (file_parser.py:132-141).
"""
from __future__ import annotations

import asyncio
import hashlib
import json
import logging
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path
from typing import Any, Optional

import pandas as pd

from .docs.docx import docx_to_text
from .docs.pdf import PdfDocument
from .docs.pdf_tables import format_tables
from .docs.xls import read_xls_frames
from .docs.xlsx import read_excel_frames

log = logging.getLogger("replisense_rfq_amd.service.parser")

HAS_PDF = True          # the in-tree PDF reader is always available (reference: HAS_PYMUPDF)
SUPPORTED_EXTENSIONS = {".txt", ".pdf", ".xlsx", ".xls", ".docx", ".csv", ".json"}


class FileParsingError(Exception):
    """Domain error mapped to HTTP 422 by the API."""


def _parse_in_process(kind: str, path: str, max_excel_rows: int) -> str:
    """Process-pool entry: the document readers are pure Python, so parallel parses
    need processes, not threads (the GIL serialises them)."""
    p = FileParser.__new__(FileParser)
    p.max_excel_rows = max_excel_rows
    fn = {"pdf": p._parse_pdf_sync, "excel": p._parse_excel_sync, "docx": p._parse_docx_sync,
          "csv": p._parse_csv_sync}[kind]
    return fn(Path(path))



def _read1(path: Path) -> bytes:
    with open(path, "rb") as f:
        return f.read(1)


def _md5_file(path: Path) -> str:
    """md5 over 8 KiB chunks (file_parser.py:122-130)."""
    h = hashlib.md5()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(8192), b""):
            h.update(chunk)
    return h.hexdigest()


def _read_text(path: Path, errors: str) -> str:
    with open(path, "r", encoding="utf-8", errors=errors) as f:
        return f.read()

class FileParser:
    def __init__(self, max_file_size_mb: int = 10, max_excel_rows: int = 1000,
                 workers: int = 4, processes: int = 0):
        """workers: the reference's 4-thread pool (file_parser.py:33).  processes > 0:
        PDF/Excel/DOCX/CSV parsing runs in that many spawned processes instead, so
        concurrent uploads parse in parallel next to the engine."""
        self.max_file_size = max_file_size_mb * 1024 * 1024
        self.max_excel_rows = max_excel_rows
        self.thread_pool = ThreadPoolExecutor(max_workers=workers)
        self.processes = processes
        self._proc_pool = None
        self.supported_extensions = set(SUPPORTED_EXTENSIONS)
        log.info("FileParser initialized with max_file_size=%sMB, max_excel_rows=%s",
                 max_file_size_mb, max_excel_rows)

    # ------------------------------------------------------------ entry points
    async def parse_file_async(self, file_path: str) -> dict[str, Any]:
        file_path = Path(file_path)
        await self._validate_file_async(file_path)
        file_hash = await self._get_file_hash_async(file_path)
        cached = self._get_cached_result(file_hash)
        if cached:
            log.info("Using cached result for %s", file_path.name)
            return cached
        ext = file_path.suffix.lower()
        try:
            if ext == ".txt":
                text = await self._parse_txt_async(file_path)
            elif ext == ".pdf":
                text = await self._in_pool(self._parse_pdf_sync, file_path, "pdf")
            elif ext in (".xlsx", ".xls"):
                text = await self._in_pool(self._parse_excel_sync, file_path, "excel")
            elif ext == ".docx":
                text = await self._in_pool(self._parse_docx_sync, file_path, "docx")
            elif ext == ".csv":
                text = await self._in_pool(self._parse_csv_sync, file_path, "csv")
            elif ext == ".json":
                text = await self._parse_json_async(file_path)
            else:
                raise FileParsingError(f"Unsupported file format: {file_path.suffix}")
            result = {
                "raw_text": text,
                "source_file": str(file_path.name),
                "file_size": file_path.stat().st_size,
                "file_hash": file_hash,
                "parsing_method": f"async_{ext[1:]}",
            }
            self._cache_result(file_hash, result)
            log.info("Successfully parsed %s (%d characters)", file_path.name, len(text))
            return result
        except Exception as e:
            log.error("Error parsing %s: %s", file_path.name, e)
            raise FileParsingError(f"Failed to parse {file_path.name}: {str(e)}")

    def parse_file(self, file_path: str) -> dict[str, Any]:
        return asyncio.run(self.parse_file_async(file_path))

    async def _in_pool(self, fn, path, kind: str):
        loop = asyncio.get_running_loop()
        if self.processes > 0:
            if self._proc_pool is None:
                import multiprocessing as mp
                from concurrent.futures import ProcessPoolExecutor

                # spawn, never fork: the serving process may own a GPU context
                self._proc_pool = ProcessPoolExecutor(self.processes,
                                                      mp_context=mp.get_context("spawn"))
            return await loop.run_in_executor(self._proc_pool, _parse_in_process, kind,
                                              str(path), self.max_excel_rows)
        return await loop.run_in_executor(self.thread_pool, fn, path)

    # -------------------------------------------------------------- validation
    async def _validate_file_async(self, file_path: Path) -> None:
        if not file_path.exists():
            raise FileNotFoundError(f"File not found: {file_path}")
        size = file_path.stat().st_size
        if size > self.max_file_size:
            raise FileParsingError(
                f"File too large: {size / 1024 / 1024:.1f}MB (max: {self.max_file_size / 1024 / 1024}MB)")
        if file_path.suffix.lower() not in self.supported_extensions:
            raise FileParsingError(f"Unsupported file type: {file_path.suffix}")
        try:
            await self._io(_read1, file_path)
        except PermissionError:
            raise FileParsingError(f"Permission denied reading file: {file_path}")

    async def _io(self, fn, *args):
        """Blocking file I/O off the event loop (the reference awaits aiofiles; the
        HTTP loop here also shares its GIL slices with the engine thread)."""
        return await asyncio.get_running_loop().run_in_executor(self.thread_pool, fn, *args)

    async def _get_file_hash_async(self, file_path: Path) -> str:
        return await self._io(_md5_file, file_path)

    def _get_cached_result(self, file_hash: str) -> Optional[dict[str, Any]]:
        return None

    def _cache_result(self, file_hash: str, result: dict[str, Any]) -> None:
        pass

    # ----------------------------------------------------------------- formats
    async def _parse_txt_async(self, file_path: Path) -> str:
        return (await self._io(_read_text, file_path, "ignore")).strip()

    def _parse_pdf_sync(self, file_path: Path) -> str:
        parts = []
        try:
            doc = PdfDocument.open(file_path)
            for i in range(len(doc)):
                t, tables = doc.page_text_and_tables(i)
                if t.strip():
                    parts.append(f"=== Page {i + 1} ===\n{t.strip()}")
                parts.extend(format_tables(tables, i + 1))
                imgs = doc.page_images(i)
                if imgs:
                    parts.append(f"\n=== Images on Page {i + 1} ===\nFound {len(imgs)} image(s)")
        except Exception as e:
            log.error("PDF parsing failed for %s: %s", file_path.name, e)
            raise FileParsingError(f"PDF parsing failed: {str(e)}")
        if not parts:
            return "PDF appears to be empty or contains no extractable text"
        return "\n\n".join(parts)

    def _parse_excel_sync(self, file_path: Path) -> str:
        parts = []
        try:
            if file_path.suffix.lower() == ".xls":
                frames = read_xls_frames(file_path, nrows=self.max_excel_rows)
            else:
                frames = read_excel_frames(file_path, nrows=self.max_excel_rows)
            for name, df in frames.items():
                if df.empty:
                    continue
                text = f"=== Sheet: {name} ===\n"
                df = df.dropna(how="all").fillna("")
                text += df.to_string(index=False, max_rows=None)
                parts.append(text)
        except Exception as e:
            raise FileParsingError(f"Excel parsing failed: {str(e)}")
        if not parts:
            return "Excel file appears to be empty or unreadable"
        return "\n\n".join(parts)

    def _parse_docx_sync(self, file_path: Path) -> str:
        try:
            return docx_to_text(file_path)
        except Exception as e:
            raise FileParsingError(f"DOCX parsing failed: {str(e)}")

    def _parse_csv_sync(self, file_path: Path) -> str:
        try:
            for enc in ("utf-8", "latin-1", "cp1252"):
                for sep in (",", ";", "\t"):
                    try:
                        df = pd.read_csv(file_path, encoding=enc, sep=sep, nrows=self.max_excel_rows)
                        if len(df.columns) > 1:
                            df = df.dropna(how="all").fillna("")
                            out = f"=== CSV Data (using {enc}, separator '{sep}') ===\n"
                            return out + df.to_string(index=False, max_rows=None)
                    except Exception:
                        continue
            raise FileParsingError(
                "Unable to parse CSV with any supported encoding/separator combination")
        except Exception as e:
            raise FileParsingError(f"CSV parsing failed: {str(e)}")

    async def _parse_json_async(self, file_path: Path) -> str:
        try:
            content = await self._io(_read_text, file_path, "strict")
            data = json.loads(content)
            return f"=== JSON Data ===\n{json.dumps(data, indent=2, ensure_ascii=False)}"
        except json.JSONDecodeError as e:
            raise FileParsingError(f"Invalid JSON format: {str(e)}")
        except Exception as e:
            raise FileParsingError(f"JSON parsing failed: {str(e)}")

    # ---------------------------------------------------------------- metadata
    def get_pdf_metadata(self, file_path: str) -> dict[str, Any]:
        file_path = Path(file_path)
        try:
            doc = PdfDocument.open(file_path)
            meta = doc.metadata
            meta.update({"page_count": len(doc), "file_size": file_path.stat().st_size,
                         "is_encrypted": doc.is_encrypted, "is_pdf": True,
                         "permissions": None})
            return meta
        except Exception as e:
            raise FileParsingError(f"Failed to extract PDF metadata: {str(e)}")

    def close(self) -> None:
        if self._proc_pool is not None:
            self._proc_pool.shutdown(wait=False, cancel_futures=True)
            self._proc_pool = None

    def __del__(self):
        if hasattr(self, "thread_pool"):
            self.thread_pool.shutdown(wait=False)
        if getattr(self, "_proc_pool", None) is not None:
            self._proc_pool.shutdown(wait=False)


async def parse_file_async(file_path: str, max_file_size_mb: int = 10) -> dict[str, Any]:
    return await FileParser(max_file_size_mb=max_file_size_mb).parse_file_async(file_path)


def get_supported_extensions() -> set:
    return set(SUPPORTED_EXTENSIONS)
