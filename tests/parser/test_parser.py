"""Document ingestion: the reference's parser tests (tests/test_file_parser.py) plus
golden byte-equality against the parses the reference recorded in cache.db
rows 11-13 (tests/assets/golden/cache_rows.json) and format round trips."""
import asyncio
import json
import os

import pytest

from replisense_rfq_amd.service.parser import FileParser, FileParsingError, get_supported_extensions
from replisense_rfq_amd.service.prompt import EXTRACTION_PROMPT_TEMPLATE
from replisense_rfq_amd.utils import docgen, synth

GOLDEN = os.path.join(os.path.dirname(__file__), "..", "assets", "golden", "cache_rows.json")
REF_ASSETS = "/root/reference/tests/assets"


def run(coro):
    return asyncio.run(coro)


def _recorded_doc(row: int) -> str:
    rows = json.load(open(GOLDEN))
    u = rows[row - 1]["user"]
    assert u.startswith(EXTRACTION_PROMPT_TEMPLATE + '\n"""\n') and u.endswith('\n"""')
    return u[len(EXTRACTION_PROMPT_TEMPLATE) + 5:-4]


@pytest.mark.parametrize("filename,row", [("attachment.docx", 11), ("attachment.xlsx", 12),
                                          ("attachment.pdf", 13)])
def test_reference_fixtures_byte_identical(reference_root, filename, row):
    path = os.path.join(REF_ASSETS, filename)
    res = run(FileParser().parse_file_async(path))
    assert list(res) == ["raw_text", "source_file", "file_size", "file_hash", "parsing_method"]
    assert res["source_file"] == filename and res["file_size"] == os.path.getsize(path)
    assert res["parsing_method"] == "async_" + filename.rsplit(".", 1)[1]
    assert len(res["file_hash"]) == 32
    assert res["raw_text"] == _recorded_doc(row)


def test_unsupported_and_missing(tmp_path):
    p = tmp_path / "test.xyz"
    p.write_text("unsupported content")
    with pytest.raises(FileParsingError, match="Unsupported file type: .xyz"):
        run(FileParser().parse_file_async(str(p)))
    with pytest.raises(FileNotFoundError):
        run(FileParser().parse_file_async("missing-file.docx"))
    big = tmp_path / "big.txt"
    big.write_bytes(b"x" * (2 * 1024 * 1024 + 10))
    with pytest.raises(FileParsingError, match=r"File too large: 2.0MB \(max: 1.0MB\)"):
        run(FileParser(max_file_size_mb=1).parse_file_async(str(big)))
    assert get_supported_extensions() == {".txt", ".pdf", ".xlsx", ".xls", ".docx", ".csv", ".json"}


def test_text_json_csv_formats(tmp_path):
    (tmp_path / "a.txt").write_text("  hello rfq \n")
    assert run(FileParser().parse_file_async(str(tmp_path / "a.txt")))["raw_text"] == "hello rfq"
    (tmp_path / "a.json").write_text(json.dumps({"rfq": "€5", "n": [1, 2]}))
    t = run(FileParser().parse_file_async(str(tmp_path / "a.json")))["raw_text"]
    assert t == '=== JSON Data ===\n{\n  "rfq": "€5",\n  "n": [\n    1,\n    2\n  ]\n}'
    (tmp_path / "a.csv").write_text("pn;qty\nX-1;5\n")
    t = run(FileParser().parse_file_async(str(tmp_path / "a.csv")))["raw_text"]
    assert t.startswith("=== CSV Data (using utf-8, separator ';') ===\n")
    (tmp_path / "b.csv").write_text("justonecolumn\nvalue\n")
    with pytest.raises(FileParsingError, match="CSV parsing failed: Unable to parse CSV"):
        run(FileParser().parse_file_async(str(tmp_path / "b.csv")))
    (tmp_path / "bad.json").write_text("{nope")
    with pytest.raises(FileParsingError, match="Failed to parse bad.json: Invalid JSON format"):
        run(FileParser().parse_file_async(str(tmp_path / "bad.json")))


@pytest.mark.parametrize("fmt", ["pdf", "xlsx", "xls", "docx"])
def test_roundtrip_synthetic(tmp_path, fmt):
    doc = synth.make_rfq(21, n_items=3, style="formal")
    p = tmp_path / f"rfq.{fmt}"
    docgen.rfq_attachment(doc, fmt, p)
    t = run(FileParser().parse_file_async(str(p)))["raw_text"]
    for it in doc.items:
        assert it.part_number in t
    if fmt in ("xlsx", "xls"):
        assert t.startswith("=== Sheet: Sheet1 ===\n") and "Part Number" in t.splitlines()[1]
    if fmt == "pdf":
        assert t.startswith("=== Page 1 ===\nREQUEST FOR QUOTATION")
    if fmt == "docx":
        assert "\n=== Tables ===\n\n--- Table 1 ---\nPart Number | Description" in t


def test_multipage_pdf_and_empty(tmp_path):
    lines = [f"line {i}" for i in range(60)]
    docgen.write_pdf(lines, tmp_path / "m.pdf")
    t = run(FileParser().parse_file_async(str(tmp_path / "m.pdf")))["raw_text"]
    assert t.count("=== Page ") == 3 and "\n\n=== Page 2 ===\nline 26" in t
    docgen.write_pdf([], tmp_path / "e.pdf")
    t = run(FileParser().parse_file_async(str(tmp_path / "e.pdf")))["raw_text"]
    assert t == "PDF appears to be empty or contains no extractable text"


def test_pdf_metadata(reference_root):
    m = FileParser().get_pdf_metadata(os.path.join(REF_ASSETS, "attachment.pdf"))
    assert m["page_count"] == 2 and m["producer"].startswith("PyFPDF")
    assert m["is_encrypted"] is False


def test_reference_uploads_parse(reference_root):
    up = "/root/reference/uploads"
    for name in sorted(os.listdir(up)):
        res = run(FileParser().parse_file_async(os.path.join(up, name)))
        assert len(res["raw_text"]) > 10


def test_process_pool_parsing_matches_threads(tmp_path):
    """processes > 0 parses in spawned workers with byte-identical output."""
    import asyncio

    from replisense_rfq_amd.service.parser import FileParser
    from replisense_rfq_amd.utils import docgen, synth

    files = []
    for i, ext in enumerate(["pdf", "docx", "xlsx", "xls", "csv"]):
        path = tmp_path / f"doc{i}.{ext}"
        docgen.rfq_attachment(synth.make_rfq(70 + i), ext, path)
        files.append(path)

    async def parse_all(p):
        return await asyncio.gather(*(p.parse_file_async(str(f)) for f in files))

    a = asyncio.run(parse_all(FileParser()))
    pp = FileParser(processes=2)
    try:
        b = asyncio.run(parse_all(pp))
    finally:
        pp.close()
    assert [x["raw_text"] for x in a] == [x["raw_text"] for x in b]
