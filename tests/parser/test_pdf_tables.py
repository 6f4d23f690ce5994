"""Ruled-table extraction in the PDF path (the reference's page.find_tables()
blocks, app/file_parser.py:183-196).  PyMuPDF is not importable here, so byte
parity with its table text is unpinned; these tests pin the in-tree detector on
generated ruled-table PDFs (m/l/S grids and stroked ``re`` cells) and the
existing fixture parse stays byte-identical (tests/parser/test_parser.py)."""
from pathlib import Path

import pytest

from replisense_rfq_amd.service.docs.pdf import PdfDocument
from replisense_rfq_amd.service.docs.pdf_tables import extract_tables
from replisense_rfq_amd.service.parser import FileParser
from replisense_rfq_amd.utils import docgen

ROWS = [["Part Number", "Description", "Qty", "Target Price"],
        ["RJF544", "RJ Field Connector, IP67", "2000", "2.85"],
        ["62IN-56T12-8S", "Circular MIL Spec", "500", ""],
        ["ACX-4015-03", "Coax Cable 3m", "1,200", "4.10"]]
HEAD = ["REQUEST FOR QUOTATION", "Please quote the items below."]
BLOCK = ("\n\n\n=== Table 1 on Page 1 ===\n"
         "Part Number | Description | Qty | Target Price\n"
         "RJF544 | RJ Field Connector, IP67 | 2000 | 2.85\n"
         "62IN-56T12-8S | Circular MIL Spec | 500 | \n"
         "ACX-4015-03 | Coax Cable 3m | 1,200 | 4.10\n")


@pytest.mark.parametrize("ruling", ["lines", "rects"])
def test_ruled_table_block(tmp_path, ruling):
    p = tmp_path / "t.pdf"
    docgen.write_pdf_table(HEAD, ROWS, p, ruling=ruling)
    text = FileParser()._parse_pdf_sync(Path(p))
    assert text.startswith("=== Page 1 ===\nREQUEST FOR QUOTATION\n")
    assert text.endswith(BLOCK)
    assert text.count("=== Table") == 1


def test_unruled_text_has_no_table(tmp_path):
    p = tmp_path / "t.pdf"
    docgen.write_pdf_table(HEAD, ROWS, p, ruling="none")
    assert "=== Table" not in FileParser()._parse_pdf_sync(Path(p))


def test_missing_cells_and_empty_rows():
    """A row with fewer cells gets None (rendered ""), an all-empty row is skipped by
    the reference's row filter."""
    h = 800.0
    seg = []
    xs, ys = [10, 110, 210], [700, 680, 660, 640]
    for y in ys:                                         # horizontal rules
        seg.append((10, y, 210, y))
    for x in (10, 210):                                  # outer verticals, all rows
        seg.append((x, 700, x, 640))
    seg.append((110, 700, 110, 680))                     # middle vertical: first row only
    seg.append((110, 660, 110, 640))                     # ... and last row
    g = lambda x, y, s: (x, x + 5 * len(s), h - (y + 8), h - (y - 2), h - y, 10.0, s)  # noqa
    glyphs = [g(15, 685, "A"), g(115, 685, "B"), g(15, 645, "C")]
    t = extract_tables(seg, glyphs, h)
    assert t == [[["A", "B"], ["", None], ["C", ""]]]
    from replisense_rfq_amd.service.docs.pdf_tables import format_tables

    assert format_tables(t, 2) == ["\n=== Table 1 on Page 2 ===\nA | B\nC | \n"]


def test_fixture_has_no_ruled_tables():
    fx = Path("/root/reference/tests/assets/attachment.pdf")      # read in place
    if not fx.exists():
        pytest.skip("fixture not present")
    doc = PdfDocument.open(fx)
    assert all(doc.page_text_and_tables(i)[1] == [] for i in range(len(doc)))


def test_pathological_grid_is_bounded():
    """table detection on untrusted uploads is bounded per page.  A
    260 x 200-line ruled grid (52,000 crossings) is skipped within a time bound; a
    dense grid under the cap (100 x 100 lines, ~10^4 cells, a glyph in each) is
    extracted with the indexed glyph lookup, also within a bound."""
    import time

    h = 800.0
    seg = [(0, float(y), 600, float(y)) for y in range(0, 780, 3)][:260]
    seg += [(float(x) * 3, 0, float(x) * 3, 780) for x in range(200)]
    t0 = time.perf_counter()
    assert extract_tables(seg, [], h) == []
    assert time.perf_counter() - t0 < 5.0
    n = 100
    seg = [(0, 7.0 * i, 7.0 * (n - 1), 7.0 * i) for i in range(n)]
    seg += [(7.0 * i, 0, 7.0 * i, 7.0 * (n - 1)) for i in range(n)]
    glyphs = [(7.0 * i + 2, 7.0 * i + 4, h - (7.0 * j + 5), h - (7.0 * j + 2), h - (7.0 * j + 2.5),
               3.0, "x") for i in range(n - 1) for j in range(n - 1)]
    t0 = time.perf_counter()
    t = extract_tables(seg, glyphs, h)
    assert time.perf_counter() - t0 < 30.0
    assert len(t) == 1 and len(t[0]) == n - 1 and all(c == "x" for c in t[0][0])


def test_pdf_set_is_multi_page_and_past_the_cap():
    """the 70B phase's fixed PDF set (BASELINE config 4, prefill-heavy)
    parses, through the service parser, to multi-page text past the 8,000-char cap of
    rfq_agent.py:147-149, so every prompt carries the full truncated document."""
    from replisense_rfq_amd.benchmarks.stream import pdf_set_requests
    from replisense_rfq_amd.service.prompt import MAX_INPUT_CHARS

    rs = pdf_set_requests(12)
    assert len(rs) == 12 and len({r["seed"] for r in rs}) == 12
    for r in rs:
        assert r["chars"] > MAX_INPUT_CHARS and r["pages"] >= 3
        assert r["messages"][1]["content"].endswith('... [truncated]\n"""')
