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
