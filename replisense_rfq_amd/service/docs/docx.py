"""Minimal WordprocessingML (.docx) reader with python-docx's text semantics.

The reference uses python-docx (app/file_parser.py:254-286), which is not
installed here.  What it reads, and how this module mirrors it:

  * ``doc.paragraphs``: the ``w:p`` children of ``w:body`` (not paragraphs inside
    tables); ``paragraph.text`` concatenates its runs and hyperlink runs, where a
    run's text maps ``w:t`` -> text, ``w:tab``/``w:ptab`` -> "\\t", ``w:br``/``w:cr``
    (text-wrapping breaks) -> "\\n", ``w:noBreakHyphen`` -> "-";
  * ``doc.tables``: the ``w:tbl`` children of ``w:body``; ``row.cells`` repeats a
    horizontally merged cell once per grid column it spans (gridSpan) and a
    vertically merged continuation cell resolves to the cell above (vMerge);
    ``cell.text`` joins the cell's paragraphs with "\\n".
"""
from __future__ import annotations

import zipfile
import xml.etree.ElementTree as ET

W = "{http://schemas.openxmlformats.org/wordprocessingml/2006/main}"


def _run_text(r) -> str:
    out = []
    for ch in r:
        tag = ch.tag
        if tag == W + "t":
            out.append(ch.text or "")
        elif tag in (W + "tab", W + "ptab"):
            out.append("\t")
        elif tag == W + "br":
            t = ch.get(W + "type")
            out.append("\n" if t in (None, "textWrapping") else "")
        elif tag == W + "cr":
            out.append("\n")
        elif tag == W + "noBreakHyphen":
            out.append("-")
    return "".join(out)


def paragraph_text(p) -> str:
    out = []
    for ch in p:
        if ch.tag == W + "r":
            out.append(_run_text(ch))
        elif ch.tag == W + "hyperlink":
            out.extend(_run_text(r) for r in ch if r.tag == W + "r")
    return "".join(out)


def _cell_text(tc) -> str:
    return "\n".join(paragraph_text(p) for p in tc if p.tag == W + "p")


def _table_rows(tbl) -> list[list[str]]:
    rows = []
    prev: list[str] = []
    for tr in tbl.findall(W + "tr"):
        cells = []
        for tc in tr.findall(W + "tc"):
            pr = tc.find(W + "tcPr")
            span = 1
            vcont = False
            if pr is not None:
                gs = pr.find(W + "gridSpan")
                if gs is not None:
                    span = int(gs.get(W + "val", "1"))
                vm = pr.find(W + "vMerge")
                if vm is not None and vm.get(W + "val", "continue") == "continue":
                    vcont = True
            col = len(cells)
            if vcont and col < len(prev):
                text = prev[col]
            else:
                text = _cell_text(tc)
            cells.extend([text] * span)
        rows.append(cells)
        prev = cells
    return rows


class DocxDocument:
    def __init__(self, path):
        with zipfile.ZipFile(path) as zf:
            root = ET.fromstring(zf.read("word/document.xml"))
        body = root.find(W + "body")
        self.paragraphs = [paragraph_text(p) for p in body if p.tag == W + "p"]
        self.tables = [_table_rows(t) for t in body if t.tag == W + "tbl"]


def docx_to_text(path) -> str:
    """app/file_parser.py:259-282 output format."""
    doc = DocxDocument(path)
    parts = []
    paras = [p.strip() for p in doc.paragraphs if p.strip()]
    if paras:
        parts.append("=== Document Text ===")
        parts.extend(paras)
    if doc.tables:
        parts.append("\n=== Tables ===")
        for i, rows in enumerate(doc.tables, 1):
            parts.append(f"\n--- Table {i} ---")
            for row in rows:
                line = " | ".join(c.strip() for c in row)
                if line.strip():
                    parts.append(line)
    result = "\n".join(parts)
    return result if result.strip() else "DOCX file appears to be empty"
