"""Minimal OOXML spreadsheet (.xlsx) reader -> per-sheet row grids.

The reference parses Excel with ``pd.read_excel(sheet_name=None, nrows=1000)``
(app/file_parser.py:222) through openpyxl, which is not installed here.  This
reader decodes the workbook directly (zip + XML: workbook, relationships, shared
strings, styles, sheets) and reproduces the cell values pandas' openpyxl adapter
hands to its TextParser:

  * empty cell -> ""; error -> NaN; bool -> bool; inline/shared/formula strings
    -> str;
  * numbers -> int when integral else float (pandas' ``_convert_cell``);
  * numbers whose number format is a date/time format -> ``datetime``;
  * trailing empty cells of a row and trailing empty rows trimmed, rows padded
    to the widest row (pandas' ``get_sheet_data``).

:func:`read_excel_frames` then feeds each grid to ``pandas.io.parsers.TextParser``
exactly like ``read_excel`` does, so dtype inference, header handling and
``to_string`` layout match the reference.
"""
from __future__ import annotations

import datetime as _dt
import math
import re
import zipfile
import xml.etree.ElementTree as ET

NS = {"m": "http://schemas.openxmlformats.org/spreadsheetml/2006/main",
      "r": "http://schemas.openxmlformats.org/officeDocument/2006/relationships",
      "pr": "http://schemas.openxmlformats.org/package/2006/relationships"}
_R_ID = "{http://schemas.openxmlformats.org/officeDocument/2006/relationships}id"

# built-in number formats that are dates/times (ECMA-376 §18.8.30)
_BUILTIN_DATE = set(range(14, 23)) | set(range(45, 48)) | {27, 30, 36, 50, 57}
_EPOCH_1900 = _dt.datetime(1899, 12, 30)
_EPOCH_1904 = _dt.datetime(1904, 1, 1)


def _is_date_format(code: str) -> bool:
    code = re.sub(r'"[^"]*"|\[[^\]]*\]|\\.|_.|\*.', "", code)
    return bool(re.search(r"[dmyhs]", code, re.I)) and "General" not in code


def _col_index(ref: str) -> int:
    n = 0
    for ch in ref:
        if ch.isalpha():
            n = n * 26 + (ord(ch.upper()) - 64)
        else:
            break
    return n - 1


def _text(el) -> str:
    # <si>/<is>: plain <t>, or rich text runs <r><t>..</t></r> (phonetic <rPh> skipped)
    t = el.find("m:t", NS)
    if t is not None and len(el.findall("m:r", NS)) == 0:
        return t.text or ""
    return "".join((r.text or "") for r in el.findall("m:r/m:t", NS))


class XlsxBook:
    def __init__(self, path):
        self.zf = zipfile.ZipFile(path)
        names = set(self.zf.namelist())
        wb = ET.fromstring(self.zf.read("xl/workbook.xml"))
        pr = wb.find("m:workbookPr", NS)
        self.date1904 = pr is not None and pr.get("date1904") in ("1", "true")
        rels = {}
        if "xl/_rels/workbook.xml.rels" in names:
            for r in ET.fromstring(self.zf.read("xl/_rels/workbook.xml.rels")):
                tgt = r.get("Target", "")
                tgt = tgt.lstrip("/") if tgt.startswith("/") else "xl/" + tgt
                rels[r.get("Id")] = tgt
        self.sheets = [(s.get("name"), rels.get(s.get(_R_ID)))
                       for s in wb.find("m:sheets", NS)]
        self.shared = []
        if "xl/sharedStrings.xml" in names:
            self.shared = [_text(si) for si in ET.fromstring(self.zf.read("xl/sharedStrings.xml"))
                           .findall("m:si", NS)]
        self.date_styles = set()
        if "xl/styles.xml" in names:
            st = ET.fromstring(self.zf.read("xl/styles.xml"))
            custom = {int(n.get("numFmtId")): n.get("formatCode", "")
                      for n in st.findall("m:numFmts/m:numFmt", NS)}
            xfs = st.find("m:cellXfs", NS)
            for i, xf in enumerate(xfs if xfs is not None else []):
                fid = int(xf.get("numFmtId", "0"))
                if fid in _BUILTIN_DATE or (fid in custom and _is_date_format(custom[fid])):
                    self.date_styles.add(i)

    def _number(self, v: str, style: int):
        f = float(v)
        if style in self.date_styles and not math.isnan(f):
            base = _EPOCH_1904 if self.date1904 else _EPOCH_1900
            d = base + _dt.timedelta(days=f)
            # openpyxl rounds to the microsecond; whole-second values are typical
            return d.replace(microsecond=round(d.microsecond / 1000) * 1000 % 1_000_000)
        val = int(f)
        return val if val == f else f

    def rows(self, target: str, nrows: int | None = None):
        root = ET.fromstring(self.zf.read(target))
        data = root.find("m:sheetData", NS)
        grid: list[list] = []
        last_nonempty = -1
        expect = 1
        for row in (data if data is not None else []):
            r_idx = int(row.get("r", expect))
            while expect < r_idx:                     # missing rows are empty rows
                grid.append([])
                expect += 1
            cells = {}
            col_auto = 0
            for c in row.findall("m:c", NS):
                ref = c.get("r")
                ci = _col_index(ref) if ref else col_auto
                col_auto = ci + 1
                t = c.get("t", "n")
                style = int(c.get("s", "0"))
                v = c.find("m:v", NS)
                if t == "inlineStr":
                    is_ = c.find("m:is", NS)
                    val = _text(is_) if is_ is not None else ""
                elif v is None or v.text is None:
                    val = ""
                elif t == "s":
                    val = self.shared[int(v.text)]
                elif t in ("str",):
                    val = v.text
                elif t == "b":
                    val = v.text.strip() in ("1", "true")
                elif t == "e":
                    val = float("nan")
                elif t == "d":
                    val = _dt.datetime.fromisoformat(v.text.rstrip("Z"))
                else:
                    val = self._number(v.text, style)
                cells[ci] = val
            width = (max(cells) + 1) if cells else 0
            line = [cells.get(i, "") for i in range(width)]
            while line and isinstance(line[-1], str) and line[-1] == "":
                line.pop()
            if line:
                last_nonempty = len(grid)
            grid.append(line)
            expect = r_idx + 1
            if nrows is not None and len(grid) >= nrows:
                break
        grid = grid[: last_nonempty + 1]
        if grid:
            w = max(len(r) for r in grid)
            grid = [r + [""] * (w - len(r)) for r in grid]
        return grid


def read_excel_frames(path, nrows: int = 1000):
    """{sheet_name: DataFrame} like ``pd.read_excel(path, sheet_name=None, nrows=nrows)``."""
    import pandas as pd
    from pandas.io.parsers import TextParser

    book = XlsxBook(path)
    out = {}
    for name, target in book.sheets:
        grid = book.rows(target, nrows + 1)   # header row + nrows data rows
        if not grid:
            out[name] = pd.DataFrame()
            continue
        parser = TextParser(grid, header=0, nrows=nrows)
        out[name] = parser.read()
    return out
