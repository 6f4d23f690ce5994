"""Writers for synthetic RFQ attachments: PDF, XLSX, XLS, DOCX, CSV, JSON, TXT.

Used to build upload workloads ("64 concurrent /upload/ PDF requests", BASELINE
config 3; mixed PDF/XLSX batches, config 5) and parser round-trip tests.  The PDF
writer emits the same structure PyFPDF 1.7 produces for the reference fixture
(one ``BT x y Td (text) Tj ET`` per line, Helvetica/WinAnsi, Flate streams); the
XLSX/DOCX writers emit minimal valid OOXML packages; the XLS writer emits a BIFF8
workbook inside an OLE2 compound file.
"""
from __future__ import annotations

import io
import json
import struct
import zipfile
import zlib
from xml.sax.saxutils import escape

# ------------------------------------------------------------------- PDF


def _pdf_escape(s: str) -> bytes:
    b = s.encode("cp1252", "replace")
    return b.replace(b"\\", b"\\\\").replace(b"(", b"\\(").replace(b")", b"\\)")


def write_pdf(lines: list[str], path=None, lines_per_page: int = 26, font_size: float = 12.0) -> bytes:
    pages = [lines[i:i + lines_per_page] for i in range(0, max(1, len(lines)), lines_per_page)]
    streams = []
    for pl in pages:
        ops = [b"2 J", b"0.57 w", b"BT /F1 %.2f Tf ET" % font_size]
        y = 795.17
        for ln in pl:
            ops.append(b"BT 31.19 %.2f Td (%s) Tj ET" % (y, _pdf_escape(ln)))
            y -= 28.35
        streams.append(ops)
    return _assemble(streams, path)


def write_pdf_table(lines: list[str], rows: list[list[str]], path=None, ruling: str = "lines",
                    col_widths: list[float] | None = None, font_size: float = 10.0) -> bytes:
    """One page: text lines, then a ruled table (the layout RFQ line items usually
    have).  ``ruling``: "lines" (m/l/S grid), "rects" (one stroked ``re`` per cell)
    or "none" (the same text with no ruling: no table may be detected)."""
    ncol = max(len(r) for r in rows)
    col_widths = col_widths or [530.0 / ncol] * ncol
    ops = [b"0.5 w", b"BT /F1 %.2f Tf ET" % font_size]
    y = 800.0
    for ln in lines:
        ops.append(b"BT 31.19 %.2f Td (%s) Tj ET" % (y, _pdf_escape(ln)))
        y -= 20.0
    top, rh, left = y - 10.0, 18.0, 31.19
    xs = [left]
    for w in col_widths:
        xs.append(xs[-1] + w)
    for r, row in enumerate(rows):
        base = top - (r + 1) * rh + 5.0
        for c, cell in enumerate(row):
            if cell:
                ops.append(b"BT %.2f %.2f Td (%s) Tj ET" % (xs[c] + 3.0, base, _pdf_escape(cell)))
    bottom = top - len(rows) * rh
    if ruling == "lines":
        for r in range(len(rows) + 1):
            yy = top - r * rh
            ops.append(b"%.2f %.2f m %.2f %.2f l S" % (xs[0], yy, xs[-1], yy))
        for x in xs:
            ops.append(b"%.2f %.2f m %.2f %.2f l S" % (x, top, x, bottom))
    elif ruling == "rects":
        for r in range(len(rows)):
            for c in range(ncol):
                ops.append(b"%.2f %.2f %.2f %.2f re S" % (xs[c], top - (r + 1) * rh,
                                                         col_widths[c], rh))
    return _assemble([ops], path)


def _assemble(page_ops: list[list[bytes]], path=None) -> bytes:
    objs: dict[int, bytes] = {}
    page_ids = []
    nxt = 3
    for ops in page_ops:
        pid, cid = nxt, nxt + 1
        nxt += 2
        raw = zlib.compress(b"\n".join(ops) + b"\n")
        objs[cid] = b"<</Filter /FlateDecode /Length %d>>\nstream\n%s\nendstream" % (len(raw), raw)
        objs[pid] = b"<</Type /Page\n/Parent 1 0 R\n/Resources 2 0 R\n/Contents %d 0 R>>" % cid
        page_ids.append(pid)
    font_id, info_id, cat_id = nxt, nxt + 1, nxt + 2
    kids = b" ".join(b"%d 0 R" % p for p in page_ids)
    objs[1] = b"<</Type /Pages\n/Kids [%s ]\n/Count %d\n/MediaBox [0 0 595.28 841.89]\n>>" % (
        kids, len(page_ids))
    objs[font_id] = b"<</Type /Font\n/BaseFont /Helvetica\n/Subtype /Type1\n/Encoding /WinAnsiEncoding\n>>"
    objs[2] = b"<<\n/ProcSet [/PDF /Text]\n/Font <<\n/F1 %d 0 R\n>>\n/XObject <<\n>>\n>>" % font_id
    objs[info_id] = b"<<\n/Producer (replisense_rfq_amd docgen)\n>>"
    objs[cat_id] = b"<<\n/Type /Catalog\n/Pages 1 0 R\n>>"
    out = io.BytesIO()
    out.write(b"%PDF-1.3\n")
    offs = {}
    for n in sorted(objs):
        offs[n] = out.tell()
        out.write(b"%d 0 obj\n%s\nendobj\n" % (n, objs[n]))
    xref = out.tell()
    size = max(objs) + 1
    out.write(b"xref\n0 %d\n0000000000 65535 f \n" % size)
    for n in range(1, size):
        out.write(b"%010d 00000 n \n" % offs.get(n, 0))
    out.write(b"trailer\n<<\n/Size %d\n/Root %d 0 R\n/Info %d 0 R\n>>\nstartxref\n%d\n%%%%EOF\n" % (
        size, cat_id, info_id, xref))
    data = out.getvalue()
    if path:
        with open(path, "wb") as f:
            f.write(data)
    return data


# ------------------------------------------------------------------ XLSX

def _col(i: int) -> str:
    s = ""
    i += 1
    while i:
        i, r = divmod(i - 1, 26)
        s = chr(65 + r) + s
    return s


def write_xlsx(sheets: dict[str, list[list]], path=None) -> bytes:
    shared: list[str] = []
    sidx: dict[str, int] = {}
    sheet_xml = []
    for rows in sheets.values():
        out = ['<?xml version="1.0" encoding="UTF-8" standalone="yes"?>'
               '<worksheet xmlns="http://schemas.openxmlformats.org/spreadsheetml/2006/main">'
               "<sheetData>"]
        for r, row in enumerate(rows, 1):
            out.append(f'<row r="{r}">')
            for c, v in enumerate(row):
                ref = f"{_col(c)}{r}"
                if v is None or v == "":
                    continue
                if isinstance(v, bool):
                    out.append(f'<c r="{ref}" t="b"><v>{int(v)}</v></c>')
                elif isinstance(v, (int, float)):
                    out.append(f'<c r="{ref}"><v>{float(v)!r}</v></c>')
                else:
                    s = str(v)
                    if s not in sidx:
                        sidx[s] = len(shared)
                        shared.append(s)
                    out.append(f'<c r="{ref}" t="s"><v>{sidx[s]}</v></c>')
            out.append("</row>")
        out.append("</sheetData></worksheet>")
        sheet_xml.append("".join(out))
    names = list(sheets)
    wb = ('<?xml version="1.0" encoding="UTF-8" standalone="yes"?>'
          '<workbook xmlns="http://schemas.openxmlformats.org/spreadsheetml/2006/main" '
          'xmlns:r="http://schemas.openxmlformats.org/officeDocument/2006/relationships"><sheets>'
          + "".join(f'<sheet name="{escape(n)}" sheetId="{i + 1}" r:id="rId{i + 1}"/>'
                    for i, n in enumerate(names)) + "</sheets></workbook>")
    rels = ('<?xml version="1.0" encoding="UTF-8" standalone="yes"?>'
            '<Relationships xmlns="http://schemas.openxmlformats.org/package/2006/relationships">'
            + "".join(f'<Relationship Id="rId{i + 1}" Type="http://schemas.openxmlformats.org/'
                      f'officeDocument/2006/relationships/worksheet" Target="worksheets/sheet{i + 1}.xml"/>'
                      for i in range(len(names))) + "</Relationships>")
    sst = ('<?xml version="1.0" encoding="UTF-8" standalone="yes"?>'
           f'<sst xmlns="http://schemas.openxmlformats.org/spreadsheetml/2006/main" count="{len(shared)}" '
           f'uniqueCount="{len(shared)}">' + "".join(f"<si><t>{escape(s)}</t></si>" for s in shared)
           + "</sst>")
    ct = ('<?xml version="1.0" encoding="UTF-8" standalone="yes"?>'
          '<Types xmlns="http://schemas.openxmlformats.org/package/2006/content-types">'
          '<Default Extension="rels" ContentType="application/vnd.openxmlformats-package.relationships+xml"/>'
          '<Default Extension="xml" ContentType="application/xml"/>'
          '<Override PartName="/xl/workbook.xml" ContentType="application/vnd.openxmlformats-officedocument.spreadsheetml.sheet.main+xml"/>'
          + "".join(f'<Override PartName="/xl/worksheets/sheet{i + 1}.xml" ContentType="application/'
                    f'vnd.openxmlformats-officedocument.spreadsheetml.worksheet+xml"/>'
                    for i in range(len(names))) + "</Types>")
    buf = io.BytesIO()
    with zipfile.ZipFile(buf, "w", zipfile.ZIP_DEFLATED) as z:
        z.writestr("[Content_Types].xml", ct)
        z.writestr("xl/workbook.xml", wb)
        z.writestr("xl/_rels/workbook.xml.rels", rels)
        z.writestr("xl/sharedStrings.xml", sst)
        for i, x in enumerate(sheet_xml):
            z.writestr(f"xl/worksheets/sheet{i + 1}.xml", x)
    data = buf.getvalue()
    if path:
        with open(path, "wb") as f:
            f.write(data)
    return data


# ------------------------------------------------------------------ DOCX

def write_docx(paragraphs: list[str], tables: list[list[list[str]]] | None = None,
               path=None) -> bytes:
    W = 'xmlns:w="http://schemas.openxmlformats.org/wordprocessingml/2006/main"'

    def p(t):
        return f'<w:p><w:r><w:t xml:space="preserve">{escape(t)}</w:t></w:r></w:p>'

    body = "".join(p(t) for t in paragraphs)
    for tb in tables or []:
        body += "<w:tbl>" + "".join(
            "<w:tr>" + "".join(f"<w:tc>{p(c)}</w:tc>" for c in row) + "</w:tr>" for row in tb
        ) + "</w:tbl>"
    doc = (f'<?xml version="1.0" encoding="UTF-8" standalone="yes"?><w:document {W}>'
           f"<w:body>{body}</w:body></w:document>")
    ct = ('<?xml version="1.0" encoding="UTF-8" standalone="yes"?>'
          '<Types xmlns="http://schemas.openxmlformats.org/package/2006/content-types">'
          '<Default Extension="xml" ContentType="application/xml"/>'
          '<Override PartName="/word/document.xml" ContentType="application/vnd.openxmlformats-'
          'officedocument.wordprocessingml.document.main+xml"/></Types>')
    buf = io.BytesIO()
    with zipfile.ZipFile(buf, "w", zipfile.ZIP_DEFLATED) as z:
        z.writestr("[Content_Types].xml", ct)
        z.writestr("word/document.xml", doc)
    data = buf.getvalue()
    if path:
        with open(path, "wb") as f:
            f.write(data)
    return data


# ------------------------------------------------------------------- XLS

def _biff(rt: int, body: bytes) -> bytes:
    return struct.pack("<HH", rt, len(body)) + body


def _xlstr(s: str, len16=True) -> bytes:
    try:
        raw, flag = s.encode("latin-1"), 0
    except UnicodeEncodeError:
        raw, flag = s.encode("utf-16-le"), 1
    n = len(s)
    return (struct.pack("<H", n) if len16 else struct.pack("<B", n)) + bytes([flag]) + raw


def write_xls(sheets: dict[str, list[list]], path=None) -> bytes:
    """BIFF8 workbook (LABEL / NUMBER cells) in an OLE2 container."""
    bof = lambda t: _biff(0x0809, struct.pack("<HHHHII", 0x0600, t, 0x0DBB, 1997, 0, 0x0600))  # noqa
    xfs = b"".join(_biff(0x00E0, struct.pack("<HHHBBBBIIH", 0, 0, 0xFFF5 if i < 15 else 0x0001,
                                               0x20, 0, 0, 0, 0, 0, 0x20C0)) for i in range(16))
    glob_head = bof(5) + _biff(0x0022, struct.pack("<H", 0)) + xfs
    sheet_streams = []
    for rows in sheets.values():
        recs = [bof(0x10)]
        for r, row in enumerate(rows):
            for c, v in enumerate(row):
                if v is None or v == "":
                    continue
                if isinstance(v, (int, float)) and not isinstance(v, bool):
                    recs.append(_biff(0x0203, struct.pack("<HHHd", r, c, 15, float(v))))
                else:
                    recs.append(_biff(0x0204, struct.pack("<HHH", r, c, 15) + _xlstr(str(v))))
        recs.append(_biff(0x000A, b""))
        sheet_streams.append(b"".join(recs))
    names = list(sheets)
    bs_len = sum(len(_biff(0x0085, struct.pack("<IBB", 0, 0, 0) + _xlstr(n, False))) for n in names)
    off = len(glob_head) + bs_len + 4
    bsheets = b""
    for n, st in zip(names, sheet_streams):
        bsheets += _biff(0x0085, struct.pack("<IBB", off, 0, 0) + _xlstr(n, False))
        off += len(st)
    wb = glob_head + bsheets + _biff(0x000A, b"") + b"".join(sheet_streams)
    # ---- OLE2: 512-B sectors, stream padded to >= 4096 (normal FAT storage)
    if len(wb) < 4096:
        wb = wb + b"\x00" * (4096 - len(wb))
    ssz = 512
    n_ws = (len(wb) + ssz - 1) // ssz
    stream = wb + b"\x00" * (n_ws * ssz - len(wb))
    n_dir = 1
    total = n_ws + n_dir
    n_fat = 1
    while n_fat * (ssz // 4) < total + n_fat:
        n_fat += 1
    fat = []
    for i in range(n_ws):                       # workbook chain: sectors 0..n_ws-1
        fat.append(i + 1 if i + 1 < n_ws else 0xFFFFFFFE)
    fat.append(0xFFFFFFFE)                      # directory sector
    fat += [0xFFFFFFFD] * n_fat                 # FAT sectors
    fat += [0xFFFFFFFF] * (n_fat * (ssz // 4) - len(fat))
    dir_sector = n_ws
    fat_start = n_ws + 1

    def dent(name, etype, start, size, child=0xFFFFFFFF):
        nm = name.encode("utf-16-le") + b"\x00\x00"
        e = nm + b"\x00" * (64 - len(nm))
        e += struct.pack("<HBB", len(nm), etype, 1)
        e += struct.pack("<III", 0xFFFFFFFF, 0xFFFFFFFF, child)
        e += b"\x00" * 16 + struct.pack("<I", 0) + b"\x00" * 16
        e += struct.pack("<IQ", start, size)
        return e

    dirs = dent("Root Entry", 5, 0xFFFFFFFE, 0, child=1) + dent("Workbook", 2, 0, len(wb))
    dirs += b"\x00" * (ssz - len(dirs))
    hdr = bytearray(512)
    hdr[:8] = _OLE_MAGIC_W
    struct.pack_into("<HHHHH", hdr, 24, 0x3E, 3, 0xFFFE, 9, 6)
    struct.pack_into("<I", hdr, 44, n_fat)
    struct.pack_into("<I", hdr, 48, dir_sector)
    struct.pack_into("<I", hdr, 56, 4096)
    struct.pack_into("<IIII", hdr, 60, 0xFFFFFFFE, 0, 0xFFFFFFFE, 0)
    difat = [fat_start + i for i in range(n_fat)] + [0xFFFFFFFF] * (109 - n_fat)
    struct.pack_into("<109I", hdr, 76, *difat)
    data = bytes(hdr) + stream + dirs + struct.pack(f"<{len(fat)}I", *fat)
    if path:
        with open(path, "wb") as f:
            f.write(data)
    return data


_OLE_MAGIC_W = b"\xd0\xcf\x11\xe0\xa1\xb1\x1a\xe1"


# ------------------------------------------------------------ RFQ attachments

def rfq_attachment(doc, fmt: str, path=None) -> bytes:
    """Render a synth.RFQDoc as an attachment of the given extension."""
    fmt = fmt.lstrip(".").lower()
    header = ["Part Number", "Description", "Quantity", "Target Price"]
    rows = [header] + [[it.part_number, it.description, it.quantity,
                        it.target_price if it.target_price is not None else ""]
                       for it in doc.items]
    if fmt == "pdf":
        return write_pdf(doc.text.splitlines(), path)
    if fmt == "xlsx":
        return write_xlsx({"Sheet1": rows}, path)
    if fmt == "xls":
        return write_xls({"Sheet1": rows}, path)
    if fmt == "docx":
        return write_docx(doc.text.splitlines(), [[[str(c) for c in r] for r in rows]], path)
    if fmt == "csv":
        import csv
        import io

        buf = io.StringIO()
        csv.writer(buf, lineterminator="\n").writerows(rows)
        data = buf.getvalue().encode()
    elif fmt == "json":
        data = json.dumps({"rfq": doc.text, "items": rows[1:]}).encode()
    else:
        data = doc.text.encode()
    if path:
        with open(path, "wb") as f:
            f.write(data)
    return data
