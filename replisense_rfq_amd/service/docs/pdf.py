"""Pure-Python PDF text extraction (PyMuPDF is not available offline).

The reference extracts PDF text with PyMuPDF ``page.get_text()``, table rows with
``page.find_tables()`` and counts images with ``page.get_images()``
(app/file_parser.py:161-212).  This module re-implements what that path needs:

  * object parser (literal/hex strings, names, arrays, dicts, refs, streams),
    object streams, FlateDecode / ASCIIHex / ASCII85 / RunLength filters with
    PNG predictors, page tree with inherited resources;
  * fonts: simple fonts (WinAnsi / MacRoman / Standard encodings + Differences,
    /Widths or standard-14 metrics) and composite Type0 fonts (Identity-H two-byte
    CIDs, /W widths, /ToUnicode bfchar/bfrange CMaps);
  * a content-stream interpreter (q/Q, cm, BT/ET, Tf, Td, TD, Tm, T*, TL, Tc, Tw,
    Tz, Ts, Tj, TJ, ', ", Form XObjects) producing positioned glyphs;
  * MuPDF-style line assembly in content order: a new line when the baseline
    moves, leading blanks of a line dropped, a space inserted across horizontal
    gaps; ``get_text`` joins lines with "\\n" (validated byte-for-byte against the
    reference's recorded parse of tests/assets/attachment.pdf, cache.db row 13);
  * ``images()``: image XObjects in the page resources (``get_images``).

  * ``page_tables()``: ruled tables (``find_tables`` "lines" strategy) from the
    painted path segments and the glyph boxes the interpreter records
    (:mod:`.pdf_tables`; byte parity with PyMuPDF unpinned).
"""
from __future__ import annotations

import logging
import re
import zlib

log = logging.getLogger("replisense_rfq_amd.service.docs.pdf")

# ------------------------------------------------------------------ lexer

WS = b" \t\r\n\f\x00"
DELIM = b"()<>[]{}/%"


class Ref(tuple):
    __slots__ = ()

    def __new__(cls, num, gen):
        return tuple.__new__(cls, (num, gen))


class Name(str):
    pass


class Stream:
    def __init__(self, d: dict, raw: bytes):
        self.dict = d
        self.raw = raw


class Lexer:
    def __init__(self, data: bytes, pos: int = 0):
        self.d = data
        self.p = pos

    def skip(self):
        d, n = self.d, len(self.d)
        while self.p < n:
            c = d[self.p]
            if c in WS:
                self.p += 1
            elif c == 0x25:  # % comment
                while self.p < n and d[self.p] not in b"\r\n":
                    self.p += 1
            else:
                break

    def token(self):
        self.skip()
        d = self.d
        if self.p >= len(d):
            return None
        c = d[self.p]
        if c == 0x2F:  # /name
            self.p += 1
            s = self.p
            while self.p < len(d) and d[self.p] not in WS and d[self.p] not in DELIM:
                self.p += 1
            raw = d[s:self.p]
            raw = re.sub(rb"#([0-9A-Fa-f]{2})", lambda m: bytes([int(m.group(1), 16)]), raw)
            return Name(raw.decode("latin-1"))
        if c == 0x28:
            return self.literal()
        if c == 0x3C:
            if d[self.p:self.p + 2] == b"<<":
                self.p += 2
                return "<<"
            return self.hexstr()
        if d[self.p:self.p + 2] == b">>":
            self.p += 2
            return ">>"
        if c in b"[]{}":
            self.p += 1
            return chr(c)
        s = self.p
        while self.p < len(d) and d[self.p] not in WS and d[self.p] not in DELIM:
            self.p += 1
        w = d[s:self.p]
        if not w:
            self.p += 1
            return chr(c)
        try:
            return int(w)
        except ValueError:
            pass
        try:
            return float(w)
        except ValueError:
            return w.decode("latin-1")

    def literal(self) -> bytes:
        d = self.d
        self.p += 1
        depth = 1
        out = bytearray()
        while self.p < len(d):
            c = d[self.p]
            self.p += 1
            if c == 0x5C:  # backslash
                e = d[self.p]
                self.p += 1
                m = {0x6E: 10, 0x72: 13, 0x74: 9, 0x62: 8, 0x66: 12}
                if e in m:
                    out.append(m[e])
                elif e in b"01234567":
                    o = bytes([e])
                    while len(o) < 3 and self.p < len(d) and d[self.p] in b"01234567":
                        o += bytes([d[self.p]])
                        self.p += 1
                    out.append(int(o, 8) & 0xFF)
                elif e == 0x0D:
                    if self.p < len(d) and d[self.p] == 0x0A:
                        self.p += 1
                elif e == 0x0A:
                    pass
                else:
                    out.append(e)
            elif c == 0x28:
                depth += 1
                out.append(c)
            elif c == 0x29:
                depth -= 1
                if depth == 0:
                    break
                out.append(c)
            else:
                out.append(c)
        return bytes(out)

    def hexstr(self) -> bytes:
        e = self.d.index(b">", self.p)
        h = re.sub(rb"\s", b"", self.d[self.p + 1:e])
        self.p = e + 1
        if len(h) % 2:
            h += b"0"
        return bytes.fromhex(h.decode())

    def obj(self):
        t = self.token()
        return self.value(t)

    def value(self, t):
        if t == "<<":
            dct = {}
            while True:
                k = self.token()
                if k == ">>" or k is None:
                    break
                dct[k] = self.obj()
            return dct
        if t == "[":
            arr = []
            while True:
                tk = self.token()
                if tk == "]" or tk is None:
                    break
                arr.append(self.value(tk))
            return self._refs(arr)
        if t == "true":
            return True
        if t == "false":
            return False
        if t == "null":
            return None
        if isinstance(t, int):
            # maybe "n g R"
            save = self.p
            t2 = self.token()
            if isinstance(t2, int):
                t3 = self.token()
                if t3 == "R":
                    return Ref(t, t2)
            self.p = save
        return t

    @staticmethod
    def _refs(arr):
        return arr


# --------------------------------------------------------------- filters

def _predict(data: bytes, parms: dict) -> bytes:
    pred = parms.get("Predictor", 1) if parms else 1
    if pred < 10:
        return data
    cols = parms.get("Columns", 1)
    colors = parms.get("Colors", 1)
    bpc = parms.get("BitsPerComponent", 8)
    bpp = max(1, colors * bpc // 8)
    rowlen = (cols * colors * bpc + 7) // 8
    out = bytearray()
    prev = bytearray(rowlen)
    i = 0
    while i < len(data):
        ft = data[i]
        row = bytearray(data[i + 1:i + 1 + rowlen])
        i += 1 + rowlen
        for j in range(len(row)):
            a = row[j - bpp] if j >= bpp else 0
            b = prev[j] if j < len(prev) else 0
            c = prev[j - bpp] if j >= bpp else 0
            if ft == 1:
                row[j] = (row[j] + a) & 0xFF
            elif ft == 2:
                row[j] = (row[j] + b) & 0xFF
            elif ft == 3:
                row[j] = (row[j] + ((a + b) >> 1)) & 0xFF
            elif ft == 4:
                pa, pb, pc = abs(b - c), abs(a - c), abs(a + b - 2 * c)
                pr = a if pa <= pb and pa <= pc else (b if pb <= pc else c)
                row[j] = (row[j] + pr) & 0xFF
        out += row
        prev = row
    return bytes(out)


def _ascii85(data: bytes) -> bytes:
    import base64

    data = re.sub(rb"\s", b"", data)
    if data.startswith(b"<~"):
        data = data[2:]
    if data.endswith(b"~>"):
        data = data[:-2]
    return base64.a85decode(data)


def _runlength(data: bytes) -> bytes:
    out = bytearray()
    i = 0
    while i < len(data):
        n = data[i]
        if n == 128:
            break
        if n < 128:
            out += data[i + 1:i + 2 + n]
            i += n + 2
        else:
            out += bytes([data[i + 1]]) * (257 - n)
            i += 2
    return bytes(out)


def decode_stream(doc, s: Stream) -> bytes:
    filters = doc.resolve(s.dict.get("Filter"))
    parms = doc.resolve(s.dict.get("DecodeParms"))
    if filters is None:
        return s.raw
    if not isinstance(filters, list):
        filters, parms = [filters], [parms]
    if not isinstance(parms, list):
        parms = [parms] * len(filters)
    data = s.raw
    for f, p in zip(filters, parms):
        p = doc.resolve(p) or {}
        if f in ("FlateDecode", "Fl"):
            try:
                data = zlib.decompress(data)
            except zlib.error:
                data = zlib.decompressobj().decompress(data)
            data = _predict(data, p)
        elif f in ("ASCIIHexDecode", "AHx"):
            h = re.sub(rb"\s", b"", data).rstrip(b">")
            data = bytes.fromhex((h + (b"0" if len(h) % 2 else b"")).decode())
        elif f in ("ASCII85Decode", "A85"):
            data = _ascii85(data)
        elif f in ("RunLengthDecode", "RL"):
            data = _runlength(data)
        else:                       # image codecs etc.: not text
            return b""
    return data


# --------------------------------------------------------------- document

class PdfDocument:
    def __init__(self, data: bytes):
        self.data = data
        self.objects: dict[int, object] = {}
        self._offsets: dict[int, int] = {}
        for m in re.finditer(rb"(?<![0-9])(\d+)\s+(\d+)\s+obj\b", data):
            self._offsets[int(m.group(1))] = m.end()   # last definition wins (incremental)
        self.trailer = self._find_trailer()
        self._load_objstms()
        root = self.resolve(self.trailer.get("Root"))
        self.catalog = root if isinstance(root, dict) else {}
        self.pages = []
        pages = self.resolve(self.catalog.get("Pages"))
        if isinstance(pages, dict):
            self._walk(pages, {})

    @classmethod
    def open(cls, path):
        with open(path, "rb") as f:
            return cls(f.read())

    def _parse_at(self, pos: int):
        lx = Lexer(self.data, pos)
        o = lx.obj()
        save = lx.p
        t = lx.token()
        if t == "stream" and isinstance(o, dict):
            p = lx.p
            if self.data[p:p + 2] == b"\r\n":
                p += 2
            elif self.data[p:p + 1] in (b"\n", b"\r"):
                p += 1
            ln = o.get("Length")
            if isinstance(ln, Ref):
                ln = self.resolve(ln)
            if isinstance(ln, int) and self.data[p + ln:p + ln + 30].lstrip().startswith(b"endstream"):
                raw = self.data[p:p + ln]
            else:
                e = self.data.index(b"endstream", p)
                raw = self.data[p:e].rstrip(b"\r\n")
            return Stream(o, raw)
        lx.p = save
        return o

    def _find_trailer(self) -> dict:
        tr = {}
        for m in re.finditer(rb"trailer\s*<<", self.data):
            lx = Lexer(self.data, m.end() - 2)
            t = lx.obj()
            if isinstance(t, dict):
                tr.update({k: v for k, v in t.items() if k not in tr or k == "Root"})
        if "Root" not in tr:                      # xref streams carry the trailer dict
            for num, pos in self._offsets.items():
                try:
                    o = self._parse_at(pos)
                except Exception:
                    continue
                if isinstance(o, Stream) and o.dict.get("Type") == "XRef" and "Root" in o.dict:
                    tr.update(o.dict)
                elif isinstance(o, dict) and o.get("Type") == "Catalog" and "Root" not in tr:
                    tr["Root"] = Ref(num, 0)
        return tr

    def _load_objstms(self):
        for num, pos in list(self._offsets.items()):
            if self.data.rfind(b"/ObjStm", pos, pos + 400) < 0:
                continue
            try:
                o = self._parse_at(pos)
            except Exception:
                continue
            if not (isinstance(o, Stream) and o.dict.get("Type") == "ObjStm"):
                continue
            body = decode_stream(self, o)
            n, first = o.dict.get("N", 0), o.dict.get("First", 0)
            lx = Lexer(body)
            idx = [(lx.token(), lx.token()) for _ in range(n)]
            for onum, off in idx:
                if isinstance(onum, int) and onum not in self.objects and onum not in self._offsets:
                    self.objects[onum] = Lexer(body, first + off).obj()

    def resolve(self, o, depth: int = 0):
        while isinstance(o, Ref) and depth < 32:
            num = o[0]
            if num not in self.objects:
                pos = self._offsets.get(num)
                self.objects[num] = self._parse_at(pos) if pos is not None else None
            o = self.objects[num]
            depth += 1
        return o

    def _walk(self, node: dict, inherited: dict):
        inh = dict(inherited)
        for k in ("Resources", "MediaBox", "CropBox", "Rotate"):
            if k in node:
                inh[k] = node[k]
        if node.get("Type") == "Pages" or "Kids" in node:
            for kid in self.resolve(node.get("Kids")) or []:
                k = self.resolve(kid)
                if isinstance(k, dict):
                    self._walk(k, inh)
        else:
            page = dict(inh)
            page.update(node)
            self.pages.append(page)

    def __len__(self):
        return len(self.pages)

    @property
    def metadata(self) -> dict:
        info = self.resolve(self.trailer.get("Info")) or {}
        out = {}
        for k in ("Title", "Author", "Subject", "Keywords", "Creator", "Producer",
                  "CreationDate", "ModDate"):
            v = self.resolve(info.get(k)) if isinstance(info, dict) else None
            out[k.lower() if k not in ("CreationDate", "ModDate") else
                ("creationDate" if k == "CreationDate" else "modDate")] = \
                _pdf_text_string(v) if isinstance(v, bytes) else (v or "")
        out["format"] = "PDF " + self.data[5:8].decode("latin-1", "ignore")
        out["encryption"] = None if "Encrypt" not in self.trailer else "encrypted"
        return out

    @property
    def is_encrypted(self) -> bool:
        return "Encrypt" in self.trailer

    # ------------------------------------------------------------- pages
    def page_text(self, i: int) -> str:
        return PageText(self, self.pages[i]).text()

    def page_text_and_tables(self, i: int) -> tuple[str, list]:
        """(get_text(), find_tables() rows) of page i from one interpreter pass."""
        from .pdf_tables import extract_tables

        pt = PageText(self, self.pages[i])
        text = pt.text()
        h = pt.height()
        glyphs = [(min(x0, x1), max(x0, x1), h - (y + ASC * s), h - (y - DESC * s), h - y, s, c)
                  for x0, x1, y, s, c in pt.glyphs]
        try:               # table failures never fail the page (file_parser.py:194-196)
            return text, extract_tables(pt.segments, glyphs, h)
        except Exception as e:  # noqa: BLE001 -- like the reference (file_parser.py:194-196),
            # a table failure never fails the page: keep its text, drop its tables
            log.warning("table extraction failed on page %d: %s", i + 1, e)
            return text, []

    def page_images(self, i: int) -> list:
        res = self.resolve(self.pages[i].get("Resources")) or {}
        xo = self.resolve(res.get("XObject")) or {}
        out = []
        for name, ref in xo.items():
            s = self.resolve(ref)
            if isinstance(s, Stream) and s.dict.get("Subtype") == "Image":
                out.append((ref[0] if isinstance(ref, Ref) else 0, name))
        return out


def _pdf_text_string(b: bytes) -> str:
    if b.startswith(b"\xfe\xff"):
        return b[2:].decode("utf-16-be", "ignore")
    return b.decode("latin-1")


# ------------------------------------------------------------------ fonts

def _winansi() -> dict:
    m = {i: chr(i) for i in range(32, 127)}
    m.update({i: chr(i) for i in range(160, 256)})
    extra = {128: "€", 130: "‚", 131: "ƒ", 132: "„", 133: "…", 134: "†", 135: "‡", 136: "ˆ",
             137: "‰", 138: "Š", 139: "‹", 140: "Œ", 142: "Ž", 145: "‘", 146: "’", 147: "“",
             148: "”", 149: "•", 150: "–", 151: "—", 152: "˜", 153: "™", 154: "š", 155: "›",
             156: "œ", 158: "ž", 159: "Ÿ", 9: "\t", 10: "\n", 13: "\r"}
    m.update(extra)
    return m


WINANSI = _winansi()
MACROMAN = {i: bytes([i]).decode("mac_roman") for i in range(32, 256) if i != 127}

# glyph names commonly used in /Differences
GLYPHS = {"space": " ", "exclam": "!", "quotedbl": '"', "numbersign": "#", "dollar": "$",
          "percent": "%", "ampersand": "&", "quotesingle": "'", "quoteright": "’",
          "parenleft": "(", "parenright": ")", "asterisk": "*", "plus": "+", "comma": ",",
          "hyphen": "-", "minus": "−", "period": ".", "slash": "/", "colon": ":",
          "semicolon": ";", "less": "<", "equal": "=", "greater": ">", "question": "?",
          "at": "@", "bracketleft": "[", "backslash": "\\", "bracketright": "]",
          "asciicircum": "^", "underscore": "_", "grave": "`", "quoteleft": "‘",
          "braceleft": "{", "bar": "|", "braceright": "}", "asciitilde": "~", "bullet": "•",
          "endash": "–", "emdash": "—", "quotedblleft": "“", "quotedblright": "”",
          "Euro": "€", "fi": "fi", "fl": "fl", "ellipsis": "…", "degree": "°",
          "zero": "0", "one": "1", "two": "2", "three": "3", "four": "4", "five": "5",
          "six": "6", "seven": "7", "eight": "8", "nine": "9"}


def glyph_to_unicode(name: str) -> str:
    if name in GLYPHS:
        return GLYPHS[name]
    if len(name) == 1:
        return name
    m = re.fullmatch(r"uni([0-9A-Fa-f]{4,})", name)
    if m:
        return chr(int(m.group(1)[:4], 16))
    m = re.fullmatch(r"u([0-9A-Fa-f]{4,6})", name)
    if m:
        return chr(int(m.group(1), 16))
    return ""


# Helvetica AFM advance widths (1/1000 em) for ASCII; other standard-14 fonts use
# their family widths where they differ materially (Courier: fixed 600).
_HELV = dict(zip(" !\"#$%&'()*+,-./0123456789:;<=>?@ABCDEFGHIJKLMNOPQRSTUVWXYZ[\\]^_`"
                 "abcdefghijklmnopqrstuvwxyz{|}~",
                 [278, 278, 355, 556, 556, 889, 667, 191, 333, 333, 389, 584, 278, 333, 278,
                  278] + [556] * 10 + [278, 278, 584, 584, 584, 556, 1015, 667, 667, 722, 722,
                  667, 611, 778, 722, 278, 500, 667, 556, 833, 722, 778, 667, 778, 722, 667,
                  611, 722, 667, 944, 667, 667, 611, 278, 278, 278, 469, 556, 333, 556, 556,
                  500, 556, 556, 278, 556, 556, 222, 222, 500, 222, 833, 556, 556, 556, 556,
                  333, 500, 278, 556, 500, 722, 500, 500, 500, 334, 260, 334, 584]))


def _std_width(base: str, ch: str) -> float:
    if "Courier" in base:
        return 600
    return _HELV.get(ch, 556)


def _parse_cmap(data: bytes) -> dict:
    m: dict[int, str] = {}

    def u(h: bytes) -> str:
        b = bytes.fromhex(h.decode())
        try:
            return b.decode("utf-16-be")
        except UnicodeDecodeError:
            return ""

    for blk in re.findall(rb"beginbfchar(.*?)endbfchar", data, re.S):
        for a, b in re.findall(rb"<([0-9A-Fa-f]+)>\s*<([0-9A-Fa-f]*)>", blk):
            m[int(a, 16)] = u(b)
    for blk in re.findall(rb"beginbfrange(.*?)endbfrange", data, re.S):
        for a, b, rest in re.findall(rb"<([0-9A-Fa-f]+)>\s*<([0-9A-Fa-f]+)>\s*(\[[^\]]*\]|<[0-9A-Fa-f]*>)",
                                     blk):
            lo, hi = int(a, 16), int(b, 16)
            if rest.startswith(b"["):
                for i, h in enumerate(re.findall(rb"<([0-9A-Fa-f]*)>", rest)):
                    m[lo + i] = u(h)
            else:
                base = u(rest[1:-1])
                if base:
                    for i in range(hi - lo + 1):
                        m[lo + i] = base[:-1] + chr(ord(base[-1]) + i)
    return m


class Font:
    def __init__(self, doc: PdfDocument, fd: dict):
        self.base = str(doc.resolve(fd.get("BaseFont")) or "")
        sub = fd.get("Subtype")
        self.composite = sub == "Type0"
        self.tounicode = {}
        tu = doc.resolve(fd.get("ToUnicode"))
        if isinstance(tu, Stream):
            self.tounicode = _parse_cmap(decode_stream(doc, tu))
        self.widths: dict[int, float] = {}
        self.dw = 1000.0
        if self.composite:
            desc = doc.resolve((doc.resolve(fd.get("DescendantFonts")) or [None])[0]) or {}
            self.dw = float(desc.get("DW", 1000))
            w = doc.resolve(desc.get("W")) or []
            i = 0
            while i < len(w):
                c0 = w[i]
                nxt = doc.resolve(w[i + 1]) if i + 1 < len(w) else None
                if isinstance(nxt, list):
                    for j, x in enumerate(nxt):
                        self.widths[c0 + j] = float(doc.resolve(x))
                    i += 2
                else:
                    c1, x = w[i + 1], doc.resolve(w[i + 2])
                    for c in range(c0, c1 + 1):
                        self.widths[c] = float(x)
                    i += 3
            self.enc = {}
        else:
            first = fd.get("FirstChar", 0)
            ws = doc.resolve(fd.get("Widths"))
            if isinstance(ws, list):
                for j, x in enumerate(ws):
                    self.widths[first + j] = float(doc.resolve(x))
            enc = doc.resolve(fd.get("Encoding"))
            base_enc = WINANSI
            diffs = None
            if isinstance(enc, dict):
                if enc.get("BaseEncoding") == "MacRomanEncoding":
                    base_enc = MACROMAN
                diffs = enc.get("Differences")
            elif enc == "MacRomanEncoding":
                base_enc = MACROMAN
            self.enc = dict(base_enc)
            if diffs:
                code = 0
                for it in doc.resolve(diffs):
                    if isinstance(it, int):
                        code = it
                    else:
                        self.enc[code] = glyph_to_unicode(str(it))
                        code += 1

    def codes(self, s: bytes):
        if self.composite:
            return [(s[i] << 8) | (s[i + 1] if i + 1 < len(s) else 0) for i in range(0, len(s), 2)]
        return list(s)

    def text(self, code: int) -> str:
        if code in self.tounicode:
            return self.tounicode[code]
        if self.composite:
            return chr(code) if 32 <= code < 0xD800 else ""
        return self.enc.get(code, chr(code) if code >= 32 else "")

    def width(self, code: int) -> float:
        if code in self.widths:
            return self.widths[code]
        if self.composite:
            return self.dw
        return _std_width(self.base, self.text(code)[:1] or " ")


# ---------------------------------------------------------- page interpreter

ASC, DESC = 0.8, 0.2                      # glyph box above / below the baseline (x font size)
PAINT_OPS = {"S", "s", "f", "F", "f*", "B", "B*", "b", "b*"}


def _mul(a, b):
    return [a[0] * b[0] + a[1] * b[2], a[0] * b[1] + a[1] * b[3],
            a[2] * b[0] + a[3] * b[2], a[2] * b[1] + a[3] * b[3],
            a[4] * b[0] + a[5] * b[2] + b[4], a[4] * b[1] + a[5] * b[3] + b[5]]


class PageText:
    def __init__(self, doc: PdfDocument, page: dict):
        self.doc = doc
        self.page = page
        self.lines: list[list] = []      # [[(x0, x1, y, size, text), ...], ...]
        self.glyphs: list[tuple] = []    # every shown glyph (x0, x1, baseline y, size, ch)
        self.segments: list[tuple] = []  # painted straight path segments (x0, y0, x1, y1)
        self._fonts: dict[int, Font] = {}

    def height(self) -> float:
        box = self.doc.resolve(self.page.get("MediaBox")) or [0, 0, 612, 792]
        try:
            return float(self.doc.resolve(box[3])) - float(self.doc.resolve(box[1]))
        except (TypeError, ValueError, IndexError):
            return 792.0

    def _font(self, res: dict, name):
        fonts = self.doc.resolve(res.get("Font")) or {}
        ref = fonts.get(name)
        key = ref[0] if isinstance(ref, Ref) else id(ref)
        if key not in self._fonts:
            fd = self.doc.resolve(ref)
            self._fonts[key] = Font(self.doc, fd if isinstance(fd, dict) else {})
        return self._fonts[key]

    def text(self) -> str:
        contents = self.doc.resolve(self.page.get("Contents"))
        if isinstance(contents, list):
            data = b"\n".join(decode_stream(self.doc, self.doc.resolve(c)) for c in contents
                              if isinstance(self.doc.resolve(c), Stream))
        elif isinstance(contents, Stream):
            data = decode_stream(self.doc, contents)
        else:
            data = b""
        res = self.doc.resolve(self.page.get("Resources")) or {}
        self._run(data, res, [1, 0, 0, 1, 0, 0], 0)
        out = []
        for line in self.lines:
            s = "".join(t for *_, t in line)
            out.append(s.rstrip())
        return "\n".join(out) + ("\n" if out else "")

    def _emit(self, x0, x1, y, size, ch):
        if self.lines:
            last = self.lines[-1]
            lx0, lx1, ly, lsize, _ = last[-1]
            same_line = abs(y - ly) <= 0.5 * max(size, lsize) and x0 >= lx0 - 0.5 * size
            if same_line:
                gap = x0 - lx1
                if ch == " ":
                    if last[-1][4] != " ":
                        last.append((x0, x1, y, size, " "))
                    return
                if gap > 0.25 * size and last[-1][4] != " ":
                    last.append((lx1, x0, y, size, " "))
                last.append((x0, x1, y, size, ch))
                return
        if ch.strip() == "" and ch != "":
            return                         # blanks never start a line
        self.lines.append([(x0, x1, y, size, ch)])

    def _run(self, data: bytes, res: dict, ctm, depth: int):
        if depth > 8:
            return
        lx = Lexer(data)
        stack: list = []
        gs = []
        tm = tlm = [1, 0, 0, 1, 0, 0]
        font, fs = None, 12.0
        tc = tw = ts = 0.0
        th = 1.0
        tl = 0.0
        pending: list = []              # segments of the path under construction
        cur = start = None

        def T(x, y):
            return (ctm[0] * x + ctm[2] * y + ctm[4], ctm[1] * x + ctm[3] * y + ctm[5])

        def show(s: bytes, adj=0.0):
            nonlocal tm
            if font is None:
                return
            for code in font.codes(s):
                ch = font.text(code)
                w0 = font.width(code) / 1000.0
                trm = _mul([fs * th, 0, 0, fs, 0, ts], _mul(tm, ctm))
                x0, y0 = trm[4], trm[5]
                adv = (w0 * fs + tc + (tw if (code == 32 and not font.composite) else 0)) * th
                size = abs(fs * (tm[3] * ctm[3] + tm[1] * ctm[2])) or fs
                x1 = x0 + adv * (tm[0] * ctm[0])
                for c in ch:
                    self._emit(x0, x1, y0, size, c)
                    self.glyphs.append((x0, x1, y0, size, c))
                tm = _mul([1, 0, 0, 1, adv, 0], tm)

        while True:
            t = lx.token()
            if t is None:
                break
            if isinstance(t, (int, float, bytes, Name)) or t in ("<<", "["):
                stack.append(lx.value(t) if t in ("<<", "[") else t)
                continue
            if t in ("true", "false", "null"):
                stack.append(t)
                continue
            op = t
            try:
                if op == "m":
                    cur = start = T(float(stack[-2]), float(stack[-1]))
                elif op == "l":
                    p = T(float(stack[-2]), float(stack[-1]))
                    if cur is not None:
                        pending.append((*cur, *p))
                    cur = p
                elif op in ("c", "v", "y"):               # curves never form table edges
                    cur = T(float(stack[-2]), float(stack[-1]))
                elif op == "h":
                    if cur is not None and start is not None and cur != start:
                        pending.append((*cur, *start))
                    cur = start
                elif op == "re":
                    x, y, w, hh = (float(v) for v in stack[-4:])
                    c4 = [T(x, y), T(x + w, y), T(x + w, y + hh), T(x, y + hh)]
                    pending.extend((*c4[k], *c4[(k + 1) % 4]) for k in range(4))
                    cur = start = c4[0]
                elif op in PAINT_OPS:
                    if op in ("s", "b", "b*") and cur is not None and start is not None \
                            and cur != start:
                        pending.append((*cur, *start))
                    self.segments.extend(pending)
                    pending, cur, start = [], None, None
                elif op == "n":
                    pending, cur, start = [], None, None
                elif op == "BI":                                # inline image: skip data
                    e = data.find(b"EI", lx.p)
                    lx.p = len(data) if e < 0 else e + 2
                elif op == "q":
                    gs.append(ctm)
                elif op == "Q":
                    ctm = gs.pop() if gs else ctm
                elif op == "cm":
                    ctm = _mul([float(v) for v in stack[-6:]], ctm)
                elif op == "BT":
                    tm = tlm = [1, 0, 0, 1, 0, 0]
                elif op == "Tf":
                    font = self._font(res, stack[-2])
                    fs = float(stack[-1])
                elif op == "Tc":
                    tc = float(stack[-1])
                elif op == "Tw":
                    tw = float(stack[-1])
                elif op == "Tz":
                    th = float(stack[-1]) / 100.0
                elif op == "TL":
                    tl = float(stack[-1])
                elif op == "Ts":
                    ts = float(stack[-1])
                elif op in ("Td", "TD"):
                    tx, ty = float(stack[-2]), float(stack[-1])
                    if op == "TD":
                        tl = -ty
                    tlm = _mul([1, 0, 0, 1, tx, ty], tlm)
                    tm = tlm
                elif op == "Tm":
                    tlm = tm = [float(v) for v in stack[-6:]]
                elif op == "T*":
                    tlm = _mul([1, 0, 0, 1, 0, -tl], tlm)
                    tm = tlm
                elif op == "Tj":
                    show(stack[-1])
                elif op == "'":
                    tlm = _mul([1, 0, 0, 1, 0, -tl], tlm)
                    tm = tlm
                    show(stack[-1])
                elif op == '"':
                    tw, tc = float(stack[-3]), float(stack[-2])
                    tlm = _mul([1, 0, 0, 1, 0, -tl], tlm)
                    tm = tlm
                    show(stack[-1])
                elif op == "TJ":
                    for it in stack[-1]:
                        if isinstance(it, bytes):
                            show(it)
                        elif isinstance(it, (int, float)):
                            tm = _mul([1, 0, 0, 1, -float(it) / 1000.0 * fs * th, 0], tm)
                elif op == "Do":
                    xo = self.doc.resolve((self.doc.resolve(res.get("XObject")) or {}).get(stack[-1]))
                    if isinstance(xo, Stream) and xo.dict.get("Subtype") == "Form":
                        m = self.doc.resolve(xo.dict.get("Matrix")) or [1, 0, 0, 1, 0, 0]
                        sub = self.doc.resolve(xo.dict.get("Resources")) or res
                        self._run(decode_stream(self.doc, xo), sub, _mul(m, ctm), depth + 1)
            except (IndexError, TypeError, ValueError, KeyError):
                pass
            stack.clear()


def pdf_pages_text(path) -> list[str]:
    doc = PdfDocument.open(path)
    return [doc.page_text(i) for i in range(len(doc))]
