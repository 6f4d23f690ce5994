"""Minimal legacy Excel (.xls, BIFF8 inside an OLE2 compound file) reader.

The reference reads .xls via ``pd.read_excel`` + xlrd (app/file_parser.py:214-252);
xlrd is not installed here.  This decodes the compound-file FAT/mini-FAT chains,
finds the Workbook stream and walks BIFF8 records: BOUNDSHEET, SST (+CONTINUE),
LABELSST, LABEL, NUMBER, RK, MULRK, FORMULA (+STRING), BOOLERR, FORMAT, XF,
DATEMODE.  Cell values are converted like pandas' xlrd adapter (numbers -> int
when integral, date-formatted numbers -> datetime, errors -> NaN), rows are
padded to the sheet's data width, and :func:`read_xls_frames` hands the grid to
``pandas.io.parsers.TextParser`` exactly as ``read_excel`` does.
"""
from __future__ import annotations

import datetime as _dt
import math
import struct

from .xlsx import _BUILTIN_DATE, _is_date_format

_OLE_MAGIC = b"\xd0\xcf\x11\xe0\xa1\xb1\x1a\xe1"
ENDOFCHAIN, FREESECT = 0xFFFFFFFE, 0xFFFFFFFF


class OleFile:
    def __init__(self, data: bytes):
        if data[:8] != _OLE_MAGIC:
            raise ValueError("not an OLE2 compound file")
        self.d = data
        ssz = 1 << struct.unpack_from("<H", data, 30)[0]
        mssz = 1 << struct.unpack_from("<H", data, 32)[0]
        n_fat, dir_start = struct.unpack_from("<II", data, 44)
        self.cutoff = struct.unpack_from("<I", data, 56)[0]
        mfat_start, n_mfat, difat_start, n_difat = struct.unpack_from("<IIII", data, 60)
        self.ssz, self.mssz = ssz, mssz
        difat = list(struct.unpack_from("<109I", data, 76))
        s = difat_start
        for _ in range(n_difat):
            if s >= ENDOFCHAIN:
                break
            vals = struct.unpack_from(f"<{ssz // 4}I", self._sector(s))
            difat += vals[:-1]
            s = vals[-1]
        self.fat = []
        for fs in difat[:n_fat]:
            if fs >= ENDOFCHAIN:
                continue
            self.fat += struct.unpack_from(f"<{ssz // 4}I", self._sector(fs))
        dir_data = self._chain(dir_start)
        self.entries = []
        for i in range(0, len(dir_data), 128):
            e = dir_data[i:i + 128]
            nlen = struct.unpack_from("<H", e, 64)[0]
            name = e[:max(0, nlen - 2)].decode("utf-16-le", "ignore")
            etype = e[66]
            start, size = struct.unpack_from("<IQ", e, 116)
            self.entries.append((name, etype, start, size & 0xFFFFFFFF))
        root = self.entries[0]
        self.ministream = self._chain(root[2])[: root[3]] if root[1] == 5 else b""
        self.minifat = list(struct.unpack_from(f"<{(n_mfat * ssz) // 4}I", self._chain(mfat_start))) \
            if n_mfat and mfat_start < ENDOFCHAIN else []

    def _sector(self, i: int) -> bytes:
        o = (i + 1) * self.ssz
        return self.d[o:o + self.ssz]

    def _chain(self, start: int) -> bytes:
        out, s, guard = [], start, 0
        while s < ENDOFCHAIN and s < len(self.fat) + 1 and guard < 1 << 22:
            out.append(self._sector(s))
            s = self.fat[s] if s < len(self.fat) else ENDOFCHAIN
            guard += 1
        return b"".join(out)

    def stream(self, name: str) -> bytes | None:
        for n, t, start, size in self.entries:
            if t == 2 and n.lower() == name.lower():
                if size < self.cutoff and self.minifat:
                    out, s = [], start
                    while s < ENDOFCHAIN and s < len(self.minifat):
                        o = s * self.mssz
                        out.append(self.ministream[o:o + self.mssz])
                        s = self.minifat[s]
                    return b"".join(out)[:size]
                return self._chain(start)[:size]
        return None


def _rk(v: int) -> float:
    if v & 2:
        x = float(v >> 2 if not (v & 0x80000000) else (v >> 2) - (1 << 30))
    else:
        x = struct.unpack("<d", struct.pack("<Q", (v & 0xFFFFFFFC) << 32))[0]
    return x / 100.0 if v & 1 else x


class _Reader:
    """Byte reader over a record payload that can continue into CONTINUE records."""

    def __init__(self, chunks: list[bytes]):
        self.chunks = chunks
        self.ci = 0
        self.p = 0

    def _need(self):
        if self.p >= len(self.chunks[self.ci]) and self.ci + 1 < len(self.chunks):
            self.ci += 1
            self.p = 0
            return True
        return False

    def u8(self):
        self._need()
        v = self.chunks[self.ci][self.p]
        self.p += 1
        return v

    def u16(self):
        return self.u8() | (self.u8() << 8)

    def u32(self):
        return self.u16() | (self.u16() << 16)

    def skip(self, n):
        for _ in range(n):
            self.u8()

    def chars(self, n: int, wide: bool) -> str:
        out = []
        while n > 0:
            if self._need():                      # string split: new option byte
                wide = bool(self.u8() & 1)
            c = self.chunks[self.ci]
            avail = (len(c) - self.p) // (2 if wide else 1)
            k = min(n, max(avail, 0))
            if k == 0:
                if self.ci + 1 >= len(self.chunks):
                    break
                self.p = len(c)
                continue
            if wide:
                out.append(c[self.p:self.p + 2 * k].decode("utf-16-le", "replace"))
                self.p += 2 * k
            else:
                out.append(c[self.p:self.p + k].decode("latin-1"))
                self.p += k
            n -= k
        return "".join(out)

    def xlstring(self, len16: bool = True) -> str:
        n = self.u16() if len16 else self.u8()
        flags = self.u8()
        rich = self.u16() if flags & 8 else 0
        ext = self.u32() if flags & 4 else 0
        s = self.chars(n, bool(flags & 1))
        self.skip(4 * rich + ext)
        return s


class XlsBook:
    def __init__(self, path):
        with open(path, "rb") as f:
            ole = OleFile(f.read())
        wb = ole.stream("Workbook") or ole.stream("Book")
        if wb is None:
            raise ValueError("no Workbook stream")
        self.data = wb
        self.sheets: list[tuple[str, int]] = []
        self.sst: list[str] = []
        self.formats: dict[int, str] = {}
        self.xf_fmt: list[int] = []
        self.date1904 = False
        self._globals()

    def _records(self, pos: int):
        d = self.data
        while pos + 4 <= len(d):
            rt, ln = struct.unpack_from("<HH", d, pos)
            yield pos, rt, d[pos + 4:pos + 4 + ln]
            pos += 4 + ln

    def _with_continue(self, it, first: bytes) -> list[bytes]:
        chunks = [first]
        return chunks

    def _globals(self):
        recs = list(self._records(0))
        i = 0
        while i < len(recs):
            pos, rt, body = recs[i]
            if rt == 0x0085:                                    # BOUNDSHEET
                off = struct.unpack_from("<I", body, 0)[0]
                kind = body[5]
                r = _Reader([body[6:]])
                name = r.xlstring(len16=False)
                if kind == 0:
                    self.sheets.append((name, off))
            elif rt == 0x00FC:                                  # SST + CONTINUEs
                chunks = [body[8:]]
                j = i + 1
                while j < len(recs) and recs[j][1] == 0x003C:
                    chunks.append(recs[j][2])
                    j += 1
                n = struct.unpack_from("<I", body, 4)[0]
                r = _Reader(chunks)
                try:
                    for _ in range(n):
                        self.sst.append(r.xlstring())
                except IndexError:
                    pass
                i = j - 1
            elif rt == 0x041E:                                  # FORMAT
                ifmt = struct.unpack_from("<H", body, 0)[0]
                self.formats[ifmt] = _Reader([body[2:]]).xlstring()
            elif rt == 0x00E0:                                  # XF
                self.xf_fmt.append(struct.unpack_from("<H", body, 2)[0])
            elif rt == 0x0022:                                  # DATEMODE
                self.date1904 = struct.unpack_from("<H", body, 0)[0] == 1
            elif rt == 0x000A:                                  # EOF of globals
                break
            i += 1

    def _is_date(self, xf: int) -> bool:
        if xf >= len(self.xf_fmt):
            return False
        f = self.xf_fmt[xf]
        return f in _BUILTIN_DATE or (f in self.formats and _is_date_format(self.formats[f]))

    def _num(self, v: float, xf: int):
        if self._is_date(xf) and not math.isnan(v):
            base = _dt.datetime(1904, 1, 1) if self.date1904 else _dt.datetime(1899, 12, 30)
            return base + _dt.timedelta(days=v)
        iv = int(v)
        return iv if iv == v else v

    def rows(self, offset: int, nrows: int | None = None):
        cells: dict[tuple[int, int], object] = {}
        pending_str = None
        for pos, rt, b in self._records(offset):
            if rt == 0x000A:
                break
            if rt == 0x00FD:
                r, c, xf, k = struct.unpack_from("<HHHI", b, 0)
                cells[(r, c)] = self.sst[k] if k < len(self.sst) else ""
            elif rt == 0x0204:
                r, c, xf = struct.unpack_from("<HHH", b, 0)
                cells[(r, c)] = _Reader([b[6:]]).xlstring()
            elif rt == 0x0203:
                r, c, xf = struct.unpack_from("<HHH", b, 0)
                cells[(r, c)] = self._num(struct.unpack_from("<d", b, 6)[0], xf)
            elif rt == 0x027E:
                r, c, xf, v = struct.unpack_from("<HHHI", b, 0)
                cells[(r, c)] = self._num(_rk(v), xf)
            elif rt == 0x00BD:
                r, c0 = struct.unpack_from("<HH", b, 0)
                n = (len(b) - 6) // 6
                for k in range(n):
                    xf, v = struct.unpack_from("<HI", b, 4 + 6 * k)
                    cells[(r, c0 + k)] = self._num(_rk(v), xf)
            elif rt == 0x0205:
                r, c, xf, val, err = struct.unpack_from("<HHHBB", b, 0)
                cells[(r, c)] = float("nan") if err else bool(val)
            elif rt == 0x0006:
                r, c, xf = struct.unpack_from("<HHH", b, 0)
                res = b[6:14]
                if res[6:8] == b"\xff\xff":
                    kind = res[0]
                    if kind == 0:
                        pending_str = (r, c)
                    elif kind == 1:
                        cells[(r, c)] = bool(res[2])
                    elif kind == 2:
                        cells[(r, c)] = float("nan")
                    else:
                        cells[(r, c)] = ""
                else:
                    cells[(r, c)] = self._num(struct.unpack("<d", res)[0], xf)
            elif rt == 0x0207 and pending_str is not None:
                cells[pending_str] = _Reader([b]).xlstring()
                pending_str = None
        if not cells:
            return []
        nr = max(r for r, _ in cells) + 1
        nc = max(c for _, c in cells) + 1
        if nrows is not None:
            nr = min(nr, nrows)
        return [[cells.get((r, c), "") for c in range(nc)] for r in range(nr)]


def read_xls_frames(path, nrows: int = 1000):
    import pandas as pd
    from pandas.io.parsers import TextParser

    book = XlsBook(path)
    out = {}
    for name, off in book.sheets:
        grid = book.rows(off, nrows + 1)
        out[name] = TextParser(grid, header=0, nrows=nrows).read() if grid else pd.DataFrame()
    return out
