"""Ruled-table detection for the in-tree PDF reader -- the role of PyMuPDF's
``page.find_tables()`` (default "lines" strategy) in the reference's PDF path
(app/file_parser.py:183-196).

Same pipeline as that strategy (the pdfplumber lattice algorithm it is built on):

  1. edges     every straight segment of a painted path (``m``/``l``/``h``) and
               the four sides of every ``re`` rectangle, horizontal or vertical
               only, at least 3 pt long, in top-left-origin page coordinates;
  2. snap      edges of one orientation within 3 pt of each other share a
               coordinate (cluster mean); collinear pieces closer than 3 pt join;
  3. points    vertical x horizontal crossings (3 pt tolerance);
  4. cells     for each point, the smallest rectangle whose four corners are
               points connected by edges (the pdfplumber cell rule);
  5. tables    cells grouped by shared corners, >= 2 cells, ordered top-left;
  6. extract   rows by cell top, columns by the table's distinct cell lefts
               (None where a row has no cell); a cell's text = the glyphs whose
               box lies more than half inside it, grouped into lines by baseline,
               lines joined by "\\n".

Untrusted uploads bound the work per page: a page with more than MAX_SEGMENTS
path segments, or whose snapped grid could hold more than MAX_POINTS crossings,
skips table detection (its page text is still emitted); the cell search stops at
the first uncovered candidate and glyphs are looked up through a top-sorted
index, so a dense ruled grid costs O(points + cells x glyphs-per-cell).

PyMuPDF is not installable here, so byte parity with its table text is
unpinned; tests/parser/test_pdf_tables.py pins this implementation on generated
ruled-table PDFs and checks that the reference fixture (no ruled tables) still
parses byte-identically.
"""
from __future__ import annotations

import bisect
from collections import defaultdict

MAX_SEGMENTS = 20_000      # painted path segments per page considered for tables
MAX_POINTS = 20_000        # horizontal x vertical snapped lines per page
SNAP = 3.0
JOIN = 3.0
ISECT = 3.0
MIN_EDGE = 3.0
ASCENT, DESCENT = 0.8, 0.2


def _cluster(values: list[float], tol: float) -> dict[float, float]:
    """value -> mean of its cluster (consecutive sorted values within tol)."""
    out: dict[float, float] = {}
    vs = sorted(set(values))
    group: list[float] = []
    for v in vs:
        if group and v - group[-1] > tol:
            m = sum(group) / len(group)
            out.update({g: m for g in group})
            group = []
        group.append(v)
    if group:
        m = sum(group) / len(group)
        out.update({g: m for g in group})
    return out


def _merge(segs: list[tuple[float, float]], tol: float) -> list[tuple[float, float]]:
    segs = sorted(segs)
    out: list[list[float]] = []
    for a, b in segs:
        if out and a <= out[-1][1] + tol:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return [(a, b) for a, b in out]


def edges_from_segments(segments, height: float):
    """segments: [(x0, y0, x1, y1)] in PDF user space -> (horizontals, verticals) as
    {y: [(x0, x1)]} / {x: [(top, bottom)]} in top-left coordinates, snapped and joined."""
    hs, vs = [], []
    for x0, y0, x1, y1 in segments:
        t0, t1 = height - y0, height - y1
        if abs(t0 - t1) <= 1e-3 * max(1.0, abs(x1 - x0)) or abs(t0 - t1) < 0.5:
            if abs(x1 - x0) >= MIN_EDGE:
                hs.append(((t0 + t1) / 2, min(x0, x1), max(x0, x1)))
        elif abs(x1 - x0) < 0.5:
            if abs(t1 - t0) >= MIN_EDGE:
                vs.append(((x0 + x1) / 2, min(t0, t1), max(t0, t1)))
    hmap = _cluster([h[0] for h in hs], SNAP)
    vmap = _cluster([v[0] for v in vs], SNAP)
    H: dict[float, list] = defaultdict(list)
    V: dict[float, list] = defaultdict(list)
    for y, a, b in hs:
        H[hmap[y]].append((a, b))
    for x, a, b in vs:
        V[vmap[x]].append((a, b))
    return ({y: _merge(s, JOIN) for y, s in H.items()},
            {x: _merge(s, JOIN) for x, s in V.items()})


def _covers(segs, a: float, b: float, tol: float) -> bool:
    """One joined segment spans [a, b]."""
    return any(s0 - tol <= a and b <= s1 + tol for s0, s1 in segs)


def _reach(coords: list, start: float, segs) -> list:
    """Sorted coords > start that the edge segs spans continuously from start."""
    out = []
    for c in coords[bisect.bisect_right(coords, start):]:
        if not _covers(segs, start, c, ISECT):
            break
        out.append(c)
    return out


def find_cells(H: dict, V: dict) -> list[tuple[float, float, float, float]]:
    points = set()
    for y, hsegs in H.items():
        for x, vsegs in V.items():
            if any(s0 - ISECT <= x <= s1 + ISECT for s0, s1 in hsegs) and \
                    any(s0 - ISECT <= y <= s1 + ISECT for s0, s1 in vsegs):
                points.add((x, y))
    pts = sorted(points, key=lambda p: (p[1], p[0]))
    xs_at_y: dict[float, list] = defaultdict(list)
    ys_at_x: dict[float, list] = defaultdict(list)
    for x, y in pts:
        xs_at_y[y].append(x)
        ys_at_x[x].append(y)
    cells = []
    for x, y in pts:
        # candidates in increasing distance; once an edge stops covering the span,
        # every farther candidate fails too (a segment covering [y, b'] covers [y, b])
        below = _reach(ys_at_x[x], y, V[x])
        right = _reach(xs_at_y[y], x, H[y])
        found = None
        for b in below:
            for r in right:
                if (r, b) in points and _covers(V[r], y, b, ISECT) and _covers(H[b], x, r, ISECT):
                    found = (x, y, r, b)
                    break
            if found:
                break
        if found:
            cells.append(found)
    return cells


def group_tables(cells) -> list[list[tuple]]:
    """Connected components of cells sharing a corner; >= 2 cells; top-left order."""
    corner_of: dict[tuple, list[int]] = defaultdict(list)
    for i, (x0, t, x1, b) in enumerate(cells):
        for c in ((x0, t), (x1, t), (x0, b), (x1, b)):
            corner_of[c].append(i)
    seen, tables = set(), []
    for i in range(len(cells)):
        if i in seen:
            continue
        comp, stack = [], [i]
        seen.add(i)
        while stack:
            j = stack.pop()
            comp.append(cells[j])
            x0, t, x1, b = cells[j]
            for c in ((x0, t), (x1, t), (x0, b), (x1, b)):
                for k in corner_of[c]:
                    if k not in seen:
                        seen.add(k)
                        stack.append(k)
        if len(comp) > 1:
            tables.append(comp)
    tables.sort(key=lambda c: (min(x[1] for x in c), min(x[0] for x in c)))
    return tables


class GlyphIndex:
    """Glyphs sorted by top: the candidates of a cell [t, b] are the glyphs whose top
    lies in [t - tallest glyph, b)."""

    def __init__(self, glyphs):
        self.glyphs = sorted(glyphs, key=lambda g: g[2])
        self.tops = [g[2] for g in self.glyphs]
        self.tallest = max((g[3] - g[2] for g in self.glyphs), default=0.0)

    def near(self, t: float, b: float):
        lo = bisect.bisect_left(self.tops, t - self.tallest)
        hi = bisect.bisect_left(self.tops, b)
        return self.glyphs[lo:hi]


def cell_text(glyphs, cell) -> str:
    """glyphs: [(x0, x1, top, bottom, baseline, size, ch)] in top-left coordinates, or
    a GlyphIndex of them."""
    x0, t, x1, b = cell
    if isinstance(glyphs, GlyphIndex):
        glyphs = glyphs.near(t, b)
    inside = []
    for g in glyphs:
        gx0, gx1, gt, gb = g[0], g[1], g[2], g[3]
        w, h = max(gx1 - gx0, 1e-3), max(gb - gt, 1e-3)
        ox = max(0.0, min(gx1, x1) - max(gx0, x0))
        oy = max(0.0, min(gb, b) - max(gt, t))
        if ox * oy > 0.5 * w * h:
            inside.append(g)
    if not inside:
        return ""
    inside.sort(key=lambda g: (g[4], g[0]))
    lines: list[list] = []
    for g in inside:
        if lines and abs(g[4] - lines[-1][-1][4]) <= 0.5 * max(g[5], lines[-1][-1][5]):
            lines[-1].append(g)
        else:
            lines.append([g])
    out = []
    for ln in lines:
        ln.sort(key=lambda g: g[0])
        s, last = "", None
        for g in ln:
            if last is not None and g[6] != " " and g[0] - last[1] > 0.25 * g[5] and \
                    not s.endswith(" "):
                s += " "
            if g[6] == " " and s.endswith(" "):
                continue
            s += g[6]
            last = g
        out.append(s.strip())
    return "\n".join(o for o in out if o)


def extract_tables(segments, glyphs, height: float) -> list[list[list]]:
    """-> tables, each a list of rows, each a list of cell strings (or None)."""
    if len(segments) > MAX_SEGMENTS:
        return []
    H, V = edges_from_segments(segments, height)
    if not H or not V or len(H) * len(V) > MAX_POINTS:
        return []
    glyphs = GlyphIndex(glyphs)
    tables = []
    for cells in group_tables(find_cells(H, V)):
        cols = sorted({round(c[0], 3) for c in cells})
        rows_by_top: dict[float, dict] = defaultdict(dict)
        for c in cells:
            rows_by_top[round(c[1], 3)][round(c[0], 3)] = c
        rows = []
        for top in sorted(rows_by_top):
            r = rows_by_top[top]
            rows.append([cell_text(glyphs, r[x]) if x in r else None for x in cols])
        tables.append(rows)
    return tables


def format_tables(tables, page_no: int) -> list[str]:
    """The reference's text blocks (app/file_parser.py:186-193), one per table."""
    parts = []
    for tnum, data in enumerate(tables, 1):
        if not data:
            continue
        txt = f"\n=== Table {tnum} on Page {page_no} ===\n"
        for row in data:
            if row and any(cell for cell in row if cell):
                txt += " | ".join(str(cell) if cell else "" for cell in row) + "\n"
        parts.append(txt)
    return parts
