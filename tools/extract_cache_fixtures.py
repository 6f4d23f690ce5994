"""Extract the reference's recorded LLM exchanges into a JSON golden fixture.

The reference ships ag2's diskcache of 14 Groq chat completions
(/root/reference/.cache/42/cache.db, table Cache).  Keys and values are pickles;
they are NEVER unpickled here: the database is opened read-only/immutable and the
pickle streams are only *disassembled* with ``pickletools.genops``, collecting the
string / number arguments in stream order.  From those we recover, per row: the
system and user messages, temperature/model/max_tokens (key), the completion
text, finish reason and Groq usage telemetry (value).

Output: tests/assets/golden/cache_rows.json
"""
from __future__ import annotations

import json
import pickletools
import sqlite3
import sys
from pathlib import Path

DB = Path("/root/reference/.cache/42/cache.db")
OUT = Path(__file__).resolve().parent.parent / "tests" / "assets" / "golden" / "cache_rows.json"

_SKIP = {"MEMOIZE", "PUT", "BINPUT", "LONG_BINPUT", "GET", "BINGET", "LONG_BINGET", "PROTO",
         "FRAME"}


def scalars(blob: bytes) -> list:
    out = []
    for op, arg, _ in pickletools.genops(blob):
        if op.name in _SKIP:
            continue
        if isinstance(arg, (str, int, float)) and not isinstance(arg, bool):
            out.append(arg)
        elif op.name in ("NEWTRUE", "NEWFALSE", "NONE"):
            out.append({"NEWTRUE": True, "NEWFALSE": False, "NONE": None}[op.name])
    return out


def after(seq: list, key: str, default=None, start: int = 0):
    for i in range(start, len(seq) - 1):
        if seq[i] == key:
            return seq[i + 1]
    return default


def parse_row(rowid: int, key: bytes, value: bytes, store_time: float) -> dict:
    k = scalars(key)
    # messages: ... 'content', <system>, 'role', 'system', 'role', 'user', 'content', <user>
    sys_msg = user_msg = None
    for i, s in enumerate(k):
        if s == "system" and i >= 3 and k[i - 1] == "role":
            sys_msg = k[i - 2]
        if s == "user" and i >= 1 and k[i - 1] == "role":
            user_msg = after(k, "content", start=i)
    v = scalars(value)
    content = after(v, "content")
    usage = {name: after(v, name) for name in (
        "completion_tokens", "prompt_tokens", "total_tokens", "queue_time", "prompt_time",
        "completion_time", "total_time")}
    return {
        "row": rowid, "store_time": store_time,
        "model": after(k, "model"), "temperature": after(k, "temperature"),
        "max_tokens": after(k, "max_tokens"),
        "system": sys_msg, "user": user_msg,
        "completion": content, "finish_reason": after(v, "finish_reason"),
        "usage": usage,
    }


def main() -> int:
    if not DB.exists():
        print("reference cache.db not found", file=sys.stderr)
        return 1
    con = sqlite3.connect(f"file:{DB}?mode=ro&immutable=1", uri=True)
    rows = con.execute("select rowid, key, value, store_time from Cache order by rowid").fetchall()
    out = [parse_row(r, k, v, t) for r, k, v, t in rows]
    OUT.parent.mkdir(parents=True, exist_ok=True)
    OUT.write_text(json.dumps(out, ensure_ascii=False, indent=1))
    print(f"wrote {len(out)} rows -> {OUT}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
