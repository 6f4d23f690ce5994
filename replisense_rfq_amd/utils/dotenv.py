"""``.env`` loading (python-dotenv is not installed offline).

The reference calls ``load_dotenv()`` at import time in app/main.py:23 and
app/rfq_agent.py:13, so ``MAX_FILE_SIZE_MB``, ``ALLOWED_ORIGINS``, ``PORT``, ... and
here the ``RFQ_*`` engine knobs can come from a ``.env`` file.  Same semantics as
python-dotenv's defaults: the first ``.env`` found walking up from the calling
module's directory (then from the working directory); existing environment
variables win (``override=False``); ``KEY=VALUE`` / ``export KEY=VALUE`` lines,
``#`` comments, single-quoted (literal) and double-quoted (escapes) values, and
``${VAR}`` / ``${VAR:-default}`` interpolation in unquoted and double-quoted values.
"""
from __future__ import annotations

import inspect
import os
import re
from pathlib import Path

_LINE = re.compile(r"^\s*(?:export\s+)?([A-Za-z_][A-Za-z0-9_.-]*)\s*=\s*(.*)$")
_VAR = re.compile(r"\$\{([A-Za-z_][A-Za-z0-9_]*)(?::-([^}]*))?\}")
_ESC = {"n": "\n", "t": "\t", "r": "\r", '"': '"', "\\": "\\", "'": "'"}


def find_dotenv(filename: str = ".env", start: str | os.PathLike | None = None) -> str:
    starts = [Path(start)] if start else []
    if not start:
        frame = inspect.currentframe()
        caller = frame.f_back.f_back if frame and frame.f_back else None
        while caller is not None and caller.f_code.co_filename == __file__:
            caller = caller.f_back
        if caller is not None and caller.f_code.co_filename and \
                not caller.f_code.co_filename.startswith("<"):
            starts.append(Path(caller.f_code.co_filename).resolve().parent)
        starts.append(Path.cwd())
    for s in starts:
        for d in [s, *s.parents]:
            cand = d / filename
            if cand.is_file():
                return str(cand)
    return ""


def _interpolate(value: str, env: dict) -> str:
    return _VAR.sub(lambda m: env.get(m.group(1)) or os.environ.get(m.group(1)) or
                    (m.group(2) or ""), value)


def _value(raw: str, env: dict) -> str:
    raw = raw.strip()
    if raw[:1] == "'":
        end = raw.find("'", 1)
        return raw[1:end] if end > 0 else raw[1:]
    if raw[:1] == '"':
        out, i = [], 1
        while i < len(raw) and raw[i] != '"':
            if raw[i] == "\\" and i + 1 < len(raw):
                out.append(_ESC.get(raw[i + 1], "\\" + raw[i + 1]))
                i += 2
                continue
            out.append(raw[i])
            i += 1
        return _interpolate("".join(out), env)
    raw = re.split(r"\s+#", raw, maxsplit=1)[0].strip()
    return _interpolate(raw, env)


def dotenv_values(path: str | os.PathLike) -> dict[str, str]:
    env: dict[str, str] = {}
    with open(path, encoding="utf-8") as f:
        for line in f:
            if not line.strip() or line.lstrip().startswith("#"):
                continue
            m = _LINE.match(line.rstrip("\n"))
            if m:
                env[m.group(1)] = _value(m.group(2), env)
    return env


def load_dotenv(path: str | os.PathLike | None = None, override: bool = False) -> bool:
    """Load ``path`` (default: :func:`find_dotenv`) into ``os.environ``; True if a
    file was read."""
    path = path or find_dotenv()
    if not path or not os.path.isfile(path):
        return False
    for k, v in dotenv_values(path).items():
        if override or k not in os.environ:
            os.environ[k] = v
    return True
