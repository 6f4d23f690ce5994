"""Exact-request response cache — the role ag2's diskcache played in the reference.

Reference: ``cache_seed 42`` made ag2 store every completion in
``.cache/42/cache.db`` (diskcache, sqlite, least-recently-stored eviction,
1 GiB limit) keyed by the request dict ``{messages, model, temperature,
max_tokens}``; an identical request was answered without calling the LLM
(SURVEY.md §2.1 X2, §5.4).  This module keeps that behaviour as an optional
wrapper around any extraction backend: an in-memory LRU plus an optional sqlite
file (JSON values only — nothing is ever unpickled).  Enable with
``RFQ_RESPONSE_CACHE=<path.sqlite>`` or ``=memory``.
"""
from __future__ import annotations

import collections
import hashlib
import json
import sqlite3
import threading


def request_key(messages: list[dict], model: str, temperature: float, max_tokens: int) -> str:
    blob = json.dumps({"messages": messages, "model": model, "temperature": temperature,
                       "max_tokens": max_tokens}, sort_keys=True, ensure_ascii=False)
    return hashlib.sha256(blob.encode()).hexdigest()


class ResponseCache:
    def __init__(self, path: str | None = None, max_entries: int = 100_000):
        self.mem: collections.OrderedDict[str, str] = collections.OrderedDict()
        self.max_entries = max_entries
        self.hits = 0
        self.misses = 0
        self._lock = threading.Lock()
        self.db = None
        if path and path != "memory":
            self.db = sqlite3.connect(path, check_same_thread=False)
            self.db.execute("CREATE TABLE IF NOT EXISTS cache (key TEXT PRIMARY KEY, value TEXT, "
                            "stored REAL DEFAULT (julianday('now')))")
            self.db.commit()

    def get(self, key: str) -> str | None:
        with self._lock:
            if key in self.mem:
                self.mem.move_to_end(key)
                self.hits += 1
                return self.mem[key]
            if self.db is not None:
                row = self.db.execute("SELECT value FROM cache WHERE key=?", (key,)).fetchone()
                if row:
                    self.hits += 1
                    self._put_mem(key, row[0])
                    return row[0]
            self.misses += 1
            return None

    def _put_mem(self, key, value):
        self.mem[key] = value
        self.mem.move_to_end(key)
        while len(self.mem) > self.max_entries:        # least-recently-stored eviction
            self.mem.popitem(last=False)

    def put(self, key: str, value: str) -> None:
        with self._lock:
            self._put_mem(key, value)
            if self.db is not None:
                self.db.execute("INSERT OR REPLACE INTO cache(key, value) VALUES (?, ?)", (key, value))
                self.db.commit()


class CachedBackend:
    """Wrap an extraction backend with the exact-request cache."""

    def __init__(self, inner, cache: ResponseCache, model: str, temperature: float,
                 max_tokens: int):
        self.inner = inner
        self.cache = cache
        self.model, self.temperature, self.max_tokens = model, temperature, max_tokens

    @property
    def healthy(self) -> bool:
        return bool(getattr(self.inner, "healthy", True))

    def _key(self, messages):
        return request_key(messages, self.model, self.temperature, self.max_tokens)

    def complete(self, messages):
        k = self._key(messages)
        hit = self.cache.get(k)
        if hit is not None:
            return hit
        out = self.inner.complete(messages)
        self.cache.put(k, out)
        return out

    async def acomplete(self, messages):
        k = self._key(messages)
        hit = self.cache.get(k)
        if hit is not None:
            return hit
        out = await self.inner.acomplete(messages)
        self.cache.put(k, out)
        return out
