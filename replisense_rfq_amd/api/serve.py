"""Server entry point (reference app/main.py:410-421).

Same environment contract: PORT (8000), ENVIRONMENT (development -> reload),
LOG_LEVEL (info).  Reload is never used with the engine backend: a reloading
worker would re-initialise the GPU engine on every file change, so it is only
honoured for RFQ_BACKEND=mock.  Engine knobs come from RFQ_* (utils/config.py).
"""
from __future__ import annotations

import argparse
import logging
import os

log = logging.getLogger("replisense_rfq_amd.api")


def server_config(host: str = "0.0.0.0", port: int | None = None) -> dict:
    reload = (os.getenv("ENVIRONMENT", "development") == "development"
              and os.getenv("RFQ_BACKEND", "") == "mock")
    return {"host": host, "port": port or int(os.getenv("PORT", "8000")), "reload": reload,
            "log_level": os.getenv("LOG_LEVEL", "info").lower(), "access_log": True,
            "timeout_keep_alive": int(os.getenv("RFQ_KEEP_ALIVE_S", "75")),
            "backlog": 4096}


def main(argv=None) -> None:
    import uvicorn

    ap = argparse.ArgumentParser(description="RFQ Processing API (MI355X engine)")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=None)
    a = ap.parse_args(argv)
    cfg = server_config(a.host, a.port)
    log.info("Starting server with config: %s", cfg)
    uvicorn.run("replisense_rfq_amd.api.main:app", **cfg)


if __name__ == "__main__":
    main()
