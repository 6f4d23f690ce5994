"""Packaging: every third-party top-level module the package imports
is declared in requirements.txt (what the Dockerfile installs) and in pyproject.toml."""
import ast
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "replisense_rfq_amd")
# import name -> distribution name where they differ
DIST = {"yaml": "pyyaml", "prometheus_client": "prometheus-client", "sklearn": "scikit-learn"}
# from the base image (ROCm PyTorch wheel) rather than pip
BASE_IMAGE = {"torch"}


def _third_party_imports() -> set:
    stdlib = set(sys.stdlib_module_names)
    mods = set()
    for dirpath, _, files in os.walk(PKG):
        for fn in files:
            if not fn.endswith(".py"):
                continue
            tree = ast.parse(open(os.path.join(dirpath, fn), encoding="utf-8").read())
            for node in ast.walk(tree):
                if isinstance(node, ast.Import):
                    names = [a.name for a in node.names]
                elif isinstance(node, ast.ImportFrom) and node.level == 0 and node.module:
                    names = [node.module]
                else:
                    continue
                for n in names:
                    top = n.split(".")[0]
                    if top not in stdlib and top != "replisense_rfq_amd":
                        mods.add(top)
    return mods


def _declared(text: str) -> set:
    out = set()
    for line in text.splitlines():
        line = line.split("#")[0].strip().strip('",')
        m = re.match(r"([A-Za-z0-9_.\-]+)", line)
        if m:
            out.add(m.group(1).lower().replace("_", "-"))
    return out


def test_every_import_is_declared():
    mods = _third_party_imports() - BASE_IMAGE
    assert {"fastapi", "numpy", "prometheus_client", "aiohttp"} <= mods
    req = _declared(open(os.path.join(ROOT, "requirements.txt")).read())
    pyproj = open(os.path.join(ROOT, "pyproject.toml")).read()
    deps = pyproj.split("dependencies = [", 1)[1].split("]", 1)[0]
    opt = pyproj.split("[project.optional-dependencies]", 1)[1].split("[", 2)
    pdeps = _declared(deps) | _declared(" ".join(opt[:2]))
    for m in sorted(mods):
        d = DIST.get(m, m).lower().replace("_", "-")
        assert d in req, f"{m} imported by the package but missing from requirements.txt"
        assert d in pdeps, f"{m} imported by the package but missing from pyproject.toml"
