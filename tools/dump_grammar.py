"""Write the compiled RFQ grammar + mask table as a flat blob for the C++
sanitizer harness (csrc/runtime/test_runtime.cpp)."""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def dump(path: str, flavor: str = "llama3") -> None:
    from replisense_rfq_amd.engine.grammar import get_grammar, pack_native

    g = get_grammar(flavor)
    d = pack_native(g.compiled, g.py.quote)
    d["mask_rows"] = np.ascontiguousarray(g.compiled.mask_rows, np.uint32)
    d["mask_words"] = np.array([g.compiled.mask_rows.shape[1]], np.int32)
    d["max_tokens"] = np.array([1200], np.int32)
    with open(path, "wb") as f:
        for k, v in d.items():
            v = np.ascontiguousarray(v)
            kind = {np.dtype(np.int32): b"i", np.dtype(np.uint8): b"b",
                    np.dtype(np.uint32): b"u"}[v.dtype]
            f.write(k.encode().ljust(32, b"\0"))
            f.write(kind + b"\0" * 7)
            f.write(np.int64(v.size).tobytes())
            f.write(v.tobytes())


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--flavor", default="llama3")
    a = ap.parse_args()
    dump(a.out, a.flavor)
