"""Host runtime under AddressSanitizer + UndefinedBehaviorSanitizer.

GPU ASan is not available on the MI355X pool, so the sanitizer pass covers the
native host code that runs on the scheduler hot path: the C++ grammar automaton,
the KV block manager and the engine core's scheduler / packer / post-processor
(csrc/runtime/test_runtime.cpp drives all three)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, "csrc", "runtime")


@pytest.mark.parametrize("flavor", ["llama3", "mixtral"])
def test_runtime_asan_ubsan(tmp_path, flavor):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = tmp_path / "test_runtime"
    subprocess.run([cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer",
                    "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
                    os.path.join(SRC, "test_runtime.cpp"), os.path.join(SRC, "grammar.cpp"),
                    os.path.join(SRC, "block_manager.cpp"), os.path.join(SRC, "engine_core.cpp"),
                    "-o", str(exe)],
                   check=True, capture_output=True, timeout=300)
    blob = tmp_path / "grammar.bin"
    from tools.dump_grammar import dump

    dump(str(blob), flavor)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([str(exe), str(blob), "300", "7"], capture_output=True, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout
