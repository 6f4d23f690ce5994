"""In-tree native build: gfx950 HIP kernels + torch op bindings + C++ runtime.

Two shared objects are produced next to this file (git-ignored, but they travel
to the GPU box with the repo snapshot):

* ``_C.so``        — every ``csrc/kernels/*.hip`` / ``csrc/comm/*.hip`` kernel
                      compiled with ``hipcc --offload-arch=gfx950`` plus
                      ``csrc/bindings/torch_ops.cpp`` (``TORCH_LIBRARY(rfq_amd)``).
                      Loaded with ``torch.ops.load_library``.
* ``_runtime.so``  — host-only C++ runtime (``csrc/runtime/*.cpp``): KV block
                      allocator, prefix hashing, JSON-grammar automaton.  pybind11
                      module, no torch dependency.

No hipify step, no CUDA shims: the sources are HIP/CDNA4 code and are compiled
directly.  Objects are cached under ``build/`` keyed by a hash of the source,
the shared headers and the flags, so a rebuild after a one-file edit recompiles
one file.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
ROOT = PKG_DIR.parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
HIPCC = str(ROCM / "bin" / "hipcc")

C_SO = PKG_DIR / "_C.so"
RT_SO = PKG_DIR / f"_runtime{sysconfig.get_config_var('EXT_SUFFIX') or '.so'}"

KERNEL_FLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-mcode-object-version=5",
    "-ffp-contract=fast", "-munsafe-fp-atomics", "-Wno-unused-result",
]


def _torch_paths():
    import torch  # noqa: WPS433 (deferred: keep `import replisense_rfq_amd` light)

    tdir = Path(torch.__file__).resolve().parent
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return tdir, abi


def _digest(paths, extra: str) -> str:
    h = hashlib.sha1(extra.encode())
    for p in paths:
        h.update(Path(p).read_bytes())
    return h.hexdigest()[:16]


def _run(cmd, what):
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"[rfq build] {what} failed:\n$ {' '.join(cmd)}\n{proc.stdout}")
    return proc.stdout


def _compile(src: Path, flags, deps, tag: str) -> Path:
    key = _digest([src, *deps], " ".join(flags) + tag)
    obj = BUILD / "obj" / f"{src.stem}.{key}.o"
    if obj.exists():
        return obj
    obj.parent.mkdir(parents=True, exist_ok=True)
    tmp = obj.with_suffix(".tmp.o")
    _run([HIPCC, *flags, "-c", str(src), "-o", str(tmp)], f"compile {src.name}")
    tmp.replace(obj)
    return obj


def _link(out: Path, objs, libs, key_extra: str):
    stamp = out.with_name(out.name + ".stamp")
    key = _digest(objs, key_extra)
    if out.exists() and stamp.exists() and stamp.read_text() == key:
        return
    tmp = out.with_suffix(".tmp.so")
    _run([HIPCC, "-shared", "-fPIC", *map(str, objs), "-o", str(tmp), *libs], f"link {out.name}")
    tmp.replace(out)
    stamp.write_text(key)


def build_kernels(jobs: int | None = None, verbose: bool = False) -> Path:
    tdir, abi = _torch_paths()
    headers = sorted((CSRC / "kernels").glob("*.h")) + sorted((CSRC / "comm").glob("*.h"))
    kernel_srcs = sorted((CSRC / "kernels").glob("*.hip")) + sorted((CSRC / "comm").glob("*.hip"))
    bind_flags = [
        "-O2", "-fPIC", "-std=c++17", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM=1",
        "-D__HIP_PLATFORM_AMD__=1", f"-I{tdir / 'include'}",
        f"-I{tdir / 'include' / 'torch' / 'csrc' / 'api' / 'include'}",
        f"-I{sysconfig.get_paths()['include']}", "-Wno-deprecated-declarations",
    ]
    jobs = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(jobs) as ex:
        futs = [ex.submit(_compile, s, KERNEL_FLAGS + [f"-I{CSRC / 'kernels'}"], headers, "k")
                for s in kernel_srcs]
        futs.append(ex.submit(_compile, CSRC / "bindings" / "torch_ops.cpp", bind_flags, [], "b"))
        futs.append(ex.submit(_compile, CSRC / "bindings" / "gemm_lt.cpp",
                              bind_flags + [f"-I{ROCM / 'include'}"], [], "b"))
        objs = [f.result() for f in futs]
    libs = [f"-L{tdir / 'lib'}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
            f"-Wl,-rpath,{tdir / 'lib'}", f"-L{ROCM / 'lib'}", "-lhipblaslt",
            f"-Wl,-rpath,{ROCM / 'lib'}"]
    _link(C_SO, objs, libs, "C" + ARCH)
    _check_stubs(C_SO)
    if verbose:
        print(f"[rfq build] {C_SO}")
    return C_SO


def _check_stubs(so: Path) -> None:
    """Fail the build when a kernel's host launch stub is undefined: clang can drop a
    kernel template's stub without an error (e.g. a device-only builtin called with
    template-dependent arguments), and the library then fails to load only on the
    GPU box (`torch.ops.load_library`: undefined symbol)."""
    nm = shutil.which("nm") or str(ROCM / "lib" / "llvm" / "bin" / "llvm-nm")
    out = _run([nm, "-D", "--undefined-only", str(so)], "nm")
    missing = [ln.split()[-1] for ln in out.splitlines() if "__device_stub__" in ln]
    if missing:
        raise RuntimeError(f"[rfq build] {so.name}: undefined kernel launch stubs {missing}")


def build_runtime(verbose: bool = False) -> Path:
    import pybind11

    # test_*.cpp are stand-alone sanitizer harnesses with their own main()
    # (tests/engine/test_runtime_sanitized.py); they never ship in _runtime.so.
    srcs = sorted(s for s in (CSRC / "runtime").glob("*.cpp") if not s.name.startswith("test_"))
    hdrs = sorted((CSRC / "runtime").glob("*.h"))
    flags = ["-O3", "-fPIC", "-std=c++17", "-fvisibility=hidden",
             f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}",
             f"-I{CSRC / 'runtime'}"]
    cxx = shutil.which("g++") or "c++"
    objs = []
    for s in srcs:
        key = _digest([s, *hdrs], " ".join(flags))
        obj = BUILD / "obj" / f"rt_{s.stem}.{key}.o"
        if not obj.exists():
            obj.parent.mkdir(parents=True, exist_ok=True)
            _run([cxx, *flags, "-c", str(s), "-o", str(obj)], f"compile {s.name}")
        objs.append(obj)
    stamp = RT_SO.with_name(RT_SO.name + ".stamp")
    key = _digest(objs, "rt")
    if not (RT_SO.exists() and stamp.exists() and stamp.read_text() == key):
        _run([cxx, "-shared", "-fPIC", *map(str, objs), "-o", str(RT_SO)], "link _runtime")
        stamp.write_text(key)
    if verbose:
        print(f"[rfq build] {RT_SO}")
    return RT_SO


def build_all(verbose: bool = True) -> None:
    build_runtime(verbose)
    build_kernels(verbose=verbose)


if __name__ == "__main__":
    build_all(verbose="-q" not in sys.argv)
