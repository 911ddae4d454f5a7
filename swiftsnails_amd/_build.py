"""In-tree native build for swiftsnails_amd.

Builds two extension modules into ``swiftsnails_amd/_lib/``:

* ``_ss_host``  — the host C++17 runtime (config parser, binary codec,
  channels / thread pool, state barriers, hash-fragment router, CPU sparse
  table, TCP message transport, master/server/worker protocol, text dump).
  Compiled with g++; needs no GPU runtime.
* ``_ss_hip``   — the gfx950 HIP kernels and the RCCL communicator, compiled
  with ``hipcc --offload-arch=gfx950``.

Objects are cached under ``build/`` and rebuilt when a source or any header in
its include directories is newer than the object.  Usage::

    python -m swiftsnails_amd._build [--force] [--only host|hip] [-j N]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_DIR = os.path.join(ROOT, "swiftsnails_amd", "_lib")
BUILD_DIR = os.path.join(ROOT, "build")
ARCH = os.environ.get("SS_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _py_includes() -> list[str]:
    import pybind11

    return ["-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"]]


def _ext_suffix() -> str:
    return ".so"


def _newest(paths) -> float:
    t = 0.0
    for p in paths:
        try:
            t = max(t, os.path.getmtime(p))
        except OSError:
            pass
    return t


def _headers(dirs) -> list[str]:
    out = []
    for d in dirs:
        out += glob.glob(os.path.join(d, "**", "*.h"), recursive=True)
    return out


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout + r.stderr)


def _compile_all(jobs, nproc):
    with cf.ThreadPoolExecutor(max_workers=nproc) as ex:
        futs = [ex.submit(_run, cmd) for cmd in jobs]
        for f in futs:
            f.result()


def _build_module(name, sources, compiler, cflags, ldflags, inc_dirs, force, nproc):
    os.makedirs(LIB_DIR, exist_ok=True)
    obj_dir = os.path.join(BUILD_DIR, name)
    os.makedirs(obj_dir, exist_ok=True)
    hdr_time = _newest(_headers(inc_dirs)) if not force else 0.0
    objs, jobs = [], []
    for src in sources:
        obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or not os.path.exists(obj) or os.path.getmtime(obj) < max(
            os.path.getmtime(src), hdr_time
        ):
            jobs.append([compiler] + cflags + ["-c", src, "-o", obj])
    _compile_all(jobs, nproc)
    out = os.path.join(LIB_DIR, name + _ext_suffix())
    if force or jobs or not os.path.exists(out) or os.path.getmtime(out) < _newest(objs):
        tmp = out + ".tmp"
        _run([compiler] + objs + ["-shared", "-o", tmp] + ldflags)
        os.replace(tmp, out)  # atomic: a running process keeps its mapped copy
    return out


def build_host(force=False, nproc=8) -> str:
    inc = [os.path.join(ROOT, "csrc", "include"), os.path.join(ROOT, "csrc", "host")]
    srcs = sorted(glob.glob(os.path.join(ROOT, "csrc", "host", "*.cpp")))
    cxx = os.environ.get("CXX", "g++")
    cflags = ["-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall", "-Wno-unused-function",
              "-pthread"] + ["-I" + d for d in inc] + _py_includes()
    return _build_module("_ss_host", srcs, cxx, cflags, ["-pthread"], inc, force, nproc)


def build_hip(force=False, nproc=8) -> str:
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    if not os.path.exists(hipcc):
        hipcc = shutil.which("hipcc") or hipcc
    inc = [os.path.join(ROOT, "csrc", "include"), os.path.join(ROOT, "csrc", "hip")]
    srcs = sorted(glob.glob(os.path.join(ROOT, "csrc", "hip", "*.hip")) +
                  glob.glob(os.path.join(ROOT, "csrc", "hip", "*.cpp")))
    cflags = ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden",
              "-Wno-unused-result", "-munsafe-fp-atomics"] + ["-I" + d for d in inc] + _py_includes()
    ldflags = ["--offload-arch=" + ARCH, "-L" + os.path.join(ROCM, "lib"), "-lrccl",
               "-Wl,-rpath," + os.path.join(ROCM, "lib")]
    return _build_module("_ss_hip", srcs, hipcc, cflags, ldflags, inc, force, nproc)


TEST_DIR = os.path.join(BUILD_DIR, "tests")
SANITIZERS = {
    "plain": [],
    # host code only (no GPU code in this binary); -O1 keeps reports readable
    "asan": ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-O1"],
    "tsan": ["-fsanitize=thread", "-O1", "-include",
             os.path.join(ROOT, "csrc", "tests", "tsan_compat.h")],
}


def build_cpp_tests(variant: str = "plain", force: bool = False) -> str:
    """Native host unit tests (csrc/tests/test_host.cpp): plain, ASan+UBSan
    or TSan build -> build/tests/test_host_<variant>."""
    os.makedirs(TEST_DIR, exist_ok=True)
    src = os.path.join(ROOT, "csrc", "tests", "test_host.cpp")
    out = os.path.join(TEST_DIR, f"test_host_{variant}")
    inc = [os.path.join(ROOT, "csrc", "include"), os.path.join(ROOT, "csrc", "host")]
    newest = max(os.path.getmtime(src), _newest(_headers(inc)))
    if not force and os.path.exists(out) and os.path.getmtime(out) >= newest:
        return out
    cxx = os.environ.get("CXX", "g++")
    flags = ["-std=c++17", "-g", "-pthread", "-Wall", "-Wno-unused-function"]
    flags += SANITIZERS[variant] or ["-O2"]
    cmd = [cxx] + flags + ["-I" + d for d in inc] + [src, "-o", out]
    subprocess.run(cmd, check=True)
    return out


def build_all(force=False, only=None, nproc=None) -> list[str]:
    nproc = nproc or min(16, os.cpu_count() or 4)
    outs = []
    if only in (None, "host"):
        outs.append(build_host(force, nproc))
    if only in (None, "hip"):
        outs.append(build_hip(force, nproc))
    return outs


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only", choices=["host", "hip"])
    ap.add_argument("-j", type=int, default=None)
    a = ap.parse_args(argv)
    for o in build_all(a.force, a.only, a.j):
        print("built", os.path.relpath(o, ROOT))


if __name__ == "__main__":
    sys.exit(main())
