"""Build libsli.so (HIP kernels + C ABI + C++ drop-in op/model layer) for gfx950, in-tree.

    python -m simplellminference_amd.build [--force] [--jobs N]

hipcc cross-compiles for gfx950 without a GPU; the shared library lands next to this file so it
travels to the GPU box with the repo snapshot (it is git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(PKG, "_build")
LIB = os.path.join(PKG, "libsli.so")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("SLI_OFFLOAD_ARCH", "gfx950")

CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
            "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "include", "base"),
            "-I", os.path.join(ROOT, "include", "memory"), "-I", os.path.join(ROOT, "include", "op"),
            "-I", os.path.join(ROOT, "include", "model"), "-I", os.path.join(ROOT, "include", "kernel")]


def sources() -> list[str]:
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    srcs += sorted(glob.glob(os.path.join(CSRC, "host", "*.cpp")))
    return srcs


def _headers() -> list[str]:
    hs = glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)
    hs += glob.glob(os.path.join(ROOT, "include", "**", "*.h"), recursive=True)
    return hs


def _obj(src: str, build_dir: str = BUILD) -> str:
    rel = os.path.relpath(src, CSRC).replace(os.sep, "__")
    return os.path.join(build_dir, rel + ".o")


def _compile(src: str, force: bool, build_dir: str = BUILD, defines: tuple = ()) -> str:
    obj = _obj(src, build_dir)
    newest_dep = max([os.path.getmtime(src)] + [os.path.getmtime(h) for h in _headers()])
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= newest_dep:
        return obj
    lang = ["-x", "hip"] if src.endswith(".cpp") else []
    # SLI_EXTRA_CXXFLAGS: extra compiler flags for an A/B variant build (tools/ab_variants.sh), e.g. code alignment
    extra = os.environ.get("SLI_EXTRA_CXXFLAGS", "").split() if build_dir != BUILD else []
    cmd = ["hipcc", *lang, *CXXFLAGS, *extra, *[f"-D{d}" for d in defines], "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, jobs: int | None = None, verbose: bool = False, variant: str | None = None,
          defines: tuple = ()) -> str:
    """variant: an A/B experiment build (tools/ab_variants.sh) — objects in _build_variants/<variant>, the
    library as libsli_<variant>.so beside libsli.so (loaded with SLI_LIB_VARIANT=<variant>), compiled
    with the extra -D defines."""
    build_dir = BUILD if variant is None else os.path.join(PKG, "_build_variants", variant)
    lib = LIB if variant is None else os.path.join(PKG, f"libsli_{variant}.so")
    os.makedirs(build_dir, exist_ok=True)
    srcs = sources()
    jobs = jobs or min(8, len(srcs), os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, force or variant is not None, build_dir, tuple(defines)), srcs))
    newest = max(os.path.getmtime(o) for o in objs)
    if force or variant is not None or not os.path.exists(lib) or os.path.getmtime(lib) < newest:
        cmd = ["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib, *objs,
               "-L", os.path.join(ROCM, "lib"), "-lrccl", f"-Wl,-rpath,{os.path.join(ROCM, 'lib')}"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"built {lib}")
    return lib


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--variant", default=None, help="A/B build: libsli_<variant>.so")
    ap.add_argument("-D", dest="defines", action="append", default=[], help="extra define for a variant build")
    a = ap.parse_args(argv)
    build(force=a.force, jobs=a.jobs, verbose=True, variant=a.variant, defines=tuple(a.defines))
    return 0


if __name__ == "__main__":
    sys.exit(main())
