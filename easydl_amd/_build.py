"""Build the native libraries in-tree (no JIT cache, no site-packages install).

* ``easydl_amd/lib/libedl_kernels.so`` – every ``csrc/kernels/*.hip`` compiled
  for gfx950 with hipcc (cross-compiles without a GPU).
* ``easydl_amd/lib/libedl_runtime.so`` – the host runtime in ``csrc/runtime``
  (process supervisor, shared-memory checkpoint store, async D2H engine,
  block checksum) linked against the HIP runtime.

Python binds both through ``ctypes`` (``easydl_amd/_native.py``): the kernels
take raw device pointers and a ``hipStream_t`` so they launch on the caller's
current stream and are capturable in HIP graphs.

Usage: ``python -m easydl_amd._build [--force]``.
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
LIBDIR = os.path.join(ROOT, "easydl_amd", "lib")
ARCH = os.environ.get("EDL_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")

KERNELS_SO = os.path.join(LIBDIR, "libedl_kernels.so")
RUNTIME_SO = os.path.join(LIBDIR, "libedl_runtime.so")


def _hipcc() -> str:
    p = shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")
    if not os.path.exists(p):
        raise RuntimeError("hipcc not found; the ROCm toolchain is required to build easydl_amd")
    return p


def _stale(target: str, sources: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"build failed: {' '.join(cmd[:6])} ...")


def _check_resolves(lib: str) -> None:
    """Fail the build (not the first GPU run) if a kernel's host launch stub is
    missing: clang's host pass can silently drop stubs of kernel templates whose
    bodies use device-only builtins."""
    r = subprocess.run(["nm", "-D", "--undefined-only", lib], capture_output=True, text=True)
    missing = [ln.split()[-1] for ln in r.stdout.splitlines() if "__device_stub__" in ln]
    if missing:
        raise RuntimeError(f"{os.path.basename(lib)}: undefined kernel launch stubs: {missing}")


# per-source extra hipcc flags (none at present: -fno-slp-vectorize on attention.hip
# measured the dK/dV kernel 12 % slower in the bench, profiles/r02_bench_kernel_stats_*)
_EXTRA_FLAGS: dict[str, list[str]] = {}


def build_kernels(force: bool = False, verbose: bool = False) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    hdrs = glob.glob(os.path.join(CSRC, "kernels", "*.h")) + glob.glob(os.path.join(CSRC, "include", "*.h"))
    deps = srcs + hdrs
    os.makedirs(LIBDIR, exist_ok=True)
    if force or _stale(KERNELS_SO, deps):
        objs = []
        for s in srcs:
            o = os.path.join(LIBDIR, "obj", os.path.basename(s) + ".o")
            os.makedirs(os.path.dirname(o), exist_ok=True)
            if force or _stale(o, [s] + hdrs):
                cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", s, "-o", o,
                       "-Wno-unused-result"] + _EXTRA_FLAGS.get(os.path.basename(s), [])
                if verbose:
                    print(" ".join(cmd))
                _run(cmd)
            objs.append(o)
        tmp = KERNELS_SO + ".tmp"
        _run([_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs)
        _check_resolves(tmp)
        os.replace(tmp, KERNELS_SO)
    return KERNELS_SO


def build_runtime(force: bool = False, verbose: bool = False) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    deps = srcs + glob.glob(os.path.join(CSRC, "runtime", "*.h")) + glob.glob(os.path.join(CSRC, "include", "*.h"))
    os.makedirs(LIBDIR, exist_ok=True)
    if not srcs:
        return ""
    if force or _stale(RUNTIME_SO, deps):
        tmp = RUNTIME_SO + ".tmp"
        # Host-only C++ (no device code): compiled by hipcc's clang in host mode,
        # linked against libamdhip64 for the pinned-memory / async-copy engine.
        cmd = [_hipcc(), "-O2", "-std=c++17", "-fPIC", "-shared", "-x", "c++", *srcs, "-o", tmp,
               "-D__HIP_PLATFORM_AMD__", f"-I{ROCM}/include", f"-L{ROCM}/lib", "-lamdhip64", "-lpthread", "-ldl",
               "-Wl,-rpath," + f"{ROCM}/lib"]
        if verbose:
            print(" ".join(cmd))
        _run(cmd)
        os.replace(tmp, RUNTIME_SO)
    return RUNTIME_SO


def build_all(force: bool = False, verbose: bool = False) -> list[str]:
    return [build_kernels(force, verbose), build_runtime(force, verbose)]


if __name__ == "__main__":
    out = build_all(force="--force" in sys.argv, verbose="-v" in sys.argv)
    print("\n".join(p for p in out if p))
