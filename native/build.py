"""Native build for hbmr: HIP kernels + C++ runtime pieces, gfx950 only.

Produces (all in-tree so they travel to the GPU box with the repo snapshot):

* ``hbmr/lib/libhbmr.so``      – HIP kernels (native/kernels/*.hip) + CPU kernels
                                  and native I/O (native/cpu/*.cc), C ABI, loaded
                                  by ``hbmr.ops`` via ctypes next to PyTorch.
* ``hbmr/lib/libhbmr_pipes.a`` – the Pipes child-side runtime (native/pipes).
* ``hbmr/lib/libhbmr_cpu.so``  – the same host-only objects as a shared library
                                  (CPU task data path: map-output sort/IFile).
* ``hbmr/lib/libhbmr_host.a``  – host-only objects (native/cpu + native/io:
                                  CPU K-Means, SequenceFile) for CPU task binaries.
* ``hbmr/bin/*``               – Pipes task executables (native/apps), e.g. the
                                  HIP K-Means GPU map binary.

No hipify, no CUDA shims: sources are HIP/C++ written for CDNA4 and compiled
with ``hipcc --offload-arch=gfx950``.  Rebuilds are incremental on mtimes
(headers included conservatively).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
NATIVE = ROOT / "native"
BUILD = ROOT / "build" / "native"
LIBDIR = ROOT / "hbmr" / "lib"
BINDIR = ROOT / "hbmr" / "bin"
ARCH = os.environ.get("HBMR_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")

HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
             "-Wno-unused-result", "-Wno-unused-value", f"-I{NATIVE / 'include'}"]
CXX_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-mavx2", "-mfma", "-pthread",
             f"-I{NATIVE / 'include'}", "-DHBMR_NO_HIP_DECLS"]


def _headers(d: Path):
    return [p for p in d.rglob("*.h")] + [p for p in d.rglob("*.hh")]


def _stale(out: Path, deps) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(str(c) for c in cmd), flush=True)
    r = subprocess.run([str(c) for c in cmd], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"native build failed: {' '.join(map(str, cmd))}\n{r.stdout}\n{r.stderr}")
    return r


def _compile_jobs(srcs, compiler, flags, objdir, hdrs):
    jobs = []
    for s in srcs:
        o = objdir / (s.relative_to(NATIVE).as_posix().replace("/", "__") + ".o")
        if _stale(o, [s, *hdrs, Path(__file__)]):
            jobs.append((s, o, [compiler, *flags, "-c", s, "-o", o]))
        else:
            jobs.append((s, o, None))
    return jobs


class _BuildLock:
    """Inter-process lock so concurrent builders (pytest-xdist workers, a test and the
    driver) never link against an object another process is still writing."""

    def __init__(self, path: Path):
        self.path = path

    def __enter__(self):
        import fcntl
        self.path.parent.mkdir(parents=True, exist_ok=True)
        self.fd = open(self.path, "w")
        fcntl.flock(self.fd, fcntl.LOCK_EX)
        return self

    def __exit__(self, *exc):
        import fcntl
        fcntl.flock(self.fd, fcntl.LOCK_UN)
        self.fd.close()


def build(verbose: bool = False, jobs: int | None = None) -> dict:
    with _BuildLock(ROOT / "build" / ".native.lock"):
        return _build(verbose, jobs)


def _build(verbose: bool, jobs: int | None) -> dict:
    BUILD.mkdir(parents=True, exist_ok=True)
    LIBDIR.mkdir(parents=True, exist_ok=True)
    BINDIR.mkdir(parents=True, exist_ok=True)
    hdrs = _headers(NATIVE)
    hip_srcs = sorted((NATIVE / "kernels").glob("*.hip"))
    cpu_srcs = sorted((NATIVE / "cpu").glob("*.cc")) + sorted((NATIVE / "io").glob("*.cc"))
    pipes_srcs = sorted((NATIVE / "pipes").rglob("*.cc"))

    work = []
    work += _compile_jobs(hip_srcs, HIPCC, HIP_FLAGS, BUILD, hdrs)
    work += _compile_jobs(cpu_srcs, CXX, CXX_FLAGS, BUILD, hdrs)
    pipes_flags = CXX_FLAGS + [f"-I{NATIVE / 'pipes' / 'api'}", f"-I{NATIVE / 'pipes'}"]
    work += _compile_jobs(pipes_srcs, CXX, pipes_flags, BUILD, hdrs)

    n = jobs or min(8, os.cpu_count() or 4)
    todo = [w for w in work if w[2] is not None]
    with cf.ThreadPoolExecutor(max_workers=n) as ex:
        list(ex.map(lambda w: _run(w[2], verbose), todo))

    objs = {s: o for s, o, _ in work}
    lib = LIBDIR / "libhbmr.so"
    lib_objs = [objs[s] for s in hip_srcs + cpu_srcs]
    if _stale(lib, lib_objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib, *lib_objs,
              "-pthread", "-lz"], verbose)
    hostlib = LIBDIR / "libhbmr_host.a"
    host_objs = [objs[s] for s in cpu_srcs]
    if _stale(hostlib, host_objs):
        if hostlib.exists():
            hostlib.unlink()
        _run(["ar", "rcs", hostlib, *host_objs], verbose)

    # host-only shared library for CPU tasks (map-output buffer, CPU K-Means,
    # SequenceFile): loadable without the HIP runtime
    cpulib = LIBDIR / "libhbmr_cpu.so"
    if _stale(cpulib, host_objs):
        _run([CXX, "-shared", "-fPIC", "-o", cpulib, *host_objs, "-pthread", "-lz"], verbose)

    out = {"libhbmr": str(lib), "libhbmr_host": str(hostlib), "libhbmr_cpu": str(cpulib)}
    if pipes_srcs:
        alib = LIBDIR / "libhbmr_pipes.a"
        pobjs = [objs[s] for s in pipes_srcs]
        if _stale(alib, pobjs):
            if alib.exists():
                alib.unlink()
            _run(["ar", "rcs", alib, *pobjs], verbose)
        out["libhbmr_pipes"] = str(alib)
        out.update(_build_apps(verbose, lib, alib, hostlib, hdrs))
    return out


def _build_apps(verbose, lib, alib, hostlib, hdrs):
    """Each native/apps/<name>.cc (CPU) or .hip (GPU) becomes hbmr/bin/<name>."""
    apps = {}
    srcs = sorted((NATIVE / "apps").glob("*.cc")) + sorted((NATIVE / "apps").glob("*.hip"))
    inc = [f"-I{NATIVE / 'include'}", f"-I{NATIVE / 'pipes' / 'api'}", f"-I{NATIVE / 'pipes'}"]
    cmds = []
    for s in srcs:
        exe = BINDIR / s.stem
        deps = [s, alib, hostlib, *hdrs]
        if s.suffix == ".hip":
            deps.append(lib)
            # compile, then link: hipcc's implicit "-x hip" would apply to the archives
            obj = BUILD / f"app__{s.stem}.o"
            cmd = [[HIPCC, *HIP_FLAGS, *inc, "-c", s, "-o", obj],
                   [HIPCC, f"--offload-arch={ARCH}", obj, "-o", exe, alib, hostlib,
                    f"-L{LIBDIR}", "-lhbmr", "-Wl,-rpath,$ORIGIN/../lib", "-pthread", "-lz"]]
        else:
            cmd = [[CXX, *CXX_FLAGS, *inc, s, "-o", exe, alib, hostlib, "-pthread", "-lz"]]
        apps[s.stem] = str(exe)
        if _stale(exe, deps):
            cmds.append(cmd)
    n = min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(max_workers=n) as ex:
        list(ex.map(lambda cs: [_run(c, verbose) for c in cs], cmds))
    return {"apps": apps}


SANITIZERS = {
    # host code only (GPU sanitizers are not available on the MI355X pool)
    "asan": ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all"],
    "tsan": ["-fsanitize=thread", "-fno-omit-frame-pointer"],
}


def build_sanitized(kind: str, verbose: bool = False) -> dict:
    """Host-only sanitizer builds (SURVEY.md §5 race detection / sanitizers):
    the Pipes runtime, CPU kernels, SequenceFile I/O and the CPU Pipes apps,
    plus native/tests/selftest.cc, compiled with ASAN+UBSAN or TSAN into
    build/sanitize/<kind>/.  Returns {name: executable}."""
    out_dir = ROOT / "build" / "sanitize" / kind
    with _BuildLock(out_dir.parent / f".{kind}.lock"):
        return _build_sanitized(kind, out_dir, verbose)


def _build_sanitized(kind: str, out_dir: Path, verbose: bool) -> dict:
    flags = SANITIZERS[kind]
    out_dir.mkdir(parents=True, exist_ok=True)
    hdrs = _headers(NATIVE)
    srcs = (sorted((NATIVE / "cpu").glob("*.cc")) + sorted((NATIVE / "io").glob("*.cc")) +
            sorted((NATIVE / "pipes").rglob("*.cc")))
    inc = [f"-I{NATIVE / 'include'}", f"-I{NATIVE / 'pipes' / 'api'}", f"-I{NATIVE / 'pipes'}"]
    base = ["-O1", "-g", "-std=c++17", "-pthread", "-DHBMR_NO_HIP_DECLS", *inc, *flags]
    work = []
    for src in srcs:
        o = out_dir / (src.relative_to(NATIVE).as_posix().replace("/", "__") + ".o")
        if _stale(o, [src, *hdrs, Path(__file__)]):
            work.append([CXX, *base, "-c", src, "-o", o])
    n = min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(max_workers=n) as ex:
        list(ex.map(lambda c: _run(c, verbose), work))
    objs = [out_dir / (src.relative_to(NATIVE).as_posix().replace("/", "__") + ".o")
            for src in srcs]
    exes = {}
    mains = sorted((NATIVE / "apps").glob("*.cc")) + sorted((NATIVE / "tests").glob("*.cc"))
    cmds = []
    for m in mains:
        exe = out_dir / m.stem
        exes[m.stem] = str(exe)
        if _stale(exe, [m, *objs, *hdrs]):
            cmds.append([CXX, *base, m, *objs, "-o", exe, "-lz"])
    with cf.ThreadPoolExecutor(max_workers=n) as ex:
        list(ex.map(lambda c: _run(c, verbose), cmds))
    return exes


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "sanitize":
        print(build_sanitized(sys.argv[2], verbose="-v" in sys.argv))
    else:
        res = build(verbose="-v" in sys.argv)
        print(res)
