"""In-tree native build of ``_C.so`` for gfx950 (MI355X).

The reference builds ``libtrt_dft_plugins.so`` with CMake driven by setup.py
(/root/reference/CMakeLists.txt:22-28, /root/reference/setup.py:30-48).  Here the HIP
kernels (no torch headers, fast) and the torch op layer (torch headers, slow) are compiled
by ``hipcc --offload-arch=gfx950`` into objects under ``build/`` and linked into a single
``tensorrt_dft_plugins_amd/_C.so`` that sits next to the package (where ``load_plugins()``
looks, like the reference's CMAKE_LIBRARY_OUTPUT_DIRECTORY).  No hipify step, no CUDA
sources, no rocFFT/hipFFT/hipBLAS link.

Usage: ``python -m tensorrt_dft_plugins_amd._build [--force] [-j N] [--out DIR] [--from-source]``

Provenance: every link embeds ``amd_dft_build_info()`` = the SHA-256 of the sources (all of
csrc/, the target and the compile flags), the host and the time.  ``build()`` skips work only
when the library's embedded digest equals the current sources' (not by file times, which a
snapshot copy does not preserve reliably); ``library_status()`` reports it, and the GPU-tier
conftest rebuilds the library from source on the GPU box before any test loads it
(``from_source=True``: every object compiled there), so the GPU tier always runs a library
compiled on that machine from exactly these sources.

``--out DIR`` builds a separate copy (objects under DIR/obj, library DIR/_C.so) without touching
the in-tree one: scripts/ci_gpu.sh compiles every source on the GPU box this way and runs the
GPU tier against that library (``MI_DFT_LIB=DIR/_C.so``), the reference's build-then-test
practice (/root/reference/build_with_docker.sh:39).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import hashlib
import os
import socket
import shutil
import subprocess
import sys
import sysconfig
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "native")
PKG = os.path.join(ROOT, "tensorrt_dft_plugins_amd")
LIB = os.path.join(PKG, "_C.so")
# host AddressSanitizer variant: the torch op layer / plan builder (host C++)
# instrumented, device code unchanged; written to build/asan/_C.so, loaded via MI_DFT_LIB with
# the ASan runtime preloaded (scripts/ci_cpu.sh)
BUILD_ASAN = os.path.join(ROOT, "build", "asan")
LIB_ASAN = os.path.join(BUILD_ASAN, "_C.so")
ASAN_FLAGS = ["-fsanitize=address", "-fno-omit-frame-pointer", "-fno-gpu-sanitize"]
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]


def _hipcc() -> str:
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    p = os.path.join(rocm, "bin", "hipcc")
    return p if os.path.exists(p) else (shutil.which("hipcc") or "hipcc")


def _torch_paths():
    import torch

    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    return inc, os.path.join(tdir, "lib"), int(torch._C._GLIBCXX_USE_CXX11_ABI)


def sources():
    """(path, needs_torch) for every native translation unit."""
    out = []
    for p in sorted(glob.glob(os.path.join(CSRC, "**", "*.hip"), recursive=True)):
        out.append((p, False))
    for p in sorted(glob.glob(os.path.join(CSRC, "**", "*.cpp"), recursive=True)):
        out.append((p, "/ops/" in p.replace(os.sep, "/")))
    return out


# bump when the compile / link command lines below change (part of the source digest)
_FLAGS_VERSION = "r5-1"
_DIGEST_MARK = b"amd_dft_source_digest="


def source_digest() -> str:
    """SHA-256 over every file of csrc/ (path + content), the target arch and the flags version."""
    h = hashlib.sha256()
    h.update(f"{ARCH}|{_FLAGS_VERSION}|{os.environ.get('MI_DFT_HIPCC_EXTRA', '')}|"
             f"{os.environ.get('MI_DFT_DEVICE_CHECKS', '0')}".encode())
    files = []
    for ext in ("hip", "cpp", "h"):
        files += glob.glob(os.path.join(CSRC, "**", f"*.{ext}"), recursive=True)
    for f in sorted(files):
        h.update(os.path.relpath(f, CSRC).replace(os.sep, "/").encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()


def embedded_digest(lib: str) -> str | None:
    """The source digest a built library carries (read from the file, without loading it)."""
    try:
        with open(lib, "rb") as f:
            data = f.read()
    except OSError:
        return None
    i = data.find(_DIGEST_MARK)
    if i < 0:
        return None
    j = i + len(_DIGEST_MARK)
    return data[j:j + 64].decode(errors="replace")


def embedded_info(lib: str) -> str | None:
    """The whole provenance string (digest, host, time) a built library carries."""
    try:
        with open(lib, "rb") as f:
            data = f.read()
    except OSError:
        return None
    i = data.find(_DIGEST_MARK)
    if i < 0:
        return None
    j = data.find(b"\0", i)
    return data[i:j if j > 0 else i + 200].decode(errors="replace")


def library_status(lib: str | None = None) -> dict:
    """{"path", "exists", "digest_ok"}: does the library match the current sources?"""
    lib = lib or os.environ.get("MI_DFT_LIB") or LIB
    d = embedded_digest(lib)
    return {"path": lib, "exists": os.path.exists(lib), "digest_ok": d is not None and d == source_digest()}


def _build_info_obj(obj_dir: str, digest: str) -> str:
    """A tiny translation unit carrying the provenance string, compiled fresh at every link."""
    src = os.path.join(obj_dir, "build_info.cpp")
    info = f"{_DIGEST_MARK.decode()}{digest} host={socket.gethostname()} time={time.strftime('%Y-%m-%dT%H:%M:%SZ', time.gmtime())}"
    with open(src, "w") as f:
        f.write('extern "C" const char* amd_dft_build_info() { return "' + info + '"; }\n')
    obj = src[:-4] + ".o"
    cmd = [_hipcc(), "-c", "-fPIC", "-x", "c++", "-o", obj, src]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{r.stdout}\n{r.stderr}")
    return obj


def _headers_digest() -> str:
    h = hashlib.sha256()
    for f in sorted(glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)):
        h.update(os.path.relpath(f, CSRC).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def _object_key(src: str, needs_torch: bool, asan: bool, hdr_digest: str) -> str:
    """What an object was compiled from: the source's content, every header's content and the
    compile configuration.  Stored next to the object (``.o.key``); an object is reused only when
    its key matches (file times are not trusted: a snapshot or ``cp -p`` can restore older source
    times over newer objects)."""
    h = hashlib.sha256()
    with open(src, "rb") as fh:
        h.update(fh.read())
    h.update(f"|{hdr_digest}|{ARCH}|{_FLAGS_VERSION}|{needs_torch}|{asan}|{os.environ.get('MI_DFT_HIPCC_EXTRA', '')}|"
             f"{os.environ.get('MI_DFT_DEVICE_CHECKS', '0')}".encode())
    return h.hexdigest()


def _key_path(obj: str) -> str:
    return obj + ".key"


def _read_key(obj: str) -> str | None:
    try:
        with open(_key_path(obj)) as f:
            return f.read().strip()
    except OSError:
        return None


def _obj_path(src: str, asan: bool = False, obj_dir: str | None = None) -> str:
    rel = os.path.relpath(src, CSRC).replace(os.sep, "_")
    if obj_dir:
        return os.path.join(obj_dir, rel + ".o")
    return os.path.join(BUILD_ASAN if asan and not src.endswith(".hip") else BUILD, rel + ".o")


def _file_flags(src: str) -> list:
    """Per-file hipcc flags from a ``// amd_dft-build-flags: ...`` line in the first lines of the
    source (e.g. -fno-slp-vectorize where SLP-packed f32 ops sit between MFMAs)."""
    with open(src) as f:
        for _, line in zip(range(40), f):
            if line.startswith("// amd_dft-build-flags:"):
                return line.split(":", 1)[1].split()
    return []


def _compile(src: str, needs_torch: bool, tinc, abi: int, asan: bool = False, obj_dir: str | None = None) -> str:
    obj = _obj_path(src, asan, obj_dir)
    cmd = [_hipcc(), "-c", "-fPIC", "-std=c++17", "-O3", "-Wall", "-Wno-unused-function",
           "-Wno-unused-variable", "-Wno-sign-compare", "-I" + CSRC,
           f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-o", obj]
    if src.endswith(".hip"):
        # -fno-slp-vectorize: SLP packs f32 pairs into v_pk_* ops plus the v_mov shuffles to feed
        # them; measured faster without on every kernel family here (scripts/ab_slp.sh:
        # afno 561->537 us, rfft2 18.8->17.9 us, AFNO R2C-W 387->320 us).
        cmd += ["-x", "hip", f"--offload-arch={ARCH}", "-munsafe-fp-atomics", "-fno-slp-vectorize"]
        cmd += _file_flags(src) + os.environ.get("MI_DFT_HIPCC_EXTRA", "").split()
        if os.environ.get("MI_DFT_DEVICE_CHECKS", "0") not in ("", "0"):
            # debug build: device-side bounds checks (csrc/fft/dev_check.h); rebuild with --force
            cmd += ["-DAMD_DFT_DEVICE_CHECKS=1"]
    else:
        # host-only C++ that includes HIP runtime headers (torch's c10/hip)
        rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
        cmd += ["-x", "c++", "-I" + os.path.join(rocm, "include"), "-D__HIP_PLATFORM_AMD__=1"]
        # the -D switches of MI_DFT_HIPCC_EXTRA (e.g. -DAMD_DFT_TUNING=1: the kernel-selection knobs
        # in the host code, csrc/ops/tuning.h) reach the host objects too
        cmd += [f for f in os.environ.get("MI_DFT_HIPCC_EXTRA", "").split() if f.startswith("-D")]
        if asan:
            cmd += ASAN_FLAGS
    if needs_torch:
        cmd += ["-O2", "-DUSE_ROCM=1", "-Wno-deprecated-declarations", "-Wno-unknown-pragmas"]
        cmd += ["-I" + p for p in tinc]
        cmd += ["-I" + sysconfig.get_paths()["include"]]
    cmd.append(src)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, jobs: int | None = None, verbose: bool = True, asan: bool = False,
          out: str | None = None, from_source: bool = False) -> str:
    """Compile every HIP/C++ source for gfx950 and link ``_C.so``; returns its path.
    ``asan``: host C++ with AddressSanitizer into build/asan/_C.so (device objects shared).
    ``out``: a separate build directory (objects in out/obj, library out/_C.so).
    ``from_source``: relink even when the library's digest matches, from objects compiled on
    THIS host (objects from another host's build directory are not reused: a per-host object
    directory), i.e. a full compile on a machine that has not built these sources yet."""
    if out and asan:
        raise ValueError("--out and --asan are exclusive")
    obj_dir = os.path.join(os.path.abspath(out), "obj") if out else None
    if from_source and not out and not asan:
        obj_dir = os.path.join(ROOT, "build", f"host-{socket.gethostname()}")
    os.makedirs(obj_dir or BUILD, exist_ok=True)
    if asan:
        os.makedirs(BUILD_ASAN, exist_ok=True)
    lib = os.path.join(os.path.abspath(out), "_C.so") if out else (LIB_ASAN if asan else LIB)
    digest = source_digest()
    if not (force or from_source) and embedded_digest(lib) == digest:
        return lib  # up to date with exactly these sources
    tinc, tlib, abi = _torch_paths()
    hdr = _headers_digest()
    srcs = sources()
    todo = []
    keys = {}
    for src, nt in srcs:
        obj = _obj_path(src, asan, obj_dir)
        keys[src] = _object_key(src, nt, asan and not src.endswith(".hip"), hdr)
        if force or not os.path.exists(obj) or _read_key(obj) != keys[src]:
            todo.append((src, nt))
    jobs = jobs or max(1, min(int(os.environ.get("MAX_JOBS", "8") or 8), os.cpu_count() or 4, 16))
    t0 = time.time()
    if todo:
        if verbose:
            print(f"[amd_dft build] compiling {len(todo)} file(s) for {ARCH} with {jobs} jobs"
                  + (" (host ASan)" if asan else ""), flush=True)
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            futs = {ex.submit(_compile, s, nt, tinc, abi, asan, obj_dir): s for s, nt in todo}
            for f in cf.as_completed(futs):
                obj = f.result()
                with open(_key_path(obj), "w") as kf:
                    kf.write(keys[futs[f]] + "\n")
                if verbose:
                    print("  built", os.path.relpath(futs[f], ROOT), flush=True)
    objs = [_obj_path(s, asan, obj_dir) for s, _ in srcs]
    # digest mismatch, --force or from_source: always relink (with a fresh provenance record); every
    # object's key was checked against its source above, so the stamped digest is true
    if True:
        objs = objs + [_build_info_obj(obj_dir or (BUILD_ASAN if asan else BUILD), digest)]
        tmp = lib + ".tmp"
        cmd = [_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + objs + [
            "-L" + tlib, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
            "-Wl,-rpath," + tlib]
        if asan:
            cmd += ["-fsanitize=address", "-shared-libasan", "-fno-gpu-sanitize"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, lib)
        if verbose:
            print(f"[amd_dft build] linked {os.path.relpath(lib, ROOT)} ({len(todo)} compiled on "
                  f"{socket.gethostname()}, {time.time() - t0:.0f} s, sources {digest[:12]})", flush=True)
    return lib


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("--asan", action="store_true", help="host AddressSanitizer build into build/asan/_C.so")
    ap.add_argument("--out", default=None, help="separate build directory (library at OUT/_C.so)")
    ap.add_argument("--from-source", action="store_true", help="compile every object on this host and relink")
    a = ap.parse_args(argv)
    build(force=a.force, jobs=a.j, asan=a.asan, out=a.out, from_source=a.from_source)


if __name__ == "__main__":
    sys.exit(main())
