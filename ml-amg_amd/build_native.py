"""Build libmlamg_hip.so (HIP kernels + C-ABI) for gfx950 with hipcc, in-tree.

Output: ml-amg_amd/mlamg/libmlamg_hip.so. Objects go to ml-amg_amd/build/ (git-ignored).
Every translation unit is compiled with -ffp-contract=off: the bitwise parity of the sparse
kernels with scipy sparsetools depends on separate multiply/add rounding (see csrc/common.hpp).
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "build")
OUT = os.path.join(HERE, "mlamg", "libmlamg_hip.so")
INCLUDE = os.path.join(ROOT, "include")

ARCH = os.environ.get("MLAMG_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")
CXXFLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-fPIC",
    "-std=c++17",
    "-ffp-contract=off",
    "-fno-gpu-rdc",
    "-Wall",
    "-Wno-unused-function",
    "-Wno-unused-variable",
    f"-I{INCLUDE}",
]
LDFLAGS = ["-shared", "-fPIC", f"--offload-arch={ARCH}", "-lrccl"]


def _sources():
    out = []
    for f in sorted(os.listdir(CSRC)):
        if f.endswith((".hip", ".cpp")):
            out.append(os.path.join(CSRC, f))
    return out


def _headers_digest():
    h = hashlib.sha1()
    for d in (CSRC, INCLUDE):
        for f in sorted(os.listdir(d)):
            if f.endswith((".hpp", ".h")):
                with open(os.path.join(d, f), "rb") as fh:
                    h.update(fh.read())
    h.update(" ".join(CXXFLAGS).encode())
    return h.hexdigest()


def _compile(src, hdr_digest, verbose):
    base = os.path.basename(src)
    obj = os.path.join(BUILD, base + ".o")
    stamp = obj + ".stamp"
    with open(src, "rb") as fh:
        key = hashlib.sha1(fh.read() + hdr_digest.encode()).hexdigest()
    if os.path.exists(obj) and os.path.exists(stamp):
        with open(stamp) as fh:
            if fh.read().strip() == key:
                return obj, False
    lang = ["-x", "hip"] if src.endswith(".hip") else []
    cmd = [HIPCC] + CXXFLAGS + lang + ["-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {base}:\n{r.stdout}\n{r.stderr}")
    if r.stderr.strip() and verbose:
        print(r.stderr, file=sys.stderr)
    with open(stamp, "w") as fh:
        fh.write(key)
    return obj, True


def build_hostext(verbose: bool = False) -> str:
    """mlamg/_hostptr: the CPython helper of the batched amg_2_v entry (csrc/hostptr.c)."""
    import sysconfig
    src = os.path.join(CSRC, "hostptr.c")
    out = os.path.join(HERE, "mlamg", "_hostptr" + sysconfig.get_config_var("EXT_SUFFIX"))
    if os.path.exists(out) and os.path.getmtime(out) >= os.path.getmtime(src):
        return out
    cc = os.environ.get("CC", shutil.which("gcc") or "cc")
    cmd = [cc, "-O2", "-shared", "-fPIC", "-Wall", f"-I{sysconfig.get_paths()['include']}", src,
           "-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"building _hostptr failed:\n{r.stdout}\n{r.stderr}")
    os.replace(out + ".tmp", out)
    return out


def build(verbose: bool = False, jobs: int | None = None) -> str:
    os.makedirs(BUILD, exist_ok=True)
    build_hostext(verbose)
    dig = _headers_digest()
    srcs = _sources()
    jobs = jobs or min(8, len(srcs))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        results = list(ex.map(lambda s: _compile(s, dig, verbose), srcs))
    objs = [o for o, _ in results]
    rebuilt = any(c for _, c in results) or not os.path.exists(OUT)
    if rebuilt:
        tmp = OUT + ".tmp"
        cmd = [HIPCC] + objs + LDFLAGS + ["-o", tmp]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
