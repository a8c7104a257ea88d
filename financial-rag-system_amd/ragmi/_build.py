"""Build libragmi.so in-tree with hipcc for gfx950 (no JIT cache, so the .so travels with
the repo snapshot to the GPU box)."""
from __future__ import annotations

import os
import subprocess

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)                      # financial-rag-system_amd/
CSRC = os.path.join(ROOT, "csrc")
LIB_PATH = os.path.join(PKG_DIR, "libragmi.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

# translation units of libragmi.so
SOURCES = ["index_capi.hip", "bert_capi.hip", "wordpiece_capi.cpp"]
HEADERS = ["device_common.hpp", "common_host.hpp", "scan_kernels.hip", "bert_kernels.hip"]


def _inputs():
    files = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    files.append(os.path.join(os.path.dirname(ROOT), "include", "ragmi.h"))
    files.append(os.path.join(os.path.dirname(ROOT), "include", "ragmi_bert.h"))
    return [f for f in files if os.path.exists(f)]


def needs_build() -> bool:
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    return any(os.path.getmtime(f) > t for f in _inputs())


def build(force: bool = False, verbose: bool = False, out: str | None = None,
          defines: tuple = ()) -> str:
    """Compile libragmi.so (in-tree unless `out`: an A/B build of the same sources with extra
    `-D` defines, loaded through RAGMI_LIB_AB)."""
    lib = out or LIB_PATH
    if not force and not out and not needs_build():
        return LIB_PATH
    srcs = [os.path.join(CSRC, s) for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]
    objs, procs = [], []
    for src in srcs:                     # translation units compile in parallel
        obj = (os.path.join(CSRC, os.path.basename(src) + ".o") if not out else
               lib + "." + os.path.basename(src) + ".o")
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
               "-fno-strict-aliasing", "-Wall", "-Wno-unused-function", *defines, "-c", src,
               "-o", obj]
        if verbose:
            print(" ".join(cmd))
        procs.append((subprocess.Popen(cmd), cmd))
        objs.append(obj)
    failed = [cmd for p, cmd in procs if p.wait() != 0]
    if failed:
        raise subprocess.CalledProcessError(1, failed[0])
    tmp = lib + ".tmp"
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(tmp, lib)
    for o in objs:
        os.remove(o)
    return lib


if __name__ == "__main__":
    import sys
    # python ragmi/_build.py [OUT.so [-DNAME=V ...]]: an A/B build beside the in-tree one
    if len(sys.argv) > 1:
        os.makedirs(os.path.dirname(os.path.abspath(sys.argv[1])), exist_ok=True)
        print(build(force=True, verbose=True, out=os.path.abspath(sys.argv[1]),
                    defines=tuple(sys.argv[2:])))
    else:
        print(build(force=True, verbose=True))
