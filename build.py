#!/usr/bin/env python3
"""In-tree native build for sharetrade.

Produces (next to the Python package, so they travel with the repo snapshot):

* ``sharetrade/_native/libsharetrade_hip.so`` — every HIP/CDNA4 kernel, built
  with ``hipcc --offload-arch=gfx950`` (C ABI, loaded with ctypes; no torch
  headers, so a full rebuild takes seconds);
* ``sharetrade/_native/libsharetrade_rt.so`` — the host-side C++ runtime
  (journal / snapshot store / checkpoint writer), built with g++.

The timing / debug builds of the flagship kernel (``csrc/ab/``) are not part of the production
library; ``python build.py --ab`` (or ``SHARETRADE_AB_BUILDS=1``) builds them into
``libsharetrade_ab.so``.

Usage: ``python build.py [--force] [--ab] [-j N]``.  Rebuilds only when a source is
newer than the library.
"""
from __future__ import annotations

import argparse
import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(ROOT, "csrc")
OUT = os.path.join(ROOT, "sharetrade", "_native")
OBJ = os.path.join(ROOT, "build", "obj")
ARCH = os.environ.get("SHARETRADE_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-ffp-contract=off", "-Wall", "-Wno-unused-function",
             "-Wno-unused-variable", "-Wno-unused-but-set-variable"]
CXX_FLAGS = ["-O2", "-std=c++17", "-fPIC", "-Wall", "-Wextra", "-Wno-unused-parameter"]

HIP_LIB = os.path.join(OUT, "libsharetrade_hip.so")
AB_LIB = os.path.join(OUT, "libsharetrade_ab.so")   # opt-in timing / debug builds (csrc/ab/)
RT_LIB = os.path.join(OUT, "libsharetrade_rt.so")


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


_INC = None


def _includes(path: str, seen=None):
    """Every local ``#include "..."`` reachable from ``path`` (recursively), so an edit to
    ``qstep_wide.hip`` rebuilds ``qstep_wide8.hip`` and its tuning variants that include it."""
    import re

    global _INC
    if _INC is None:
        _INC = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)
    seen = set() if seen is None else seen
    try:
        with open(path) as f:
            txt = f.read()
    except OSError:
        return seen
    for name in _INC.findall(txt):
        dep = os.path.normpath(os.path.join(os.path.dirname(path), name))
        if dep not in seen and os.path.exists(dep):
            seen.add(dep)
            _includes(dep, seen)
    return seen


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout)
        raise RuntimeError(f"build step failed: {cmd[0]} {cmd[-1]}")
    return r.stdout


def build_hip(force: bool = False, jobs: int = 8, ab: bool = False) -> str:
    """Production kernels: every ``csrc/*.hip`` -> libsharetrade_hip.so.  With ``ab``: the timing / debug
    builds of the flagship kernel (``csrc/ab/*.hip``: per-phase stamps, phases skipped or run twice, several
    computing wrong results by design) -> their own libsharetrade_ab.so, which only an opted-in process
    (SHARETRADE_AB_BUILDS=1) loads."""
    lib_path = AB_LIB if ab else HIP_LIB
    srcs = sorted(glob.glob(os.path.join(CSRC, "ab" if ab else "", "*.hip")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "*.h")))
    manifest = lib_path + ".srcs"   # the sources linked last time: a removed / moved source forces a relink
    listing = "\n".join(os.path.relpath(s, ROOT) for s in srcs) + "\n"
    try:
        with open(manifest) as f:
            same_srcs = f.read() == listing
    except OSError:
        same_srcs = True   # no record (first build or an older tree): the mtime rule alone decides
    if not force and same_srcs and not _newer(lib_path, srcs + hdrs + ([os.path.join(CSRC, "qstep_ws.hip")] if ab else [])):
        return lib_path   # library newer than every source: nothing to do (the object dir need not exist)
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(OUT, exist_ok=True)
    objs = []
    todo = []
    for s in srcs:
        o = os.path.join(OBJ, ("ab_" if ab else "") + os.path.basename(s) + ".o")
        objs.append(o)
        if force or _newer(o, [s] + hdrs + sorted(_includes(s))):
            todo.append((s, o))
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(lambda so: _run([HIPCC] + HIP_FLAGS + ["-c", so[0], "-o", so[1]]), todo))
    if force or todo or not same_srcs or _newer(lib_path, objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib_path] + objs)
    with open(manifest, "w") as f:
        f.write(listing)
    return lib_path


def build_rt(force: bool = False) -> str:
    srcs = sorted(f for f in glob.glob(os.path.join(CSRC, "runtime", "*.cpp"))
                  if not f.endswith("selftest.cpp"))   # standalone sanitizer driver (tests/test_sanitizers.py)
    hdrs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.h")))
    if not srcs:
        return ""
    os.makedirs(OUT, exist_ok=True)
    if force or _newer(RT_LIB, srcs + hdrs):
        _run(["g++"] + CXX_FLAGS + ["-shared", "-o", RT_LIB] + srcs + ["-lpthread"])
    return RT_LIB


def build_all(force: bool = False, jobs: int = 8, ab: bool = False):
    """Build (or confirm up to date) both libraries.  Serialised across processes by an exclusive
    lock on ``build/.lock``: the ranks of a multi-GPU job all call this before they initialise the
    process group, the first one builds, the others wait on the lock and find the libraries current
    (no rank sits in a collective while another compiles)."""
    import fcntl

    os.makedirs(os.path.dirname(OBJ), exist_ok=True)
    with open(os.path.join(os.path.dirname(OBJ), ".lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            libs = [build_hip(force, jobs)]
            if ab or os.environ.get("SHARETRADE_AB_BUILDS", "") not in ("", "0"):
                libs.append(build_hip(force, jobs, ab=True))
            rt = build_rt(force)
            if rt:
                libs.append(rt)
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)
    return libs


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--ab", action="store_true", help="also build the opt-in timing / debug kernels (csrc/ab/)")
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 1))
    a = ap.parse_args()
    for lib in build_all(a.force, a.j, a.ab):
        print(lib)
