"""In-tree build of the native HIP/C++ libraries for gfx950.

``python -m rnb_amd.build [--force] [-j N]`` compiles every library below with
``hipcc --offload-arch=gfx950`` into ``rnb_amd/_native/``. The libraries are
plain C-ABI shared objects loaded with ctypes (``rnb_amd/ops/native.py``), so
they do not depend on the PyTorch C++ ABI. Every source compiles to its own
object under ``build/obj/`` in parallel (``-j``) and the objects link into the
.so; an object is rebuilt only when its source, a ``csrc`` header or this file
is newer than it, and a library only when one of its objects is.
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
OUT = os.path.join(ROOT, "rnb_amd", "_native")
ARCH = os.environ.get("RNB_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")

# name -> (sources, extra flags, extra link libs)
LIBRARIES = {
    "librnb_kernels.so": (["conv_igemm.hip", "conv_halo.hip", "conv_temporal.hip",
                           "video_ops.hip", "bn_ops.hip", "conv_halo_ws.hip", "conv21.hip",
                           "conv_f32.hip", "conv_wino_f32.hip", "conv_wino_x6.hip",
                           "conv_x6.hip", "conv_h3.hip", "conv_h3stem.hip", "conv_h3p.hip",
                           "conv_h3w.hip"],
                          [], []),
    "librnb_runtime.so": (["runtime.cpp"], [], []),
    "librnb_tracer.so": (["tracer.cpp"], [], ["-L%s/lib" % ROCM, "-lrocprofiler-sdk",
                                               "-Wl,-rpath,%s/lib" % ROCM]),
}

# experiment kernels measured slower than the autotune set (profiles/NOTES.md
# round 5: the wave-specialised temporal conv_h3u and the stride-2 row-band
# conv_h3s), kept out of the product library: ``--exp`` builds them into
# rnb_amd/_native/exp/, where ops/native.py picks them up if present (their
# launches then resolve the range flag from librnb_kernels.so)
EXP_LIBRARIES = {
    "exp/librnb_h3exp.so": (["bench/conv_h3u.hip", "bench/conv_h3s.hip"], [], []),
}


def hipcc() -> str:
    exe = shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")
    if not os.path.exists(exe):
        raise RuntimeError("hipcc not found (ROCM_PATH=%s)" % ROCM)
    return exe


def _stale(target: str, sources) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    headers = [os.path.join(CSRC, h) for h in sorted(os.listdir(CSRC)) if h.endswith(".h")]
    deps = list(sources) + headers + [os.path.abspath(__file__)]
    return any(os.path.getmtime(s) > t for s in deps)


def _compile(src: str, obj: str, flags, verbose: bool) -> str:
    os.makedirs(os.path.dirname(obj), exist_ok=True)
    tmp = obj + ".tmp.%d" % os.getpid()
    cmd = [hipcc(), "--offload-arch=%s" % ARCH, "-O3", "-std=c++17", "-fPIC", "-c",
           "-Wall", "-Wno-unused-function", "-Wno-unused-variable",
           "-Wno-unused-result"] + list(flags) + [src, "-o", tmp]
    if verbose:
        print(" ".join(cmd), flush=True)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError("compiling %s failed:\n%s\n%s" % (src, res.stdout, res.stderr))
    os.replace(tmp, obj)
    return obj


def build_one(name: str, force: bool = False, verbose: bool = False, pool=None) -> str:
    srcs, flags, libs = LIBRARIES[name] if name in LIBRARIES else EXP_LIBRARIES[name]
    srcs = [os.path.join(CSRC, s) for s in srcs]
    missing = [s for s in srcs if not os.path.exists(s)]
    if missing:
        raise FileNotFoundError("missing sources for %s: %s" % (name, missing))
    target = os.path.join(OUT, name)
    objdir = os.path.join(ROOT, "build", "obj", ARCH)
    objs = [os.path.join(objdir, os.path.basename(s) + ".o") for s in srcs]
    todo = [(s, o) for s, o in zip(srcs, objs) if force or _stale(o, [s])]
    if todo:
        if pool is None:
            for s, o in todo:
                _compile(s, o, flags, verbose)
        else:
            for f in [pool.submit(_compile, s, o, flags, verbose) for s, o in todo]:
                f.result()
    if not force and not todo and os.path.exists(target) and \
            all(os.path.getmtime(o) <= os.path.getmtime(target) for o in objs):
        return target
    os.makedirs(os.path.dirname(target), exist_ok=True)
    tmp = target + ".tmp.%d" % os.getpid()
    cmd = [hipcc(), "--offload-arch=%s" % ARCH, "-fPIC", "-shared"] + objs + ["-o", tmp] + libs
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError("linking %s failed:\n%s\n%s" % (name, res.stdout, res.stderr))
    os.replace(tmp, target)
    return target


def build_all(force: bool = False, jobs: int = 8, verbose: bool = False, exp: bool = False):
    # one pool compiles the objects of every library; the libraries link in turn
    names = list(LIBRARIES) + (list(EXP_LIBRARIES) if exp else [])
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        return {n: build_one(n, force, verbose, ex) for n in names}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=8)
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--exp", action="store_true",
                    help="also build the experiment kernels (csrc/bench) into _native/exp/")
    args = ap.parse_args(argv)
    for name, path in build_all(args.force, args.jobs, args.verbose, args.exp).items():
        print("built %-22s -> %s" % (name, os.path.relpath(path, ROOT)))
    return 0


if __name__ == "__main__":
    sys.exit(main())
