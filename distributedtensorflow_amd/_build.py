"""In-tree build of the native extensions (no JIT cache, no site-packages install).

* ``_lib/_dtf_hip*.so``    — HIP/CDNA4 kernels (``csrc/kernels/*.hip``) + pybind11 bindings,
  compiled by ``hipcc --offload-arch=gfx950``.  The .so's ``NEEDED libamdhip64.so.7`` resolves
  to the HIP runtime torch already loaded (same soname), so the process has ONE runtime and our
  launches go on torch's streams.
* ``_lib/_dtf_native*.so`` — host runtime (crc32c, TFRecord/tfevents, TF-V2 tensor bundle,
  MNIST idx reader, prefetching batcher) in C++17 with pybind11, compiled by g++.

Incremental: object files are cached under ``build/`` keyed on source+header mtimes and flags.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import hashlib
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributedtensorflow_amd")
LIBDIR = os.path.join(PKG, "_lib")
BUILD = os.path.join(ROOT, "build")
ARCH = os.environ.get("DTF_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _ext_suffix():
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _py_includes():
    import pybind11
    return [pybind11.get_include(), sysconfig.get_paths()["include"]]


def _hash(paths, flags):
    h = hashlib.sha1()
    for p in sorted(paths):
        h.update(p.encode())
        h.update(str(os.path.getmtime(p)).encode())
    h.update(" ".join(flags).encode())
    return h.hexdigest()[:16]


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def _compile_all(jobs, max_workers):
    with cf.ThreadPoolExecutor(max_workers=max_workers) as ex:
        futs = [ex.submit(_run, j) for j in jobs]
        for f in futs:
            f.result()


def build_hip(verbose=False, jobs=None):
    src_dir = os.path.join(ROOT, "csrc", "kernels")
    srcs = sorted(glob.glob(os.path.join(src_dir, "*.hip")) + glob.glob(os.path.join(src_dir, "*.cpp")))
    headers = glob.glob(os.path.join(src_dir, "*.h")) + glob.glob(os.path.join(src_dir, "*.cuh"))
    flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result",
             "-munsafe-fp-atomics", "-ffp-contract=fast"]
    # experiment builds only (e.g. -DDTF_HALO_FREG_D2=6); part of the object-cache key
    flags += os.environ.get("DTF_HIP_EXTRA_FLAGS", "").split()
    inc = ["-I" + src_dir] + ["-I" + p for p in _py_includes()]
    os.makedirs(os.path.join(BUILD, "hip"), exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    objs, todo = [], []
    for s in srcs:
        key = _hash([s] + headers, flags)
        o = os.path.join(BUILD, "hip", os.path.basename(s) + "." + key + ".o")
        objs.append(o)
        if not os.path.exists(o):
            x = ["-x", "hip"] if s.endswith(".hip") else []
            todo.append([HIPCC] + flags + inc + x + ["-c", s, "-o", o])
    _compile_all(todo, jobs or min(8, os.cpu_count() or 4))
    out = os.path.join(LIBDIR, "_dtf_hip" + _ext_suffix())
    key = _hash(objs, flags)
    stamp = out + ".stamp"
    if not (os.path.exists(out) and os.path.exists(stamp) and open(stamp).read() == key):
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", out] + objs)
        with open(stamp, "w") as f:
            f.write(key)
    if verbose:
        print("built", out)
    return out


def build_native(verbose=False):
    src_dir = os.path.join(ROOT, "csrc", "native")
    srcs = sorted(glob.glob(os.path.join(src_dir, "*.cpp")))
    if not srcs:
        return None
    headers = glob.glob(os.path.join(src_dir, "*.h"))
    flags = ["-O3", "-std=c++17", "-fPIC", "-shared", "-msse4.2", "-pthread",
             "-fvisibility=hidden"]
    out = os.path.join(LIBDIR, "_dtf_native" + _ext_suffix())
    key = _hash(srcs + headers, flags)
    stamp = out + ".stamp"
    os.makedirs(LIBDIR, exist_ok=True)
    if not (os.path.exists(out) and os.path.exists(stamp) and open(stamp).read() == key):
        inc = ["-I" + src_dir] + ["-I" + p for p in _py_includes()]
        _run(["g++"] + flags + inc + srcs + ["-o", out, "-lrt"])
        with open(stamp, "w") as f:
            f.write(key)
    if verbose:
        print("built", out)
    return out


def build_all(verbose=False):
    build_native(verbose)
    build_hip(verbose)


if __name__ == "__main__":
    build_all(verbose=True)
    sys.exit(0)
