"""In-tree native build (no hipify, no JIT cache).

Two shared objects are produced next to this file so they travel to the GPU box with
the repository snapshot:

* ``_smprt*.so`` -- the host runtime (mailbox transport, timeline, grad counter):
  plain C++17 + pybind11, built with g++.
* ``_C*.so``     -- the CDNA4 kernels (``csrc/kernels/*.hip``, compiled by hipcc for
  ``gfx950`` only) plus their torch bindings (``csrc/kernels/bindings.cpp``).

Builds are incremental: an object is rebuilt when its source, any header in its
directory or the flags change.

Usage: ``python -m smdistributed_modelparallel_amd._build [--jobs N] [--only runtime|kernels]``.
"""
import argparse
import concurrent.futures as cf
import glob
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
BUILD_DIR = os.path.join(os.path.dirname(PKG_DIR), "build", "native")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX")
ARCH = os.environ.get("SMP_OFFLOAD_ARCH", "gfx950")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


def _py_includes():
    import pybind11

    return [sysconfig.get_paths()["include"], pybind11.get_include()]


def _torch_paths():
    import torch

    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    return inc, os.path.join(tdir, "lib"), int(torch._C._GLIBCXX_USE_CXX11_ABI)


def _digest(paths, flags):
    h = hashlib.sha1()
    for p in sorted(paths):
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(" ".join(flags).encode())
    return h.hexdigest()


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def _compile_many(jobs, tasks, verbose):
    """tasks: list of (src, obj, cmd, deps, flags). Rebuild when stamp differs."""
    todo = []
    for src, obj, cmd, deps, flags in tasks:
        stamp = obj + ".stamp"
        digest = _digest([src] + deps, flags)
        if os.path.exists(obj) and os.path.exists(stamp) and open(stamp).read() == digest:
            continue
        todo.append((obj, cmd, stamp, digest))
    if not todo:
        return False

    def one(t):
        obj, cmd, stamp, digest = t
        os.makedirs(os.path.dirname(obj), exist_ok=True)
        _run(cmd, verbose)
        with open(stamp, "w") as f:
            f.write(digest)
        return obj

    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for fut in [ex.submit(one, t) for t in todo]:
            fut.result()
    return True


def build_runtime(jobs=8, verbose=False):
    src_dir = os.path.join(CSRC, "runtime")
    srcs = sorted(glob.glob(os.path.join(src_dir, "*.cpp")))
    hdrs = sorted(glob.glob(os.path.join(src_dir, "*.h")))
    flags = ["-O2", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall", "-Wno-unused-result"]
    inc = ["-I" + p for p in _py_includes()]
    tasks = []
    objs = []
    for s in srcs:
        obj = os.path.join(BUILD_DIR, "runtime", os.path.basename(s) + ".o")
        objs.append(obj)
        tasks.append((s, obj, ["g++"] + flags + inc + ["-c", s, "-o", obj], hdrs, flags))
    changed = _compile_many(jobs, tasks, verbose)
    out = os.path.join(PKG_DIR, "_smprt" + EXT_SUFFIX)
    if changed or not os.path.exists(out):
        _run(["g++", "-shared", "-o", out] + objs + ["-lpthread", "-ldl"], verbose)
    return out


# per-translation-unit extra flags (measured per kernel: profiles/r3/s3_rehearsal.md)
_TU_FLAGS = {"attention_d64_dq.hip": ["-fno-slp-vectorize"], "attention_d64.hip": ["-fno-slp-vectorize"]}


def build_kernels(jobs=8, verbose=False):
    src_dir = os.path.join(CSRC, "kernels")
    hip_srcs = sorted(glob.glob(os.path.join(src_dir, "*.hip")))
    rt_dir = os.path.join(CSRC, "torchrt")  # torch-aware runtime (grad tracker, IPC P2P)
    cpp_srcs = sorted(glob.glob(os.path.join(src_dir, "*.cpp"))) + sorted(glob.glob(os.path.join(rt_dir, "*.cpp")))
    hdrs = sorted(glob.glob(os.path.join(src_dir, "*.h"))) + sorted(glob.glob(os.path.join(rt_dir, "*.h")))
    tinc, tlib, abi = _torch_paths()
    common = [
        "-O3",
        "-std=c++17",
        "-fPIC",
        f"--offload-arch={ARCH}",
        "-D__HIP_PLATFORM_AMD__=1",
        "-DUSE_ROCM=1",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-munsafe-fp-atomics",
        "-Wno-unused-result",
    ]
    tasks, objs = [], []
    for s in hip_srcs:
        # kernel TUs do not include torch headers: fast to build, reusable outside torch
        obj = os.path.join(BUILD_DIR, "kernels", os.path.basename(s) + ".o")
        objs.append(obj)
        flags = common + ["-I" + src_dir] + _TU_FLAGS.get(os.path.basename(s), [])
        tasks.append((s, obj, [HIPCC] + flags + ["-c", s, "-o", obj], hdrs, flags))
    for s in cpp_srcs:
        obj = os.path.join(BUILD_DIR, "kernels", os.path.basename(s) + ".o")
        objs.append(obj)
        flags = (
            common
            + ["-I" + src_dir]
            + ["-I" + p for p in tinc + _py_includes()]
            + ["-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H", "-DHIPBLAS_V2"]
        )
        tasks.append((s, obj, [HIPCC] + flags + ["-x", "hip", "-c", s, "-o", obj], hdrs, flags))
    changed = _compile_many(jobs, tasks, verbose)
    out = os.path.join(PKG_DIR, "_C" + EXT_SUFFIX)
    if changed or not os.path.exists(out):
        _run(
            [HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", out]
            + objs
            + [
                "-L" + tlib,
                f"-Wl,-rpath,{tlib}",
                "-lc10",
                "-lc10_hip",
                "-ltorch",
                "-ltorch_cpu",
                "-ltorch_hip",
                "-ltorch_python",
                "-lamdhip64",
            ],
            verbose,
        )
    return out


def build_all(jobs=8, verbose=False, only=None):
    outs = []
    if only in (None, "runtime"):
        outs.append(build_runtime(jobs, verbose))
    if only in (None, "kernels"):
        outs.append(build_kernels(jobs, verbose))
    return outs


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--only", choices=["runtime", "kernels"], default=None)
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    for o in build_all(a.jobs, a.verbose, a.only):
        print("built", o)
    sys.exit(0)
