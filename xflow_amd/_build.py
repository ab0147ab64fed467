"""In-tree native build of xflow-amd (no setuptools, no JIT cache).

Products (all under the repo, so they travel to the GPU box with the tree):
  xflow_amd/_xflow_native<EXT_SUFFIX>   pybind11 module (engine, kernels, reader)
  build/lib/libxflow_api.so             C API (XFCreate / XFStartTrain ...)
  build/bin/xflow_lr                    native CLI, argv-compatible with the reference

HIP sources are compiled for gfx950 only (``hipcc --offload-arch=gfx950``).
Host C++ is compiled with g++.  Objects are rebuilt when their source or any
header under csrc/ is newer.  Usage: ``python -m xflow_amd._build [-j N] [--force]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build")
# XFLOW_DEVICE_ASSERT=1: debug build with device-side bounds asserts
# (XF_DASSERT in csrc/hip/hip_util.h); objects go to their own directory
DEVICE_ASSERT = os.environ.get("XFLOW_DEVICE_ASSERT", "0") not in ("", "0")
# XFLOW_KTIMING=1: diagnostic build with per-phase cycle counters in the
# standard-FM producer (XF_KT in csrc/hip/kernels_model.hip), own directory
KTIMING = os.environ.get("XFLOW_KTIMING", "0") not in ("", "0")
OBJ = os.path.join(BUILD, "obj-dassert" if DEVICE_ASSERT else ("obj-ktime" if KTIMING else "obj"))
PKG = os.path.join(ROOT, "xflow_amd")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("XFLOW_OFFLOAD_ARCH", "gfx950")

HIPCC = os.path.join(ROCM, "bin", "hipcc")
CXX = os.environ.get("CXX", "g++")

COMMON_FLAGS = ["-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function", "-ffp-contract=off",
                "-I" + os.path.join(CSRC, "include"), "-I" + os.path.join(CSRC, "capi")]
# -ffp-contract=off: keep the device FTRL / loss math bit-identical to the CPU
# backend and the reference (no silent FMA contraction).
HIP_FLAGS = ["--offload-arch=" + ARCH, "-ffp-contract=off", "-mcode-object-version=5",
             "-I" + os.path.join(CSRC, "hip"), "-Wno-unused-result"] + \
            (["-DXFLOW_DEVICE_ASSERT=1"] if DEVICE_ASSERT else []) + \
            (["-DXFLOW_KTIMING=1"] if KTIMING else [])

HOST_SOURCES = ["io/reader.cpp", "cpu/cpu_backend.cpp", "engine/engine.cpp", "engine/trainer.cpp"]


def native_module_path() -> str:
    return os.path.join(PKG, "_xflow_native" + sysconfig.get_config_var("EXT_SUFFIX"))


def _headers_mtime() -> float:
    hs = glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def _obj_path(src: str) -> str:
    rel = os.path.relpath(src, CSRC).replace(os.sep, "_")
    return os.path.join(OBJ, rel + ".o")


def _stale(target: str, deps: list[str], hdr_mtime: float) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps) or hdr_mtime > t


def _run(cmd: list[str], verbose: bool) -> None:
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build step failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    if r.stdout.strip() and verbose:
        print(r.stdout)


def _compile_cmd(src: str) -> list[str]:
    out = _obj_path(src)
    if src.endswith(".hip"):
        return [HIPCC, "-c", src, "-o", out] + COMMON_FLAGS + HIP_FLAGS
    if src.endswith(("rccl_comm.cpp", "peer_window.cpp")):  # host code against the HIP runtime
        return [HIPCC, "-c", src, "-o", out] + COMMON_FLAGS
    flags = list(COMMON_FLAGS)
    if src.endswith("module.cpp"):
        import pybind11

        flags += ["-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"],
                  "-fvisibility=hidden"]
    return [CXX, "-c", src, "-o", out] + flags


def build(jobs: int | None = None, force: bool = False, verbose: bool = False) -> dict:
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(os.path.join(BUILD, "lib"), exist_ok=True)
    os.makedirs(os.path.join(BUILD, "bin"), exist_ok=True)
    hdr = _headers_mtime()
    hip_srcs = sorted(glob.glob(os.path.join(CSRC, "hip", "*.hip")))
    host_srcs = [os.path.join(CSRC, s) for s in HOST_SOURCES]
    mod_src = os.path.join(CSRC, "python", "module.cpp")
    comm_src = os.path.join(CSRC, "comm", "rccl_comm.cpp")
    step_src = os.path.join(CSRC, "comm", "sharded_step.cpp")
    aps_srcs = [os.path.join(CSRC, "comm", f) for f in ("async_ps.cpp", "peer_window.cpp")]
    capi_src = os.path.join(CSRC, "capi", "c_api.cpp")
    cli_src = os.path.join(CSRC, "tools", "xflow_lr.cpp")
    all_srcs = hip_srcs + host_srcs + [mod_src, comm_src, step_src, capi_src, cli_src] + aps_srcs
    todo = [s for s in all_srcs if force or _stale(_obj_path(s), [s], hdr)]
    jobs = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = [ex.submit(_run, _compile_cmd(s), verbose) for s in todo]
        for f in futs:
            f.result()

    core_objs = [_obj_path(s) for s in hip_srcs + host_srcs]
    link = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC"]
    rocm_lib = os.path.join(ROCM, "lib")
    products = {}

    # Python module: resolve libamdhip64 from torch's bundled ROCm first, so a
    # process that imports torch and this module shares ONE HIP runtime.
    torch_lib = None
    try:
        import importlib.util

        spec = importlib.util.find_spec("torch")
        if spec and spec.submodule_search_locations:
            torch_lib = os.path.join(list(spec.submodule_search_locations)[0], "lib")
    except Exception:  # pragma: no cover
        torch_lib = None
    rpaths = ([torch_lib] if torch_lib else []) + [rocm_lib]
    mod_out = native_module_path()
    mod_objs = core_objs + [_obj_path(mod_src), _obj_path(comm_src), _obj_path(step_src)] + \
        [_obj_path(s) for s in aps_srcs]
    if force or _stale(mod_out, mod_objs, 0.0):
        # librccl.so.1 resolves to the RCCL torch has already loaded (same SONAME)
        _run(link + mod_objs + ["-o", mod_out, "-L" + rocm_lib, "-lrccl", "-lrt"] +
             [f"-Wl,-rpath,{p}" for p in rpaths], verbose)
    products["module"] = mod_out

    capi_out = os.path.join(BUILD, "lib", "libxflow_api.so")
    capi_objs = core_objs + [_obj_path(capi_src)]
    if force or _stale(capi_out, capi_objs, 0.0):
        _run(link + capi_objs + ["-o", capi_out, f"-Wl,-rpath,{rocm_lib}", "-lpthread"], verbose)
    products["capi"] = capi_out
    shutil.copyfile(os.path.join(CSRC, "capi", "c_api.h"), os.path.join(BUILD, "lib", "c_api.h"))

    cli_out = os.path.join(BUILD, "bin", "xflow_lr")
    cli_objs = core_objs + [_obj_path(cli_src)]
    if force or _stale(cli_out, cli_objs, 0.0):
        _run([HIPCC, "--offload-arch=" + ARCH] + cli_objs +
             ["-o", cli_out, f"-Wl,-rpath,{rocm_lib}", "-lpthread"], verbose)
    products["cli"] = cli_out
    # what this call compiled (an object newer than its source and every
    # header is reused: a fresh checkout compiles all of them)
    products["compiled"] = f"{len(todo)} of {len(all_srcs)} sources"
    return products


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    prods = build(a.jobs, a.force, a.verbose)
    for k, v in prods.items():
        print(f"{k}: {v}")


if __name__ == "__main__":
    sys.exit(main())
