"""Build the native extension ``mamba_distributed_amd/_C.so`` for gfx950 (MI355X) — in-tree.

  python -m mamba_distributed_amd.csrc.build [--jobs N] [--force] [--debug]

* ``kernels/*.hip``  pure HIP/CDNA4 device code + host launchers (no torch headers -> fast
  compiles), ``hipcc -c --offload-arch=gfx950 -O3``.
* ``runtime/*.cpp``  host-only C++ runtime pieces (``token_loader.cpp``: mmap'd .npy shards +
  prefetch thread, ``torch.classes.mamba_amd.TokenLoader``), g++ against torch's headers.
* ``bindings.cpp``   the PyTorch operator registrations (``TORCH_LIBRARY(mamba_amd, ...)``),
  compiled against torch's headers.
* Linked with hipcc into ``_C.so`` against torch's own libraries (the HIP runtime is the one
  torch already loaded: same soname ``libamdhip64.so.7``).

Incremental: an object is rebuilt only when its source or a header in csrc/ is newer.
No hipify, no CUDA sources, no dual code paths: gfx950 only.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig
import time

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
BUILD = os.path.join(HERE, "build")
OUT = os.path.join(PKG, "_C.so")
ARCH = os.environ.get("MAMBA_AMD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
# MFMA accumulators in arch VGPRs instead of AGPRs where the kernels fit in 256 VGPRs anyway: the
# SSD chunk walks touch their running state with VALU every chunk (decay, bf16 staging), and in
# AGPRs each touch costs a v_accvgpr_read/write pair (~100 extra VALU per chunk in the forward).
PER_FILE_FLAGS = {"ssd.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"],
                  # the persistent GEMM's one-lane tile claim: without this the atomic optimizer consumes the
                  # returned value on the spot (s_waitcnt vmcnt(0) behind every in-flight K-tile DMA)
                  "gemm_pipe.hip": ["-mllvm", "-amdgpu-atomic-optimizer-strategy=None"]}


def torch_paths():
    import torch
    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    return tdir, inc, os.path.join(tdir, "lib"), int(torch._C._GLIBCXX_USE_CXX11_ABI)


def _newer(src, obj, headers):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return os.path.getmtime(src) > t or any(os.path.getmtime(h) > t for h in headers)


def _run(cmd):
    t0 = time.time()
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    return p.returncode, p.stdout, time.time() - t0, cmd


def build(jobs: int = 8, force: bool = False, debug: bool = False, verbose: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    tdir, tinc, tlib, abi = torch_paths()
    headers = glob.glob(os.path.join(HERE, "**", "*.h"), recursive=True)
    opt = ["-O0", "-g"] if debug else ["-O3"]
    common = ["-fPIC", "-std=c++17", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-I", HERE]
    hip_flags = common + opt + [f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
                                "-fno-gpu-rdc",
                                "-Wno-unused-result"]
    py_inc = sysconfig.get_paths()["include"]
    bind_flags = common + ["-O2", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DTORCH_EXTENSION_NAME=_C",
                           "-I", os.path.join(ROCM, "include"), "-I", py_inc] + sum([["-I", i] for i in tinc], [])
    jobs_list = []
    objs = []
    for src in sorted(glob.glob(os.path.join(HERE, "kernels", "*.hip"))):
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _newer(src, obj, headers) or _newer(os.path.abspath(__file__), obj, []):
            jobs_list.append([HIPCC, "-c", src, "-o", obj] + hip_flags + PER_FILE_FLAGS.get(os.path.basename(src), []))
    for src in sorted(glob.glob(os.path.join(HERE, "runtime", "*.cpp"))):
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _newer(src, obj, headers):
            jobs_list.append(["g++", "-c", src, "-o", obj, "-O3", "-pthread"] + bind_flags)
    bsrc = os.path.join(HERE, "bindings.cpp")
    bobj = os.path.join(BUILD, "bindings.cpp.o")
    objs.append(bobj)
    if force or _newer(bsrc, bobj, headers):
        jobs_list.append(["g++", "-c", bsrc, "-o", bobj] + bind_flags)
    failed = False
    if jobs_list:
        with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            for rc, out, dt, cmd in ex.map(_run, jobs_list):
                name = os.path.basename(cmd[2])
                if rc != 0:
                    failed = True
                    print(f"[build] FAILED {name} ({dt:.1f}s)\n{out}", file=sys.stderr)
                else:
                    print(f"[build] {name} ({dt:.1f}s)" + (f"\n{out}" if (verbose and out.strip()) else ""))
    if failed:
        raise RuntimeError("native build failed")
    if force or not os.path.exists(OUT) or any(os.path.getmtime(o) > os.path.getmtime(OUT) for o in objs):
        link = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", OUT] + objs + [
            "-L", tlib, "-Wl,-rpath," + tlib, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
            "-lamdhip64", "-pthread"]
        rc, out, dt, _ = _run(link)
        if rc != 0:
            print(out, file=sys.stderr)
            raise RuntimeError("native link failed")
        print(f"[build] linked {OUT} ({dt:.1f}s)")
    return OUT


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 4))
    p.add_argument("--force", action="store_true")
    p.add_argument("--debug", action="store_true")
    p.add_argument("--verbose", action="store_true")
    a = p.parse_args(argv)
    out = build(a.jobs, a.force, a.debug, a.verbose)
    # link-time check: the extension must resolve all its symbols against torch (loads on CPU too)
    import torch
    torch.ops.load_library(out)


if __name__ == "__main__":
    main()
