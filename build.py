#!/usr/bin/env python3
"""In-tree build of the native layer (no pip install, no JIT cache: the .so files travel with the repo snapshot).

Products (all under ``actor_critic_algs_on_tensorflow_amd/_C/``):
  * ``libacamd.so``   -- gfx950 HIP kernels (``csrc/kernels/*.hip``, ``hipcc --offload-arch=gfx950``) + the torch op
                         registrations (``csrc/bindings.cpp``), loaded with ``torch.ops.load_library`` and exposed as
                         ``torch.ops.acamd.*``.
  * ``_tfbundle*.so`` -- the C++ TensorFlow tensor-bundle (V2 checkpoint) codec, a pybind11 module with no torch or
                         GPU dependency (``csrc/tfbundle/``).

A ``build.ninja`` is generated under ``build/`` and driven with ninja (incremental, parallel).
Usage: ``python build.py [-j N] [--clean] [--verbose]``.
"""
from __future__ import annotations

import argparse
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "actor_critic_algs_on_tensorflow_amd")
OUT_DIR = os.path.join(PKG, "_C")
BUILD_DIR = os.path.join(ROOT, "build")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")

KERNELS = ["env_classic", "env_atari", "heads", "returns", "optim", "gemm", "gemm_plain", "gemm_conv", "gemm_group", "gemm_big",
           "conv", "conv_wgrad",
           "loss", "cnn_fused", "mlp", "ppo_head", "fc_rollout", "fc_bwd"]
# env kernels must round exactly like the PyTorch oracles: no fma contraction (the Pong physics carries its own
# `fp contract(off)` pragma, so env_atari.hip compiles like cnn_fused.hip: their shared policy-head maths rounds alike)
NO_CONTRACT = {"env_classic"}


def _torch_paths():
    import torch
    import torch.utils.cpp_extension as ce
    tdir = os.path.dirname(torch.__file__)
    return (ce.include_paths(), os.path.join(tdir, "lib"), int(torch._C._GLIBCXX_USE_CXX11_ABI))


def _pybind_include():
    import pybind11
    return pybind11.get_include()


def write_ninja(verbose=False):
    incs, tlib, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    ext_suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    lines = []
    w = lines.append
    w("ninja_required_version = 1.3")
    w(f"hipcc = {hipcc}")
    w("cxx = g++")
    w(f"kflags = -O3 -std=c++17 -fPIC --offload-arch={ARCH} -munsafe-fp-atomics -I{ROOT}/csrc/kernels "
      f"-Wno-unused-result")
    binc = " ".join(f"-isystem {p}" for p in incs)
    w(f"bflags = -O2 -std=c++17 -fPIC -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 -D_GLIBCXX_USE_CXX11_ABI={abi} "
      f"-isystem {ROCM}/include {binc} -I{ROOT}/csrc/kernels -Wno-deprecated-declarations")
    w(f"tbflags = -O2 -std=c++17 -fPIC -isystem {py_inc} -isystem {_pybind_include()} -I{ROOT}/csrc/tfbundle")
    w(f"ldflags = -shared -L{tlib} -Wl,-rpath,{tlib} -lamdhip64 -lc10 -lc10_hip -ltorch -ltorch_cpu -ltorch_hip -lrccl")
    w("rule hipcc\n  command = $hipcc $kflags $extra -c $in -o $out\n  description = HIPCC $in")
    w("rule cxx\n  command = $cxx $bflags -c $in -o $out\n  description = CXX $in")
    w("rule tbcxx\n  command = $cxx $tbflags -c $in -o $out\n  description = CXX $in")
    w("rule link\n  command = $cxx $in $ldflags -o $out\n  description = LINK $out")
    w("rule tblink\n  command = $cxx -shared $in -o $out\n  description = LINK $out")
    objs = []
    # every kernel header is an implicit dependency of every object (pong_env.h, cnn_head.h, ... are shared by
    # several translation units; a stale object would silently diverge from the oracles)
    hdr = " ".join(sorted(glob.glob(os.path.join(ROOT, "csrc", "kernels", "*.h"))))
    for k in KERNELS:
        src = os.path.join(ROOT, "csrc", "kernels", k + ".hip")
        obj = os.path.join(BUILD_DIR, k + ".o")
        extra = "-ffp-contract=off" if k in NO_CONTRACT else ""
        w(f"build {obj}: hipcc {src} | {hdr}\n  extra = {extra}")
        objs.append(obj)
    bobj = os.path.join(BUILD_DIR, "bindings.o")
    w(f"build {bobj}: cxx {os.path.join(ROOT, 'csrc', 'bindings.cpp')} | {hdr}")
    objs.append(bobj)
    w(f"build {os.path.join(OUT_DIR, 'libacamd.so')}: link {' '.join(objs)}")
    # TF-bundle codec (pybind11, no torch)
    tb_srcs = ["tf_bundle.cpp", "module.cpp"]
    tb_objs = []
    for s in tb_srcs:
        o = os.path.join(BUILD_DIR, "tb_" + s.replace(".cpp", ".o"))
        w(f"build {o}: tbcxx {os.path.join(ROOT, 'csrc', 'tfbundle', s)} | "
          f"{os.path.join(ROOT, 'csrc', 'tfbundle', 'tf_bundle.h')}")
        tb_objs.append(o)
    w(f"build {os.path.join(OUT_DIR, '_tfbundle' + ext_suffix)}: tblink {' '.join(tb_objs)}")
    os.makedirs(BUILD_DIR, exist_ok=True)
    with open(os.path.join(BUILD_DIR, "build.ninja"), "w") as f:
        f.write("\n".join(lines) + "\n")


def build(jobs=None, clean=False, verbose=False):
    if clean and os.path.isdir(BUILD_DIR):
        shutil.rmtree(BUILD_DIR)
    os.makedirs(OUT_DIR, exist_ok=True)
    write_ninja(verbose)
    ninja = shutil.which("ninja") or os.path.join(os.path.dirname(sys.executable), "ninja")
    cmd = [ninja, "-C", BUILD_DIR]
    j = jobs or int(os.environ.get("MAX_JOBS", "0") or 0) or min(8, os.cpu_count() or 4)
    cmd += ["-j", str(min(j, 16))]
    if verbose:
        cmd.append("-v")
    subprocess.run(cmd, check=True)
    return os.path.join(OUT_DIR, "libacamd.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    print(build(a.jobs, a.clean, a.verbose))


if __name__ == "__main__":
    main()
