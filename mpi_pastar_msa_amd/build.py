"""Build the native parts of the engine in-tree (hipcc for gfx950).

  libpastar_gpu.so   HIP kernels + C-ABI (include/pastar_gpu.h)
  bin/msa_pastar     C++ CLI mirroring the reference's msa_pastar

The .so files land next to this file so that they travel with the repository
snapshot to the GPU box (they are git-ignored, not gpurun-ignored).
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libpastar_gpu.so")
CLI = os.path.join(HERE, "bin", "msa_pastar")
LISTS_DEMO = os.path.join(HERE, "bin", "pastar_lists_astar")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

# -ffp-contract=off keeps the host weight pipeline in plain IEEE single
# arithmetic (no FMA contraction), as the reference's g++ build computes it.
# no packed-FP32 instructions (hipcc -O3 forms them from ordinary float code;
# the engine's device arithmetic is integer, the flag keeps it that way for
# any float code the compiler meets; the host pass does not know the feature
# and says so, harmlessly)
COMMON = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
          "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops",
          "-I" + os.path.join(ROOT, "include"), "-I" + CSRC]
# diagnostics builds, e.g. PASTAR_HIPCC_FLAGS=-DPASTAR_PHASE_TIMERS (block-0
# phase timers of the expand kernel, read with PASTAR_TIMING_MASK=5)
COMMON += os.environ.get("PASTAR_HIPCC_FLAGS", "").split()

LIB_SOURCES = ["pastar_gpu.hip", "host_model.cpp", "wire.cpp"]
LIB_DEPS = LIB_SOURCES + ["device.hpp", "kernels.hpp", "host_model.hpp", "solo.hpp", "lists.hpp", "selftest.hpp"]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    print("+", " ".join(cmd), flush=True)
    subprocess.check_call(cmd)


def build_lib(force=False):
    deps = [os.path.join(CSRC, s) for s in LIB_DEPS] + [os.path.join(ROOT, "include", "pastar_gpu.h")]
    if not force and not _stale(LIB, deps):
        return LIB
    objs = []
    for s in LIB_SOURCES:
        src = os.path.join(CSRC, s)
        obj = os.path.join(CSRC, os.path.splitext(s)[0] + ".o")
        _run([HIPCC] + COMMON + ["-c", src, "-o", obj])
        objs.append(obj)
    _run([HIPCC, "--offload-arch=gfx950", "-shared", "-o", LIB] + objs +
         ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"])
    for o in objs:
        os.remove(o)
    return LIB


def build_cli(force=False):
    src = os.path.join(CSRC, "msa_pastar_main.cpp")
    deps = [src, LIB, os.path.join(ROOT, "include", "pastar_gpu.h")]
    if not force and not _stale(CLI, deps):
        return CLI
    os.makedirs(os.path.dirname(CLI), exist_ok=True)
    _run(["g++", "-O2", "-std=c++17", "-I" + os.path.join(ROOT, "include"), src, "-o", CLI,
          "-L" + HERE, "-lpastar_gpu", "-Wl,-rpath,$ORIGIN/.."])
    return CLI


def build_lists_demo(force=False):
    """The reference's serial worker loop over the OpenList / ClosedList
    facades (include/pastar_lists.hpp)."""
    src = os.path.join(CSRC, "lists_astar_main.cpp")
    deps = [src, LIB, os.path.join(ROOT, "include", "pastar_gpu.h"), os.path.join(ROOT, "include", "pastar_lists.hpp")]
    if not force and not _stale(LISTS_DEMO, deps):
        return LISTS_DEMO
    os.makedirs(os.path.dirname(LISTS_DEMO), exist_ok=True)
    _run(["g++", "-O2", "-std=c++17", "-Wall", "-I" + os.path.join(ROOT, "include"), src, "-o", LISTS_DEMO,
          "-L" + HERE, "-lpastar_gpu", "-Wl,-rpath,$ORIGIN/.."])
    return LISTS_DEMO


def build_all(force=False):
    build_lib(force)
    build_cli(force)
    build_lists_demo(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
