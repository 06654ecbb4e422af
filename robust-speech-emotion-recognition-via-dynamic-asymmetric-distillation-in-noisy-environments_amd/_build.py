"""Build libdad_hip.so (the C-ABI library of include/dad.h) in-tree for gfx950.

Plain `hipcc --offload-arch=gfx950` per translation unit + one shared-library link; the
result lands in <package>/lib/ so it travels with the repo snapshot to the GPU box.
"""
import concurrent.futures
import os
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
LIB_DIR = os.path.join(PKG_DIR, "lib")
OBJ_DIR = os.path.join(PKG_DIR, "build")
LIB_PATH = os.path.join(LIB_DIR, "libdad_hip.so")
SOURCES = ["encode.hip", "encode_ws.hip", "tail.hip", "wgrad.hip", "optim.hip", "dad_abi.hip", "rccl_dp.hip", "collate.hip", "eval.hip", "utils_abi.hip", "prep.hip"]
HEADERS = ["dad_common.h", "dad_kernels.h", "dad_probe.h", "dad_prep.h", os.path.join("..", "..", "include", "dad.h")]
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
ARCH = os.environ.get("DAD_OFFLOAD_ARCH", "gfx950")
CFLAGS = ["--offload-arch=" + ARCH, "-O3", "-fPIC", "-std=c++17", "-ffp-contract=off",
          "-I" + os.path.join(ROCM, "include")]


def _newest(paths):
    return max(os.path.getmtime(p) for p in paths)


def lib_path(variant=None):
    """Diagnostic builds (e.g. DAD_PROBE_* kernels) live beside the product library."""
    return LIB_PATH if not variant else os.path.join(LIB_DIR, "libdad_hip_%s.so" % variant)


def _compile(src, variant=None, extra=()):
    odir = OBJ_DIR if not variant else os.path.join(OBJ_DIR, variant)
    obj = os.path.join(odir, os.path.splitext(src)[0] + ".o")
    deps = [os.path.join(CSRC, src)] + [os.path.join(CSRC, h) for h in HEADERS]
    if os.path.exists(obj) and os.path.getmtime(obj) >= _newest(deps):
        return obj
    cmd = [HIPCC] + CFLAGS + list(extra) + ["-c", os.path.join(CSRC, src), "-o", obj]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed for %s:\n%s" % (src, r.stdout))
    return obj


def build(verbose=True, variant=None, extra=()):
    """Compile (incrementally) and link; returns the library path.

    variant/extra: a diagnostic build with extra compiler flags into lib/libdad_hip_<variant>.so
    (loaded only when DAD_LIB_VARIANT names it; the product library is never replaced).
    """
    path = lib_path(variant)
    os.makedirs(OBJ_DIR if not variant else os.path.join(OBJ_DIR, variant), exist_ok=True)
    os.makedirs(LIB_DIR, exist_ok=True)
    jobs = min(len(SOURCES), int(os.environ.get("MAX_JOBS", "8")))
    with concurrent.futures.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, variant, extra), SOURCES))
    if not os.path.exists(path) or os.path.getmtime(path) < _newest(objs):
        cmd = [HIPCC, "-shared", "-o", path] + objs + ["-L" + os.path.join(ROCM, "lib"), "-lrccl"]
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n%s" % r.stdout)
    if verbose:
        print("built", path)
    return path


if __name__ == "__main__":
    build()
    sys.exit(0)
