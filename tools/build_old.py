"""Build lib/libdad_hip_<name>.so from the csrc/ and include/ of an earlier commit (A/B runs of
tools/gpu_ab.sh against the working tree's libdad_hip.so).

    python tools/build_old.py <git-rev> [name=old] [extra hipcc flags...]
"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = "robust-speech-emotion-recognition-via-dynamic-asymmetric-distillation-in-noisy-environments_amd"
sys.path.insert(0, os.path.join(ROOT, PKG))
import _build  # noqa: E402


def main():
    rev = sys.argv[1]
    name = sys.argv[2] if len(sys.argv) > 2 else "old"
    extra = sys.argv[3:]
    tmp = tempfile.mkdtemp(prefix="dadold_")
    os.makedirs(os.path.join(tmp, PKG, "csrc"))
    os.makedirs(os.path.join(tmp, "include"))
    files = subprocess.run(["git", "ls-tree", "--name-only", rev, PKG + "/csrc/"], cwd=ROOT, check=True,
                           stdout=subprocess.PIPE, text=True).stdout.split()
    for f in files + ["include/dad.h"]:
        data = subprocess.run(["git", "show", "%s:%s" % (rev, f)], cwd=ROOT, check=True, stdout=subprocess.PIPE).stdout
        open(os.path.join(tmp, f), "wb").write(data)
    srcs = [f for f in files if f.endswith(".hip")]
    objs = []
    for s in srcs:
        o = os.path.join(tmp, os.path.basename(s) + ".o")
        subprocess.run([_build.HIPCC] + _build.CFLAGS + extra + ["-c", os.path.join(tmp, s), "-o", o], check=True)
        objs.append(o)
    out = _build.lib_path(name)
    subprocess.run([_build.HIPCC, "-shared", "-o", out] + objs + ["-L" + os.path.join(_build.ROCM, "lib"), "-lrccl"],
                   check=True)
    print("built", out, "from", rev)


if __name__ == "__main__":
    main()
