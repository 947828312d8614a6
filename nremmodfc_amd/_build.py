"""Build libwcsde.so (all HIP sources under csrc/) for gfx950, in-tree.

The shared library is the product: every compute entry point of the package
goes through it (nremmodfc_amd/_lib.py).  Built with plain ``hipcc`` so the
C ABI in include/wcsde.h is exactly what ships.  Each source compiles to its own
object (in parallel) under build/, then one link.

``--diag`` builds libwcsde_diag.so instead: the same sources with -DWCSDE_DIAG,
which adds the ablation entry point of csrc/wcsde_diag.h (tools/diag_*.py load
it through WCSDE_LIB_OVERRIDE).  The product library never contains it.
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libwcsde.so")
DIAG_LIB = os.path.join(HERE, "libwcsde_diag.so")
# A/B timing of two builds (or the diag build) in one session (tools/): load another in-tree library
LIB_LOAD = os.environ.get("WCSDE_LIB_OVERRIDE", LIB)
ARCH = os.environ.get("WCSDE_ARCH", "gfx950")


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False, diag=False):
    srcs = sources()
    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    headers.append(os.path.join(ROOT, "include", "wcsde.h"))
    out = DIAG_LIB if diag else LIB
    if not force and not _stale(out, srcs + headers):
        return out
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    objdir = os.path.join(ROOT, "build", "diag" if diag else "product")
    os.makedirs(objdir, exist_ok=True)
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-I", os.path.join(ROOT, "include")]
    if diag:
        flags.append("-DWCSDE_DIAG")

    def compile_one(src):
        obj = os.path.join(objdir, os.path.basename(src)[:-4] + ".o")
        if force or _stale(obj, [src] + headers):
            cmd = [hipcc, *flags, "-c", src, "-o", obj + ".tmp"]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            subprocess.run(cmd, check=True)
            os.replace(obj + ".tmp", obj)
        return obj

    jobs = max(1, min(len(srcs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(compile_one, srcs))
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True, diag="--diag" in sys.argv))
