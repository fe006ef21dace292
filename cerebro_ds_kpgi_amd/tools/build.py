"""Build the native libraries in-tree (no JIT cache, no site-packages).

* ``libcerebro_hip.so`` — every ``csrc/hip/*.hip`` compiled for gfx950 with
  hipcc (``--offload-arch=gfx950``), loaded by ``ops._hip`` through ctypes
  *after* torch so it binds to the HIP runtime torch already loaded.
* ``libcerebro_da.so``  — the C++ Direct-Access reader / pglz codec
  (``csrc/da/*.cpp``), host-only.

Objects are cached by source/header mtime; ``python -m
cerebro_ds_kpgi_amd.tools.build`` rebuilds what changed.
"""

import concurrent.futures as cf
import glob
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
LIBDIR = os.path.join(ROOT, "cerebro_ds_kpgi_amd", "_lib")
OBJDIR = os.path.join(ROOT, "build", "obj")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")

HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=" + ARCH, "-munsafe-fp-atomics",
             "-Wno-unused-result"]
CXX_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-pthread", "-Wall", "-Wno-unused-function"]


def _newer(src, obj, headers):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(f) > t for f in [src] + headers)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed: {}\n{}".format(" ".join(cmd), r.stdout))
    return r.stdout


def _build(kind, srcs, headers, out, compiler, flags, link_flags, jobs):
    os.makedirs(OBJDIR, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    objs, todo = [], []
    for s in srcs:
        o = os.path.join(OBJDIR, kind + "_" + os.path.basename(s) + ".o")
        objs.append(o)
        if _newer(s, o, headers):
            todo.append((s, o))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = [ex.submit(_run, [compiler] + flags + ["-c", s, "-o", o]) for s, o in todo]
        for f in futs:
            f.result()
    if todo or not os.path.exists(out) or any(os.path.getmtime(o) > os.path.getmtime(out)
                                               for o in objs):
        _run([compiler] + flags + ["-shared", "-o", out] + objs + link_flags)
    return out


def build_hip(jobs=8, variant="", defines=()):
    """``variant`` + ``defines`` (e.g. ``pf1``, ``["CER_FP32_PF=1"]``) build an
    A/B twin ``libcerebro_hip_{variant}.so`` loaded with ``CER_HIP_LIB``."""
    srcs = sorted(glob.glob(os.path.join(ROOT, "csrc", "hip", "*.hip")))
    if not srcs:
        return None
    headers = glob.glob(os.path.join(ROOT, "csrc", "hip", "*.h"))
    name = "libcerebro_hip{}.so".format("_" + variant if variant else "")
    out = os.path.join(LIBDIR, name)
    flags = HIP_FLAGS + ["-D" + d for d in defines]
    return _build("hip" + ("_" + variant if variant else ""), srcs, headers, out, HIPCC, flags,
                  [], jobs)


def build_da(jobs=8):
    srcs = sorted(glob.glob(os.path.join(ROOT, "csrc", "da", "*.cpp")))
    if not srcs:
        return None
    headers = glob.glob(os.path.join(ROOT, "csrc", "da", "*.h"))
    out = os.path.join(LIBDIR, "libcerebro_da.so")
    return _build("da", srcs, headers, out, os.environ.get("CXX", "g++"), CXX_FLAGS, [], jobs)


def build_all(jobs=8):
    return build_hip(jobs), build_da(jobs)


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("jobs", nargs="?", type=int, default=8)
    ap.add_argument("--variant", default="")
    ap.add_argument("-D", dest="defines", action="append", default=[])
    a = ap.parse_args()
    if a.variant:
        print(build_hip(a.jobs, a.variant, a.defines))
    else:
        print(build_all(a.jobs))
