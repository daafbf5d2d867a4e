"""Build libsdrgpu.so (gfx950 HIP kernels + C ABI) and the oracle library in-tree.

Explicit hipcc/gcc command lines, no build system: each translation unit is
compiled to an object under build/ and linked into sdrpp_amd/lib/libsdrgpu.so.
Host-side design code (windows, taps) is compiled with -ffp-contract=off so it
rounds exactly like the reference source; device code keeps the default FMA
contraction (its parity bar is a stated tolerance).
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "sdrpp_amd", "csrc")
LIBDIR = os.path.join(ROOT, "sdrpp_amd", "lib")
BUILD = os.path.join(ROOT, "build")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

SOURCES = [
    # (file, extra flags)
    ("host_design.cpp", ["-ffp-contract=off"]),
    ("capi.cpp", []),
    ("fft.hip", []),
    ("fft64.hip", []),
    ("blocks.hip", []),
    ("channelizer.hip", []),
    ("loops.hip", ["-ffp-contract=off"]),   # bit-exact serial recurrences
    ("frontend.hip", []),
    ("consumers.hip", ["-ffp-contract=off"]),   # bit-exact encoders
    ("file_source.cpp", []),
    ("gather.cpp", []),
]


def _run(cmd):
    print("+", " ".join(cmd), flush=True)
    subprocess.check_call(cmd)


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _defs(defines):
    """-D NAME[=V] per define; an entry starting with '-' is passed as compiler flags (A/B builds,
    e.g. '-mllvm -amdgpu-sched-strategy=max-ilp')."""
    out = []
    for d in defines:
        out += d.split() if d.startswith("-") else ["-D" + d]
    return out


def build_lib(force=False, variant=None, defines=()):
    """variant: an A/B build of the same ABI with extra -D defines, into build/<variant>/ and
    sdrpp_amd/lib_<variant>/libsdrgpu.so (loaded through SDRGPU_LIB_PATH; tools/session.sh)."""
    libdir = LIBDIR if not variant else os.path.join(ROOT, "sdrpp_amd", "lib_" + variant)
    build = BUILD if not variant else os.path.join(BUILD, variant)
    os.makedirs(libdir, exist_ok=True)
    os.makedirs(build, exist_ok=True)
    headers = [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")]
    headers.append(os.path.join(ROOT, "include", "sdrgpu.h"))
    objs, cmds = [], []
    for src, extra in SOURCES:
        path = os.path.join(CSRC, src)
        obj = os.path.join(build, src + ".o")
        objs.append(obj)
        if force or _stale(obj, [path] + headers):
            lang = ["-x", "hip"] if src.endswith(".hip") else []
            cmds.append([HIPCC, "--offload-arch=" + ARCH, "-O3", "-fPIC", "-std=c++17",
                         "-Wall", "-Wno-unused-function", "-Wno-unused-variable",
                         "-I", os.path.join(ROOT, "include")] + _defs(defines) + extra + lang +
                        ["-c", path, "-o", obj])
    # translation units compile in parallel (at most 8 hipcc processes: the CPU share here and well
    # under the GPU box's -j16)
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        list(ex.map(_run, cmds))
    lib = os.path.join(libdir, "libsdrgpu.so")
    if force or _stale(lib, objs):
        _run([HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", lib] + objs + ["-ldl"])
    return lib


def build_oracle():
    """The checker (test infrastructure): the C restatement, and -- where the reference tree is
    mounted (dev container only) -- oracle/_ref/ref_probe built from the reference's own headers."""
    odir = os.path.join(ROOT, "oracle")
    _run(["make", "-C", odir, "-s"])
    if os.path.isdir("/root/reference/core/src/dsp"):
        _run(["make", "-C", odir, "-s", "ref"])
    return os.path.join(odir, "libsdr_oracle.so")


if __name__ == "__main__":
    force = "--force" in sys.argv
    args = [a for a in sys.argv[1:] if a != "--force"]
    if args and args[0] == "--variant":   # python sdrpp_amd/build.py --variant NAME DEF [DEF ...]
        build_lib(True, args[1], args[2:])
    else:
        build_lib(force)
    build_oracle()
