"""Register budget of every kernel in a built device object: VGPR / AGPR / SGPR counts, spills, LDS
and scratch (from the code object's metadata notes), filtered by a name regex.
  python tools/kernel_regs.py build/blocks.hip.o [regex]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def code_object(obj, tmp):
    fat = os.path.join(tmp, "x.fatbin")
    co = os.path.join(tmp, "x.co")
    subprocess.run(["objcopy", "--dump-section", ".hip_fatbin=" + fat, obj], check=True, capture_output=True)
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--input=" + fat, "--output=" + co],
                   check=True, capture_output=True)
    return co


def kernels(obj):
    with tempfile.TemporaryDirectory() as tmp:
        notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", code_object(obj, tmp)],
                               check=True, capture_output=True, text=True).stdout
    out, cur = [], None
    for ln in notes.splitlines():
        m = re.match(r"\s*-?\s*\.(\w+):\s+(.*)$", ln)
        if not m:
            continue
        k, v = m.group(1), m.group(2).strip()
        if k == "args":
            continue
        if k == "agpr_count":   # first key of a kernel's record
            cur = {}
            out.append(cur)
        if cur is not None and k in ("agpr_count", "vgpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
                                     "group_segment_fixed_size", "private_segment_fixed_size", "name"):
            cur[k] = v
    return out


if __name__ == "__main__":
    rx = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    for k in kernels(sys.argv[1]):
        name = k.get("name", "?")
        if rx.search(name):
            print(f"v{k.get('vgpr_count')} a{k.get('agpr_count')} s{k.get('sgpr_count')} spill v{k.get('vgpr_spill_count')}"
                  f" s{k.get('sgpr_spill_count')} lds {k.get('group_segment_fixed_size')} scratch "
                  f"{k.get('private_segment_fixed_size')}  {name[:150]}")
