"""Static check of the built gfx950 code for the store-data hazard that made the round-2 / round-3
1M pass A nondeterministic ("buffer_store_dwordx4 with an SGPR soffset").

A buffer store of more than 64 bits reads its data VGPRs after issue, so a VALU write of those
VGPRs needs one wait state after it. hipcc (ROCm 7.2) inserts that wait only when the store's
soffset is an inline constant: with an SGPR soffset the next instruction may overwrite the data
and the store writes it half-updated, differently from run to run. This test disassembles every
device object of the build and fails on any >64-bit buffer store with an SGPR soffset whose very
next instructions write one of its data VGPRs (CPU only: it reads build/*.o).

The scan is conservative: it looks at the next WINDOW = 2 instructions after the store
(stopping early at an s_nop or s_waitcnt, which provide the wait state), and treats any instruction
whose first operand is a VGPR or VGPR range as a write of it -- VALU, v_writelane, DS / global /
buffer loads and MFMA results alike -- except stores, whose first operand is their data source."""
import glob
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
STORE = re.compile(r"^\s*buffer_store_dword(x3|x4)\s+v\[(\d+):(\d+)\],\s*[^,]+,\s*s\[\d+:\d+\],\s*(s\d+)\b")
DEST = re.compile(r"^\s*([a-z_0-9]+)\s+v(?:\[(\d+):(\d+)\]|(\d+)(?!\d))")
NO_DEST = re.compile(r"^(buffer|global|flat|scratch)_store|^ds_write|^ds_store|^buffer_atomic|^global_atomic")
STOP = re.compile(r"^\s*s_(nop|waitcnt)\b")
WINDOW = 2


def _disasm(obj, tmp):
    fat = os.path.join(tmp, os.path.basename(obj) + ".fatbin")
    co = os.path.join(tmp, os.path.basename(obj) + ".co")
    subprocess.run(["objcopy", "--dump-section", ".hip_fatbin=" + fat, obj], check=True, capture_output=True)
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--input=" + fat, "--output=" + co],
                   check=True, capture_output=True)
    out = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", co], check=True,
                         capture_output=True, text=True).stdout
    return [ln.split("//")[0] for ln in out.splitlines()]


def _violations(lines):
    bad = []
    for i, ln in enumerate(lines[:-1]):
        m = STORE.match(ln)
        if not m:
            continue
        lo, hi = int(m.group(2)), int(m.group(3))
        nxts = [x for x in lines[i + 1:i + 12] if x.strip()][:WINDOW]
        for nxt in nxts:
            if STOP.match(nxt):
                break
            d = DEST.match(nxt)
            if not d or NO_DEST.match(d.group(1)):
                continue
            a = int(d.group(2) or d.group(4))
            b = int(d.group(3) or d.group(4))
            if a <= hi and b >= lo:
                bad.append((ln.strip(), nxt.strip()))
                break
    return bad


def test_no_wide_buffer_store_data_hazard(tmp_path):
    objs = [o for o in glob.glob(os.path.join(ROOT, "build", "*.hip.o"))]
    if not objs or not os.path.exists(os.path.join(LLVM, "llvm-objdump")):
        pytest.skip("no device objects built here")
    found = {}
    for o in objs:
        v = _violations(_disasm(o, str(tmp_path)))
        if v:
            found[os.path.basename(o)] = v[:3]
    assert not found, found


def test_checker_flags_the_round3_pattern():
    """The pattern the checker must catch (from the first version of fft_passA_1m_kernel)."""
    lines = ["\tbuffer_store_dwordx4 v[66:69], v178, s[16:19], s38 offen",
             "\tv_mul_f64 v[66:67], v[72:73], v[76:77]"]
    assert _violations(lines)
    ok = ["\tbuffer_store_dwordx4 v[66:69], v70, s[16:19], 0 offen", "\ts_nop 1", "\tv_mul_f64 v[66:67], v[82:83], v[76:77]"]
    assert not _violations(ok)
    # an unrelated instruction in between does not hide it (conservative window of 2)
    gap = ["\tbuffer_store_dwordx4 v[66:69], v178, s[16:19], s38 offen", "\tv_add_u32 v1, v2, v3",
           "\tv_mov_b32 v68, v90"]
    assert _violations(gap)
    # non-VALU writers of the data registers: a DS read, a global load, an MFMA result, v_writelane
    for w in ["\tds_read_b64 v[68:69], v5", "\tglobal_load_dwordx2 v[66:67], v[4:5], off",
              "\tv_mfma_f32_16x16x4_f32 v[64:67], v1, v2, v[64:67]", "\tv_writelane_b32 v69, s4, 3"]:
        assert _violations(["\tbuffer_store_dwordx3 v[66:68], v178, s[16:19], s38 offen", w] if "69" not in w
                           else ["\tbuffer_store_dwordx4 v[66:69], v178, s[16:19], s38 offen", w]), w
    # a store reading the same registers is no write
    assert not _violations(["\tbuffer_store_dwordx4 v[66:69], v178, s[16:19], s38 offen",
                            "\tglobal_store_dwordx4 v[4:5], v[66:69], off"])
