"""Static instruction mix of kernels in a hipcc --save-temps .s file (gfx950).

  python tools/isa_stats.py FILE.s [SUBSTRING ...]

For every kernel whose mangled name contains all SUBSTRINGs: instruction count, VALU (v_*), packed
fp32 (v_pk_*), fp64, LDS (ds_*), VMEM, scalar, waitcnt, VGPR / AGPR / spill counts, and the 25 most
frequent opcodes. Static counts (loops count once): a guide for A/B variants, not a profile."""
import re
import sys
from collections import Counter


def kernels(text):
    for m in re.finditer(r"^(_Z\S+):\s*;\s*@\1\n(.*?)^\.Lfunc_end\d+:", text, re.S | re.M):
        yield m.group(1), m.group(2)


def meta(text, name, key):
    m = re.search(re.escape(name) + r"\." + key + r", (\d+)", text)
    return int(m.group(1)) if m else None


def main():
    path, subs = sys.argv[1], sys.argv[2:]
    text = open(path).read()
    for name, body in kernels(text):
        if not all(s in name for s in subs):
            continue
        ops = [ln.split()[0] for ln in (l.strip() for l in body.split("\n"))
               if ln and not ln.startswith((".", ";", "_Z")) and not ln.endswith(":")]
        c = Counter(ops)
        cnt = lambda pred: sum(v for k, v in c.items() if pred(k))
        print(name)
        print(f"  instr {len(ops)}  valu {cnt(lambda k: k.startswith('v_'))}  pk {cnt(lambda k: k.startswith('v_pk'))}"
              f"  f64 {cnt(lambda k: k.endswith('_f64'))}  ds {cnt(lambda k: k.startswith('ds_'))}"
              f"  vmem {cnt(lambda k: k.startswith(('global_', 'buffer_')))}  salu {cnt(lambda k: k.startswith('s_'))}"
              f"  waitcnt {c['s_waitcnt']}  vgpr {meta(text, name, 'num_vgpr')}  agpr {meta(text, name, 'num_agpr')}"
              f"  scratch {cnt(lambda k: k.startswith('scratch_'))}")
        print("  " + ", ".join(f"{k} {v}" for k, v in c.most_common(25)))


if __name__ == "__main__":
    main()
