"""LDS bank-conflict model of the 1M pass B (fft_passB_1m_kernel) after stage 1, per sequence stride.

  python tools/lds_bank_model.py [LS ...]

Lanes: sL = tid % 8 (sequence), tL = tid / 8 (butterfly). Instruction forms from the gfx950 ISA of the
kernel: the middle radix-16 stage reads with ds_read2_b64 and writes with ds_write2_b64 (each access
4 groups of 16 lanes, bank = float2 index mod 16 as a pair of dwords), the last radix-4 stage reads
with ds_read_b64 (2 groups of 32 lanes, float2 index mod 32). Banking rules: MI355X_MICROARCH.md
LDS table. Prints LDS cycles per access relative to conflict-free (1.0 = no conflicts)."""
import sys


def pad16(j):
    return j + j // 16


def cycles(addrs, group, mod):
    c = 0
    for g0 in range(0, 64, group):
        banks = {}
        for a in addrs[g0:g0 + group]:
            banks.setdefault(a % mod, set()).add(a)
        c += max(len(v) for v in banks.values())
    return c


def model(LS, S=8):
    tot = {"mid_read": 0, "mid_write": 0, "last_read": 0}
    base = dict.fromkeys(tot, 0)
    for w in range(8):
        tid = [64 * w + l for l in range(64)]
        sL = [t % S for t in tid]
        tL = [t // S for t in tid]
        for r in range(16):
            tot["mid_read"] += cycles([s * LS + pad16(j) + 68 * r for s, j in zip(sL, tL)], 16, 16)
            idx = [(j // 16) * 256 + j % 16 for j in tL]
            tot["mid_write"] += cycles([s * LS + pad16(d) + 17 * r for s, d in zip(sL, idx)], 16, 16)
            base["mid_read"] += 4
            base["mid_write"] += 4
        for b in range(4):
            for r in range(4):
                tot["last_read"] += cycles([s * LS + pad16(j + 64 * b) + 272 * r for s, j in zip(sL, tL)], 32, 32)
                base["last_read"] += 2
    return {k: round(tot[k] / base[k], 2) for k in tot}


if __name__ == "__main__":
    for LS in [int(a) for a in sys.argv[1:]] or [1089, 1090, 1092]:
        print(LS, "mod 32 =", LS % 32, model(LS))
