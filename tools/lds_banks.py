#!/usr/bin/env python3
"""LDS bank-conflict model for the wgrad kernel's staged tiles (MI355X_MICROARCH.md §LDS):
ds_write_b128 = 8 groups x 8 contiguous lanes, bank (a/4)%32; ds_read_b64_tr_b16 = 2 groups x 32
lanes, bank (a/4)%64. Extra cycles per group = max distinct addresses on one bank - 1."""
import itertools


def conflicts(groups, nbanks, width):
    extra = 0
    for acc in groups:
        banks = {}
        for a in acc:
            for w in range(width // 4):
                b = (a // 4 + w) % nbanks
                banks.setdefault(b, set()).add(a)
        extra += max(len(v) for v in banks.values()) - 1
    return extra


def writes(nch, swz, a_ch):
    """one K block: 64 rows x nch 16B chunks; thread t: row = t // tpr, chunk = t % tpr + j*tpr"""
    tpr = nch // a_ch
    tot = 0
    for w in range(4):
        for j in range(a_ch):
            addrs = []
            for lane in range(64):
                t = 64 * w + lane
                row, cc = t // tpr, t % tpr + j * tpr
                addrs.append(row * nch * 16 + swz(row, cc, nch) * 16)
            tot += conflicts([addrs[8 * g:8 * g + 8] for g in range(8)], 32, 16)
    return tot


def reads(nch, swz, wcols):
    """mma fragment reads: lane (g, q, p): row = ks*32 + 8g + q (+4), col = base + i*16 + 4p"""
    tot = 0
    for ks in range(2):
        for half in range(2):
            for base in range(0, nch * 8, 16):
                addrs = []
                for lane in range(64):
                    g, q, p = lane >> 4, (lane & 15) >> 2, lane & 3
                    row = ks * 32 + 8 * g + q + 4 * half
                    col = base + 4 * p
                    addrs.append(row * nch * 16 + swz(row, col >> 3, nch) * 16 + (col & 7) * 2)
                tot += conflicts([addrs[:32], addrs[32:]], 64, 8)
    return tot


def swz_old(row, ch, nch):
    if nch == 16:
        return ch ^ ((((row & 3) | ((row >> 1) & 4)) << 1) & 15)
    return ch ^ ((((row & 3) << 1) ^ (((row >> 3) & 1) << 1)) & 7)


def swz_new(row, ch, nch):
    if nch == 32:  # 256-wide tiles (8 waves): row bits 0,1,3 -> chunk bits 1,2,3
        return ch ^ (((row & 1) << 1) | ((row & 2) << 1) | (row & 8))
    if nch == 16:  # bit2 <- row bit0 (write pairs), bit1 <- row bit1, bit3 <- row bit3 (read sets)
        return ch ^ ((((row & 1) << 2) | (row & 2) | (row & 8)) & 15)
    return ch ^ ((((row & 1) << 2) ^ (row & 2) ^ (((row >> 3) & 1) << 2)) & 7)


if __name__ == "__main__":
    for nch, a_ch in ((32, 4), (16, 4), (8, 2)):
        for name, f in (("old", swz_old), ("new", swz_new)):
            print(f"nch={nch} {name}: write extra cycles {writes(nch, f, a_ch)}, read extra cycles {reads(nch, f, 0)}")
