#!/usr/bin/env python3
"""Bank-conflict check of the W-operand LDS swizzle of gemm_pipe_kernel (csrc/kernels/gemm.hip, swW) for
the permuted 16x16x32 fragment reads: lane (fr, fq) of a wave reads W row wn + 4 NI (fr >> 2) + (fr & 3)
+ 4 ni, 16-byte k chunk 4 kk + fq, for every column block ni at an immediate offset -- so the swizzle must
not change with ni -- and each ds_read_b128 lane group (MI355X_MICROARCH.md, LDS table) must hit 16
distinct 16-byte slots of the 256-byte bank row.  usage: lds_swizzle_check.py"""
import numpy as np

GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
          list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
GROUPS += [[lane + 32 for lane in g] for g in GROUPS]


def sw_w(r, NI):
    """gemm.hip swW."""
    if NI in (3, 6):
        j = (r % (16 * NI)) // (4 * NI)
        return (1 if j in (1, 2) else 0) ^ (2 * j + ((r & 3) >> 1))
    lg = {2: 1, 4: 2, 8: 3}[NI]
    return (r & 2) | (((r >> (2 + lg)) & 1) << 2)


def conflicts(NI, WGN):
    bad = 0
    for w in range(WGN):
        for kk in range(2):
            for ni in range(NI):
                slots = []
                for lane in range(64):
                    fr, fq = lane & 15, lane >> 4
                    row_b = w * 16 * NI + (fr >> 2) * (4 * NI) + (fr & 3)
                    r = row_b + 4 * ni
                    assert sw_w(r, NI) == sw_w(row_b, NI), "swizzle changes with the column block"
                    slots.append((r & 1) * 8 + ((kk * 4 + fq) ^ sw_w(row_b, NI)))
                slots = np.array(slots)
                bad += sum(len(set(slots[g].tolist())) != 16 for g in GROUPS)
    return bad


if __name__ == "__main__":
    for NI, WGN in ((2, 4), (3, 4), (4, 4), (4, 2), (6, 2), (8, 2)):
        print(f"NI={NI} WGN={WGN}: {conflicts(NI, WGN)} conflicting lane groups")
