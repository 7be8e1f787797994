"""LDS bank-conflict simulator for the gfx950 lane-group model (MI355X_MICROARCH.md §LDS).

    python tools/lds_sim.py        # checks the access patterns of the hand-written kernels

ds_read_b128 is serviced in 4 lane groups of 16 ({0-3,12-15,20-27}, {4-11,16-19,28-31}, ...), one LDS
cycle each when conflict-free; bank = (addr / 4) mod 64; identical addresses broadcast.
"""
B128_GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
               list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32)),
               list(range(32, 36)) + list(range(44, 48)) + list(range(52, 60)),
               list(range(36, 44)) + list(range(48, 52)) + list(range(60, 64))]


def cycles_b128(addrs):
    tot = 0
    for g in B128_GROUPS:
        banks = {}
        for l in g:
            a = addrs[l]
            for k in range(4):
                b = (a // 4 + k) % 64
                banks.setdefault(b, set()).add(a // 16)
        tot += max(len(v) for v in banks.values())
    return tot  # 4 == conflict-free


def conv_l1():
    hswz = lambda R: R & 7
    pix = lambda fr: fr if fr < 4 else (fr - 8 if fr >= 12 else fr + 4)
    wswz = lambda co, c: (c & ~7) | ((c & 7) ^ ((co >> 1) & 7))
    worst_b = worst_a = 0
    W, XP = 56, 58
    for g0 in (0, 4, 8, 11):
        for j in range(4):
            for tap in range(9):
                tr, tu = divmod(tap, 3)
                for kk in range(2):
                    addrs = []
                    for lane in range(64):
                        fr, fq = lane & 15, lane >> 4
                        px = (g0 + j) * 16 + pix(fr)
                        if px >= 224:
                            continue
                        r, w = divmod(px, W)
                        R = r * XP + w + tr * XP + tu
                        addrs.append(R * 128 + (((kk * 4 + fq) ^ hswz(R)) << 4))
                    if len(addrs) < 64:
                        continue
                    worst_b = max(worst_b, cycles_b128(addrs))
    for wtap in range(9):
        for kk in range(2):
            for i in range(4):
                addrs = []
                for lane in range(64):
                    fr, fq = lane & 15, lane >> 4
                    co = i * 16 + fr
                    c = wtap * 8 + kk * 4 + fq
                    addrs.append(co * 1152 + wswz(co, c) * 16)
                worst_a = max(worst_a, cycles_b128(addrs))
    print(f"conv_l1: B (halo) worst {worst_b} cycles, A (weights) worst {worst_a} cycles (4 = conflict-free)")


def stem():
    # A: fragment i, lane row fr -> weight row 16*(fr >> 2) + 4*i + (fr & 3) (16 consecutive output channels per
    # lane for 16-byte stores); 448-byte rows, 16-byte chunk c stored at c ^ ((row >> 4) & 2) (csrc/kernels/stem.hip).
    # The round-5 layout (480-byte padded rows, no swizzle) measures 8 cycles here: 2-way conflicts.
    worst_a = worst_b = 0
    for r in range(7):
        for i in range(4):
            addrs = []
            for l in range(64):
                fr, fq = l & 15, l >> 4
                row = (fr >> 2) * 16 + i * 4 + (fr & 3)
                addrs.append(row * 448 + ((r * 4 + fq) ^ ((row >> 4) & 2)) * 16)
            worst_a = max(worst_a, cycles_b128(addrs))
        for w in range(4):
            for g in range(7):
                addrs = [(2 * w * 230 * 8 + ((l & 15) + (l >> 4)) * 16 + r * 230 * 8 + g * 256) for l in range(64)]
                worst_b = max(worst_b, cycles_b128(addrs))
    print(f"stem: A worst {worst_a}, B worst {worst_b}")


def conv_fwd_generic():
    # 16-B chunks XOR (row >> 1) & (CHUNKS - 1); fragments rows fr, chunk kk*4 + fq
    for ROWB in (64, 128):
        CH = ROWB // 16
        worst = 0
        for base in range(0, 64, 16):
            for kk in range(ROWB // 64):
                addrs = []
                for l in range(64):
                    fr, fq = l & 15, l >> 4
                    row = base + fr
                    addrs.append(row * ROWB + (((kk * 4 + fq) ^ ((row >> 1) & (CH - 1))) << 4))
                worst = max(worst, cycles_b128(addrs))
        print(f"conv_fwd ROWB={ROWB}: worst {worst}")


if __name__ == "__main__":
    conv_l1()
    stem()
    conv_fwd_generic()


def stem_search():
    import itertools
    best = None
    for pitch in range(448, 528, 16):
        for perm in itertools.permutations(range(4)):
            tau = lambda fr: perm[fr >> 2] * 4 + (fr & 3)
            worst = 0
            for r in range(7):
                for i in range(4):
                    addrs = [((i * 16 + tau(l & 15)) * pitch + (r * 4 + (l >> 4)) * 16) for l in range(64)]
                    worst = max(worst, cycles_b128(addrs))
            if best is None or worst < best[0]:
                best = (worst, pitch, perm)
    print("stem A best (cycles, pitch, block perm):", best)
