"""LDS bank-conflict model of the fused kernel's hot access patterns (gfx950 rules from
MI355X_MICROARCH.md §LDS: lane groups per instruction, 64 x 4-B banks for b64/b128 reads,
32 for b32 and writes).  Prints LDS-array cycles per wave-instruction vs the conflict-free
minimum, so a layout change can be checked on the CPU before it goes to the GPU."""
import itertools

G128 = [[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27],
        [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]]
G128 = G128 + [[l + 32 for l in g] for g in G128]
G64 = [list(range(32)), list(range(32, 64))]
GW128 = [list(range(8 * i, 8 * i + 8)) for i in range(8)]


def cycles(addrs, groups, nbytes, nbanks):
    tot = 0
    for g in groups:
        banks = {}
        for l in g:
            a = addrs[l]
            if a is None:
                continue
            for d in range(nbytes // 4):
                dw = a // 4 + d
                banks.setdefault(dw % nbanks, set()).add(dw)
        tot += max((len(v) for v in banks.values()), default=1)
    return tot


def report(name, gen, kind="r128"):
    groups, nb, nbanks = {"r128": (G128, 16, 64), "r64": (G64, 8, 64), "w128": (GW128, 16, 32)}[kind]
    worst, total, n = 0, 0, 0
    for addrs in gen():
        c = cycles(addrs, groups, nb, nbanks)
        total += c
        n += 1
        worst = max(worst, c)
    ideal = len(groups)
    print(f"{name:42s} {kind}: avg {total / n:5.2f} cycles (ideal {ideal}), worst {worst}  [{n} instr]")


REGB = 96256
lanes = range(64)


def fr(l): return l & 15
def fg(l): return l >> 4


def r1b(row, x):
    return row * 32 + (x ^ ((row & 1) * 9 ^ ((row >> 1) & 1) * 4 ^ ((row >> 2) & 1) * 2))


def phaseB():
    # conv1 over output-pixel pairs (lenet_fused.hip phase B a_index): 25 tiles x 4 K-steps;
    # A-row fr = (window wl = fr >> 1 of the tile, output row dy = fr & 1)
    for t in range(25):
        for sk in range(4):
            a = []
            for l in lanes:
                wl, dy = fr(l) >> 1, fr(l) & 1
                q = min(8 * t + wl, 195)
                y, x = 2 * (q // 14) + dy, 2 * (q % 14)
                pr = min(4 * sk + fg(l), 14)
                a.append(REGB + ((pr // 5 * 32 + y + pr % 5) * 29 + x) * 16)
            yield a


def phaseC():
    for t in range(7):
        for sk in range(8):
            a = []
            for l in lanes:
                wi, pi = fr(l) >> 2, fr(l) & 3
                q = min(4 * t + wi, 24)
                y, x = 2 * (q // 5) + (pi >> 1), 2 * (q % 5) + (pi & 1)
                prc = min(4 * sk + fg(l), 29)
                a.append(REGB + ((prc // 5 * 14 + y + prc % 5) * 13 + x) * 16)
            yield a


def fc1_fwd():
    for w in range(8):
        for ks in range(13):
            yield [2 * (min(16 * w + fr(l), 119) * 400 + 32 * ks + 8 * fg(l)) for l in lanes]


def fc1_tr():
    for nt in range(25):
        for ks in range(4):
            for half in range(2):
                a = []
                for l in lanes:
                    l16 = l & 15
                    q, p, g = l16 >> 2, l16 & 3, l >> 4
                    r = min(32 * ks + 8 * g + 4 * half + q, 119)
                    a.append(2 * (r * 400 + 16 * nt + 4 * p))
                yield a


def r3(o, yy, x):
    return (o * 18 + yy) * 16 + (x ^ (yy & 7))


def dgrad2():
    for mt in range(14):
        for kk in range(20):
            a = []
            for l in lanes:
                y, x = mt, min(fr(l), 13)
                o, kyp = 4 * (kk % 4) + fg(l), kk // 4
                a.append(r3(o, y + kyp, x) * 16)
            yield a


def dgrad2_wf():
    for kk in range(20):
        yield [REGB + 17472 + ((4 * kk + fg(l)) * 16 + fr(l)) * 16 for l in lanes]


def wgrad2():
    for nt in range(10):
        for sk in range(5):
            a, b = [], []
            for l in lanes:
                n = nt * 16 + fr(l)
                nc = min(n, 149)
                c, ky, kx = nc // 25, (nc % 25) // 5, nc % 5
                y, x0 = 2 * sk + (fg(l) >> 1), 8 * (fg(l) & 1)
                a.append(64512 + 2 * (fr(l) * 176 + y * 16 + x0))  # (DY2_CS = 176)
                b.append(REGB + ((c * 14 + y + ky) * 13 + x0 + kx) * 16)
            yield a
            yield b


# lenet_fused.hip kF1Col: phase F's column of lane fr of wave w (bit 7: padding lane)
F1COL = [73, 39, 201, 19, 35, 65, 56, 42, 30, 27, 59, 33, 38, 3, 25, 62, 74, 20, 17, 0, 57, 23, 72, 36, 13, 53, 10, 4, 22, 202, 18, 34, 54, 182, 67, 41, 68, 28, 2, 71, 31, 11, 55, 15, 40, 6, 9, 58, 49, 51, 37, 177, 43, 44, 12, 63, 21, 26, 24, 14, 60, 61, 48, 64, 50, 7, 70, 47, 46, 69, 45, 1, 8, 16, 32, 5, 66, 29, 178, 52]


def wgrad1(which, table=True):
    def gen():
        for w in range(5):
            for k in range(28):
                a = []
                for l in lanes:
                    n = w * 16 + fr(l)
                    nc = F1COL[n] & 127 if table else min(n, 74)
                    c, ky, kx = nc // 25, (nc % 25) // 5, nc % 5
                    if which == "A":
                        a.append(fr(l) * 1824 + fg(l) * 16 + k * 64)
                    else:
                        a.append(REGB + ((c * 32 + ky) * 29 + 8 * fg(l) + kx + k * 29) * 16)
                yield a
    return gen


def r1_write(fwd):
    # build_r1_part: thread t -> (row, q); writes records x = 8q .. 8q+7
    def gen():
        for w in range(6):
            for x in range(8):
                a = []
                for l in lanes:
                    t = 64 * w + l
                    row, q = (t & 7) + 8 * (t >> 5), (t >> 3) & 3
                    r = r1b(row, 8 * q + x) if fwd else row * 29 + 8 * q + x
                    a.append(REGB + r * 16 if 8 * q + x < 29 else None)
                yield a
    return gen


def r3_write():
    for w in range(5):
        for xr in range(14):
            a = []
            for l in lanes:
                t = 64 * w + l
                if t >= 288:
                    a.append(None)
                    continue
                o, yy = t // 18, t % 18
                a.append(r3(o, yy, xr) * 16)
            yield a


if __name__ == "__main__":
    report("B  conv1 A (R1 records)", phaseB)
    report("C  conv2 A (R2 records)", phaseC)
    report("D  fc1 fwd B (fc1 rows, ld 400)", fc1_fwd)
    report("D' fc1 dgrad B (tr16, ld 400)", fc1_tr, "r64")
    report("E  conv2 dgrad A (R3 records)", dgrad2)
    report("E  conv2 dgrad B (WF)", dgrad2_wf)
    report("E  conv2 wgrad A/B (DY2, R2)", wgrad2)
    report("F  conv1 wgrad A (DY1 rows)", wgrad1("A"))
    report("F  conv1 wgrad B (R1 records)", wgrad1("B"))
    report("F  conv1 wgrad B, column order", wgrad1("B", table=False))
    report("A/F R1 record build (write)", r1_write(False), "w128")
    report("E  R3 record build (write)", r3_write, "w128")
