"""Search R1-record layouts for LDS bank conflicts of the three access patterns that share the
R1 records (tools/lds_banks.py model, gfx950 rules): phase B's conv1 A reads, phase F's conv1
wgrad B reads and the record build's writes.  Candidates: row stride RS, channel stride CS and
an XOR swizzle of the record index by row bits; then, for phase B alone, every assignment of
the tile's 4 pooling windows to MFMA row groups.  Results: profiles/r4/lds_model/README.md."""
import itertools
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import lds_banks as L  # noqa: E402


def cost_b(addr):
    tot = 0
    for t in range(49):
        for sk in range(4):
            a = []
            for ln in range(64):
                wi, pi = (ln & 15) >> 2, (ln & 15) & 3
                q = 4 * t + wi
                y, x = 2 * (q // 14) + (pi >> 1), 2 * (q % 14) + (pi & 1)
                pr = min(4 * sk + (ln >> 4), 14)
                a.append(addr(pr // 5, y + pr % 5, x) * 16)
            tot += L.cycles(a, L.G128, 16, 64)
    return tot


def cost_f(addr):
    tot = 0
    for w in range(5):
        for k in range(28):
            a = []
            for ln in range(64):
                nc = min(w * 16 + (ln & 15), 74)
                c, ky, kx = nc // 25, (nc % 25) // 5, nc % 5
                a.append(addr(c, ky + k, 8 * (ln >> 4) + kx) * 16)
            tot += L.cycles(a, L.G128, 16, 64)
    return tot


def cost_w(addr):  # build_r1_part: thread -> (row, q), records x = 8q .. 8q + 7 of rows c * 32 + y
    tot = 0
    for w in range(6):
        for x in range(8):
            a = []
            for ln in range(64):
                t = 64 * w + ln
                row, q = (t & 7) + 8 * (t >> 5), (t >> 3) & 3
                xx = 8 * q + x
                a.append(addr(row // 32, row % 32, xx) * 16 if xx < 29 else None)
            tot += L.cycles(a, L.GW128, 16, 32)
    return tot


def main():
    base = lambda c, y, x: (c * 32 + y) * 29 + x  # noqa: E731  (the kernel's layout)
    b, f, w = cost_b(base), cost_f(base), cost_w(base)
    print(f"current layout (RS 29): B {b}  F {f}  build {w}  total {b + f + w} LDS cycles per workgroup "
          f"(conflict-free: B 784, F 560, build 384)")
    fams = {}
    for m in range(16):
        fams[f"y*{m}"] = lambda y, m=m: (y * m) & 15
        fams[f"(y&7)*{m}"] = lambda y, m=m: ((y & 7) * m) & 15
        fams[f"(y&3)*{m}"] = lambda y, m=m: ((y & 3) * m) & 15
        fams[f"(y&1)*8^(y>>1&1)*{m}"] = lambda y, m=m: (((y & 1) * 8) ^ ((y >> 1) & 1) * m) & 15
    res = []
    for rs in (29, 30, 31, 32, 33, 34, 36, 40):
        cs = 32 * rs
        if 3 * cs * 16 > 44544 + 7536:  # R1 region + the free LDS
            continue
        for name, g in fams.items():
            if rs < 32 and name != "y*0":
                continue  # (a swizzled index needs 32 records per row)
            addr = lambda c, y, x, g=g, rs=rs, cs=cs: c * cs + y * rs + (x ^ g(y))  # noqa: E731
            b, f, w = cost_b(addr), cost_f(addr), cost_w(addr)
            res.append((b + f + w, b, f, w, rs, name))
    res.sort()
    print("best layouts (total, B, F, build, row stride, swizzle):")
    for r in res[:8]:
        print("  ", r)
    # phase B alone: which two of the tile's 4 windows share a lane group (row stride 29)
    rs = 29
    costs = []
    for perm in itertools.permutations(range(4)):
        rec = lambda w, pi: (pi >> 1) * rs + 2 * perm[w] + (pi & 1)  # noqa: E731
        ga = [rec(w, p) % 16 for w in (0, 3) for p in range(4)] + [(rec(w, p) + rs) % 16 for w in (1, 2) for p in range(4)]
        gb = [rec(w, p) % 16 for w in (1, 2) for p in range(4)] + [(rec(w, p) + rs) % 16 for w in (0, 3) for p in range(4)]
        costs.append((max(ga.count(v) for v in ga) + max(gb.count(v) for v in gb), perm))
    costs.sort()
    ident = dict((p, c) for c, p in costs)[(0, 1, 2, 3)]
    print(f"phase B window-to-row-group permutations (2 lane groups, 1 = conflict-free each): best {costs[0]}, "
          f"current (0, 1, 2, 3): {ident}")


if __name__ == "__main__":
    main()
