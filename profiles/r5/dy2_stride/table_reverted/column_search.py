import random, collections, math, sys
sys.path.insert(0, '/root/repo/tools')
from lds_banks import G128
REGB = 96256
def units_of(n, sk, fg):
    nc = min(n, 149)
    c, ky, kx = nc // 25, (nc % 25) // 5, nc % 5
    y, x0 = 2 * sk + (fg >> 1), 8 * (fg & 1)
    rec = (c * 14 + y + ky) * 13 + x0 + kx
    return rec
def tile_cost(cols):  # cols: 16 column ids (150 = pad -> reads 149)
    tot = 0
    for sk in range(5):
        for g in G128:
            units = collections.defaultdict(set)
            for l in g:
                rec = units_of(cols[l & 15], sk, l >> 4)
                units[rec % 16].add(rec)
            tot += max(len(s) for s in units.values())
    return tot  # ideal 5*4 = 20 per tile
random.seed(5)
slots = list(range(150)) + [150] * 10
ident = sum(tile_cost(slots[16*t:16*t+16]) for t in range(10))
random.shuffle(slots)
tc = [tile_cost(slots[16*t:16*t+16]) for t in range(10)]
cur = sum(tc); best = cur; bestsl = slots[:]
T = 3.0
for it in range(400000):
    i, j = random.randrange(160), random.randrange(160)
    ti, tj = i // 16, j // 16
    if slots[i] == slots[j]: continue
    slots[i], slots[j] = slots[j], slots[i]
    ci = tile_cost(slots[16*ti:16*ti+16]); cj = tile_cost(slots[16*tj:16*tj+16]) if tj != ti else ci
    new = cur - tc[ti] + ci - (tc[tj] - cj if tj != ti else 0)
    if new <= cur or random.random() < math.exp((cur - new) / T):
        cur = new; tc[ti] = ci; tc[tj] = cj
        if cur < best: best = cur; bestsl = slots[:]
    else:
        slots[i], slots[j] = slots[j], slots[i]
    T = max(0.05, T * 0.99998)
    if best == 200: break
print("identity", ident, "best", best, "ideal 200", "iters", it)
print(", ".join(map(str, bestsl)))
