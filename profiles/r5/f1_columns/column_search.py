import random, collections, math
def rec_of(n, fg):
    c, r = divmod(n, 25); ky, kx = divmod(r, 5)
    return (c * 32 + ky) * 29 + 8 * fg + kx
groups = [list(range(0,4)) + list(range(12,16)) + list(range(20,28)), list(range(4,12)) + list(range(16,20)) + list(range(28,32))]
groups += [[l + 32 for l in g] for g in groups]
def wave_cost(lanes):  # lanes: 16 column ids (pads: same column as some lane -> just a column id)
    tot = 0
    for g in groups:
        units = collections.defaultdict(set)
        for l in g:
            rec = rec_of(lanes[l & 15], l >> 4)
            units[rec % 16].add(rec)
        tot += max(len(s) for s in units.values())
    return tot  # ideal 4 (one cycle per group)
random.seed(3)
slots = list(range(75)) + [None] * 5  # None = pad
def resolve(sl):
    # pads read the column of lane (fr ^ 1)'s... choose: the first real column in the wave
    out = []
    for w in range(5):
        ws = sl[16 * w:16 * w + 16]
        real = [x for x in ws if x is not None]
        out.append([x if x is not None else real[0] for x in ws])
    return out
def cost(sl):
    return sum(wave_cost(ws) for ws in resolve(sl))
random.shuffle(slots)
cur = cost(slots); best = cur; bestsl = slots[:]
T = 2.0
for it in range(300000):
    i, j = random.randrange(80), random.randrange(80)
    if i == j: continue
    slots[i], slots[j] = slots[j], slots[i]
    c = cost(slots)
    if c <= cur or random.random() < math.exp((cur - c) / T):
        cur = c
        if c < best: best = c; bestsl = slots[:]
    else:
        slots[i], slots[j] = slots[j], slots[i]
    T = max(0.05, T * 0.99997)
    if best == 20: break
print("best cost", best, "(ideal 20, identity:", cost(list(range(75)) + [None]*5), ")")
print(bestsl)
