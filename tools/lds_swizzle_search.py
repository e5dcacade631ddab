#!/usr/bin/env python3
"""Search the transpose-scratch layout of stft1024 for bank conflicts, using the gfx950
LDS bank model of MI355X_MICROARCH.md §LDS (lane groups and bank functions per
instruction).  Index unit: float2 (8 B).  Access patterns (lane l, register r):
  pass-1 write  n = 8 l + r, r even, ds_write_b128  (8 groups of 8 lanes, bank (a/4)%32)
  pass-1 read   n = l + 64 r,        ds_read_b64    (2 groups of 32, bank (a/4)%64)
  pass-2 write  n = 64 (l>>3) + (l&7) + 8 r, ds_write_b64 (4 groups of 16, bank (a/4)%32)
  pass-3 read   n = pi(l) + 64 r,    ds_read_b64
Cost = sum over lane groups of the max number of distinct dword addresses on one bank."""
import itertools


def pi_of(i):
    return 0 if i == 0 else 32 if i == 1 else (64 - (i >> 1) if i & 1 else i >> 1)


def cost(addr_dwords, groups, nbanks):
    c = 0
    for g in groups:
        banks = {}
        for l in g:
            for a in addr_dwords[l]:
                banks.setdefault(a % nbanks, set()).add(a)
        c += max(len(s) for s in banks.values())
    return c


G8 = [list(range(i, i + 8)) for i in range(0, 64, 8)]
G16 = [list(range(i, i + 16)) for i in range(0, 64, 16)]
G32 = [list(range(0, 32)), list(range(32, 64))]


def total(phys, pis=pi_of):
    t = 0
    for r in range(0, 8, 2):  # pass-1 writes (16 B)
        t += cost({l: [2 * phys(8 * l + r) + k for k in range(4)] for l in range(64)}, G8, 32)
    for r in range(8):
        t += cost({l: [2 * phys(l + 64 * r), 2 * phys(l + 64 * r) + 1] for l in range(64)}, G32, 64)
        n = lambda l: 64 * (l >> 3) + (l & 7) + 8 * r
        t += cost({l: [2 * phys(n(l)), 2 * phys(n(l)) + 1] for l in range(64)}, G16, 32)
        t += cost({l: [2 * phys(pis(l) + 64 * r), 2 * phys(pis(l) + 64 * r) + 1] for l in range(64)}, G32, 64)
    return t


def ideal():
    return 4 * 8 + 8 * (2 + 4 + 2)  # one cycle per group


cands = {"identity": lambda n: n, "pad2/16 (current)": lambda n: n + ((n >> 4) << 1)}
for a, b, c, d in itertools.product(range(3, 9), range(1, 5), range(3, 9), range(1, 5)):
    if (a, b) >= (c, d):
        continue
    cands[f"xor n{a}->b{b}, n{c}->b{d}"] = (lambda a, b, c, d: lambda n: n ^ (((n >> a) & 1) << b) ^
                                            (((n >> c) & 1) << d))(a, b, c, d)
res = sorted((total(f), k) for k, f in cands.items())
print("ideal", ideal())
for t, k in res[:8]:
    print(t, k)
print("current", total(cands["pad2/16 (current)"]), "identity", total(cands["identity"]))


def breakdown(phys, pis=pi_of):
    out = {}
    out["p1w"] = sum(cost({l: [2 * phys(8 * l + r) + k for k in range(4)] for l in range(64)}, G8, 32)
                     for r in range(0, 8, 2))
    out["p1r"] = sum(cost({l: [2 * phys(l + 64 * r), 2 * phys(l + 64 * r) + 1] for l in range(64)}, G32, 64)
                     for r in range(8))
    out["p2w"] = sum(cost({l: [2 * phys(64 * (l >> 3) + (l & 7) + 8 * r), 2 * phys(64 * (l >> 3) + (l & 7) + 8 * r) + 1]
                           for l in range(64)}, G16, 32) for r in range(8))
    out["p3r"] = sum(cost({l: [2 * phys(pis(l) + 64 * r), 2 * phys(pis(l) + 64 * r) + 1] for l in range(64)}, G32, 64)
                     for r in range(8))
    return out


print("breakdown current", breakdown(cands["pad2/16 (current)"]), "ideal p1w 32 p1r 16 p2w 32 p3r 16")
# richer family: padding p per 2^s plus one xor term
best = []
for s in range(3, 8):
    for p in (0, 1, 2, 4):
        for a in range(3, 9):
            for b in range(0, 5):
                f = (lambda s, p, a, b: lambda n: (n ^ ((((n >> a) & 1) << b) if b else 0)) + (n >> s) * p)(s, p, a, b)
                # b128 writes need even phys for even n
                if any(f(8 * l + r) % 2 for l in range(64) for r in range(0, 8, 2)):
                    continue
                best.append((total(f), s, p, a, b))
best.sort()
print(best[:10])

f = lambda n: (n ^ (((n >> 3) & 1) << 3)) + 2 * (n >> 4)
print("best1 breakdown", breakdown(f))
best = []
for s in (4, 5):
    for p in (2, 4):
        for a, b, c, d in itertools.product(range(3, 8), range(1, 5), range(3, 8), range(1, 5)):
            if (a, b) >= (c, d):
                continue
            f = (lambda s, p, a, b, c, d: lambda n: (n ^ (((n >> a) & 1) << b) ^ (((n >> c) & 1) << d)) + (n >> s) * p)(s, p, a, b, c, d)
            if any(f(8 * l + r) % 2 for l in range(64) for r in range(0, 8, 2)):
                continue
            if len({f(n) for n in range(512)}) != 512:
                continue
            best.append((total(f), s, p, a, b, c, d))
best.sort()
print(best[:6])
t, s, p, a, b, c, d = best[0]
f = lambda n: (n ^ (((n >> a) & 1) << b) ^ (((n >> c) & 1) << d)) + (n >> s) * p
print("best2 breakdown", breakdown(f), "max phys", max(f(n) for n in range(512)))


def find_grouping(f):
    """Split the 32 conjugate lane pairs {0,32}, {j, 64-j} into two halves of 16 whose 32
    pass-3 read addresses are distinct modulo 32 float2 (conflict-free ds_read_b64)."""
    pairs = [(0, 32)] + [(j, 64 - j) for j in range(1, 32)]
    vals = [tuple(f(x) % 32 for x in p) for p in pairs]
    if any(a == b for a, b in vals):
        return None
    best = None

    def rec(i, A, used_a, B, used_b):
        nonlocal best
        if best is not None:
            return
        if i == len(pairs):
            best = (A, B)
            return
        a, b = vals[i]
        if len(A) < 16 and a not in used_a and b not in used_a and (i > 0 or True):
            rec(i + 1, A + [pairs[i]], used_a | {a, b}, B, used_b)
        if i > 0 and len(B) < 16 and a not in used_b and b not in used_b:
            rec(i + 1, A, used_a, B + [pairs[i]], used_b | {a, b})

    rec(0, [], set(), [], set())
    return best


found = []
for s in (4, 5, 6):
    for p in (2, 4):
        for a, b, c, d in itertools.product(range(3, 8), range(1, 5), range(3, 8), range(0, 5)):
            f = (lambda s, p, a, b, c, d: lambda n: (n ^ (((n >> a) & 1) << b) ^ ((((n >> c) & 1) << d) if d else 0)) + (n >> s) * p)(s, p, a, b, c, d)
            if any(f(8 * l + r) % 2 for l in range(64) for r in range(0, 8, 2)):
                continue
            if len({f(n) for n in range(512)}) != 512:
                continue
            bd = breakdown(f)
            if bd["p1w"] + bd["p1r"] + bd["p2w"] > 80:
                continue
            g = find_grouping(f)
            if g:
                found.append((s, p, a, b, c, d, max(f(n) for n in range(512)), g))
print(len(found))
for x in found[:5]:
    print(x[:7])
if found:
    s, p, a, b, c, d, mx, (A, B) = found[0]
    lanes = [None] * 64
    for i, pr in enumerate(A):
        lanes[2 * i], lanes[2 * i + 1] = pr
    for i, pr in enumerate(B):
        lanes[32 + 2 * i], lanes[32 + 2 * i + 1] = pr
    f = lambda n: (n ^ (((n >> a) & 1) << b) ^ ((((n >> c) & 1) << d) if d else 0)) + (n >> s) * p
    print("pi table", lanes)
    print("breakdown", breakdown(f, lambda l: lanes[l]), "total", total(f, lambda l: lanes[l]))


def find_assignment(f):
    """Also make the tile writes conflict-free: rows k = pi + 64 r written as ds_write_b64 at
    pitch 34 floats → within each 16-lane group the pi must be distinct mod 16."""
    pairs = [(0, 32)] + [(j, 64 - j) for j in range(1, 32)]
    pv = [tuple(f(x) % 32 for x in pr) for pr in pairs]
    tv = [tuple(x % 16 for x in pr) for pr in pairs]
    groups = [[] for _ in range(4)]
    res = None

    def ok(g, i):
        if len(groups[g]) >= 8:
            return False
        half = g // 2
        used_p = {v for gg in (2 * half, 2 * half + 1) for k in groups[gg] for v in pv[k]}
        used_t = {v for k in groups[g] for v in tv[k]}
        a, b = pv[i]
        c, d = tv[i]
        return a != b and c != d and a not in used_p and b not in used_p and c not in used_t and d not in used_t

    def rec(i):
        nonlocal res
        if res is not None:
            return
        if i == len(pairs):
            res = [list(g) for g in groups]
            return
        for g in ([0] if i == 0 else range(4)):
            if ok(g, i):
                groups[g].append(i)
                rec(i + 1)
                groups[g].pop()

    rec(0)
    if res is None:
        return None
    lanes = []
    for g in res:
        for k in g:
            lanes += list(pairs[k])
    return lanes


for cand in found:
    s, p, a, b, c, d, mx, _ = cand
    f = (lambda s, p, a, b, c, d: lambda n: (n ^ (((n >> a) & 1) << b) ^ ((((n >> c) & 1) << d) if d else 0)) + (n >> s) * p)(s, p, a, b, c, d)
    lanes = find_assignment(f)
    if lanes:
        print("swizzle", (s, p, a, b, c, d), "max", mx)
        print("pi", lanes)
        print(breakdown(f, lambda l: lanes[l]))
        tw = sum(cost({l: [34 * (lanes[l] + 64 * r), 34 * (lanes[l] + 64 * r) + 1] for l in range(64)}, G16, 32)
                 for r in range(8))
        print("tile writes cost", tw, "(ideal 32)")
        break
else:
    print("no assignment")


def find_assignment2(f):
    """As find_assignment, but pairs whose two rows share k mod 16 ((0,32),(8,56),(16,48),
    (24,40)) are unavoidable 2-way tile-write conflicts: allow one of them per 16-lane group."""
    pairs = [(0, 32)] + [(j, 64 - j) for j in range(1, 32)]
    pv = [tuple(f(x) % 32 for x in pr) for pr in pairs]
    tv = [tuple(x % 16 for x in pr) for pr in pairs]
    groups = [[] for _ in range(4)]
    res = None

    def ok(g, i):
        if len(groups[g]) >= 8:
            return False
        half = g // 2
        used_p = {v for gg in (2 * half, 2 * half + 1) for k in groups[gg] for v in pv[k]}
        a, b = pv[i]
        if a == b or a in used_p or b in used_p:
            return False
        used_t = [v for k in groups[g] for v in tv[k]]
        c, d = tv[i]
        if c == d:
            if any(tv[k][0] == tv[k][1] for k in groups[g]):
                return False
            return c not in used_t
        return c not in used_t and d not in used_t

    def rec(i):
        nonlocal res
        if res is not None:
            return
        if i == len(pairs):
            res = [list(g) for g in groups]
            return
        for g in ([0] if i == 0 else range(4)):
            if ok(g, i):
                groups[g].append(i)
                rec(i + 1)
                groups[g].pop()

    rec(0)
    if res is None:
        return None
    lanes = []
    for g in res:
        for k in g:
            lanes += list(pairs[k])
    return lanes


for cand in found:
    s, p, a, b, c, d, mx, _ = cand
    f = (lambda s, p, a, b, c, d: lambda n: (n ^ (((n >> a) & 1) << b) ^ ((((n >> c) & 1) << d) if d else 0)) + (n >> s) * p)(s, p, a, b, c, d)
    lanes = find_assignment2(f)
    if lanes:
        print("swizzle", (s, p, a, b, c, d), "max", mx)
        print("pi", lanes)
        print(breakdown(f, lambda l: lanes[l]))
        tw = sum(cost({l: [34 * (lanes[l] + 64 * r), 34 * (lanes[l] + 64 * r) + 1] for l in range(64)}, G16, 32)
                 for r in range(8))
        print("tile writes cost", tw, "(ideal 32)")
        cur_tw = sum(cost({l: [34 * (pi_of(l) + 64 * r), 34 * (pi_of(l) + 64 * r) + 1] for l in range(64)}, G16, 32)
                     for r in range(8))
        print("current tile writes cost", cur_tw)
        break
else:
    print("no assignment")
