"""LDS bank-conflict model of one blind-rotation pair step (k=1, N=2048, E=8):
every LDS access of the kernel's step, per wave, priced with the b32 rule of
MI355X_MICROARCH.md §LDS (two 32-lane groups, bank = dword mod 32, one cycle
per distinct address on the busiest bank).  Prints extra (conflict) cycles per
access kind, summed over the 16 waves of a workgroup."""
import collections

N, E, LOG, e = 2048, 8, 11, 3
T = N // E
NPH = (LOG + e - 1) // e


def lo(p):
    return max(LOG - (p + 1) * e, 0)


def base(p, tl):
    L = lo(p)
    return ((tl >> L) << (L + e)) | (tl & ((1 << L) - 1))


def pad(i):
    return i + (i >> 4)


def idx(p, tl, m):
    return base(p, tl) + (m << lo(p))


def cycles(addrs):
    """addrs: 64 dword addresses (None = inactive) -> LDS cycles (b32 rule)"""
    tot = 0
    for g in (addrs[:32], addrs[32:]):
        banks = collections.defaultdict(set)
        for a in g:
            if a is not None:
                banks[a % 32].add(a)
        tot += max((len(s) for s in banks.values()), default=1)
    return tot


def brv(x, bits):
    r = 0
    for _ in range(bits):
        r = (r << 1) | (x & 1)
        x >>= 1
    return r


def main():
    stats = collections.Counter()
    ideal = collections.Counter()
    for w in range(T // 64):
        lanes = [w * 64 + l for l in range(64)]
        acc = []
        # exchanges p -> p+1 (forward) and p -> p-1 (inverse): write layout p, read layout p'
        for p in range(NPH - 1):
            for (pf, pt, kind) in ((p, p + 1, "fwd_x%d" % p), (p + 1, p, "inv_x%d" % (p + 1))):
                for m in range(E):
                    acc.append(("w " + kind, [pad(idx(pf, tl, m)) for tl in lanes]))
                    acc.append(("r " + kind, [pad(idx(pt, tl, m)) for tl in lanes]))
        # twiddle reads: forward stage s in phase p: zt[(1<<s) + (idx >> (LOG - s))] per butterfly
        for p in range(NPH):
            for s in range(p * e, min((p + 1) * e, LOG)):
                dm = 1 << (LOG - 1 - s - lo(p))
                for m in range(E):
                    if m & dm:
                        continue
                    fw = [(1 << s) + (idx(p, tl, m) >> (LOG - s)) for tl in lanes]
                    acc.append(("tw fwd s%d" % s, fw))
                    acc.append(("tw inv s%d" % s, [3 * (1 << s) - 1 - (idx(p, tl, m) >> (LOG - s)) for tl in lanes]))
        for kind, a in acc:
            c = cycles(a)
            stats[kind.split()[0] + " " + kind.split()[1][:6]] += c
            ideal[kind.split()[0] + " " + kind.split()[1][:6]] += 2
    tot = sum(stats.values()) - sum(ideal.values())
    for k in sorted(stats):
        print(f"{k:14s} cycles {stats[k]:6d}  conflict-free {ideal[k]:6d}  extra {stats[k] - ideal[k]:6d}")
    print("total extra cycles per step per workgroup (2 polys x 2 primes share the pattern):", tot * 4)


main()
