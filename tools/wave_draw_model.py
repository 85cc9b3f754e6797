"""Model of stable_wave_draw's lane schedule (bayesbridge_amd/csrc/bb_sampler.h) against the
sequential double rejection loop of retstable.cpp:162-256: random, counter-keyed inner and outer
acceptances; the schedule's accepted (outer, inner) attempt must equal the sequential loop's
for every coefficient.  Also the rounds per wave of fixed groups against the adaptive schedule.
    python tools/wave_draw_model.py
"""
# Python model of stable_wave_draw's lane scheduling against the sequential double rejection loop
import random, hashlib
def h(*a):
    return int.from_bytes(hashlib.blake2b(repr(a).encode(), digest_size=8).digest(), 'little') / 2**64
def inner(seed, c, o, i, pin): return h(seed, 'in', c, o, i) < pin
def outer(seed, c, o, i, pout): return h(seed, 'out', c, o, i) < pout
def sequential(seed, c, pin, pout):
    o = 0
    while True:
        i = 0
        while True:
            if inner(seed, c, o, i, pin):
                if outer(seed, c, o, i, pout): return (o, i)
                break
            i += 1
        o += 1
def popc(x): return bin(x).count('1')
def nth(x, k):
    for _ in range(k):
        if not x: break
        x &= x - 1
    return (x & -x).bit_length() - 1 if x else -1
def ffs(x): return (x & -x).bit_length()  # 1-based, 0 if none
def wave(seed, active, pin, pout, L0=8):
    I = 8; NC = 64 // L0
    home = [l // L0 for l in range(64)]; ii = [l % 8 for l in range(64)]
    o0 = [0]*64; ib = [0]*64; jc = [home[l] for l in range(64)]
    res = [None]*64
    um = 0
    for c in range(NC):
        if active[c]: um |= 1 << c
    um_prev, G_prev = um, L0
    c_cur = list(home)
    rounds = 0
    def gbase(c, um, G): return L0 * c if G == L0 else popc(um & ((1 << c) - 1)) * G
    while um:
        rounds += 1
        m = popc(um)
        G = L0
        while m * G * 2 <= 64 and G < 64: G *= 2
        # G = max(L0, 64/next_pow2(m))
        if G > L0:
            new = [0]*64
            src = []
            for l in range(64):
                slot = l // G; cn = nth(um, slot)
                s = gbase(cn, um_prev, G_prev) if cn >= 0 else l
                src.append((cn, s))
            o0n = [o0[s] for _, s in src]; ibn = [ib[s] for _, s in src]; jcn = [jc[s] for _, s in src]
            o0, ib, jc = o0n, ibn, jcn
            c_cur = [cn for cn, _ in src]
        serve = [c_cur[l] >= 0 and (um >> c_cur[l]) & 1 for l in range(64)]
        base = [(l & ~(L0 - 1)) if G == L0 else (l // G) * G for l in range(64)]
        O = G // I
        seg = [(l - base[l]) >> 3 for l in range(64)]
        acc = [False]*64
        for l in range(64):
            if serve[l]:
                o = o0[l] + seg[l]
                acc[l] = inner(seed, jc[l], o, (ib[l] if seg[l] == 0 else 0) + ii[l], pin)
        ball = sum(1 << l for l in range(64) if acc[l])
        sb = [(ball >> (base[l] + 8 * seg[l])) & 0xff for l in range(64)]
        wsrc = [base[l] + 8 * seg[l] + (ffs(sb[l]) - 1 if sb[l] else 0) for l in range(64)]
        # inner winner index
        win_i = [None]*64
        for l in range(64):
            s = wsrc[l]
            win_i[l] = (ib[s] if seg[s] == 0 else 0) + ii[s]
        oacc = [False]*64
        for l in range(64):
            if serve[l] and sb[l]:
                oacc[l] = outer(seed, jc[l], o0[l] + seg[l], win_i[l], pout)
        hb_all = sum(1 << l for l in range(64) if ii[l] == 0 and sb[l] != 0)
        ab_all = sum(1 << l for l in range(64) if ii[l] == 0 and oacc[l])
        fin = [False]*64; rr = [None]*64
        for l in range(64):
            hb = hb_all >> base[l]; ab = ab_all >> base[l]
            H = A = 0
            for k in range(O):
                H |= ((hb >> (8 * k)) & 1) << k; A |= ((ab >> (8 * k)) & 1) << k
            stop = (~H & ((1 << O) - 1)) | A
            k = ffs(stop) - 1 if stop else O
            if serve[l]:
                if k == O: o0[l] += O; ib[l] = 0
                elif (A >> k) & 1:
                    # the accepted (o, i)
                    s = base[l] + 8 * k
                    rr[l] = (o0[l] + k, win_i[s]); fin[l] = True
                else:
                    ib[l] = ib[l] + I if k == 0 else I; o0[l] += k
        fb = sum(1 << l for l in range(64) if fin[l] and l == base[l])
        fm = 0; x = fb
        while x:
            b = ffs(x) - 1; x &= x - 1
            fm |= 1 << (b // L0 if G == L0 else nth(um, b // G))
        for l in range(64):
            if (fm >> home[l]) & 1:
                res[l] = rr[gbase(home[l], um, G)]
        um_prev, G_prev = um, G
        um &= ~fm
    return [res[c * L0] for c in range(NC)], rounds
def fixed_rounds(seed, active, pin, pout, L0=8):
    # rounds of stable_spec_draw<L0, 8>: each coefficient's rounds with O = L0/8 outer attempts
    NC = 64 // L0; O = L0 // 8; mx = 0
    for c in range(NC):
        if not active[c]: continue
        o0, ib, r = 0, 0, 0
        while True:
            r += 1
            # evaluate O segments
            done = False
            for k in range(O):
                o = o0 + k; st = ib if k == 0 else 0
                acc = [inner(seed, c, o, st + i, pin) for i in range(8)]
                if not any(acc):
                    ib = st + 8 if k == 0 else 8; o0 = o; break
                i = acc.index(True)
                if outer(seed, c, o, st + i, pout): done = True; break
                if k == O - 1: o0 = o + 1; ib = 0
            if done: break
        mx = max(mx, r)
    return mx


def check(trials=3000, seed=1):
    """Every coefficient's accepted (outer, inner) attempt under the schedule equals the
    sequential loop's; returns the number of waves checked."""
    rng = random.Random(seed)
    n = 0
    for L0 in (8, 16):
        for _ in range(trials):
            s = rng.random()
            pin = rng.choice([0.05, 0.3, 0.6])
            pout = rng.choice([0.2, 0.7, 0.95])
            NC = 64 // L0
            active = [rng.random() < 0.9 for _ in range(NC)]
            got, _ = wave(s, active, pin, pout, L0)
            for c in range(NC):
                want = sequential(s, c, pin, pout) if active[c] else None
                assert got[c] == want, (L0, c, got[c], want, pin, pout)
            n += 1
    return n


def rounds(trials=2000, seed=2, pin=0.3, pout=0.7):
    import statistics
    rng = random.Random(seed)
    out = {}
    for L0 in (8, 16):
        fr, ar = [], []
        for _ in range(trials):
            s = rng.random()
            active = [True] * (64 // L0)
            fr.append(fixed_rounds(s, active, pin, pout, L0))
            ar.append(wave(s, active, pin, pout, L0)[1])
        out[L0] = (statistics.mean(fr), statistics.mean(ar))
    return out


if __name__ == "__main__":
    print("schedule == sequential loop on", check(), "waves")
    for L0, (f, a) in rounds().items():
        print(f"{L0} lanes per coefficient: fixed groups {f:.2f} rounds per wave, adaptive {a:.2f}")
