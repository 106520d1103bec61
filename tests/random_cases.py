"""Seeded random AllReduce cases over valid FlexTree topologies (incl. lonely ranks)."""
import random

import oracle_lib


def factorizations(n):
    out = []

    def rec(m, cur):
        if m == 1:
            if cur:
                out.append(list(cur))
            return
        for f in range(2, m + 1):
            if m % f == 0:
                rec(m // f, cur + [f])
    rec(n, [])
    return out


def random_topology(rng, P):
    """(topo string, lonely) valid for P, or None."""
    opts = [("1", 0)] + [(",".join(map(str, f)), 0) for f in factorizations(P)]
    for L in range(1, P):
        S = P - L
        for f in factorizations(S):
            if len(f) >= 2 and L * f[0] <= S:
                opts.append((",".join(map(str, f)), L))
    return rng.choice(opts)


def cases(seed, count, max_p=12, max_n=40000, P_fixed=None):
    """count cases; P uniform in 2..max_p, or P_fixed for every case."""
    import ftar_inputs as fi
    rng = random.Random(seed)
    out = []
    while len(out) < count:
        P = P_fixed or rng.randint(2, max_p)
        topo, lonely = random_topology(rng, P)
        n = rng.choice([0, 1, P - 1, P, P + 1, rng.randint(2, 200), rng.randint(200, max_n)])
        dt = rng.choice(["f32", "f32", "f32", "bf16", "f64", "i32", "u8", "i16", "i64", "bool"])
        op = "band" if dt in ("i32", "u8", "i16", "i64") and rng.random() < 0.3 else "sum"
        oop = rng.random() < 0.3
        chunk = rng.choice([0, 256, 1024, 1 << 14])
        seed_ = rng.randint(0, 1 << 30)
        ins = [fi.fill(dt, seed_, r, n) for r in range(P)]
        try:
            ref = oracle_lib.allreduce(ins, topo, lonely, fi.BY_NAME[dt], 0 if op == "sum" else 1, outofplace=oop)
        except RuntimeError:
            continue  # not a schedule the reference can run
        out.append(dict(P=P, topo=topo, lonely=lonely, n=n, dtype=dt, op=op, oop=oop, chunk=chunk, ins=ins, ref=ref))
    return out
