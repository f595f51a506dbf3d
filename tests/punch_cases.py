"""Realm punch test datagrams shared by the emulated and GPU tiers (no side effects)."""


def punch_batch(n, m, seed):
    """Datagrams for the realm punch matcher: packets under each attempt, corrupted
    ones, wrong lengths and junk; returns (packets, attempts [(nonce, key)], metas)."""
    import random
    from hysteria_amd import realm
    from oracle import realm_ref as rref
    rng = random.Random(seed)
    atts = [(rng.randbytes(16), rng.randbytes(32)) for _ in range(m)]
    pk = []
    for i in range(n):
        nonce, key = atts[rng.randrange(m)]
        p = bytearray(rref.encode(rng.choice([1, 2]), nonce, key, rng.randbytes(8), rng.randbytes(rng.choice([0, 1, 7, 300, 1024]))))
        k = rng.randrange(6)
        if k == 1:
            p[8 + rng.randrange(25)] ^= 0x10
        elif k == 2:
            p = p[:rng.randrange(rref.MIN_WIRE)]
        elif k == 3:
            p = p + bytes(rref.MAX_WIRE + 1 - len(p))
        elif k == 4:
            p = bytearray(rng.randbytes(rng.randrange(0, 200)))
        pk.append(bytes(p))
    metas = [realm.PunchMetadata(a.hex(), b.hex()) for a, b in atts]
    return pk, atts, metas
