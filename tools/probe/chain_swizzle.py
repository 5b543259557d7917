"""Search for the chains' LDS image swizzle keys (csrc/reschain.hip, EcGeo::KEYS): key(u) for tokens u = 0..15 of a
16-token group (the decoder's zero rows u = -1 / 16 read with the fixed keys 15 / 0), such that
  * every ds_read_b128 lane group of a B-fragment read (lanes {0-3,12-15,20-27}, {4-11,16-19,28-31} and the g + 2
    halves; lane = 16 g + li reads token li + s, logical chunk 4 kk + g, physical chunk (4 kk + g) ^ key) hits 16
    distinct 16-B bank slots for each tap shift s (decoder: -1, 0, +1; encoder: 0);
  * the epilogue's ds_write_b64 (16 contiguous lanes = tokens 0..15 of one g) keeps two lanes per bank at most
    (key mod 8 takes each value exactly twice);
  * every ds_read_b128 lane group of the global-store path's slice reads (EcStore::ir: lane -> token 8 p + (lane >> 3),
    logical chunk 8 w + (lane & 7), physical chunk (8 w + c8) ^ key) hits 16 distinct bank slots, for p = 0, 1 and
    either parity of the wave w (round 6: the identity keys of the encoder and the round-5 decoder keys both put two
    lanes of each group on one slot there -- the encoder chains' 21-23 % LDS bank-conflict rate).
usage: python tools/probe/chain_swizzle.py   (CPU; prints both tables and their packed 64-bit constants)"""
A = set(range(0, 4)) | set(range(12, 16))   # li of g-parity-0 lanes in the first b128 group
B = set(range(4, 12))
G1 = set(range(0, 4)) | set(range(12, 16)) | set(range(20, 28))
G2 = set(range(4, 12)) | set(range(16, 20)) | set(range(28, 32))
GROUPS = [G1, G2, {lane + 32 for lane in G1}, {lane + 32 for lane in G2}]


def frag_ok(f, shifts):
    for s in shifts:
        vals = set()
        for li in range(16):
            tp = li + s
            if tp not in f:
                continue
            v = f[tp] ^ (1 if li in B else 0)
            if v in vals:
                return False
            vals.add(v)
    return True


def write_ok(f):
    cnt = {}
    for tp in range(16):
        if tp in f:
            r = f[tp] % 8
            cnt[r] = cnt.get(r, 0) + 1
            if cnt[r] > 2:
                return False
    return True


def store_ok(f):
    for grp in GROUPS:
        for p in (0, 1):
            for wb in (0, 1):
                seen = set()
                for lane in grp:
                    row = 8 * p + (lane >> 3)
                    if row not in f:
                        continue
                    s = ((8 * wb + (lane & 7)) ^ f[row]) & 15
                    if s in seen:
                        return False
                    seen.add(s)
    return True


def ok(f, shifts=(-1, 0, 1)):
    return frag_ok(f, shifts) and write_ok(f) and store_ok(f)


def search(shifts, k=0, f=None):
    f = {-1: 15, 16: 0} if f is None else f
    if k == 16:
        return dict(f)
    for v in range(16):
        f[k] = v
        if ok(f, shifts):
            r = search(shifts, k + 1, f)
            if r:
                return r
        del f[k]
    return None


def packed(f):
    return sum(f[u] << (4 * u) for u in range(16))


if __name__ == "__main__":
    for name, shifts in (("encoder (taps 1)", (0,)), ("decoder (taps 3)", (-1, 0, 1))):
        f = search(shifts)
        print(f"{name}: keys u = 0..15: {[f[u] for u in range(16)]}  packed 0x{packed(f):016x}")
