"""Search for the decoder chain's image swizzle keys (csrc/reschain.hip, EcGeo::KEYS): key(u) for tokens u = 0..15 of
a 16-token window plus the zero rows u = -1 / 16, such that
  * every ds_read_b128 lane group of a B-fragment read (lanes {0-3,12-15,20-27}, {4-11,16-19,28-31} and the g + 2
    halves; lane = 16 g + li reads token li + s, logical chunk 4 kk + g, physical chunk (4 kk + g) ^ key) hits 16
    distinct 16-B bank slots for each tap shift s in {-1, 0, +1};
  * the epilogue's ds_write_b64 (16 contiguous lanes = tokens 0..15 of one g) keeps two lanes per bank at most
    (key mod 8 takes each value exactly twice).
usage: python tools/probe/chain_swizzle.py   (CPU; prints the table and its packed 64-bit constant)"""
A = set(range(0, 4)) | set(range(12, 16))   # li of g-parity-0 lanes in the first b128 group
B = set(range(4, 12))


def ok(f):
    for s in (-1, 0, 1):
        vals = set()
        for li in range(16):
            tp = li + s
            if tp not in f:
                continue
            v = f[tp] ^ (1 if li in B else 0)
            if v in vals:
                return False
            vals.add(v)
    cnt = {}
    for tp in range(16):
        if tp in f:
            r = f[tp] % 8
            cnt[r] = cnt.get(r, 0) + 1
            if cnt[r] > 2:
                return False
    return True


def search(order, k, f):
    if k == len(order):
        return dict(f)
    tp = order[k]
    for v in range(16):
        f[tp] = v
        if ok(f):
            r = search(order, k + 1, f)
            if r:
                return r
        del f[tp]
    return None


if __name__ == "__main__":
    f = search(list(range(16)) + [-1, 16], 0, {})
    print("keys u = -1..16:", [f[t] for t in range(-1, 17)])
    print("packed u = 0..15: 0x%016x" % sum(f[u] << (4 * u) for u in range(16)))
