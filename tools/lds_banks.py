"""LDS bank-conflict model of the attention v2 tile image (csrc/attention.hip
Img<D>): extra LDS cycles of the k_product row reads (ds_read_b128) and the
v_product transposed reads (ds_read_b64_tr_b16) for one 32-row half tile,
using the gfx950 lane groups and bank rule of MI355X_MICROARCH.md §LDS.

    python tools/lds_banks.py      # prints padded vs swizzled, asserts Img<D> is conflict-free
"""
G128 = [list(range(0,4))+list(range(12,16))+list(range(20,28)), list(range(4,12))+list(range(16,20))+list(range(28,32))]
G128 += [[x+32 for x in g] for g in G128]
G64 = [list(range(32)), list(range(32,64))]

def cost(addrs, nbytes, groups):
    """extra cycles (conflicts) for one wave instruction"""
    extra = 0
    for g in groups:
        banks = {}
        for l in g:
            a = addrs[l]
            for w in range(nbytes // 4):
                b = (a // 4 + w) % 64
                banks.setdefault(b, set()).add(a // 4 + w)
        extra += max(len(v) for v in banks.values()) - 1
    return extra

def k_reads(D, off):
    tot = 0
    for s in range(D // 16):
        addrs = []
        for l in range(64):
            row, h = l & 31, l >> 5
            col = 8 * h + 16 * s
            addrs.append(off(row, col))
        tot += cost(addrs, 16, G128)
    return tot

def v_reads(D, off, rows=64):
    tot = 0
    for s in range(2):
        for db in range(D // 32):
            for hi in (0, 8):
                addrs = []
                for l in range(64):
                    h, g, i = l >> 5, (l >> 4) & 1, l & 15
                    q, p = i >> 2, i & 3
                    row = 16 * s + 4 * h + q + hi
                    col = db * 32 + 16 * g + 4 * p
                    addrs.append(off(row, col))
                tot += cost(addrs, 8, G64)
    return tot

def plain(RS):
    return lambda row, col: (row * RS + col) * 2



def swz(RS, D, f):
    def off(row, col):
        c2 = (col // 8) ^ f(row)
        assert 0 <= c2 < D // 8
        return row * RS * 2 + c2 * 16 + (col % 8) * 2
    return off


IMG = {  # csrc/attention.hip Img<D>: (row stride, chunk XOR)
    32: (40, lambda r: 0),
    64: (64, lambda r: ((r & 3) << 1) ^ ((r >> 2) & 3)),
    96: (96, lambda r: (r & 1) ^ ((r >> 2) & 3)),
    128: (128, lambda r: ((r & 3) << 2) ^ ((r >> 2) & 3)),
}

if __name__ == "__main__":
    for D, (RS, f) in IMG.items():
        o = swz(RS, D, f)
        k, v = k_reads(D, o), v_reads(D, o)
        pk, pv = k_reads(D, plain(D + 8)), v_reads(D, plain(D + 8))
        print(f"D={D}: D+8 pad k={pk} v={pv} extra cycles | Img k={k} v={v}")
        if D != 32:
            assert k == 0 and v == 0
