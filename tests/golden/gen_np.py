import numpy as np, sys
def gen(L, C, p, seed, pre, width=0, variant=0):
    rng = np.random.default_rng(seed)
    A = np.frombuffer(b"ACGT", dtype=np.uint8)
    code = rng.integers(0, 4, L)
    ref = A[code]
    def wr(f, s):
        b = s.tobytes()
        if width:
            for k in range(0, len(b), width): f.write(b[k:k+width] + b"\n")
        else: f.write(b + b"\n")
    with open(pre + ".ref.fa", "wb") as f:
        f.write(b">ref\n"); wr(f, ref)
    with open(pre + ".coll.fa", "wb") as f:
        for k in range(C):
            c = code.copy()
            m = rng.random(L) < p
            if variant == 0:
                c[m] = (c[m] + rng.integers(1, 4, int(m.sum()))) % 4
            f.write(b">copy_%d\n" % k); wr(f, A[c])
    with open(pre + ".list", "w") as f:
        f.write(pre + ".ref.fa\n" + pre + ".coll.fa\n")
if __name__ == "__main__":
    L, C, p, seed, pre = int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    width = int(sys.argv[6]) if len(sys.argv) > 6 else 0
    gen(L, C, p, seed, pre, width)


def gen_arrays(L, C, p, seed, leading_empty=True):
    """Same draws as gen(), returned as (ref bytes, concatenated copies as a
    uint8 array, document offsets) -- FASTA's leading '>' gives an empty first
    document, reproduced by leading_empty."""
    rng = np.random.default_rng(seed)
    A = np.frombuffer(b"ACGT", dtype=np.uint8)
    code = rng.integers(0, 4, L)
    ref = A[code].tobytes()
    text = np.empty(C * L, dtype=np.uint8)
    for k in range(C):
        c = code.copy()
        m = rng.random(L) < p
        c[m] = (c[m] + rng.integers(1, 4, int(m.sum()))) % 4
        text[k * L:(k + 1) * L] = A[c]
    off = [0] if leading_empty else []
    off = np.array(off + [k * L for k in range(C + 1)], dtype=np.uint64)
    return ref, text, off
