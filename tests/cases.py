"""Input cases shared by the CPU and GPU tests.

Each case is (name, reference file bytes, collection file bytes, -p prefix).
They cover the reference's document semantics:
leading '>' (empty first document), blank lines, an unterminated last line,
headerless multi-line input, -p cuts, plus workload shapes: repetitive copies
at several SNP rates, identical copies (deep head-string suffix sort),
unrelated random text (a head at almost every position), multi-line FASTA,
CRLF line ends, tiny documents, and references on both the small (_n < 1e6,
FN:1792) and large path."""
import os

import numpy as np

UINT64_MAX = (1 << 64) - 1
ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)


def _rng(seed):
    return np.random.default_rng(seed)


def rand_dna(rng, n):
    return ACGT[rng.integers(0, 4, n)].tobytes()


def mutate(rng, s: bytes, p: float) -> bytes:
    a = np.frombuffer(s, dtype=np.uint8).copy()
    code = np.searchsorted(ACGT, a)
    m = rng.random(len(a)) < p
    code[m] = (code[m] + rng.integers(1, 4, int(m.sum()))) % 4
    return ACGT[code].tobytes()


def fasta(seqs, width=0, names=None, nl=b"\n", final_nl=True):
    out = []
    for k, s in enumerate(seqs):
        out.append(b">" + (names[k] if names else b"seq%d" % k) + nl)
        if width:
            lines = [s[i:i + width] for i in range(0, len(s), width)] or [b""]
            out.append(nl.join(lines) + nl)
        else:
            out.append(s + nl)
    b = b"".join(out)
    if not final_nl:
        b = b[: -len(nl)]
    return b


def copies_case(seed, L, C, p, width=0):
    rng = _rng(seed)
    ref = rand_dna(rng, L)
    seqs = [mutate(rng, ref, p) for _ in range(C)]
    return fasta([ref], width), fasta(seqs, width)


def small_cases():
    """Cases on the small-reference path (_n < 1e6); fast on the oracle."""
    cases = []
    r, c = copies_case(1, 5000, 5, 0.01)
    cases.append(("copies_5k_1pct", r, c, UINT64_MAX))
    r, c = copies_case(2, 20000, 8, 0.001, width=60)
    cases.append(("copies_20k_multiline", r, c, UINT64_MAX))
    r, c = copies_case(3, 3000, 6, 0.05)
    cases.append(("copies_3k_5pct", r, c, UINT64_MAX))
    # identical copies: deep ties in the head string
    rng = _rng(4)
    ref = rand_dna(rng, 4000)
    cases.append(("identical_copies", fasta([ref]), fasta([ref] * 6), UINT64_MAX))
    # unrelated random collection: heads almost everywhere
    rng = _rng(5)
    ref = rand_dna(rng, 3000)
    cases.append(("unrelated_random", fasta([ref]), fasta([rand_dna(rng, 2500), rand_dna(rng, 1800)]),
                  UINT64_MAX))
    # repeats inside the reference itself
    rng = _rng(6)
    unit = rand_dna(rng, 300)
    ref = (unit * 7)[:2000] + rand_dna(rng, 500)
    cases.append(("repetitive_ref", fasta([ref]), fasta([mutate(rng, ref, 0.02) for _ in range(4)]),
                  UINT64_MAX))
    # document-boundary semantics
    rng = _rng(7)
    ref = rand_dna(rng, 2000)
    s = [mutate(rng, ref, 0.01) for _ in range(3)]
    blank = b">a\n" + s[0][:700] + b"\n" + s[0][700:] + b"\n\n" + s[1] + b"\n>b\n>c\n" + s[2] + b"\n"
    cases.append(("blank_lines_and_empty_docs", fasta([ref]), blank, UINT64_MAX))
    cases.append(("no_trailing_newline", fasta([ref]), fasta(s, final_nl=False), UINT64_MAX))
    headerless = b"\n".join([s[0][i:i + 80] for i in range(0, len(s[0]), 80)]) + b"\n"
    cases.append(("headerless_multiline", fasta([ref]), headerless, UINT64_MAX))
    cases.append(("headerless_single_line_tail", fasta([ref]), s[1] + b"\n", UINT64_MAX))
    cases.append(("prefix_cut", fasta([ref]), fasta(s), 3000))
    cases.append(("prefix_cut_at_separator", fasta([ref]), fasta(s), 2003))
    cases.append(("crlf_lines", fasta([ref]), fasta(s, nl=b"\r\n"), UINT64_MAX))
    tiny = b">t1\nA\n>t2\nAC\n>t3\nG\n>t4\n" + s[0][:40] + b"\n"
    cases.append(("tiny_docs", fasta([ref]), tiny, UINT64_MAX))
    # raw (non-FASTA) reference with a trailing '$' and other letters
    rng = _rng(8)
    raw = rand_dna(rng, 1500) + b"NNNNACGTN" + rand_dna(rng, 800) + b"$\n"
    cases.append(("raw_reference_with_N", raw, fasta([mutate(rng, raw[:-2], 0.01) for _ in range(3)]),
                  UINT64_MAX))
    return cases


def no_document_cases():
    """Collections the reader turns into zero documents: an empty file and one
    unterminated line (dropped by getline().good(), FN:1138).  With no heads the
    reference's j-scan runs `size() - 1` wrapped and writes phrasesVector[-1]
    (FN:1359-1385): undefined behaviour, rejected with CMSBWT_EINPUT here."""
    rng = _rng(12)
    ref = fasta([rand_dna(rng, 2000)])
    return [("empty_file", ref, b"", UINT64_MAX),
            ("single_unterminated_line", ref, rand_dna(rng, 300), UINT64_MAX)]


def large_cases():
    """Large-reference path (_n >= 1e6, FN:1795)."""
    r, c = copies_case(9, 1_000_000, 3, 0.001)
    return [("large_1m_3copies", r, c, UINT64_MAX)]


def materialise(tmpdir, case):
    name, ref, coll, prefix = case
    d = os.path.join(str(tmpdir), name)
    os.makedirs(d, exist_ok=True)
    rp, cp = os.path.join(d, "ref.fa"), os.path.join(d, "coll.fa")
    with open(rp, "wb") as f:
        f.write(ref)
    with open(cp, "wb") as f:
        f.write(coll)
    with open(os.path.join(d, "list.txt"), "w") as f:
        f.write(rp + "\n" + cp + "\n")
    return d, rp, cp, prefix


def brute_force_bwt(docs):
    """Multi-string BWT: every document ends with its own terminator; terminators
    sort below every symbol and among themselves by document index; a suffix
    starting a document gets 0x02."""
    m = len(docs)
    suf = []
    for k, d in enumerate(docs):
        a = [c + m for c in d] + [k]
        for p in range(len(a)):
            suf.append((a[p:], k, p))
    suf.sort(key=lambda t: t[0])
    out = bytearray()
    for _, k, p in suf:
        out.append(docs[k][p - 1] if p > 0 else 2)
    return bytes(out)


def py_read_docs(coll: bytes, prefix: int = UINT64_MAX, file_size: int = None):
    """Python restatement of the reference's collection reader (FN:1138-1275):
    returns (documents, sn).  Only '\\n'-terminated lines count (getline().good());
    an empty line or a '>' line ends the current document; -p cuts the line at
    which charactersRead reaches _sn-1 (uint64 wrap kept)."""
    M = (1 << 64) - 1
    size = len(coll) if file_size is None else file_size
    sn = min(size, prefix)
    docs, content, read = [], b"", 0
    pos, stopped = 0, False
    while True:
        e = coll.find(b"\n", pos)
        if e < 0:
            break
        line = coll[pos:e]
        pos = e + 1
        if len(line) == 0 or line[:1] == b">":
            read += 1
            docs.append(content)
            content = b""
        else:
            read += len(line)
            if read >= (sn - 1) & M:
                take = (len(line) - ((read - sn) & M) - 1) & M
                content += line[:min(take, len(line))]
                stopped = True
                break
            content += line
    if content:
        read += 1
        if read < (sn - 1) & M:
            sn = read
        docs.append(content)
    return docs, sn


# Text bytes of the ambiguity cases: >= 0x80 compare below DNA as signed chars
# (FN:55) but sort above it in the suffix array; none is '\n', '\r', '>' or 0x02.
AMBIG_BYTES = (0x81, 0x85, 0x8A, 0x9F, 0xC3, 0x10, 0x1F, 0x7E, 0x7F)


def ambiguity_case(seed, ref_len, n_motifs=6, n_docs=80):
    """A collection on which match.h's comparator is not a strict weak order.
    The reference holds unique 24-mers U_k, each followed by a byte >= 0x90,
    and every byte of AMBIG_BYTES followed by DNA.  Documents are pieces
    U_k[s:e] + b + DNA: at (pos U_k + s, len e - s) the singleton mismatch test
    (FN:54-55, signed chars) makes b >= 0x80 smaller=true and 0x7E/0x7F
    smaller=false, while isaNext (the suffix starting with b, unsigned order)
    puts the smaller=true keys above the smaller=false ones."""
    rng = _rng(seed)
    motifs = [rand_dna(rng, 24) for _ in range(n_motifs)]
    ref = bytearray(rand_dna(rng, ref_len))
    inserts = [m + bytes([int(rng.integers(0x90, 0x100))]) + rand_dna(rng, 40) for m in motifs]
    inserts += [bytes([b]) + rand_dna(rng, 40) for b in AMBIG_BYTES for _ in range(2)]
    step = ref_len // (len(inserts) + 1)
    for i, s in enumerate(inserts):
        o = (i + 1) * step
        ref[o:o + len(s)] = s
    docs = []
    for _ in range(n_docs):
        d = b""
        for _ in range(int(rng.integers(1, 4))):
            m = motifs[int(rng.integers(0, n_motifs))]
            s = int(rng.integers(0, 7))
            e = int(rng.integers(s + 14, 25))
            b = AMBIG_BYTES[int(rng.integers(0, len(AMBIG_BYTES)))]
            d += m[s:e] + bytes([b]) + rand_dna(rng, int(rng.integers(0, 60)))
        docs.append(d)
    return fasta([bytes(ref)]), fasta(docs)


def ambiguity_cases():
    """Comparator-ambiguity inputs on both reference paths
    (_n < 1e6 writes the counter side file, FN:1795)."""
    out = []
    for name, seed, L, nd in (("amb_small_ref", 31, 200_000, 80), ("amb_small_ref_many", 32, 300_000, 400),
                              ("amb_large_ref", 33, 1_100_000, 200)):
        r, c = ambiguity_case(seed, L, n_docs=nd)
        out.append((name, r, c, UINT64_MAX))
    return out
