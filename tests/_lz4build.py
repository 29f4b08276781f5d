"""Test helper: LZ4 blocks from explicit sequence lists, with their decoded
bytes.  The block format is the one lz4ada.adb:716-788 parses (token, 15 +
255... length extensions, 2-byte LE offset, match length + 4); a block may
end after a match (the reference's loop stops once its index passes the
block end, :780-782).  Pure Python, test infrastructure only."""
import random


def _ext(v):
    out = bytearray()
    v -= 15
    while v >= 255:
        out.append(255)
        v -= 255
    out.append(v)
    return bytes(out)


def encode(seqs, final_lits=None):
    """seqs: list of (literal bytes, offset, match length >= 4); final_lits:
    the literal-only last sequence (None: the block ends after the last
    match) -> (payload, decoded bytes).  Offsets must be <= bytes decoded so
    far unless the caller wants a reference before the block start."""
    comp = bytearray()
    raw = bytearray()
    for lits, off, ml in seqs:
        L = len(lits)
        m4 = ml - 4
        comp.append(((15 if L >= 15 else L) << 4) | (15 if m4 >= 15 else m4))
        if L >= 15:
            comp += _ext(L)
        comp += lits
        comp += bytes([off & 255, off >> 8])
        if m4 >= 15:
            comp += _ext(m4)
        raw += lits
        if 0 < off <= len(raw):
            pat = raw[len(raw) - off:]
            raw += (pat * (ml // off + 1))[:ml]
        else:
            raw += bytes(ml)  # not decodable: the caller expects an error
    if final_lits is not None:
        L = len(final_lits)
        comp.append((15 if L >= 15 else L) << 4)
        if L >= 15:
            comp += _ext(L)
        comp += final_lits
        raw += final_lits
    return bytes(comp), bytes(raw)


def sparse_seqs(rng: random.Random, out_bytes, lit_lo=100, lit_hi=800, offs=None, mls=None):
    """Literal-heavy sequences (long literal runs, matches of varied offset
    and length: periods 1-15, wraps at 16-31, far sources) until about
    out_bytes are decoded."""
    offs = offs or [1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 23, 31, 32, 33, 64, 100, 1000, None]
    mls = mls or [4, 5, 7, 8, 12, 15, 16, 17, 19, 31, 32, 33, 64, 100, 300, 1000, 2500]
    seqs, pos = [], 0
    while pos < out_bytes:
        lits = rng.randbytes(rng.randint(lit_lo, lit_hi))
        pos += len(lits)
        off = rng.choice(offs)
        if off is None or off > pos:
            off = rng.randint(1, min(pos, 65535))
        ml = rng.choice(mls)
        seqs.append((lits, off, ml))
        pos += ml
    return seqs
