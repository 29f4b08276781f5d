"""The test-side LZ4 block builder (tests/_lz4build.py) agrees with the
oracle, so GPU tests built on it compare against reference semantics."""
import random

import _lz4build as B
import _oracle as O
import lz4frame


def test_builder_matches_oracle():
    rng = random.Random(3)
    blocks = []
    for i, n in enumerate([70_000, 30_000, 5_000]):
        seqs = B.sparse_seqs(rng, n)
        blocks.append(B.encode(seqs, None if i == 1 else rng.randbytes(50)))
    frame, raw = lz4frame.build_frame([(c, r, False) for c, r in blocks], 256 << 10,
                                      block_cksum=True, content_cksum=True)
    st, out, _, msg = O.decode_stream(frame)
    assert st == O.OK, msg
    assert out == raw


def test_builder_offset0_is_an_error():
    seqs = B.sparse_seqs(random.Random(4), 2000)
    lits, _, ml = seqs[1]
    seqs[1] = (lits, 0, ml)
    comp, raw = B.encode(seqs, b"x" * 20)
    frame, _ = lz4frame.build_frame([(comp, raw, False)], 64 << 10)
    st, _, _, msg = O.decode_stream(frame)
    assert st != O.OK and "Offset = 0" in msg
