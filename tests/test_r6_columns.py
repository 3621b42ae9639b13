"""Range-mode R6 period columns (dprf_amd/csrc/dprf_kernels_r6.hip r6_pat_words, r6_round's UNI block read,
r6_store_k's bounded wrap copy): for every password length the column holds every word a read touches, and every
byte a block actually uses is either the period or a wrap byte that r6_store_k writes.  The function is restated
here from the source (and the source is checked to still contain that statement)."""
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "..", "dprf_amd", "csrc", "dprf_kernels_r6.hip")


def pat_words(mode, lmax):
    if mode != 0:
        return ((lmax + 63) >> 2) + 5
    mx = ((lmax + 16) >> 2) + 5
    for bs in (32, 48, 64):
        Lp = lmax + bs
        g = 16
        while Lp % g:
            g >>= 1
        for o in range(0, Lp, g):
            mx = max(mx, (o >> 2) + (5 if o & 3 else 4))
    return mx


def test_source_still_matches_restatement():
    src = open(SRC).read()
    body = src[src.index("static uint32_t r6_pat_words"):]
    body = body[:body.index("\n}\n")]
    for frag in ("((lmax + 63u) >> 2) + 5u", "((lmax + 16u) >> 2) + 5u", "bs <= 64; bs += 16",
                 "while (Lp % g) g >>= 1", "(o >> 2) + ((o & 3u) ? 5u : 4u)"):
        assert frag in body, frag
    assert "lw[4] = (o & 3u) ? col[4 * 64] : lw[3];" in src
    assert "for (uint32_t k = 0; k < 16 && Lp + k < colbytes; k++)" in src


def test_every_read_fits_and_every_used_byte_is_written():
    for lmax in range(1, 33):
        words = pat_words(0, lmax)
        assert words >= 16                                  # r6_begin writes the 16 password words
        assert ((lmax + 16) >> 2) + 5 <= words               # r6_load_k's second 5-word read
        for bs in (32, 48, 64):
            Lp = lmax + bs
            written = set(range(Lp)) | {Lp + k for k in range(16) if Lp + k < 4 * words}
            o = 0
            for _ in range(4 * Lp):                          # the blocks of one round (Lp units x 4)
                nwords = 5 if o & 3 else 4
                assert (o >> 2) + nwords <= words, (lmax, bs, o)
                used = range(o, o + 16)
                assert all(b in written for b in used), (lmax, bs, o)
                o = (o + 16) % Lp
        # list mode keeps the full wrap and the fifth word of every block
        assert pat_words(1, lmax) >= pat_words(0, lmax)


def test_minus_pr6_saves_a_word():
    assert pat_words(0, 6) == 21 and pat_words(1, 6) == 22
