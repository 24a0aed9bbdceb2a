"""CPU checks of the row-band arithmetic of the MIME rows kernel
(async_amd/csrc/b64x_kernels.hip: k_rows_prep fills RowModel::nb/ru/mx/rg,
k_decode_rows_lines maps a lane's band offset F to (row in band, slot q) with
one 32-bit multiply-high).  Restated here in Python; no GPU needed."""
import math

import pytest

K_THREADS = 256
K_ROWS_U = 4


def band_constants(sx):
    """k_rows_prep's nb, ru, mx for Sx slots per row (Sx < 4096)."""
    low = sx & -sx
    g = low if low < K_THREADS else K_THREADS
    return sx // g, K_THREADS // g, (0xFFFFFFFF + sx) // sx


@pytest.mark.parametrize("sx", [1, 2, 3, 10, 64, 86, 255, 256, 342, 512, 1000, 2048, 4095])
def test_band_tiles_rows_exactly(sx):
    """NB blocks of 256 lanes cover exactly Ru rows of Sx slots (NB * 256 =
    Ru * Sx = lcm(256, Sx)), so U consecutive bands tile the batch."""
    nb, ru, _ = band_constants(sx)
    assert nb * K_THREADS == ru * sx == math.lcm(K_THREADS, sx)


def test_band_division_is_exact_for_every_sx():
    """umulhi(F, ceil(2^32 / Sx)) == F // Sx for every lane offset F of a band
    (F < NB * 256 = Ru * Sx) and every Sx below 4096 -- the kernel's bound.
    The error F * (mx * Sx - 2^32) grows with F, so the largest F decides."""
    for sx in range(1, 4096):
        nb, ru, mx = band_constants(sx)
        fmax = nb * K_THREADS - 1
        assert fmax * (mx * sx - (1 << 32)) < (1 << 32), sx
        for f in (0, 1, sx - 1, sx, fmax // 2, fmax):
            assert (f * mx) >> 32 == f // sx, (sx, f)


def test_band_division_fails_past_the_bound():
    """The prep gates the bands at Sx < 4096: past it the multiply-high is no
    longer exact for every offset of a band (so the gate is needed)."""
    bad = 0
    for sx in range(4096, 4096 + 512):
        nb, ru, mx = band_constants(sx)
        fmax = nb * K_THREADS - 1
        if fmax * (mx * sx - (1 << 32)) >= (1 << 32):
            bad += 1
    assert bad > 0


def test_band_offsets_fit_32_bits_for_config4():
    """Config 4 in CRLF-76 lines: 1,404-byte rows, dense 1,032-byte output
    rows: U bands of rows span well under 2^31 bytes (RowModel::rg)."""
    sx = 1032 // 12  # 86 slots per output row
    nb, ru, mx = band_constants(sx)
    assert (nb, ru) == (43, 128)
    assert K_ROWS_U * ru * 1404 + 1404 + 32 < (1 << 31)
    assert K_ROWS_U * ru * 1032 < (1 << 31)
