"""The XCD-aware block order of the conv kernels (`xcd_block` in csrc/ica_common.h) must be a bijection of
the grid's linear block ids for every grid size, or tiles would be skipped / computed twice.  This restates
its index arithmetic and checks it exhaustively for the grid sizes the launchers can produce (any size,
including sizes that are not multiples of 8), plus that each XCD's range is contiguous."""
import re
from pathlib import Path

import pytest

HDR = Path(__file__).resolve().parents[1] / "imagecompression_adversarial_amd" / "csrc" / "ica_common.h"


def remap(lin: int, total: int) -> int:
    q, r, x = total >> 3, total & 7, lin & 7
    return x * q + min(x, r) + (lin >> 3)


def test_header_formula_is_the_restated_one():
    src = HDR.read_text()
    assert re.search(r"q = total >> 3, r = total & 7, x = lin & 7;", src)
    assert re.search(r"L = x \* q \+ \(x < r \? x : r\) \+ \(lin >> 3\);", src)


@pytest.mark.parametrize("total", list(range(1, 300)) + [768, 1023, 12288, 98307, 131072])
def test_remap_is_bijective_and_contiguous_per_xcd(total):
    ids = [remap(lin, total) for lin in range(total)]
    assert sorted(ids) == list(range(total))
    for x in range(8):
        mine = [ids[lin] for lin in range(x, total, 8)]
        assert mine == list(range(mine[0], mine[0] + len(mine))) if mine else True
