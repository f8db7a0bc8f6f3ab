"""LDS bank model of the conv kernels' operand images (MI355X_MICROARCH.md §LDS): the MFMA fragment
reads (ds_read_b128: four 16-lane groups, bank = (a/4) mod 64) of the [rows][BK] stage images are
conflict-free under csrc/conv_igemm_kernel.h ``fswz<BK>`` for both stage depths (BK = 64: 128-B
rows; BK = 32: 64-B rows of the 4-slot rings)."""
import pytest

# ds_read_b128 lane groups (one LDS cycle each when conflict-free)
GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
          list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
GROUPS += [[l + 32 for l in g] for g in GROUPS]


def fswz(bk, row):
    return ((row >> 1) & 7) if bk == 64 else (((row >> 3) & 1) << 1)


def extra_cycles(addrs):
    """Sum over lane groups of (max distinct addresses on one bank - 1) for 16-B accesses."""
    extra = 0
    for g in GROUPS:
        banks = {}
        for lane in g:
            a = addrs[lane]
            for w in range(4):
                banks.setdefault((a // 4 + w) % 64, set()).add(a)
        extra += max(len(v) for v in banks.values()) - 1
    return extra


@pytest.mark.parametrize("bk", [64, 32])
def test_fragment_reads_conflict_free(bk):
    row_bytes = bk * 2
    for base_row in range(0, 256, 16):        # every 16-row MFMA fragment of a 256-row image
        for ks in range(bk // 32):            # k32 steps of the stage
            addrs = []
            for lane in range(64):
                row = base_row + (lane & 15)
                ch = ks * 4 + (lane >> 4)
                addrs.append(row * row_bytes + ((ch ^ fswz(bk, row)) * 16))
            assert extra_cycles(addrs) == 0, (bk, base_row, ks)


@pytest.mark.parametrize("bk", [64, 32])
def test_swizzle_is_a_permutation_per_row(bk):
    """Each row's chunks land on distinct positions (the DMA source-side inverse is well defined)."""
    cpr = bk // 8
    for row in range(256):
        assert sorted(c ^ fswz(bk, row) for c in range(cpr)) == list(range(cpr))
