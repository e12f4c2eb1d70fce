"""Host model of the half-tile rings' LDS layout (csrc/wmx_gemm.hip: gemm256_kernel with WMX_G256_BK = 64 and
gemm_mx8_256_kernel with WMX_MX8_BK = 128).  A unit row r is 128 B; its 16-B chunk c sits at position
c ^ ((r >> 1) & 7).  Checked here, without a GPU:
  * the DMA side: the 8 lanes of a row (lane & 7 = LDS position) read every source chunk of the row exactly once;
  * the read side: for every fragment read the kernels issue, each ds_read_b128 lane group (gfx950 serves the wave in
    four 16-lane groups, MI355X_MICROARCH.md LDS table) touches 16 distinct (row parity, position) slots, i.e. all
    64 banks once: conflict-free;
  * the unit maps cover the tile: A units 0 / 3 and W units 1 / 2 hold every row of the 256-row panels once."""
import itertools

GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
          list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
GROUPS += [[l + 32 for l in g] for g in GROUPS]


def pos(r, c):
    return c ^ ((r >> 1) & 7)


def bank_slots(addrs):
    # a 16-B ds_read_b128 at byte address a covers banks (a / 4) % 64 .. + 3; rows are 128 B: slot = (row parity, pos)
    return [((a // 128) & 1, (a % 128) // 16) for a in addrs]


def test_dma_reads_every_chunk_once():
    for r in range(128):
        srcs = [pos(r, p) for p in range(8)]  # lane with LDS position p reads source chunk p ^ sw(r) = pos(r, p)
        assert sorted(srcs) == list(range(8)), r


def test_bf16_fragment_reads_conflict_free():
    # lane (fr = l & 15, fq = l >> 4) reads row base + fr, chunk 4 s + fq (k32 half s); bases are multiples of 16
    for base, s in itertools.product(range(0, 128, 16), (0, 1)):
        addr = [(base + (l & 15)) * 128 + pos(base + (l & 15), 4 * s + (l >> 4)) * 16 for l in range(64)]
        for g in GROUPS:
            slots = bank_slots([addr[l] for l in g])
            assert len(set(slots)) == 16, (base, s, g, slots)


def test_mx8_fragment_reads_conflict_free():
    # lane (fr = l & 31, g = l >> 5) reads row base + fr, chunks 4 s + g and 4 s + 2 + g (K-step s); bases multiples of 32
    for base, s, h in itertools.product(range(0, 128, 32), (0, 1), (0, 2)):
        addr = [(base + (l & 31)) * 128 + pos(base + (l & 31), 4 * s + h + (l >> 5)) * 16 for l in range(64)]
        for g in GROUPS:
            slots = bank_slots([addr[l] for l in g])
            assert len(set(slots)) == 16, (base, s, h, g, slots)


def test_unit_maps_cover_the_panels():
    a_rows = sorted([(r >> 6) * 128 + (r & 63) for r in range(128)] + [(r >> 6) * 128 + 64 + (r & 63) for r in range(128)])
    w_rows = sorted([(r >> 5) * 64 + (r & 31) for r in range(128)] + [(r >> 5) * 64 + 32 + (r & 31) for r in range(128)])
    assert a_rows == list(range(256)) and w_rows == list(range(256))
    # the wave's fragment rows live in its own units: A rows 128 wm + [0, 64) = unit 0 rows 64 wm + [0, 64)
    for wm in (0, 1):
        assert [(r >> 6) * 128 + (r & 63) for r in range(64 * wm, 64 * wm + 64)] == list(range(128 * wm, 128 * wm + 64))
    for wn in range(4):
        assert [(r >> 5) * 64 + (r & 31) for r in range(32 * wn, 32 * wn + 32)] == list(range(64 * wn, 64 * wn + 32))
