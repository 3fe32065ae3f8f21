"""Host restatement of the per-XCD unit-queue partition (rp_device.h fetch_pixel, rp_api.cpp render_shard):
queue g of G serves the chunks g, g + G, ... of C consecutive tiles of the tile order, nk(g) tiles, its i-th
tile being (i / C) * G * C + g * C + i % C.  Every tile must be served by exactly one queue, whatever K, G, C
(the GPU test test_unit_queues_bitwise checks the kernel itself renders identical frames)."""
import pytest


def queue_tiles(K, G, C, g):
    GC = G * C
    rest = K % GC
    nk = (K // GC) * C + min(rest - min(rest, g * C), C)
    return [(i // C) * GC + g * C + i % C for i in range(nk)]


@pytest.mark.parametrize("K", [1, 2, 7, 8, 9, 63, 64, 65, 255, 2040])
@pytest.mark.parametrize("G,C", [(1, 1), (8, 1), (8, 2), (8, 3), (8, 16), (3, 5)])
def test_queues_partition_the_tiles(K, G, C):
    seen = []
    for g in range(G):
        tiles = queue_tiles(K, G, C, g)
        assert tiles == sorted(tiles)  # each queue keeps the order's sequence
        seen += tiles
    assert sorted(seen) == list(range(K))


@pytest.mark.parametrize("K", [1, 6, 8, 2040, 4999])
def test_regions_mode_is_one_chunk_per_queue(K):
    """XCD_REGIONS = chunk ceil(K / G): queue g serves one contiguous run of the order."""
    G = 8
    C = (K + G - 1) // G
    for g in range(G):
        tiles = queue_tiles(K, G, C, g)
        assert tiles == list(range(min(g * C, K), min((g + 1) * C, K)))
