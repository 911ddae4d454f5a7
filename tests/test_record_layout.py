"""The record exchange's bucket layout (bdedup.hip, the kBdRecLayout bit of a
deduper's layout argument; host-side layout functions, no GPU): a source's
bucket holds 3584 / N records so that server bucket k — the union of the N
sources' bucket k — holds about one one-rank bucket (~3584 records, the
one-GPU dedup's tuned size), up to the bucket-count cap; the unique-key layout
is unchanged by the bit's existence, and the scratch is sized for the layout
a deduper will actually use."""
import pytest

from swiftsnails_amd._native import hip

N_BENCH = 262144 * 39


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_record_layout_server_bucket_size(world):
    h = hip()
    bit = h.bd_record_layout_bit()
    P = h.bd_buckets(N_BENCH, world, world | bit)
    assert P % world == 0
    server_bucket = world * N_BENCH / P  # records of N sources per server bucket
    if world <= 4:
        assert 3400 < server_bucket < 3700, server_bucket
    else:  # the 16K bucket cap: ~5000 records, ~2000 distinct keys at the bench shape
        assert P <= 16384 + 64 and server_bucket < 6000, (P, server_bucket)
    # the layout helpers all see the bit: offsets / scratch agree with the count
    assert h.bd_offsets(N_BENCH, world, world | bit)[0] == P
    assert h.bd_scratch_words(N_BENCH, world, world | bit) > P


def test_unique_layout_unchanged_by_the_bit():
    h = hip()
    bit = h.bd_record_layout_bit()
    # one rank: the same layout either way (no servers merging sources)
    assert h.bd_buckets(N_BENCH, 1, 1 | bit) == h.bd_buckets(N_BENCH, 1, 1)
    # N > 1 unique keys: ~3072 occurrences per source bucket (SS_BD_TARGET_DIST), split
    # by the servers into sub-buckets of a table's size
    tg = h.bd_target_dist()
    for world in (2, 4, 8):
        P = h.bd_buckets(N_BENCH, world, world)
        assert 0.9 * tg < N_BENCH / P < 1.1 * tg
        m = h.srv_sub_buckets(world)
        assert world * (N_BENCH / P) * 1.25 / m <= 3000  # <= ~3000 keys per server table


@pytest.mark.parametrize("world", [2, 4, 8])
def test_grouped_record_layout_uses_the_unique_buckets(world):
    """Grouped records (the kBdRecGroup bit beside kBdRecLayout, N > 1): the
    record placement with the unique layout's ~3072-occurrence source buckets
    (the servers split them into the unique layout's sub-buckets, each run's
    records grouped by them after the scatter) — not the 3584 / N records
    whose bucket count reaches the 16K cap at N = 8."""
    h = hip()
    bits = h.bd_record_layout_bit() | h.bd_record_group_bit()
    P = h.bd_buckets(N_BENCH, world, world | bits)
    assert P == h.bd_buckets(N_BENCH, world, world)
    assert P < h.bd_buckets(N_BENCH, world, world | h.bd_record_layout_bit())
    assert h.bd_offsets(N_BENCH, world, world | bits)[0] == P
    assert h.bd_scratch_words(N_BENCH, world, world | bits) > P
    # the servers' split of a grouped layout is the unique one's
    m = h.srv_sub_buckets(world, N_BENCH, world)
    assert m > 1 and world * (N_BENCH / P) * 1.25 / m <= 3000
