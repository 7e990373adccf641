"""Synthetic-study generator (vent_analysis_amd/synth.py): the fixtures pin vary=False volumes by
sha256, so the per-study geometry of benchmark batches (vary=True) must leave them unchanged."""
import numpy as np

from vent_analysis_amd.synth import synth_batch, synth_volume, volume_digest


def test_vary_false_is_the_fixture_generator():
    a = synth_volume(40, 36, 9, 3)
    b = synth_volume(40, 36, 9, 3, vary=False)
    assert volume_digest(*a) == volume_digest(*b)


def test_vary_true_changes_geometry_per_seed():
    counts = [int(synth_volume(64, 64, 12, s, vary=True)[1].sum()) for s in range(6)]
    fixed = int(synth_volume(64, 64, 12, 0)[1].sum())
    assert len(set(counts)) == len(counts)          # every study its own lung geometry
    assert min(counts) < 0.95 * fixed < 1.05 * fixed < max(counts)


def test_batch_repeats_unique_studies():
    hp, mk = synth_batch(24, 20, 6, 5, base_seed=7, unique=2, vary=True)
    assert np.array_equal(hp[0], hp[2]) and np.array_equal(mk[1], mk[3])
    assert not np.array_equal(mk[0], mk[1])
