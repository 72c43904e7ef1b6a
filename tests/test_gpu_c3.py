"""C3 (BASELINE configs[2]): the 100-pulsar HD GWB workload (30 modes, K = 60, no
per-pulsar noise) streamed in 4096-realization batches with per-realization checksums only — the
realization-sharded job of fakepta_amd.batch.simulate_sharded (reference loop: correlated_noises.py:153-160).

Size-independent checks at the full array size over >= 3 batches:
  * realizations picked from the resident blocks match the oracle (its own Philox stream) to 1e-10;
  * per-realization checksums are bit-identical whatever batch a realization is drawn in (batch 4096 vs
    3000), and through the single-process multi-device driver (fpta_multi_synth, two contexts sharing
    the card: the sharding logic of a 2-GPU job);
  * the gathered checksums agree with the downloaded picks.
"""
import numpy as np
import pytest

from oracle import fakepta_oracle as O
from tests.conftest import assert_parity
from tests.helpers import oracle_segments

pytestmark = pytest.mark.gpu
TOL = 1e-10
N_REAL, BATCH, SEED = 10000, 4096, 4321  # 3 batches: 4096, 4096, 1808


@pytest.fixture(scope="module")
def c3():
    from fakepta import correlated_noises as cn
    from fakepta import fake_pta as fp
    from fakepta_amd import _capi
    from fakepta_amd.batch import BatchSimulator
    ctx = _capi.Context(0)
    np.random.seed(0)
    psrs = fp.make_fake_array(npsrs=100, Tobs=10, ntoas=2000, gaps=False, isotropic=True, toaerr=1e-7,
                              backends="NUPPI.1400", custom_model={"RN": None, "DM": None, "Sv": None})
    cn.add_common_correlated_noise(psrs, orf="hd", log10_A=-15, gamma=13 / 3, components=30)
    sim = BatchSimulator(psrs, white=False, ctx=ctx)
    assert ctx.batch_info()["K"] == 60 and sim.n_toa == 200000
    yield psrs, sim, ctx
    ctx.close()


def test_c3_streamed_checksums_and_picks(c3):
    from fakepta_amd.batch import simulate_sharded
    psrs, sim, ctx = c3
    picks = {0: None, 4095: None, 4096: None, 8191: None, 9999: None}

    def grab(s, first, n):
        for r in picks:
            if first <= r < first + n:
                picks[r] = ctx.batch_download(r - first, 1)[0]

    sums = simulate_sharded(sim, N_REAL, seed=SEED, batch=BATCH, on_batch=grab)
    assert sums.shape == (N_REAL, 2) and np.all(np.isfinite(sums))
    assert ctx.batch_grid_info()["last_path"] == 4  # the default (gridded) path served the job
    segs = oracle_segments(sim)
    for r, row in picks.items():
        want = O.batch_synth(sim.offs, sim.toas, sim.freqs, segs, SEED, r, 1)[0]
        assert_parity(row, want, TOL)
        np.testing.assert_allclose(sums[r, 1], (row ** 2).sum(), rtol=1e-12)
        np.testing.assert_allclose(sums[r, 0], row.sum(), rtol=1e-9, atol=1e-12 * np.abs(row).sum())
    # a different batch split draws every realization bit-identically
    again = simulate_sharded(sim, N_REAL, seed=SEED, batch=3000)
    np.testing.assert_array_equal(again, sums)


def test_c3_multi_device_driver_matches(c3):
    """fpta_multi_synth with two contexts on the card (the 2-device sharding of the C-ABI driver) returns the
    same checksums, in global order, as the single-context stream."""
    from fakepta_amd import _capi
    from fakepta_amd.batch import simulate_sharded
    psrs, sim, ctx = c3
    want = simulate_sharded(sim, 6000, seed=SEED, real0=123, batch=2500)
    m = _capi.MultiContext([0, 0])
    try:
        m.set_toas(sim.offs, sim.toas, sim.freqs)
        for s in sim.segments:
            m.add_signal(s["kind"], s["f"], s["amp"], idx=s["idx"], L=s["L"], mask=s["mask"])
        got = m.synth_checksums(SEED, 123, 6000, batch=2500)
        np.testing.assert_array_equal(got, want)
        got1 = m.synth_checksums(SEED, 123, 6000, batch=1000)
        np.testing.assert_array_equal(got1, want)
        assert m.context(1).batch_grid_info()["last_path"] == 4
    finally:
        m.close()


@pytest.mark.parametrize("pgroup", [1, 4, 7, 16])
def test_fused_checksums_match_full_pass(c3, pgroup):
    """FPTA_OPT_FUSE_CHECKSUMS: the interpolation's partial checksums, reduced in a fixed order, agree with a full
    pass over the resident block (rounding only), including a ragged realization count and the white epilogue, for
    partial rows of 1, 4, 7 and 16 (default) chunks (FPTA_OPT_PART_GROUP; 7 and 16 leave a short last group)."""
    from fakepta_amd import _capi
    psrs, sim, ctx = c3
    ctx.set_option(_capi.OPT_PART_GROUP, pgroup)
    try:
        for n, white in ((1808, False), (333, True)):
            if white:
                ctx.batch_set_white(np.full(sim.n_toa, 1e-7), [], [])
            ctx.set_option(_capi.OPT_FUSE_CHECKSUMS, 0)
            sim.synth(n, seed=SEED, real0=77, to_host=False)
            full = ctx.batch_checksums()
            ctx.set_option(_capi.OPT_FUSE_CHECKSUMS, 1)
            sim.synth(n, seed=SEED, real0=77, to_host=False)
            fused = ctx.batch_checksums()
            assert ctx.batch_grid_info()["last_path"] == 4
            np.testing.assert_allclose(fused[:, 1], full[:, 1], rtol=1e-12)
            np.testing.assert_allclose(fused[:, 0], full[:, 0], rtol=1e-9, atol=1e-12 * np.abs(full[:, 0]).max())
            assert not np.array_equal(fused, full) or n < 2  # the fused route ran (different summation order)
    finally:
        ctx.set_option(_capi.OPT_FUSE_CHECKSUMS, 0)
        ctx.set_option(_capi.OPT_PART_GROUP, 16)
        ctx.batch_set_white(None, [], [])


def test_tail_batch_below_mfma_min_real_is_split_invariant(c3):
    """A streamed job whose last batch is smaller than FPTA_OPT_MFMA_MIN_REAL (16) draws it on the job's path, not
    the direct one: checksums are bit-identical for batch 4096 (tail 1), 4097 (one batch), 1000 (tail 97) and 13
    realizations at a time; in-library streaming, per-batch consumers and the two-context driver agree."""
    from fakepta_amd import _capi
    from fakepta_amd.batch import simulate_sharded
    psrs, sim, ctx = c3
    n = 4097
    want = simulate_sharded(sim, n, seed=SEED, real0=11, batch=4097)
    for batch in (4096, 1000):
        np.testing.assert_array_equal(simulate_sharded(sim, n, seed=SEED, real0=11, batch=batch), want)
    np.testing.assert_array_equal(
        simulate_sharded(sim, n, seed=SEED, real0=11, batch=4096, on_batch=lambda s, first, k: None), want)
    assert ctx.get_option(_capi.OPT_MFMA_MIN_REAL) == 16  # the context's own setting is restored
    small = simulate_sharded(sim, 40, seed=SEED, real0=11 + 4000, batch=13)
    np.testing.assert_array_equal(small, want[4000:4040])
    m = _capi.MultiContext([0, 0])
    try:
        m.set_toas(sim.offs, sim.toas, sim.freqs)
        for s in sim.segments:
            m.add_signal(s["kind"], s["f"], s["amp"], idx=s["idx"], L=s["L"], mask=s["mask"])
        np.testing.assert_array_equal(m.synth_checksums(SEED, 11, n, batch=2048), want)  # shards 2048 + 2049
        np.testing.assert_array_equal(m.synth_checksums(SEED, 11 + 4000, 40, batch=7), want[4000:4040])
    finally:
        m.close()


def test_async_partial_reductions_are_bitwise_identical(c3):
    """FPTA_OPT_ASYNC_SUMS: reducing each block's partial checksums on a stream of their own (two partials buffers,
    beside the next block) returns the same checksums as on the context stream, in-library and two-context driver."""
    from fakepta_amd import _capi
    from tests.helpers import assert_variant_refused, variant_build
    psrs, sim, ctx = c3
    if not variant_build(_capi):  # measured slower: a variant-build option
        assert_variant_refused(ctx, _capi, _capi.OPT_ASYNC_SUMS, 1)
        return
    try:
        res = {}
        for asy in (0, 1):
            ctx.set_option(_capi.OPT_ASYNC_SUMS, asy)
            res[asy] = ctx.batch_synth_checksums(SEED, 99, 9000, batch=2048)
        np.testing.assert_array_equal(res[0], res[1])
    finally:
        ctx.set_option(_capi.OPT_ASYNC_SUMS, 0)
