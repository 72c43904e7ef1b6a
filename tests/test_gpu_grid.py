"""Gridded synthesis path (FPTA_OPT_SYNTH_PATH 4, grid.hip) against the CPU oracle.

The gridded path evaluates the same Fourier sums as the direct kernels through an oversampled
phase grid (real DFT) and a banded exponential-of-semicircle interpolation.
It is an approximation with a bounded aliasing error: at the shipped defaults (width 15,
oversampling 1.5; a-priori bound exp(-pi w sqrt(1 - 1/sigma)) = 1.5e-12) the error is <= ~6e-12
relative for a FLAT spectrum (every mode weighs equally, the worst case) and smaller for red
spectra (width 14 reaches 3.1e-11 on these cases: tools/grid_width_errors.py, profiles/r03l_grid_width_errors.jsonl).
Tolerance: the suite's
1e-10; the accuracy tests below also check the tighter bound GRID_TOL the defaults are
designed for, AT the shipped defaults (the fixture restores the context's own options after every test
instead of writing fixed values).
"""
import numpy as np
import pytest

from oracle import fakepta_oracle as O
from tests.conftest import assert_parity, rel_err
from tests.helpers import (assert_variant_refused, common_signal, oracle_segments, per_psr_signal, random_layout,
                           variant_build)

pytestmark = pytest.mark.gpu

TOL = 1e-10
GRID_TOL = 2e-11


@pytest.fixture(scope="module")
def capi():
    from fakepta_amd import _capi
    return _capi


@pytest.fixture(scope="module")
def ctx(capi):
    c = capi.Context(0)
    yield c
    c.close()


SHIPPED_WIDTH, SHIPPED_SIGMA100 = 15, 150  # capi.hip fpta_ctx defaults


def _diag_build(capi):
    """The loaded library holds the diagnostic kernels (make variant DEFS=-DFPTA_DIAG_KERNELS)."""
    return bool(capi.build_flags() & capi.BUILD_DIAG)


def _assert_refused(ctx, capi, ws):
    old = ctx.get_option(capi.OPT_INTERP_WS)
    with pytest.raises(capi.FptaError, match="diagnostic"):
        ctx.set_option(capi.OPT_INTERP_WS, ws)
    assert ctx.get_option(capi.OPT_INTERP_WS) == old


@pytest.fixture(scope="module")
def shipped(ctx, capi):
    """The options of a fresh context: the shipped defaults every test must run at unless it says otherwise."""
    opts = ctx.options()
    assert opts[capi.OPT_GRID_WIDTH] == SHIPPED_WIDTH and opts[capi.OPT_GRID_SIGMA] == SHIPPED_SIGMA100
    return opts


@pytest.fixture(params=[(1, 1), (1, 0), (0, 1)], ids=["dft_gen", "dft_mfma", "dft_valu"])
def gridded(ctx, capi, shipped, request):
    """Gridded path with the DFT drawing its per-pulsar coefficients itself (k_grid_dft_gen, the default), or reading
    them from the coefficient buffer on fp64 MFMA (FPTA_OPT_DFT_GEN 0: a variant-build option) or VALU
    (FPTA_OPT_GRID_MFMA bit 0, which draws through the buffer whatever DFT_GEN); the interpolation is on MFMA in every
    case. The context's options are restored to the shipped snapshot afterwards."""
    if request.param[1] == 0 and not variant_build(capi):
        pytest.skip("FPTA_OPT_DFT_GEN 0 is a variant-build option")
    ctx.set_option(capi.OPT_SYNTH_PATH, 4)
    ctx.set_option(capi.OPT_GRID_MFMA, request.param[0])
    ctx.set_option(capi.OPT_DFT_GEN, request.param[1])
    yield ctx
    ctx.set_options(shipped)


def _flat_layout(ctx, rng, P=4, n_range=(100, 300), n_modes=100, idx=2.0, t0=4.5e9):
    offs, toas, nu = random_layout(rng, P, n_range, t_max=1.6e8)
    toas = toas + t0
    ctx.batch_set_toas(offs, toas, nu)
    f, _ = per_psr_signal(rng, offs, toas, n_modes)
    a = np.full_like(f, 1e-7)
    ctx.batch_add_signal(0, f, a, idx=idx)
    return offs, toas, nu, [O.Segment(0, 2 * np.pi * f, a, idx)]


@pytest.mark.parametrize("n_modes", [1, 30, 100, 257])
def test_flat_spectrum_real_epochs(gridded, capi, n_modes):
    """Worst case for the aliasing error: flat spectrum, real-MJD-like epochs (t ~ 5e9 s), at the shipped
    width / oversampling."""
    assert gridded.get_option(capi.OPT_GRID_WIDTH) == SHIPPED_WIDTH
    assert gridded.get_option(capi.OPT_GRID_SIGMA) == SHIPPED_SIGMA100
    rng = np.random.default_rng(n_modes)
    offs, toas, nu, segs = _flat_layout(gridded, rng, n_modes=n_modes)
    got = gridded.batch_synth(5, 0, 64)
    want = O.batch_synth(offs, toas, nu, segs, 5, 0, 64)
    assert rel_err(got, want) <= GRID_TOL
    assert_parity(got, want, TOL)


def test_width_and_oversampling_options(gridded, capi):
    """The kernel width sets the error (a narrow kernel is measurably worse); a lower oversampling
    with a wider kernel stays within tolerance."""
    rng = np.random.default_rng(3)
    offs, toas, nu, segs = _flat_layout(gridded, rng, n_modes=60)
    want = O.batch_synth(offs, toas, nu, segs, 8, 0, 32)
    gridded.set_option(capi.OPT_GRID_WIDTH, 6)
    coarse = rel_err(gridded.batch_synth(8, 0, 32), want)
    gridded.set_option(capi.OPT_GRID_WIDTH, 16)
    gridded.set_option(capi.OPT_GRID_SIGMA, 150)
    fine = rel_err(gridded.batch_synth(8, 0, 32), want)
    assert 1e-9 < coarse < 1e-3
    assert fine <= GRID_TOL


def test_auto_path_respects_error_bound(ctx, capi, shipped):
    """Auto selection (path 0) takes the gridded path at the shipped defaults, refuses it (and says why) when
    the width / oversampling pair's a-priori bound exceeds 2e-11, and reports the bound in grid_info."""
    rng = np.random.default_rng(4)
    # 2000-TOA pulsars: the gridded plan needs well under half the direct FMAs (auto's cost rule)
    offs, toas, nu = random_layout(rng, 4, (2000, 2000), ragged=False)
    ctx.batch_set_toas(offs, toas, nu)
    f, a = per_psr_signal(rng, offs, toas, 30)
    ctx.batch_add_signal(0, f, a, idx=2.0)
    segs = [O.Segment(0, 2 * np.pi * f, a, 2.0)]
    try:
        ctx.batch_synth(3, 0, 64, to_host=False)
        gi = ctx.batch_grid_info()
        assert gi["last_path"] == 4 and gi["path_reason"] == "", gi
        assert gi["width"] == SHIPPED_WIDTH
        assert abs(gi["err_bound"] - np.exp(-np.pi * SHIPPED_WIDTH * np.sqrt(1 / 3))) < 1e-15
        ctx.set_option(capi.OPT_GRID_WIDTH, 8)
        got = ctx.batch_synth(3, 0, 64)
        gi = ctx.batch_grid_info()
        assert gi["last_path"] == 3 and "error bound" in gi["path_reason"]
        assert_parity(got, O.batch_synth(offs, toas, nu, segs, 3, 0, 64), TOL)
        ctx.set_options(shipped)
        ctx.batch_synth(3, 0, 8, to_host=False)  # below FPTA_OPT_MFMA_MIN_REAL: direct
        gi = ctx.batch_grid_info()
        assert gi["last_path"] == 1 and "n_real" in gi["path_reason"]
    finally:
        ctx.set_options(shipped)


def test_unsorted_and_clustered_toas(gridded):
    """TOAs in any order (chunks shrink where the band would exceed the row cap) and clustered
    epochs with long gaps (make_fake_array gaps=True)."""
    rng = np.random.default_rng(17)
    P = 6
    n = rng.integers(50, 400, size=P)
    offs = np.concatenate([[0], np.cumsum(n)]).astype(np.int64)
    parts = []
    for p, k in enumerate(n):
        centers = rng.uniform(0, 3e8, 5)
        t = np.concatenate([c + rng.uniform(0, 3e5, k // 5 + 1) for c in centers])[:k]
        if p % 2:
            rng.shuffle(t)
        parts.append(t)
    toas = np.concatenate(parts)
    nu = rng.uniform(700, 3000, offs[-1])
    gridded.batch_set_toas(offs, toas, nu)
    segs = []
    for nm, idx in ((30, 0.0), (100, 2.0)):
        f, a = per_psr_signal(rng, offs, toas, nm)
        gridded.batch_add_signal(0, f, a, idx=idx)
        segs.append(O.Segment(0, 2 * np.pi * f, a, idx))
    f, a, L, _ = common_signal(rng, offs, toas, 30)
    gridded.batch_add_signal(1, f, a, L=L)
    segs.append(O.Segment(1, 2 * np.pi * f, a, 0.0, L=L))
    for real0, R in ((0, 130), (3, 17)):
        got = gridded.batch_synth(42, real0, R)
        want = O.batch_synth(offs, toas, nu, segs, 42, real0, R)
        assert_parity(got, want, TOL)


@pytest.mark.parametrize("real0", [0, 7])
def test_fused_white_matches_separate_pass(gridded, capi, real0):
    rng = np.random.default_rng(23)
    offs, toas, nu = random_layout(rng, 5, (30, 200))
    gridded.batch_set_toas(offs, toas, nu)
    f, a = per_psr_signal(rng, offs, toas, 30)
    gridded.batch_add_signal(0, f, a, idx=0.0)
    sigma = rng.uniform(1e-7, 1e-6, offs[-1])
    blocks = [np.arange(s, min(s + 3, offs[-1])) for s in range(0, offs[-1], 4)]
    es = rng.uniform(1e-8, 1e-7, len(blocks))
    gridded.batch_set_white(sigma, blocks, es)
    fused = gridded.batch_synth(77, real0, 131)
    gridded.set_option(capi.OPT_FUSE_WHITE, 0)
    separate = gridded.batch_synth(77, real0, 131)
    assert_parity(fused, separate, 1e-13)
    block_of = -np.ones(offs[-1], dtype=np.int64)
    for b, q in enumerate(blocks):
        block_of[q] = b
    want = O.batch_synth(offs, toas, nu, [O.Segment(0, 2 * np.pi * f, a, 0.0)], 77, real0, 131, sigma=sigma,
                         block_of=block_of, ecorr_sigma=es)
    assert_parity(fused, want, TOL)


def test_split_invariance_bitwise(gridded):
    rng = np.random.default_rng(8)
    offs, toas, nu = random_layout(rng, 6, (40, 300))
    gridded.batch_set_toas(offs, toas, nu)
    f, a = per_psr_signal(rng, offs, toas, 41)
    gridded.batch_add_signal(0, f, a, idx=2.0)
    full = gridded.batch_synth(2024, 0, 200)
    parts = np.concatenate([gridded.batch_synth(2024, r0, n) for r0, n in ((0, 64), (64, 100), (164, 36))])
    np.testing.assert_array_equal(full, parts)


def test_non_harmonic_grid_is_refused(gridded, capi):
    rng = np.random.default_rng(2)
    offs, toas, nu = random_layout(rng, 3, (20, 50))
    gridded.batch_set_toas(offs, toas, nu)
    f = np.sort(rng.uniform(1e-9, 1e-7, (3, 10)), axis=1)
    gridded.batch_add_signal(0, f, np.full_like(f, 1e-7))
    with pytest.raises(capi.FptaError, match="harmonic"):
        gridded.batch_synth(1, 0, 32)


def test_c2_full_size_gridded_vs_seeded(ctx, capi):
    """BASELINE configs[1] (100 psr x 2000 TOAs, RN30 + DM100 + HD30, R = 1024): the gridded path and
    the exact seeded VALU path agree over the whole block (size-independent cross-check of two
    different algorithms on the same device coefficients)."""
    from fakepta import correlated_noises as cn
    from fakepta import fake_pta as fp
    from fakepta_amd.batch import BatchSimulator
    np.random.seed(0)
    psrs = fp.make_fake_array(npsrs=100, Tobs=10, ntoas=2000, gaps=False, isotropic=True, toaerr=1e-7,
                              backends="NUPPI.1400", custom_model={"RN": 30, "DM": 100, "Sv": None})
    cn.add_common_correlated_noise(psrs, orf="hd", log10_A=-15, gamma=13 / 3)
    sim = BatchSimulator(psrs, white=False, ctx=ctx)
    try:
        ctx.set_option(capi.OPT_SYNTH_PATH, 4)
        sim.synth(1024, seed=99, to_host=False)
        ctx.debug_fill_out(np.nan)  # every sample written
        grid = sim.synth(1024, seed=1234)
        # the shipped C2 kernel (bench.py's): the fused draws + DFTs + half-chunk-band interpolation, GEN (draws in the
        # kernel), even first realization
        assert ctx.batch_grid_info()["interp_kernel"] == "k_grid_fused<8, false, true, true>", ctx.batch_grid_info()
        ctx.set_option(capi.OPT_SYNTH_PATH, 3)
        exact = sim.synth(1024, seed=1234)
    finally:
        ctx.set_option(capi.OPT_SYNTH_PATH, 0)
    assert np.all(np.isfinite(grid))
    assert rel_err(grid, exact) <= GRID_TOL
    per_real = np.linalg.norm(grid - exact, axis=1) / np.linalg.norm(exact, axis=1)
    assert per_real.max() <= 5 * GRID_TOL
    # realizations across the block against the oracle's own batch semantics: its Philox draws, its ORF mixing and the
    # direct sums (no device coefficients involved)
    segs = oracle_segments(sim)
    for r in (0, 1, 511, 1023):
        want = O.batch_synth(sim.offs, sim.toas, sim.freqs, segs, 1234, r, 1)[0]
        assert_parity(grid[r], want, TOL)


@pytest.mark.parametrize("path", [4, 3, 1])
def test_side_stream_draws_are_bitwise_identical(ctx, capi, shipped, path):
    """FPTA_OPT_OVERLAP: coefficients drawn on the side stream (consumers wait per signal) give bit-identical
    blocks and coefficients to the single-stream order, on the gridded, exact and direct paths, across
    consecutive batches (the side stream must not overwrite a block's coefficients while it is still read)."""
    rng = np.random.default_rng(31)
    offs, toas, nu = random_layout(rng, 70, (40, 120))
    ctx.batch_set_toas(offs, toas, nu)
    f, a = per_psr_signal(rng, offs, toas, 30)
    ctx.batch_add_signal(0, f, a, idx=0.0)
    f, a = per_psr_signal(rng, offs, toas, 50)
    ctx.batch_add_signal(0, f, a, idx=2.0)
    f, a, L, _ = common_signal(rng, offs, toas, 20)
    ctx.batch_add_signal(1, f, a, L=L)
    try:
        ctx.set_option(capi.OPT_SYNTH_PATH, path)
        runs, blocks = {}, {}
        for ov in (0, 1):
            ctx.set_option(capi.OPT_OVERLAP, ov)
            runs[ov] = [ctx.batch_synth(99, r0, 200, coeffs=True) for r0 in (0, 200, 400)]
            # device-only batches back to back: the next block's draws overlap this block's interpolation
            blk = []
            for r0 in (600, 800, 1000, 1200):
                ctx.batch_synth(99, r0, 200, to_host=False)
                blk.append(ctx.batch_download(0, 200))
            blocks[ov] = blk
        for (o0, c0), (o1, c1) in zip(runs[0], runs[1]):
            np.testing.assert_array_equal(o0, o1)
            np.testing.assert_array_equal(c0, c1)
        for b0, b1 in zip(blocks[0], blocks[1]):
            np.testing.assert_array_equal(b0, b1)
    finally:
        ctx.set_options(shipped)


@pytest.mark.parametrize("fuse", [0, 1])
def test_lds_interpolation_is_bitwise_identical(ctx, capi, shipped, fuse):
    """FPTA_OPT_INTERP_LDS: the LDS-staged interpolation (chunk groups, union rows staged once per workgroup)
    returns the register-tiled kernel's block and checksums bit for bit, on a ragged multi-signal layout with
    pulsar boundaries inside chunk groups and unsorted TOAs. A diagnostic kernel (measured slower, not adopted): only
    in libraries built with -DFPTA_DIAG_KERNELS; the product library refuses the option."""
    if not capi.build_flags() & capi.BUILD_DIAG:
        with pytest.raises(capi.FptaError, match="diagnostic"):
            ctx.set_option(capi.OPT_INTERP_LDS, 1)
        assert ctx.get_option(capi.OPT_INTERP_LDS) == 0
        return
    rng = np.random.default_rng(41)
    offs, toas, nu = random_layout(rng, 23, (31, 260))
    perm = rng.permutation(offs[1] - offs[0])
    toas[offs[0]:offs[1]] = toas[offs[0]:offs[1]][perm]  # one pulsar with TOAs out of order
    ctx.batch_set_toas(offs, toas, nu)
    f, a = per_psr_signal(rng, offs, toas, 30)
    ctx.batch_add_signal(0, f, a, idx=0.0)
    f, a = per_psr_signal(rng, offs, toas, 100)
    ctx.batch_add_signal(0, f, a, idx=2.0)
    f, a, L, _ = common_signal(rng, offs, toas, 30)
    ctx.batch_add_signal(1, f, a, L=L)
    try:
        ctx.set_option(capi.OPT_SYNTH_PATH, 4)
        ctx.set_option(capi.OPT_FUSE_CHECKSUMS, fuse)
        ctx.set_option(capi.OPT_PART_GROUP, 1)  # the diagnostic kernels write one partial row per chunk
        res = {}
        for lds in (0, 1):
            ctx.set_option(capi.OPT_INTERP_LDS, lds)
            res[lds] = (ctx.batch_synth(5, 300, 333), ctx.batch_checksums())
        np.testing.assert_array_equal(res[0][0], res[1][0])
        np.testing.assert_array_equal(res[0][1], res[1][1])
    finally:
        ctx.set_options(shipped)


def _shared_span_layout(ctx, rng, P=12, n=(300, 700), nu_const=True, with_masked=False):
    """Pulsars on one common span T (as make_fake_array with equal Tobs): red noise, DM (idx 2) and a common
    GWB all sit on f_k = k / T. At a single radio frequency (nu == freqf) DM's chromatic weight is 1, so the
    three share w0 and the weight per TOA and coalesce into one grid signal; with several radio frequencies
    only RN and the GWB do. A masked signal (backend noise) never joins an unmasked one."""
    counts = rng.integers(n[0], n[1], size=P)
    offs = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    t0, t1 = 4.4e9, 4.4e9 + 3.15e8
    toas = np.concatenate([np.concatenate([[t0], np.sort(rng.uniform(t0, t1, k - 2)), [t1]]) for k in counts])
    nu = np.full(offs[-1], 1400.0) if nu_const else rng.choice([800.0, 1400.0, 2500.0], size=offs[-1])
    T = t1 - t0
    ctx.batch_set_toas(offs, toas, nu)
    segs = []
    for nm, idx in ((30, 0.0), (100, 2.0)):
        f = np.tile(np.arange(1, nm + 1) / T, (P, 1))
        a = np.sqrt(O.powerlaw(f, rng.uniform(-14.5, -13.5, (P, 1)), 3.0) / T)
        ctx.batch_add_signal(0, f, a, idx=idx)
        segs.append(O.Segment(0, 2 * np.pi * f, a, idx))
    fc = np.arange(1, 31) / T
    ac = np.sqrt(O.powerlaw(fc, -14.0, 13 / 3) / T)
    v = rng.normal(size=(P, 3))
    L = O.mvn_factor(O.orf_hd(v / np.linalg.norm(v, axis=1)[:, None]))
    ctx.batch_add_signal(1, fc, ac, L=L)
    segs.append(O.Segment(1, 2 * np.pi * fc, ac, 0.0, L=L))
    if with_masked:
        mask = (np.arange(offs[-1]) % 3 == 0).astype(np.uint8)
        f = np.tile(np.arange(1, 21) / T, (P, 1))
        a = np.sqrt(O.powerlaw(f, -13.8, 2.0) / T)
        ctx.batch_add_signal(0, f, a, idx=0.0, mask=mask)
        segs.append(O.Segment(0, 2 * np.pi * f, a, 0.0, mask=mask.astype(bool)))
    return offs, toas, nu, segs


@pytest.mark.parametrize("nu_const,with_masked,n_grid", [(True, False, 1), (False, False, 2), (True, True, 2)])
def test_coalesced_grid_signals(ctx, capi, shipped, nu_const, with_masked, n_grid):
    """FPTA_OPT_GRID_COALESCE: signals sharing w0 and the chromatic weight share one grid; the block matches the
    oracle at the gridded tolerance and the un-coalesced plan to rounding, coefficient downloads still return
    every signal's own draws (taken before the merge), and the side stream gives bit-identical blocks."""
    rng = np.random.default_rng(53 + n_grid + 7 * with_masked)
    offs, toas, nu, segs = _shared_span_layout(ctx, rng, nu_const=nu_const, with_masked=with_masked)
    try:
        ctx.set_option(capi.OPT_SYNTH_PATH, 4)
        got, co = ctx.batch_synth(11, 5, 150, coeffs=True)
        gi = ctx.batch_grid_info()
        assert gi["grid_signals"] == n_grid and gi["signals"] == len(segs), gi
        want = O.batch_synth(offs, toas, nu, segs, 11, 5, 150)
        assert rel_err(got, want) <= GRID_TOL
        assert_parity(got, want, TOL)
        ctx.set_option(capi.OPT_OVERLAP, 0)
        np.testing.assert_array_equal(ctx.batch_synth(11, 5, 150), got)
        ctx.set_option(capi.OPT_OVERLAP, 1)
        ctx.set_option(capi.OPT_GRID_COALESCE, 0)
        sep, co_sep = ctx.batch_synth(11, 5, 150, coeffs=True)
        assert ctx.batch_grid_info()["grid_signals"] == len(segs)
        np.testing.assert_array_equal(co, co_sep)
        assert rel_err(got, sep) <= GRID_TOL
    finally:
        ctx.set_options(shipped)


@pytest.mark.parametrize("fuse", [0, 1])
@pytest.mark.parametrize("layout", ["coalesced", "single"])
def test_pipelined_batches_are_bitwise_identical(ctx, capi, shipped, fuse, layout):
    """Pipelined gridded batches (FPTA_OPT_OVERLAP 1): a streamed shard draws, merges and transforms block b + 1 on
    the side stream into the other grid buffer while block b interpolates; the per-realization checksums of 5
    back-to-back blocks (no host round trip) equal the single-stream ones bit for bit, with and without fused
    checksums, for a coalesced multi-signal layout and a one-signal (C3-like) layout; and so do they with the
    per-pulsar DM grid signal drawn and transformed on a second side stream (FPTA_OPT_SIDE_SPLIT 1, or 2: after the
    common draws) or not."""
    rng = np.random.default_rng(61)
    if layout == "coalesced":
        _shared_span_layout(ctx, rng, nu_const=False)
    else:
        offs, toas, nu = random_layout(rng, 20, (100, 400))
        ctx.batch_set_toas(offs, toas, nu)
        f, a, L, _ = common_signal(rng, offs, toas, 30)
        ctx.batch_add_signal(1, f, a, L=L)
    try:
        ctx.set_option(capi.OPT_SYNTH_PATH, 4)
        ctx.set_option(capi.OPT_FUSE_CHECKSUMS, fuse)
        res = {}
        runs = ((0, 2), (1, 1), (1, 0), (1, 2)) if variant_build(capi) else ((0, 2), (1, 2))  # SIDE_SPLIT 0 / 1: variant
        for ov, split in runs:
            ctx.set_option(capi.OPT_OVERLAP, ov)
            ctx.set_option(capi.OPT_SIDE_SPLIT, split)
            res[ov, split] = ctx.batch_synth_checksums(21, 3, 5 * 256 - 17, batch=256)
        for k in runs[1:]:
            np.testing.assert_array_equal(res[0, 2], res[k])
    finally:
        ctx.set_options(shipped)


def test_pipelined_layout_switches_are_bitwise_identical(ctx, capi, shipped):
    """Pipelined blocks across layout changes on one context: a 70-pulsar layout (DM on the second side stream, the
    GWB mix adding into red noise), a 12-pulsar one with other coefficient columns, then a 70-pulsar one again. Each
    run of blocks returns the single-stream checksums bit for bit: the two side streams join at every block start,
    so no stream writes coefficient columns or a grid buffer the other, or an earlier layout's block, still reads."""
    def run(ov, split):
        ctx.set_option(capi.OPT_OVERLAP, ov)
        ctx.set_option(capi.OPT_SIDE_SPLIT, split)
        out = []
        for v, P in enumerate((70, 12, 70)):
            ctx.batch_clear()
            _shared_span_layout(ctx, np.random.default_rng(71 + v), P=P, n=(120, 300), nu_const=False)
            ctx.set_option(capi.OPT_SYNTH_PATH, 4)
            out.append(ctx.batch_synth_checksums(5, 3, 3 * 256 - 5, batch=256))
        return out
    try:
        ref = run(0, 2)
        for ov, split in ((1, 1), (1, 0), (1, 2)) if variant_build(capi) else ((1, 2),):
            for a, b in zip(ref, run(ov, split)):
                np.testing.assert_array_equal(a, b)
    finally:
        ctx.batch_clear()
        ctx.set_options(shipped)


@pytest.mark.parametrize("fuse,pgroup", [(0, 16), (1, 1), (1, 3), (1, 16)])
@pytest.mark.parametrize("R", [333, 1024, 1100])
def test_warp_specialised_interpolation_is_bitwise_identical(ctx, capi, shipped, fuse, pgroup, R):
    """FPTA_OPT_INTERP_WS: the warp-specialised interpolation (producer waves fill an LDS ring, compute waves run the
    same MFMA steps and only store) returns the register-pipelined kernel's block and checksums bit for bit, on a
    ragged multi-signal layout with unsorted TOAs, for realization counts that leave compute waves idle (R_pad not a
    multiple of 512), and with the fused partial checksums summed over groups of 1, 3 or 16 chunks
    (FPTA_OPT_PART_GROUP: 23 pulsars' chunks leave a short last group). FPTA_OPT_INTERP_WS 0 / 2 / 3 are variant-build
    options (measured slower): the product library refuses them."""
    if not variant_build(capi):
        for ws in (0, 2, 3):
            assert_variant_refused(ctx, capi, capi.OPT_INTERP_WS, ws)
        return
    rng = np.random.default_rng(43)
    offs, toas, nu = random_layout(rng, 23, (31, 260))
    perm = rng.permutation(offs[1] - offs[0])
    toas[offs[0]:offs[1]] = toas[offs[0]:offs[1]][perm]
    ctx.batch_set_toas(offs, toas, nu)
    f, a = per_psr_signal(rng, offs, toas, 30)
    ctx.batch_add_signal(0, f, a, idx=0.0)
    f, a = per_psr_signal(rng, offs, toas, 100)
    ctx.batch_add_signal(0, f, a, idx=2.0)
    f, a, L, _ = common_signal(rng, offs, toas, 30)
    ctx.batch_add_signal(1, f, a, L=L)
    try:
        ctx.set_option(capi.OPT_SYNTH_PATH, 4)
        ctx.set_option(capi.OPT_FUSE_CHECKSUMS, fuse)
        ctx.set_option(capi.OPT_PART_GROUP, pgroup)
        res = {}
        # 2: WS also for fused-checksum blocks; 3: k_grid_interp_ws2 (two workgroups per CU); 4: k_grid_interp_st
        # (storer waves, diagnostic builds only: one partial row per chunk)
        variants = (1, 2, 3, 4) if _diag_build(capi) and (not fuse or pgroup == 1) else (1, 2, 3)
        for ws in (0,) + variants:
            ctx.set_option(capi.OPT_INTERP_WS, ws)
            res[ws] = (ctx.batch_synth(5, 300, R), ctx.batch_checksums())
        for ws in variants:
            np.testing.assert_array_equal(res[0][0], res[ws][0])
            np.testing.assert_array_equal(res[0][1], res[ws][1])
    finally:
        ctx.set_options(shipped)


@pytest.mark.parametrize("ws", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("R", [1100, 1696])
def test_partial_realization_blocks_write_every_sample(ctx, capi, shipped, ws, R):
    """Regression: R_pad not a multiple of 512 (a C3 shard's last batch of 1696) gives persistent interpolation
    waves tiles of a realization block past R_pad between valid ones. Every sample must be written (the block is
    poisoned with NaN first) and the fused partial checksums must match a full pass over the block; the register
    kernel once exited on its first tile's block (dropping later valid tiles) and let later invalid tiles write
    another chunk's partials."""
    if ws != 1 and not _diag_build(capi):
        pytest.skip("FPTA_OPT_INTERP_WS 0 / 2 / 3 / 4 are variant-build options (make variant DEFS=-DFPTA_DIAG_KERNELS)")
    rng = np.random.default_rng(47)
    offs, toas, nu = random_layout(rng, 40, (300, 900))
    ctx.batch_set_toas(offs, toas, nu)
    f, a, L, _ = common_signal(rng, offs, toas, 30)
    ctx.batch_add_signal(1, f, a, L=L)
    segs = [O.Segment(1, 2 * np.pi * f, a, 0.0, L=L)]
    try:
        ctx.set_option(capi.OPT_SYNTH_PATH, 4)
        ctx.set_option(capi.OPT_INTERP_WS, ws)
        ctx.set_option(capi.OPT_FUSE_CHECKSUMS, 1)
        ctx.batch_synth(9, 0, R, to_host=False)
        ctx.debug_fill_out(np.nan)
        got = ctx.batch_synth(9, 64, R)
        sums = ctx.batch_checksums()
        assert np.all(np.isfinite(got))
        want = O.batch_synth(offs, toas, nu, segs, 9, 64, R)
        assert rel_err(got, want) <= GRID_TOL
        np.testing.assert_allclose(sums[:, 0], got.sum(axis=1), rtol=1e-10, atol=1e-12 * np.abs(got).max())
        np.testing.assert_allclose(sums[:, 1], (got * got).sum(axis=1), rtol=1e-10)
    finally:
        ctx.set_options(shipped)


@pytest.mark.parametrize("fuse", [0, 1])
@pytest.mark.parametrize("R,real0", [(128, 5), (256, 8), (333, 5), (1100, 8)])
def test_storer_interpolation_white_ecorr_is_bitwise_identical(ctx, capi, shipped, fuse, R, real0):
    """FPTA_OPT_INTERP_WS 4 (k_grid_interp_st: compute waves hand their sums to storer waves through LDS; the storers
    add white noise and ECORR, store, and reduce the partial checksums) returns the register kernel's block and
    checksums bit for bit with the white / ECORR epilogue, on a ragged layout whose pulsars start at odd TOA offsets
    (the misaligned white-noise words), at odd and even first realizations (the one-normal-per-call path), for
    realization counts whose last tile holds fewer than four units; and the block matches the oracle
    (/root/reference/fakepta/fake_pta.py:201-230). A diagnostic kernel (measured, not adopted): the product library
    refuses the option."""
    if not _diag_build(capi):
        _assert_refused(ctx, capi, 4)
        return
    rng = np.random.default_rng(59)
    offs, toas, nu = random_layout(rng, 9, (31, 180))
    ctx.batch_set_toas(offs, toas, nu)
    f, a = per_psr_signal(rng, offs, toas, 30)
    ctx.batch_add_signal(0, f, a, idx=0.0)
    f2, a2 = per_psr_signal(rng, offs, toas, 60)
    ctx.batch_add_signal(0, f2, a2, idx=2.0)
    sigma = rng.uniform(1e-7, 1e-6, offs[-1])
    blocks = [np.arange(s, min(s + 3, offs[-1])) for s in range(0, offs[-1], 5)]
    es = rng.uniform(1e-8, 1e-7, len(blocks))
    ctx.batch_set_white(sigma, blocks, es)
    try:
        ctx.set_option(capi.OPT_SYNTH_PATH, 4)
        ctx.set_option(capi.OPT_FUSE_CHECKSUMS, fuse)
        ctx.set_option(capi.OPT_PART_GROUP, 1)  # the diagnostic kernels write one partial row per chunk
        res = {}
        for ws in (0, 4):
            ctx.set_option(capi.OPT_INTERP_WS, ws)
            ctx.batch_synth(13, 0, R, to_host=False)
            ctx.debug_fill_out(np.nan)
            res[ws] = (ctx.batch_synth(13, real0, R), ctx.batch_checksums())
        for key in (4,):
            assert np.all(np.isfinite(res[key][0]))
            np.testing.assert_array_equal(res[0][0], res[key][0])
            np.testing.assert_array_equal(res[0][1], res[key][1])
        block_of = -np.ones(offs[-1], dtype=np.int64)
        for b, q in enumerate(blocks):
            block_of[q] = b
        segs = [O.Segment(0, 2 * np.pi * f, a, 0.0), O.Segment(0, 2 * np.pi * f2, a2, 2.0)]
        want = O.batch_synth(offs, toas, nu, segs, 13, real0, R, sigma=sigma, block_of=block_of, ecorr_sigma=es)
        assert_parity(res[4][0], want, TOL)
    finally:
        ctx.batch_set_white()
        ctx.set_options(shipped)


@pytest.mark.parametrize("fuse", [0, 1])
@pytest.mark.parametrize("layout,R", [("two", 333), ("two", 1024), ("one", 1100), ("shared", 256)])
def test_union_interpolation_is_bitwise_identical(ctx, capi, shipped, fuse, layout, R):
    """FPTA_OPT_INTERP_WS 5 (k_grid_interp_u: the union of 4 consecutive chunks' band rows staged once in LDS, weights
    made on the fly by the weight tables' own expression) returns the register kernel's block and checksums bit for
    bit: two grid signals (red noise + DM at several radio frequencies, one pulsar with unsorted TOAs), one signal
    (a common GWB, C3-like, ragged pulsars: partial chunks and groups), and the coalesced C2-like layout; realization
    counts off the 512 tile; every sample written (NaN-poisoned block). The kernel must be the one that ran. A
    diagnostic kernel (measured, not adopted): the product library refuses the option."""
    if not _diag_build(capi):
        _assert_refused(ctx, capi, 5)
        return
    rng = np.random.default_rng(67)
    if layout == "shared":
        _shared_span_layout(ctx, rng, nu_const=False)
    else:
        offs, toas, nu = random_layout(rng, 11, (31, 400))
        if layout == "two":
            perm = rng.permutation(offs[1] - offs[0])
            toas[offs[0]:offs[1]] = toas[offs[0]:offs[1]][perm]
        ctx.batch_set_toas(offs, toas, nu)
        if layout == "two":
            for nm, idx in ((30, 0.0), (100, 2.0)):
                f, a = per_psr_signal(rng, offs, toas, nm)
                ctx.batch_add_signal(0, f, a, idx=idx)
        else:
            f, a, L, _ = common_signal(rng, offs, toas, 30)
            ctx.batch_add_signal(1, f, a, L=L)
    try:
        ctx.set_option(capi.OPT_SYNTH_PATH, 4)
        ctx.set_option(capi.OPT_FUSE_CHECKSUMS, fuse)
        ctx.set_option(capi.OPT_PART_GROUP, 1)  # the diagnostic kernels write one partial row per chunk
        res = {}
        for ws in (0, 5):
            ctx.set_option(capi.OPT_INTERP_WS, ws)
            ctx.batch_synth(7, 0, R, to_host=False)
            ctx.debug_fill_out(np.nan)
            res[ws] = (ctx.batch_synth(7, 64, R), ctx.batch_checksums())
            if ws == 5:
                assert ctx.batch_grid_info()["interp_kernel"] == f"k_grid_interp_u<{'true' if fuse else 'false'}>"
        assert np.all(np.isfinite(res[5][0]))
        np.testing.assert_array_equal(res[0][0], res[5][0])
        np.testing.assert_array_equal(res[0][1], res[5][1])
    finally:
        ctx.set_options(shipped)


@pytest.mark.parametrize("layout", ["coalesced", "dm_only", "masked", "many_modes"])
def test_dft_gen_matches_buffered_draws(ctx, capi, shipped, layout):
    """k_grid_dft_gen (FPTA_OPT_DFT_GEN 1) draws the per-pulsar members' coefficients with k_gen's counters and sums
    a grid signal's terms in the merge order (anchor, then the others; products rounded first): its blocks equal
    the buffered path's (k_gen -> coefficient buffer -> k_coef_merge / mix epilogue -> k_grid_dft_mfma) bit for
    bit, pipelined or not, over realization counts off every tile multiple; and they match the oracle. The buffered
    path (FPTA_OPT_DFT_GEN 0) is a variant-build option: the product library runs the oracle half only."""
    rng = np.random.default_rng(zlib_crc(layout))
    if layout in ("coalesced", "masked"):
        offs, toas, nu, segs = _shared_span_layout(ctx, rng, nu_const=False, with_masked=layout == "masked")
    elif layout == "dm_only":
        offs, toas, nu, segs = _flat_layout(ctx, rng, P=9, n_modes=100)
    else:  # 257 modes: seven 32-row chunks of the quarter range, several per wave
        offs, toas, nu, segs = _flat_layout(ctx, rng, P=3, n_modes=257)
    try:
        ctx.set_option(capi.OPT_SYNTH_PATH, 4)
        for R, real0 in ((150, 5), (333, 1000), (16, 7)):
            res = {}
            for gen in (0, 1) if variant_build(capi) else (1,):
                ctx.set_option(capi.OPT_DFT_GEN, gen)
                for ov in (0, 1):
                    ctx.set_option(capi.OPT_OVERLAP, ov)
                    res[gen, ov] = ctx.batch_synth(13, real0, R)
            for k in res:
                np.testing.assert_array_equal(res[k], res[1, 0])
            want = O.batch_synth(offs, toas, nu, segs, 13, real0, R)
            assert_parity(res[1, 1], want, TOL)
    finally:
        ctx.set_options(shipped)


def zlib_crc(s):
    import zlib
    return zlib.crc32(s.encode())


@pytest.mark.parametrize("factor", ["cholesky", "svd", "dipole_rank3"])
def test_gen_mix_matches_two_kernels(ctx, capi, shipped, factor):
    """k_gen_mix (FPTA_OPT_GEN_MIX 1, 2 and 3) draws a common signal's normals into LDS and mixes them on fp64 MFMA in one
    kernel: same counters, same products in the same k-step order as k_gen + k_mix_mfma, so blocks are bit-identical
    on the gridded (with and without k_grid_dft_gen) and exact paths, for a triangular (Cholesky) and a dense (SVD)
    ORF factor and the batch path's rank-3 factor of the singular dipole ORF (columns past the third exactly zero:
    both kernels mix, and k_gen_mix draws, only those three), 70 and 160 pulsars (two and three 64-pulsar tiles).
    GEN_MIX 0 / 1 / 3 and DFT_GEN 0 are variant-build options: the product library runs the shipped kernels against
    the oracle only."""
    variant = variant_build(capi)
    from fakepta_amd.batch import batch_factor
    rng = np.random.default_rng({"cholesky": 71, "svd": 72}.get(factor, 73))
    for P in (70, 160):
        offs, toas, nu = random_layout(rng, P, (40, 120))
        ctx.batch_set_toas(offs, toas, nu)
        f, a = per_psr_signal(rng, offs, toas, 20)
        ctx.batch_add_signal(0, f, a)
        fc, ac, _, pos = common_signal(rng, offs, toas, 30)
        gam = O.orf_hd(pos) if factor != "dipole_rank3" else O.orf_dipole(pos)
        L = np.linalg.cholesky(gam) if factor == "cholesky" else (O.mvn_factor(gam) if factor == "svd" else
                                                                   batch_factor(gam))
        if factor == "dipole_rank3":
            assert np.all(L[:, 3:] == 0) and np.any(L[:, 2] != 0)
        ctx.batch_add_signal(1, fc, ac, L=L)
        segs = [O.Segment(0, 2 * np.pi * f, a, 0.0), O.Segment(1, 2 * np.pi * fc, ac, 0.0, L=L)]
        try:
            for path, dft_gen in ((4, 1), (4, 0), (3, 0), (2, 0)) if variant else ((4, 1), (3, 1), (2, 1)):
                ctx.set_option(capi.OPT_SYNTH_PATH, path)
                ctx.set_option(capi.OPT_DFT_GEN, dft_gen)
                res = {}
                # 2: k_gen_mix with 16-realization waves (twice the waves per workgroup); 3: and 16-realization
                # workgroups
                for gm in (0, 1, 2, 3) if variant else (2,):
                    ctx.set_option(capi.OPT_GEN_MIX, gm)
                    res[gm] = ctx.batch_synth(17, 40, 300)
                for gm in res:
                    np.testing.assert_array_equal(res[2], res[gm])
                assert_parity(res[2], O.batch_synth(offs, toas, nu, segs, 17, 40, 300), TOL)
        finally:
            ctx.set_options(shipped)


@pytest.mark.parametrize("case", ["common", "common_short", "per_psr", "modes40"])
@pytest.mark.parametrize("fuse,pgroup", [(0, 16), (1, 1), (1, 16)])
@pytest.mark.parametrize("R", [333, 1100])
def test_psr_interpolation_is_bitwise_identical(ctx, capi, shipped, case, fuse, pgroup, R):
    """FPTA_OPT_INTERP_PSR (k_grid_interp_psr: a workgroup makes one pulsar's grid for 64 realizations in LDS with
    k_grid_dft_mfma's MFMA steps and butterfly, then interpolates the pulsar's chunks from it) returns the two-kernel
    path's block and partial checksums bit for bit: a common 30-mode GWB on ragged pulsars (C3-like; one pulsar of a
    single short chunk in "common_short"), a per-pulsar red noise drawn into the coefficient buffer (FPTA_OPT_DFT_GEN
    0), and 40 modes (nf = 124, the largest one-block grid); partial rows of 1 and 16 chunks; every sample written
    (NaN-poisoned block); the kernel that ran is the per-pulsar one."""
    if case == "per_psr" and not variant_build(capi):
        pytest.skip("a per-pulsar signal drawn into the coefficient buffer: FPTA_OPT_DFT_GEN 0, a variant-build option")
    rng = np.random.default_rng(83 + len(case))
    # dense TOAs (bands of <= 32 rows: a 32-TOA chunk spans a few grid cells), ragged counts
    offs, toas, nu = random_layout(rng, 13, (700, 2100))
    if case == "common_short":  # plus a pulsar of 5 TOAs within a day: one short chunk
        offs = np.append(offs, offs[-1] + 5)
        toas = np.concatenate([toas, 2e8 + np.sort(rng.uniform(0, 86400.0, 5))])
        nu = np.concatenate([nu, np.full(5, 1400.0)])
    ctx.batch_set_toas(offs, toas, nu)
    if case == "per_psr":
        f, a = per_psr_signal(rng, offs, toas, 30)
        ctx.batch_add_signal(0, f, a, idx=0.0)
    else:
        f, a, L, _ = common_signal(rng, offs, toas, 40 if case == "modes40" else 30)
        ctx.batch_add_signal(1, f, a, L=L)
    try:
        ctx.set_option(capi.OPT_SYNTH_PATH, 4)
        ctx.set_option(capi.OPT_DFT_GEN, 0 if case == "per_psr" else 1)
        ctx.set_option(capi.OPT_FUSE_CHECKSUMS, fuse)
        ctx.set_option(capi.OPT_PART_GROUP, pgroup)
        res = {}
        for psr in (0, 1):
            ctx.set_option(capi.OPT_INTERP_PSR, psr)
            ctx.batch_synth(7, 0, R, to_host=False)
            ctx.debug_fill_out(np.nan)
            res[psr] = (ctx.batch_synth(7, 64, R), ctx.batch_checksums())
            name = ctx.batch_grid_info()["interp_kernel"]
            assert name.startswith("k_grid_interp_psr") == bool(psr), name
        assert np.all(np.isfinite(res[1][0]))
        np.testing.assert_array_equal(res[0][0], res[1][0])
        np.testing.assert_array_equal(res[0][1], res[1][1])
    finally:
        ctx.set_options(shipped)


def test_psr_interpolation_not_taken_outside_its_layouts(ctx, capi, shipped):
    """k_grid_interp_psr serves one grid signal of <= 124 grid points without fused white noise: 60 modes (nf > 124),
    two grid signals and a white-noise block take the other kernels."""
    rng = np.random.default_rng(89)
    offs, toas, nu = random_layout(rng, 12, (100, 300))
    try:
        ctx.set_option(capi.OPT_SYNTH_PATH, 4)
        for case in ("modes60", "two", "white"):
            ctx.batch_clear()
            ctx.batch_set_toas(offs, toas, nu)
            f, a, L, _ = common_signal(rng, offs, toas, 60 if case == "modes60" else 30)
            ctx.batch_add_signal(1, f, a, L=L)
            if case == "two":
                f2, a2 = per_psr_signal(rng, offs, toas, 100)
                ctx.batch_add_signal(0, f2, a2, idx=2.0)
            if case == "white":
                ctx.batch_set_white(np.full(offs[-1], 1e-7), [], [])
            ctx.batch_synth(3, 0, 256, to_host=False)
            assert not ctx.batch_grid_info()["interp_kernel"].startswith("k_grid_interp_psr"), case
            ctx.batch_set_white()
    finally:
        ctx.batch_clear()
        ctx.set_options(shipped)


@pytest.mark.parametrize("fuse", [0, 1])
def test_psr_pipelined_batches_are_bitwise_identical(ctx, capi, shipped, fuse):
    """Pipelined per-pulsar blocks (two coefficient buffers: block b + 1 draws into one while block b's interpolation
    reads the other): the checksums of 7 back-to-back blocks equal the single-stream and the two-kernel ones bit for
    bit, and so do they when the layout switches between a per-pulsar and a two-signal plan on one context."""
    rng = np.random.default_rng(97)
    offs, toas, nu = random_layout(rng, 30, (600, 1500))
    f, a, L, _ = common_signal(rng, offs, toas, 30)
    f2, a2 = per_psr_signal(rng, offs, toas, 100)

    def layout(two):
        ctx.batch_clear()
        ctx.batch_set_toas(offs, toas, nu)
        ctx.batch_add_signal(1, f, a, L=L)
        if two:
            ctx.batch_add_signal(0, f2, a2, idx=2.0)
        ctx.set_option(capi.OPT_SYNTH_PATH, 4)

    try:
        ctx.set_option(capi.OPT_FUSE_CHECKSUMS, fuse)
        res = {}
        for psr, ov in ((0, 0), (1, 0), (1, 1), (0, 1)):
            ctx.set_option(capi.OPT_INTERP_PSR, psr)
            ctx.set_option(capi.OPT_OVERLAP, ov)
            out = []
            for two in (False, True, False):
                layout(two)
                out.append(ctx.batch_synth_checksums(13, 5, 7 * 256 - 3, batch=256))
            res[psr, ov] = out
        for key in ((1, 0), (1, 1), (0, 1)):
            for x, y in zip(res[0, 0], res[key]):
                np.testing.assert_array_equal(x, y)
    finally:
        ctx.batch_clear()
        ctx.set_options(shipped)


@pytest.mark.parametrize("layout", ["shared", "two_unsorted", "dense"])
@pytest.mark.parametrize("R", [256, 1024, 1100])
def test_window_ring_interpolation_is_bitwise_identical(ctx, capi, shipped, layout, R):
    """FPTA_OPT_INTERP_WR (k_grid_interp_wr: each grid signal's band rows kept in a ring of LDS rows across consecutive
    chunks, only the rows the previous chunk did not hold loaded) returns the warp-specialised kernel's block bit for
    bit: the coalesced C2-like two-signal layout, two signals on ragged pulsars with one pulsar's TOAs in two sorted
    runs, the later first (the bands jump: a fresh chunk inside a pulsar), dense TOAs; every sample written
    (NaN-poisoned block). R_pad not a multiple of 256 (R = 1100) takes the other kernels. A diagnostic kernel
    (measured slower, not adopted): the product library refuses the option."""
    if not _diag_build(capi):
        with pytest.raises(capi.FptaError, match="diagnostic"):
            ctx.set_option(capi.OPT_INTERP_WR, 1)
        assert ctx.get_option(capi.OPT_INTERP_WR) == 0
        return
    rng = np.random.default_rng(101 + len(layout))
    if layout == "shared":
        _shared_span_layout(ctx, rng, n=(1500, 2400), nu_const=False)
    else:
        offs, toas, nu = random_layout(rng, 17, (2000, 2400))  # bands of <= 40 rows over both signals
        if layout == "two_unsorted":  # one pulsar's TOAs as two sorted runs, the later half first: the bands jump
            k = (offs[2] - offs[1]) // 2
            toas[offs[1]:offs[2]] = np.roll(toas[offs[1]:offs[2]], k)
        ctx.batch_set_toas(offs, toas, nu)
        for nm, idx in ((30, 0.0), (100, 2.0)):
            f, a = per_psr_signal(rng, offs, toas, nm)
            ctx.batch_add_signal(0, f, a, idx=idx)
    try:
        ctx.set_option(capi.OPT_SYNTH_PATH, 4)
        res = {}
        for wr in (0, 1):
            ctx.set_option(capi.OPT_INTERP_WR, wr)
            ctx.batch_synth(3, 0, R, to_host=False)
            ctx.debug_fill_out(np.nan)
            res[wr] = ctx.batch_synth(3, 32, R)
            name = ctx.batch_grid_info()["interp_kernel"]
            assert (name == "k_grid_interp_wr") == (wr == 1 and R % 256 == 0), name
        assert np.all(np.isfinite(res[1]))
        np.testing.assert_array_equal(res[0], res[1])
    finally:
        ctx.set_options(shipped)
