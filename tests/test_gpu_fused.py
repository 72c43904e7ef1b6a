"""k_grid_fused (FPTA_OPT_INTERP_FUSED): the whole gridded synthesis of one pulsar x 32 realizations in one workgroup
(coefficient draws, every grid signal's quarter-range DFT into LDS, the interpolation from LDS), against the two-kernel
path it replaces (k_grid_dft_gen / k_grid_dft_mfma + k_grid_interp_ws) bit for bit, and against the oracle.

Half-chunk bands (FPTA_OPT_INTERP_FUSED 1 where they pay, 3 forced: TOAs 0..15 and 16..31 of a chunk each on their
own band rows) are NOT bit-identical to the two-kernel path: a half's band starts at another row, so its 4-row MFMA
k-steps group the products differently and the sums differ by rounding. They are checked against the oracle at the
path's tolerance and against whole-chunk bands (option 2) at HALF_TOL, far below it.

Reference loops the kernel evaluates: /root/reference/fakepta/fake_pta.py:372-387 (per-pulsar coefficients and
F @ c) and correlated_noises.py:153-160 (the ORF-mixed common signal).
"""
import numpy as np
import pytest

from oracle import fakepta_oracle as O
from tests.conftest import assert_parity, rel_err
from tests.helpers import common_signal, per_psr_signal, random_layout, variant_build
from tests.test_gpu_grid import GRID_TOL, TOL, _flat_layout, _shared_span_layout

pytestmark = pytest.mark.gpu

# half-chunk vs whole-chunk bands: the same products summed in other groups (rounding only)
HALF_TOL = 1e-12


@pytest.fixture(scope="module")
def capi():
    from fakepta_amd import _capi
    return _capi


@pytest.fixture(scope="module")
def ctx(capi):
    c = capi.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def shipped(ctx, capi):
    opts = ctx.options()
    assert opts[capi.OPT_INTERP_FUSED] == 1
    return opts


def _c2_like(ctx, rng, P=23, n=(31, 700), unsorted=True):
    """C2's signal mix on ragged pulsars over one common span T (make_fake_array with equal Tobs): RN30 (idx 0), DM100
    (idx 2, three radio bands) and the HD GWB30 on f_k = k / T, so RN and the GWB coalesce into one grid signal (two grid
    signals, four 32-row DFT chunks); a pulsar of 31 TOAs (wide bands) and one pulsar's TOAs unsorted (bands jump)."""
    counts = rng.integers(n[0], n[1], size=P)
    counts[1] = 31
    offs = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    t0, t1 = 4.4e9, 4.4e9 + 3.15e8
    toas = np.concatenate([np.concatenate([[t0], np.sort(rng.uniform(t0, t1, k - 2)), [t1]]) for k in counts])
    if unsorted:
        perm = rng.permutation(offs[1] - offs[0])
        toas[offs[0]:offs[1]] = toas[offs[0]:offs[1]][perm]
    nu = rng.choice([800.0, 1400.0, 2500.0], size=offs[-1])
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
    return offs, toas, nu, segs


def _layout(ctx, rng, layout):
    if layout == "c2_like":
        return _c2_like(ctx, rng)
    if layout == "coalesced":
        return _shared_span_layout(ctx, rng, nu_const=False)
    if layout == "one_grid":  # RN + DM + GWB at one radio frequency: a single coalesced grid signal
        return _shared_span_layout(ctx, rng, nu_const=True)
    if layout == "dm_only":
        return _flat_layout(ctx, rng, P=9, n_modes=100)
    raise ValueError(layout)


def _run(ctx, capi, fused, seed, real0, R):
    ctx.set_option(capi.OPT_INTERP_FUSED, fused)
    ctx.batch_synth(seed, 0, R, to_host=False)
    ctx.debug_fill_out(np.nan)
    out = ctx.batch_synth(seed, real0, R)
    return out, ctx.batch_grid_info()["interp_kernel"]


@pytest.mark.parametrize("layout", ["c2_like", "coalesced", "one_grid", "dm_only"])
@pytest.mark.parametrize("dft_gen", [1, 0])
def test_fused_synthesis_is_bitwise_identical(ctx, capi, shipped, layout, dft_gen):
    """The fused kernel returns the two-kernel path's block bit for bit: draws inside the kernel (FPTA_OPT_DFT_GEN 1:
    k_grid_dft_gen's terms) or from the merged coefficient buffer (0: k_grid_dft_mfma's operand), one or two grid
    signals (one to four DFT waves with a job), realization counts off every tile multiple and odd first realizations (the
    Philox pair boundary), every sample written (NaN-poisoned block); the kernel that ran is the fused one. And the
    block matches the oracle."""
    if dft_gen == 0 and not variant_build(capi):
        pytest.skip("FPTA_OPT_DFT_GEN 0 is a variant-build option")
    rng = np.random.default_rng(211 + len(layout))
    offs, toas, nu, segs = _layout(ctx, rng, layout)
    try:
        ctx.set_option(capi.OPT_SYNTH_PATH, 4)
        ctx.set_option(capi.OPT_DFT_GEN, dft_gen)
        for R, real0 in ((333, 5), (1024, 0), (1100, 77), (16, 3)):
            ref, k0 = _run(ctx, capi, 0, 13, real0, R)
            got, k1 = _run(ctx, capi, 2, 13, real0, R)
            assert k1.startswith("k_grid_fused") and k1.endswith(", false>"), k1
            assert not k0.startswith("k_grid_fused"), k0
            assert np.all(np.isfinite(got))
            np.testing.assert_array_equal(ref, got)
            half, k3 = _run(ctx, capi, 3, 13, real0, R)  # half-chunk bands: rounding-level differences only
            assert k3.startswith("k_grid_fused") and k3.endswith(", true>"), k3
            assert np.all(np.isfinite(half))
            assert rel_err(half, got) <= HALF_TOL
            if R == 333:
                want = O.batch_synth(offs, toas, nu, segs, 13, real0, R)
                for blk in (got, half):
                    assert rel_err(blk, want) <= GRID_TOL
                    assert_parity(blk, want, TOL)
    finally:
        ctx.batch_clear()
        ctx.set_options(shipped)


@pytest.mark.parametrize("R,real0", [(256, 0), (333, 7), (64, 32)])
def test_fused_dft_waves_join_long_pulsars(ctx, capi, shipped, R, real0):
    """C4's shape at small scale: one 100-mode common (ORF-mixed) signal, so the DFT waves only load their terms, and
    pulsars of thousands of TOAs (hundreds of chunks per item): the DFT waves take chunk tickets of the item being
    interpolated before they build the next one (FusedArgs.join_reserve), beside the interpolation waves. Ragged
    pulsars (one short: an item whose chunks all go to the interpolation waves), the block bit-identical to the
    two-kernel path and every sample written; and the oracle."""
    rng = np.random.default_rng(229)
    counts = np.array([6000, 4100, 90, 5200])
    offs = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    t0, t1 = 4.4e9, 4.4e9 + 3.15e8
    toas = np.concatenate([np.concatenate([[t0], np.sort(rng.uniform(t0, t1, k - 2)), [t1]]) for k in counts])
    nu = np.full(offs[-1], 1400.0)
    ctx.batch_set_toas(offs, toas, nu)
    f, a, L, _ = common_signal(rng, offs, toas, 100)
    ctx.batch_add_signal(1, f, a, L=L)
    segs = [O.Segment(1, 2 * np.pi * f, a, 0.0, L=L)]
    try:
        ctx.set_option(capi.OPT_SYNTH_PATH, 4)
        ref, k0 = _run(ctx, capi, 0, 31, real0, R)
        got, k1 = _run(ctx, capi, 2, 31, real0, R)
        assert k1.startswith("k_grid_fused"), k1
        assert np.all(np.isfinite(got))
        np.testing.assert_array_equal(ref, got)
        half, k3 = _run(ctx, capi, 3, 31, real0, R)
        assert k3.endswith(", true>"), k3
        assert np.all(np.isfinite(half))
        assert rel_err(half, got) <= HALF_TOL
        want = O.batch_synth(offs, toas, nu, segs, 31, real0, R)
        for blk in (got, half):
            assert rel_err(blk, want) <= GRID_TOL
            assert_parity(blk, want, TOL)
    finally:
        ctx.batch_clear()
        ctx.set_options(shipped)


@pytest.mark.parametrize("seed", range(12))
def test_fused_randomized_layouts(ctx, capi, shipped, seed):
    """Random layouts on a common span (so the fused kernel serves them): 1 to 40 pulsars of 1 to 3000 TOAs (one-TOA
    pulsars included: items of a single short chunk), red noise of 1 to 40 modes, DM of 10 to 100, with or without a
    common GWB, realization counts and first realizations off every tile and parity. The block equals the two-kernel
    path's bit for bit and every sample is written (NaN-poisoned block); item queues, chunk tickets and the DFT waves'
    join are exercised with whatever shapes come."""
    rng = np.random.default_rng(1000 + seed)
    P = int(rng.integers(1, 41))
    counts = rng.integers(1, 3001, size=P)
    counts[rng.integers(0, P)] = 1
    offs = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    t0, t1 = 4.4e9, 4.4e9 + 3.15e8
    toas = np.concatenate([np.sort(rng.uniform(t0, t1, k)) if k < 3 else
                           np.concatenate([[t0], np.sort(rng.uniform(t0, t1, k - 2)), [t1]]) for k in counts])
    nu = rng.choice([800.0, 1400.0, 2500.0], size=offs[-1])
    T = t1 - t0
    ctx.batch_set_toas(offs, toas, nu)
    for nm, idx in ((int(rng.integers(1, 41)), 0.0), (int(rng.integers(10, 101)), 2.0)):
        f = np.tile(np.arange(1, nm + 1) / T, (P, 1))
        a = np.sqrt(O.powerlaw(f, rng.uniform(-14.5, -13.5, (P, 1)), 3.0) / T)
        ctx.batch_add_signal(0, f, a, idx=idx)
    if P >= 2 and rng.random() < 0.7:
        nc = int(rng.integers(1, 31))
        fc = np.arange(1, nc + 1) / T
        v = rng.normal(size=(P, 3))
        ctx.batch_add_signal(1, fc, np.sqrt(O.powerlaw(fc, -14.0, 13 / 3) / T),
                             L=O.mvn_factor(O.orf_hd(v / np.linalg.norm(v, axis=1)[:, None])))
    R, real0 = int(rng.integers(16, 701)), int(rng.integers(0, 5000))
    try:
        ctx.set_option(capi.OPT_SYNTH_PATH, 4)
        ref, k0 = _run(ctx, capi, 0, 41 + seed, real0, R)
        got, k1 = _run(ctx, capi, 2, 41 + seed, real0, R)
        assert np.all(np.isfinite(got))
        np.testing.assert_array_equal(ref, got)
        half, k3 = _run(ctx, capi, 3, 41 + seed, real0, R)
        assert np.all(np.isfinite(half))
        print(f"layout {seed}: P {P}, {offs[-1]} TOAs, R {R}, real0 {real0}: {k1} / {k3} (two-kernel {k0})")
        if not k1.startswith("k_grid_fused"):  # a layout the fused kernel does not serve (e.g. a grid over LDS)
            assert k1 == k0 == k3, (k0, k1, k3)
            np.testing.assert_array_equal(ref, half)
        else:
            assert k3.endswith(", true>"), k3
            assert rel_err(half, got) <= HALF_TOL
    finally:
        ctx.batch_clear()
        ctx.set_options(shipped)


def test_fused_pipelined_blocks(ctx, capi, shipped):
    """Pipelined blocks (FPTA_OPT_OVERLAP 1) on the fused kernel: the next block's common draws go into the other
    coefficient buffer on the side stream while this block's kernel reads its own. Blocks queued back to back without a
    host round trip: the last block equals its one-stream run bit for bit; so does every block of a run of synth calls
    that each read their block back, and the per-block checksums."""
    rng = np.random.default_rng(223)
    _c2_like(ctx, rng, P=40, n=(200, 900), unsorted=False)
    try:
        ctx.set_option(capi.OPT_SYNTH_PATH, 4)
        res = {}
        for ov in (0, 1):
            ctx.set_option(capi.OPT_OVERLAP, ov)
            for b in range(4):
                ctx.batch_synth(29, 256 * b, 256, to_host=False)
            res[ov, "last"] = ctx.batch_synth(29, 256 * 4, 256)
            assert ctx.batch_grid_info()["interp_kernel"].startswith("k_grid_fused")
            res[ov, "each"] = [(ctx.batch_synth(29, 300 * b + 1, 300), ctx.batch_checksums()) for b in range(3)]
        np.testing.assert_array_equal(res[0, "last"], res[1, "last"])
        for (x, xs), (y, ys) in zip(res[0, "each"], res[1, "each"]):
            np.testing.assert_array_equal(x, y)
            np.testing.assert_array_equal(xs, ys)
    finally:
        ctx.batch_clear()
        ctx.set_options(shipped)


def test_fused_not_taken_outside_its_blocks(ctx, capi, shipped):
    """Blocks k_grid_fused does not serve take the two-kernel path: white / ECORR epilogue, fused partial checksums
    (streamed jobs), three grid signals (a masked backend signal), grids too large for LDS (600 modes: 1,804 grid
    rows), and FPTA_OPT_INTERP_FUSED 0 (k_grid_fused_w, which could take the first and third, is opt-in:
    FPTA_OPT_FUSED_WHITE, tests/test_gpu_fused_w.py)."""
    rng = np.random.default_rng(227)
    try:
        offs, toas, nu, segs = _c2_like(ctx, rng, P=12, n=(100, 300))
        ctx.set_option(capi.OPT_SYNTH_PATH, 4)
        ctx.batch_synth(3, 0, 256, to_host=False)
        assert ctx.batch_grid_info()["interp_kernel"].startswith("k_grid_fused")
        ctx.batch_set_white(np.full(offs[-1], 1e-7), [], [])
        ctx.batch_synth(3, 0, 256, to_host=False)
        assert not ctx.batch_grid_info()["interp_kernel"].startswith("k_grid_fused")
        ctx.batch_set_white()
        ctx.set_option(capi.OPT_FUSE_CHECKSUMS, 1)
        ctx.batch_synth(3, 0, 256, to_host=False)
        assert not ctx.batch_grid_info()["interp_kernel"].startswith("k_grid_fused")
        ctx.set_option(capi.OPT_FUSE_CHECKSUMS, 0)
        ctx.set_option(capi.OPT_INTERP_FUSED, 0)
        ctx.batch_synth(3, 0, 256, to_host=False)
        assert not ctx.batch_grid_info()["interp_kernel"].startswith("k_grid_fused")
        for build in (lambda: _shared_span_layout(ctx, rng, nu_const=False, with_masked=True),
                      lambda: _flat_layout(ctx, rng, P=3, n_modes=600)):
            ctx.set_options(shipped)
            ctx.batch_clear()
            build()
            ctx.set_option(capi.OPT_SYNTH_PATH, 4)
            ctx.batch_synth(3, 0, 256, to_host=False)
            k = ctx.batch_grid_info()["interp_kernel"]
            assert not k.startswith("k_grid_fused"), k
    finally:
        ctx.batch_set_white()
        ctx.batch_clear()
        ctx.set_options(shipped)


def test_fused_launch_timing_events(ctx, capi, shipped):
    """With profiling on, the fused launch and k_gen_mix take their timing events as the dispatch's own start / stop
    (hipExtLaunchKernel): one K_SYNTH and one K_MIX record per block, each a positive duration shorter than the block's
    wall time; with profiling off, no record and the same block bit for bit."""
    import time
    rng = np.random.default_rng(97)
    _c2_like(ctx, rng, P=70, n=(200, 400), unsorted=False)  # 70 pulsars: the HD mix on k_gen_mix (64 <= P <= 256)
    try:
        ctx.set_option(capi.OPT_SYNTH_PATH, 4)
        ref = ctx.batch_synth(5, 0, 256)
        assert ctx.batch_grid_info()["interp_kernel"].startswith("k_grid_fused")
        ctx.set_option(capi.OPT_PROFILE, 1)
        ctx.reset_stats()
        n_blocks = 3
        t0 = time.perf_counter()
        for _ in range(n_blocks):
            got = ctx.batch_synth(5, 0, 256)
        wall_ms = (time.perf_counter() - t0) * 1e3
        np.testing.assert_array_equal(ref, got)
        for which in (capi.K_SYNTH, capi.K_MIX):
            n, ms = ctx.kernel_stats(which)
            assert n == n_blocks, (which, n)
            assert 0.0 < ms < wall_ms, (which, ms, wall_ms)
        ctx.set_option(capi.OPT_PROFILE, 0)
        ctx.reset_stats()
        np.testing.assert_array_equal(ref, ctx.batch_synth(5, 0, 256))
        assert ctx.kernel_stats(capi.K_SYNTH)[0] == 0
    finally:
        ctx.set_option(capi.OPT_PROFILE, 0)
        ctx.batch_clear()
        ctx.set_options(shipped)
