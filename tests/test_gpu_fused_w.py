"""k_grid_fused_w (FPTA_OPT_FUSED_WHITE 1, opt-in: measured slower than the two-kernel path on C5): the
fused gridded synthesis for white / ECORR blocks and three-grid-signal blocks (C5's shape:
RN + HD / monopole / dipole common signals in one grid signal, DM and Sv in two more, white noise + 2-TOA ECORR
epochs), pulsar x 16 realizations per item, against the two-kernel white path it replaces (k_grid_dft_gen +
k_grid_interp_mfma<true, ..>, FPTA_OPT_INTERP_FUSED 0) and against the oracle.

The kernel sums a chunk's band steps in two chains (even and odd steps) and adds them, so its GP sums differ from the
two-kernel path's by rounding (checked at W_TOL); the white and ECORR terms are the same operations on the same normals.

Reference loops: /root/reference/fakepta/fake_pta.py:201-253 (white / ECORR), 372-387 (per-pulsar GP),
correlated_noises.py:153-160 (ORF-mixed common signals).
"""
import numpy as np
import pytest

from oracle import fakepta_oracle as O
from tests.conftest import assert_parity, rel_err
from tests.test_gpu_grid import GRID_TOL, TOL

pytestmark = pytest.mark.gpu

W_TOL = 1e-12  # the same products summed in two chains instead of one (rounding only)


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
    assert opts[capi.OPT_INTERP_FUSED] == 1 and opts[capi.OPT_FUSED_WHITE] == 0
    return opts


@pytest.fixture(autouse=True)
def fused_white(ctx, capi, shipped):
    ctx.set_option(capi.OPT_FUSED_WHITE, 1)
    yield
    ctx.set_options(shipped)


def _c5_like(ctx, rng, P=17, n=(40, 500), white=True, ecorr=True, sv=True, commons=("hd", "monopole", "dipole")):
    """C5's signal mix on ragged pulsars over one common span: every epoch observed by two backends (np.repeat, as
    fake_pta.Pulsar), RN30, DM100 (idx 2), Sv60 (idx 4), the common signals on f_k = k / T (ORF factors of rank P,
    1 and 3), per-TOA white sigma and one 2-TOA ECORR block per (backend, epoch pair); one pulsar of 7 TOAs, one of 33.
    Returns the oracle's segments and white parameters."""
    counts = rng.integers(n[0], n[1], size=P) // 2 * 2
    counts[2], counts[3] = 6, 34
    offs = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    t0, t1 = 4.4e9, 4.4e9 + 3.15e8
    toas, nu = [], []
    for k in counts:
        ep = np.concatenate([[t0], np.sort(rng.uniform(t0, t1, k // 2 - 2)), [t1]]) if k >= 4 else np.array([t0, t1])
        toas.append(np.repeat(ep, 2))
        nu.append(np.abs(np.tile([1400.0, 800.0], k // 2) + rng.normal(0, 10, k)))
    toas, nu = np.concatenate(toas), np.concatenate(nu)
    T = t1 - t0
    ctx.batch_set_toas(offs, toas, nu)
    segs = []
    for nm, idx in ((30, 0.0), (100, 2.0)) + (((60, 4.0),) if sv else ()):
        f = np.tile(np.arange(1, nm + 1) / T, (P, 1))
        a = np.sqrt(O.powerlaw(f, rng.uniform(-14.5, -13.5, (P, 1)), 3.0) / T)
        ctx.batch_add_signal(0, f, a, idx=idx)
        segs.append(O.Segment(0, 2 * np.pi * f, a, idx))
    v = rng.normal(size=(P, 3))
    pos = v / np.linalg.norm(v, axis=1)[:, None]
    orfs = {"hd": O.orf_hd, "monopole": O.orf_monopole, "dipole": O.orf_dipole}
    from fakepta_amd.batch import batch_factor
    for name in commons:
        fc = np.arange(1, 31) / T
        ac = np.sqrt(O.powerlaw(fc, -14.5, 13 / 3) / T)
        L = batch_factor(orfs[name](pos))
        ctx.batch_add_signal(1, fc, ac, L=L)
        segs.append(O.Segment(1, 2 * np.pi * fc, ac, 0.0, L=L))
    sigma = rng.uniform(0.5e-7, 2e-7, offs[-1]) if white else None
    blocks, esig, block_of = [], [], -np.ones(offs[-1], dtype=np.int64)
    if ecorr:
        for p in range(P):
            idx = np.arange(offs[p], offs[p + 1])
            for b in (0, 1):  # backend b: TOAs of the backend, epochs of two consecutive times
                tb = idx[b::2]
                for j in range(0, len(tb), 2):
                    blocks.append(tb[j:j + 2])
        esig = rng.uniform(0.5e-7, 1.5e-7, len(blocks))
        for i, q in enumerate(blocks):
            block_of[q] = i
    ctx.batch_set_white(sigma, blocks if ecorr else [], esig if ecorr else [])
    return offs, toas, nu, segs, sigma, (block_of if ecorr else None), (np.asarray(esig) if ecorr else None)


def _run(ctx, capi, fused, seed, real0, R):
    ctx.set_option(capi.OPT_INTERP_FUSED, fused)
    ctx.batch_synth(seed, 0, R, to_host=False)
    ctx.debug_fill_out(np.nan)
    out = ctx.batch_synth(seed, real0, R)
    return out, ctx.batch_grid_info()["interp_kernel"]


@pytest.mark.parametrize("case", ["white_ecorr", "white", "ecorr", "plain", "two_grid_white"])
def test_fused_w_matches_two_kernel_path_and_oracle(ctx, capi, shipped, case):
    """k_grid_fused_w against the two-kernel path (INTERP_FUSED 0) at W_TOL and the oracle at the gridded tolerance:
    realization counts off the 16-realization items (R_pad padding), odd first realizations (the ODD draws and the
    white stream's misaligned quads), every sample written (NaN-poisoned block), the kernel that ran named."""
    rng = np.random.default_rng(401 + len(case))
    kw = dict(white=case in ("white_ecorr", "white", "two_grid_white"), ecorr=case in ("white_ecorr", "ecorr"),
              sv=case != "two_grid_white")
    offs, toas, nu, segs, sigma, block_of, esig = _c5_like(ctx, rng, **kw)
    try:
        ctx.set_option(capi.OPT_SYNTH_PATH, 4)
        for R, real0 in ((333, 5), (16, 0), (100, 77), (1024, 3)):
            ref, k0 = _run(ctx, capi, 0, 13, real0, R)
            got, k1 = _run(ctx, capi, 1, 13, real0, R)
            assert k1 == f"k_grid_fused_w<16, {'true' if real0 & 1 else 'false'}>", k1
            assert not k0.startswith("k_grid_fused"), k0
            assert np.all(np.isfinite(got))
            assert rel_err(got, ref) <= W_TOL, (R, real0, rel_err(got, ref))
            if R in (333, 100):
                want = O.batch_synth(offs, toas, nu, segs, 13, real0, R, sigma=sigma, block_of=block_of,
                                     ecorr_sigma=esig)
                assert rel_err(got, want) <= GRID_TOL
                assert_parity(got, want, TOL)
    finally:
        ctx.batch_set_white()
        ctx.batch_clear()
        ctx.set_options(shipped)


def test_fused_w_pipelined_blocks_and_determinism(ctx, capi, shipped):
    """Pipelined blocks (FPTA_OPT_OVERLAP 1: the next block's common draws into the other coefficient buffer on the
    side stream while this block's kernel reads its own) equal one-stream blocks bit for bit, run to run, with their
    checksums; batch-split invariance (a realization's samples do not depend on the block it is drawn in)."""
    rng = np.random.default_rng(433)
    _c5_like(ctx, rng, P=20, n=(200, 700))
    try:
        ctx.set_option(capi.OPT_SYNTH_PATH, 4)
        res = {}
        for ov in (0, 1):
            ctx.set_option(capi.OPT_OVERLAP, ov)
            for b in range(3):
                ctx.batch_synth(29, 256 * b, 256, to_host=False)
            res[ov, "last"] = ctx.batch_synth(29, 256 * 3, 256)
            assert ctx.batch_grid_info()["interp_kernel"].startswith("k_grid_fused_w")
            res[ov, "each"] = [(ctx.batch_synth(29, 300 * b + 1, 300), ctx.batch_checksums()) for b in range(3)]
        np.testing.assert_array_equal(res[0, "last"], res[1, "last"])
        for (x, xs), (y, ys) in zip(res[0, "each"], res[1, "each"]):
            np.testing.assert_array_equal(x, y)
            np.testing.assert_array_equal(xs, ys)
        whole = ctx.batch_synth(29, 100, 64)
        split = np.concatenate([ctx.batch_synth(29, 100, 17), ctx.batch_synth(29, 117, 47)])
        np.testing.assert_array_equal(whole, split)
    finally:
        ctx.batch_set_white()
        ctx.batch_clear()
        ctx.set_options(shipped)


def test_fused_w_not_taken_outside_its_blocks(ctx, capi, shipped):
    """Blocks k_grid_fused_w does not serve take the other kernels: fused partial checksums (streamed jobs), grids
    too large for LDS at 16 realizations (three signals of 600 modes), FPTA_OPT_INTERP_FUSED 0; and a plain block of
    a two-grid-signal layout stays on k_grid_fused."""
    rng = np.random.default_rng(439)
    try:
        offs, toas, nu, segs, sigma, block_of, esig = _c5_like(ctx, rng, P=8, n=(100, 300))
        ctx.set_option(capi.OPT_SYNTH_PATH, 4)
        ctx.batch_synth(3, 0, 256, to_host=False)
        assert ctx.batch_grid_info()["interp_kernel"].startswith("k_grid_fused_w")
        ctx.set_option(capi.OPT_FUSE_CHECKSUMS, 1)
        ctx.batch_synth(3, 0, 256, to_host=False)
        assert not ctx.batch_grid_info()["interp_kernel"].startswith("k_grid_fused")
        ctx.set_option(capi.OPT_FUSE_CHECKSUMS, 0)
        ctx.set_option(capi.OPT_INTERP_FUSED, 0)
        ctx.batch_synth(3, 0, 256, to_host=False)
        assert not ctx.batch_grid_info()["interp_kernel"].startswith("k_grid_fused")
        ctx.set_options(shipped)
        ctx.set_option(capi.OPT_FUSED_WHITE, 1)
        ctx.batch_set_white()
        ctx.batch_clear()
        _c5_like(ctx, rng, P=6, n=(100, 300), white=False, ecorr=False, sv=False)
        ctx.set_option(capi.OPT_SYNTH_PATH, 4)
        ctx.batch_synth(3, 0, 256, to_host=False)
        k = ctx.batch_grid_info()["interp_kernel"]
        assert k.startswith("k_grid_fused<"), k
        ctx.batch_clear()
        # three 600-mode signals: 3 x 1,804 grid rows do not fit in LDS even at 16 realizations
        P = 3
        offs = np.array([0, 200, 400, 600], dtype=np.int64)
        t = np.sort(rng.uniform(4.4e9, 4.4e9 + 3.15e8, 600))
        ctx.batch_set_toas(offs, t, rng.choice([800.0, 1400.0, 2500.0], size=600))
        T = t.max() - t.min()
        for idx in (0.0, 2.0, 4.0):
            f = np.tile(np.arange(1, 601) / T, (P, 1))
            ctx.batch_add_signal(0, f, np.sqrt(O.powerlaw(f, -14.0, 3.0) / T), idx=idx)
        ctx.batch_set_white(np.full(600, 1e-7), [], [])
        ctx.batch_synth(3, 0, 64, to_host=False)
        assert not ctx.batch_grid_info()["interp_kernel"].startswith("k_grid_fused")
    finally:
        ctx.batch_set_white()
        ctx.batch_clear()
        ctx.set_options(shipped)
