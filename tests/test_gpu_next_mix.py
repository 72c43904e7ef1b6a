"""FPTA_OPT_FUSED_NEXT_MIX: a pipelined k_grid_fused block also draws and ORF-mixes the common signal of the block
that follows it (same seed and size, first realization real0 + the last stride when that is a whole number of
blocks, else real0 + n_real) as spare-time tickets of its waves
(fused_mix_tile), into the coefficient buffer that block swaps in; that block then launches no k_gen_mix.

Checked against the same block sequences with the option off (every block runs k_gen_mix): bit for bit, since the
tickets draw k_gen_mix's normals and sum the same products per k-step in the same order (for a lower-triangular
factor they stop at the 16-pulsar tile's diagonal, where k_gen_mix adds exact zeros). Sequences mix hits (the next
realizations), misses (a jump, another size, another seed, an odd first realization, a layout change, OVERLAP 0 or
a coefficient download in between: the call then waits for the previous kernel before anything writes the buffer)
and blocks queued without a host sync in between. One hit block is checked against the oracle as well.

Reference loop the mix replaces: /root/reference/fakepta/correlated_noises.py:153-160 (the ORF-correlated draws of
add_common_correlated_noise); per-pulsar signals fake_pta.py:372-387.
"""
import numpy as np
import pytest

from oracle import fakepta_oracle as O
from tests.conftest import assert_parity, rel_err
from tests.test_gpu_grid import GRID_TOL, TOL

pytestmark = pytest.mark.gpu


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
    assert opts[capi.OPT_FUSED_NEXT_MIX] == 1 and opts[capi.OPT_OVERLAP] == 1 and opts[capi.OPT_INTERP_FUSED] == 1
    return opts


def _layout(ctx, rng, P, factor="cholesky", n=(40, 260)):
    """C2's signal mix on P ragged pulsars over one common span: RN30 (idx 0), DM100 (idx 2, three radio bands) and a
    common GWB30 on f_k = k / T (RN and the GWB share a grid signal, mixed by the factor: Cholesky of HD (lower-
    triangular), numpy's SVD factor of HD (full), or the monopole's rank-1 factor)."""
    from fakepta_amd.batch import batch_factor
    counts = rng.integers(n[0], n[1], size=P)
    offs = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    t0, t1 = 4.4e9, 4.4e9 + 3.15e8
    toas = np.concatenate([np.concatenate([[t0], np.sort(rng.uniform(t0, t1, k - 2)), [t1]]) for k in counts])
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
    pos = v / np.linalg.norm(v, axis=1)[:, None]
    if factor == "cholesky":
        L = batch_factor(O.orf_hd(pos))
        assert np.all(np.triu(L, 1) == 0.0)
    elif factor == "svd":
        L = O.mvn_factor(O.orf_hd(pos))
    else:
        L = batch_factor(O.orf_monopole(pos))
    ctx.batch_add_signal(1, fc, ac, L=L)
    segs.append(O.Segment(1, 2 * np.pi * fc, ac, 0.0, L=L))
    ctx.set_option(1, 4)  # FPTA_OPT_SYNTH_PATH: gridded (auto may take the exact paths at these sizes)
    return offs, toas, nu, segs


# (seed, real0, n_real, fetch): fetch = download the block (a host sync); else the next call is queued behind it
_SEQ = [(7, 0, 256, True), (7, 256, 256, True), (7, 512, 256, False), (7, 768, 256, True),   # hits from block 3
        (7, 1100, 256, False), (7, 1356, 256, True),                                          # jump: miss, hit
        (7, 1612, 100, False), (7, 1712, 100, True),                                          # size: miss, hit
        (9, 1812, 100, False), (9, 1912, 100, True),                                          # seed: miss, hit
        (9, 2013, 100, False), (9, 2113, 100, False), (9, 2213, 100, True)]                   # odd first: hits


def _run_seq(ctx, capi, on, seq):
    ctx.set_option(capi.OPT_FUSED_NEXT_MIX, on)
    outs, used, made = [], [], []
    for seed, real0, R, fetch in seq:
        out = ctx.batch_synth(seed, real0, R, to_host=fetch)
        if not fetch:
            out = None
        gi = ctx.batch_grid_info()
        assert gi["interp_kernel"].startswith("k_grid_fused<"), gi["interp_kernel"]
        outs.append(out)
        used.append(gi["next_mix_used"])
        made.append(gi["next_mix_made"])
    ctx.synchronize()
    return outs, used, made


def _hits_expected(seq):
    """Blocks whose mix the previous block's kernel made: the key follows on, and the previous block itself was not
    the first two of the context's pipelined run (the first has no second coefficient buffer grown yet)."""
    exp = [False] * len(seq)
    for i in range(2, len(seq)):
        s0, r0, n0, _ = seq[i - 1]
        s1, r1, n1, _ = seq[i]
        exp[i] = s0 == s1 and r1 == r0 + n0 and n0 == n1
    return exp


@pytest.mark.parametrize("P,factor", [(100, "cholesky"), (70, "svd"), (200, "cholesky"), (64, "monopole")])
def test_next_mix_bitwise_vs_gen_mix(ctx, capi, shipped, P, factor):
    """Hit and miss sequences with the option on equal the same sequences with every block on k_gen_mix, bit for bit;
    hits exactly where the key follows on; one hit block against the oracle."""
    rng = np.random.default_rng(701 + P)
    offs, toas, nu, segs = _layout(ctx, rng, P, factor)
    try:
        ref, used0, made0 = _run_seq(ctx, capi, 0, _SEQ)
        assert not any(used0) and not any(made0)
        got, used1, made1 = _run_seq(ctx, capi, 1, _SEQ)
        for i, (x, y) in enumerate(zip(ref, got)):
            if x is not None:
                assert np.all(np.isfinite(y))
                np.testing.assert_array_equal(y, x, err_msg=f"block {i} {_SEQ[i]}")
        exp = _hits_expected(_SEQ)
        # the context ran blocks before this sequence (the option-off run): its second coefficient buffer exists, so
        # block 1 can hit too
        exp[1] = True
        assert used1 == exp, (used1, exp)
        assert all(made1), made1
        i = 3  # a hit
        seed, real0, R, _ = _SEQ[i]
        want = O.batch_synth(offs, toas, nu, segs, seed, real0, R)
        assert rel_err(got[i], want) <= GRID_TOL
        assert_parity(got[i], want, TOL)
    finally:
        ctx.batch_clear()
        ctx.set_options(shipped)


def test_next_mix_rank_strides(ctx, capi, shipped):
    """Blocks at a stride of G blocks (rank g of G in bench.py: real0 = (s G + g) R): from the third block on the
    prediction follows the stride (a whole number of blocks) and every block hits; a jump that is not a whole number
    of blocks predicts real0 + n_real again. Bit for bit against the option off."""
    rng = np.random.default_rng(751)
    _layout(ctx, rng, 100, "cholesky")
    R = 128
    seq = [(11, (s * 4 + 1) * R, R, s % 2 == 1) for s in range(6)]                      # rank 1 of 4
    seq += [(11, 5000, R, False), (11, 5000 + R, R, True), (11, 5000 + 2 * R, R, True)]  # a jump, then consecutive
    try:
        ctx.synchronize()
        ref, _, _ = _run_seq(ctx, capi, 0, seq)
        got, used, made = _run_seq(ctx, capi, 1, seq)
        for i, (x, y) in enumerate(zip(ref, got)):
            if x is not None:
                np.testing.assert_array_equal(y, x, err_msg=f"block {i} {seq[i]}")
        assert used == [False, False, True, True, True, True, False, True, True], used
        assert all(made)
    finally:
        ctx.batch_clear()
        ctx.set_options(shipped)


def test_next_mix_invalidated_by_changes(ctx, capi, shipped):
    """A block after a layout change (another amplitude), OVERLAP 0, or a coefficient download takes no precomputed
    mix and equals the option-off result; the block after it hits again."""
    rng = np.random.default_rng(733)
    offs, toas, nu, segs = _layout(ctx, rng, 96, "cholesky")
    try:
        def seq(on):
            ctx.set_option(capi.OPT_FUSED_NEXT_MIX, on)
            res = []
            for real0 in (0, 128, 256):
                ctx.batch_synth(5, real0, 128, to_host=False)
            # OVERLAP 0 for the block the previous kernel mixed for
            ctx.set_option(capi.OPT_OVERLAP, 0)
            res.append((ctx.batch_synth(5, 384, 128), ctx.batch_grid_info()["next_mix_used"]))
            ctx.set_option(capi.OPT_OVERLAP, 1)
            for real0 in (512, 640):
                res.append((ctx.batch_synth(5, real0, 128), ctx.batch_grid_info()["next_mix_used"]))
            # a coefficient download (the draws leave the fused kernel: GEN = false, k_gen_mix runs)
            out, co = ctx.batch_synth(5, 768, 128, coeffs=True)
            res.append((out, ctx.batch_grid_info()["next_mix_used"]))
            res.append((ctx.batch_synth(5, 896, 128), ctx.batch_grid_info()["next_mix_used"]))
            res.append((ctx.batch_synth(5, 1024, 128), ctx.batch_grid_info()["next_mix_used"]))
            return res

        ref = seq(0)
        got = seq(1)
        for (x, _), (y, u) in zip(ref, got):
            np.testing.assert_array_equal(y, x)
        assert [u for _, u in got] == [False, False, True, False, False, True]
        # a layout change between two blocks that follow on: the new layout's block must not take the old mix
        ctx.set_option(capi.OPT_FUSED_NEXT_MIX, 1)
        ctx.batch_synth(5, 0, 128, to_host=False)
        ctx.batch_synth(5, 128, 128, to_host=False)
        ctx.batch_clear()
        offs, toas, nu, segs = _layout(ctx, np.random.default_rng(739), 96, "cholesky")
        got = ctx.batch_synth(5, 256, 128)
        assert not ctx.batch_grid_info()["next_mix_used"]
        ctx.set_option(capi.OPT_FUSED_NEXT_MIX, 0)
        want = ctx.batch_synth(5, 256, 128)
        np.testing.assert_array_equal(got, want)
    finally:
        ctx.batch_clear()
        ctx.set_options(shipped)


def test_next_mix_taken_by_a_white_block(ctx, capi, shipped):
    """A white / ECORR block whose mix the previous (plain) block's kernel made takes it (the key does not cover the
    white noise) and runs the two-kernel white path, whose DFT reads the mixed columns on a side stream after that
    kernel: equal to the option-off sequence bit for bit, queued without host syncs."""
    rng = np.random.default_rng(757)
    offs, toas, nu, segs = _layout(ctx, rng, 100, "cholesky")
    n = int(offs[-1])
    sigma = rng.uniform(0.5e-7, 2e-7, n)
    blocks = [np.arange(i, min(i + 2, n)) for i in range(0, n - 1, 2)]
    esig = rng.uniform(0.5e-7, 1.5e-7, len(blocks))
    try:
        def seq(on):
            ctx.set_option(capi.OPT_FUSED_NEXT_MIX, on)
            ctx.batch_set_white()
            for real0 in (0, 256):
                ctx.batch_synth(21, real0, 256, to_host=False)
            ctx.batch_set_white(sigma, blocks, esig)
            out = ctx.batch_synth(21, 512, 256)
            gi = ctx.batch_grid_info()
            ctx.batch_set_white()
            return out, gi["next_mix_used"], gi["interp_kernel"]
        ref, u0, _ = seq(0)
        got, u1, k1 = seq(1)
        assert not u0 and u1
        assert not k1.startswith("k_grid_fused"), k1
        np.testing.assert_array_equal(got, ref)
    finally:
        ctx.batch_set_white()
        ctx.batch_clear()
        ctx.set_options(shipped)


def test_next_mix_not_made_outside_its_layouts(ctx, capi, shipped):
    """No successor mix for layouts k_gen_mix does not serve alone: fewer than 64 pulsars (k_mix path), more than
    256, two common signals; and none with the option off."""
    rng = np.random.default_rng(743)
    try:
        for P in (40, 300):
            _layout(ctx, rng, P, "cholesky", n=(40, 120))
            for real0 in (0, 128, 256):
                ctx.batch_synth(3, real0, 128, to_host=False)
                gi = ctx.batch_grid_info()
                assert not gi["next_mix_made"] and not gi["next_mix_used"]
            ctx.batch_clear()
        _layout(ctx, rng, 80, "cholesky", n=(40, 120))
        T = 3.15e8
        fc = np.arange(1, 11) / T
        ctx.batch_add_signal(1, fc, np.sqrt(O.powerlaw(fc, -15.0, 13 / 3) / T), L=np.eye(80))
        for real0 in (0, 128, 256):
            ctx.batch_synth(3, real0, 128, to_host=False)
            gi = ctx.batch_grid_info()
            assert not gi["next_mix_made"] and not gi["next_mix_used"]
        ctx.synchronize()
    finally:
        ctx.batch_clear()
        ctx.set_options(shipped)


def test_next_mix_c2_full_size(ctx, capi, shipped):
    """BASELINE configs[1] at full size (100 psr x 2000 TOAs, RN30 + DM100 + HD30, R = 1024), blocks streamed as
    bench.py runs them: the third block takes the mix the second block's kernel made (no k_gen_mix), equals the
    option-off block bit for bit, and its realizations 0, 1, 511, 1023 match the oracle's own batch semantics."""
    from fakepta import correlated_noises as cn
    from fakepta import fake_pta as fp
    from fakepta_amd.batch import BatchSimulator
    from tests.helpers import oracle_segments
    np.random.seed(0)
    psrs = fp.make_fake_array(npsrs=100, Tobs=10, ntoas=2000, gaps=False, isotropic=True, toaerr=1e-7,
                              backends="NUPPI.1400", custom_model={"RN": 30, "DM": 100, "Sv": None})
    cn.add_common_correlated_noise(psrs, orf="hd", log10_A=-15, gamma=13 / 3)
    sim = BatchSimulator(psrs, white=False, ctx=ctx)
    try:
        ctx.set_option(capi.OPT_SYNTH_PATH, 4)
        outs = {}
        for on in (0, 1):
            ctx.set_option(capi.OPT_FUSED_NEXT_MIX, on)
            for real0 in (0, 1024):
                sim.synth(1024, seed=1234, real0=real0, to_host=False)
            ctx.debug_fill_out(np.nan)
            outs[on] = sim.synth(1024, seed=1234, real0=2048)
            gi = ctx.batch_grid_info()
            assert gi["interp_kernel"] == "k_grid_fused<8, false, true, true>", gi["interp_kernel"]
            assert gi["next_mix_used"] == bool(on)
        assert np.all(np.isfinite(outs[1]))
        np.testing.assert_array_equal(outs[1], outs[0])
        segs = oracle_segments(sim)
        for r in (0, 1, 511, 1023):
            want = O.batch_synth(sim.offs, sim.toas, sim.freqs, segs, 1234, 2048 + r, 1)[0]
            assert_parity(outs[1][r], want, TOL)
    finally:
        ctx.batch_clear()
        ctx.set_options(shipped)
