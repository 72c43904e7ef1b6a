"""Host-side logic of the drop-in package against the reference's fixtures (CPU only:
nothing here launches a kernel)."""
import os

import numpy as np
import pytest

from fakepta import correlated_noises as cn
from fakepta import fake_pta as fp
from fakepta import spectrum as sp
from tests.conftest import assert_parity


def test_psd_registry_matches_reference_names():
    assert sorted(fp.spec) == ["broken_powerlaw", "powerlaw", "t_process", "t_process_adapt", "turnover",
                               "turnover_knee"]
    assert fp.spec_params["powerlaw"] == ["log10_A", "gamma"]
    assert fp.spec_params["turnover_knee"] == ["log10_A", "gamma", "lfb", "lfk", "kappa", "delta"]


def test_psds_bitwise_vs_reference(golden):
    import json
    g = golden("g1_psd.npz")
    for key, params in json.loads(str(g["meta_json"])).items():
        name, gi, _ = key.split("__")
        p = {k: (np.array(v) if isinstance(v, list) else v) for k, v in params.items()}
        np.testing.assert_allclose(getattr(sp, name)(g["grid" + gi[1:]].copy(), **p), g[key], rtol=1e-14)


def test_pulsar_construction_rng_parity(golden):
    """Same np.random draws as the reference constructor: jittered radio frequencies, flags, name."""
    g = golden("g2_single_psr.npz")
    rng = np.random.default_rng(7)
    yr = 365.25 * 24 * 3600
    keep = rng.random(330) < 0.75
    cadence = 12.3 * 24 * 3600
    epochs = 0.35 * yr + np.arange(1, 331)[keep] * cadence
    np.random.seed(11)
    psr = fp.Pulsar(epochs, 3e-7, 1.1, 4.2, pdist=(1.0, 0.2), freqs=[1400], backends=["A.1400", "B.800"],
                    custom_model={"RN": 30, "DM": 100, "Sv": 30})
    np.testing.assert_array_equal(psr.toas, g["toas"])
    np.testing.assert_array_equal(psr.freqs, g["freqs"])
    np.testing.assert_array_equal(psr.backend_flags.astype("U"), g["backend_flags"])
    assert psr.name == str(g["name"]) and psr.Tspan == g["Tspan"]


@pytest.mark.parametrize("backends", [["NUPPI.1400"], ["NUPPI.1400", "LEAP.1396", "X.2500"], ["backend"],
                                      ["A.1400", "b"]])
def test_backend_flags_fast_path_matches_per_toa_loop(backends):
    """get_freqs_and_backends parses each distinct flag once when every flag names its frequency; otherwise it walks
    the TOAs drawing np.random.choice(freqs) per unnamed flag, as fake_pta.py:63-74. Both give the per-TOA loop's
    frequencies, flags (dtype included) and leave the global RNG in the same state."""
    def per_toa(nepochs, freqs, backends):
        flags = np.tile(backends, nepochs)
        radio = []
        for i, flag in enumerate(flags):
            try:
                radio.append(float(flag.split('.')[-1]))
            except ValueError:
                choice = np.random.choice(freqs)
                flags[i] = flags[i] + '.' + str(int(choice))
                radio.append(choice)
        return np.array(radio), flags

    class Stub:
        nepochs = 7
    np.random.seed(3)
    got = fp.Pulsar.get_freqs_and_backends(Stub(), [1400, 2000], backends)
    after_got = np.random.random()
    np.random.seed(3)
    want = per_toa(7, [1400, 2000], backends)
    after_want = np.random.random()
    np.testing.assert_array_equal(got[0], want[0])
    assert got[0].dtype == want[0].dtype and got[1].dtype == want[1].dtype
    np.testing.assert_array_equal(got[1], want[1])
    assert after_got == after_want


def test_tutorial_names(golden):
    """examples/tutorial.ipynb cell 5: names of the 25-pulsar isotropic array."""
    names = golden("g5_tutorial.json")["names_npsrs25_isotropic"]
    i = np.arange(25, dtype=float) + 0.5
    cost = 1 - 2 * i / 25
    phis = np.mod(2 * np.pi * i / ((1 + 5 ** 0.5) / 2), 2 * np.pi)
    got = []
    for c, ph in zip(cost, phis):
        p = fp.Pulsar.__new__(fp.Pulsar)
        p.theta, p.phi = np.arccos(c), ph
        got.append(p.get_psrname())
    assert got == names


def test_g4_names_and_design_matrix(golden):
    g = golden("g4_make_fake_array.npz")
    assert len(g["names"]) == 25 and g["Mmat0"].shape[1] == 8


def test_quantise_ecorr_verbatim(golden):
    g = golden("g2_single_psr.npz")
    p = fp.Pulsar.__new__(fp.Pulsar)
    p.toas, p.backend_flags = g["q_toas"], g["q_flags"]
    p.backends = np.unique(p.backend_flags)
    q = p.quantise_ecorr()
    assert [len(b) for b in q] == list(g["q_lens"])
    np.testing.assert_array_equal(np.concatenate(q), g["q_idx"])
    full = p.ecorr_blocks()
    assert sorted(np.concatenate(full).tolist()) == list(range(len(p.toas)))


@pytest.mark.parametrize("orf", ["hd", "monopole", "dipole", "curn"])
def test_orfs_and_factor(golden, orf):
    g = golden("g3_common.npz")

    class P:
        def __init__(self, pos):
            self.pos = pos
    psrs = [P(x) for x in g["pos"]]
    gam = cn.ORF_FUNCS[orf](psrs)
    np.testing.assert_allclose(gam, g[f"{orf}_orf"], rtol=1e-14, atol=1e-15)
    L = cn.orf_factor(gam)
    np.testing.assert_allclose(L.T, g[f"{orf}_svdM"], atol=1e-13)
    assert_parity(L @ L.T, gam, 1e-12)


def test_mvn_draw_order_equivalence():
    """numpy's legacy multivariate_normal == standard_normal(P) @ (sqrt(s) vt): the host draws
    z in that order and the GPU applies L = M^T."""
    rng_cov = np.random.default_rng(1).normal(size=(7, 7))
    cov = rng_cov @ rng_cov.T
    np.random.seed(3)
    a = np.random.multivariate_normal(np.zeros(7), cov)
    np.random.seed(3)
    z = np.random.standard_normal(7)
    np.testing.assert_allclose(cn.orf_factor(cov) @ z, a, rtol=1e-12, atol=1e-12)


def test_noisedict_conventions():
    p = fp.Pulsar.__new__(fp.Pulsar)
    p.name, p.backends = "J0000+0000", np.array(["A", "B"])
    p.init_noisedict(None)
    assert p.noisedict["J0000+0000_A_efac"] == 1.0 and len(p.noisedict) == 8
    p.init_noisedict({"J0000+0000_A_efac": 2.0, "J1111+1111_A_efac": 3.0, "red_noise_gamma": 1})
    assert p.noisedict == {"J0000+0000_A_efac": 2.0}
    p.init_noisedict({"A_efac": 1.1, "A_log10_tnequad": -7, "B_efac": 1.2, "B_log10_tnequad": -6,
                      "A_log10_t2equad": -7, "A_log10_ecorr": -8, "red_noise_log10_A": -14,
                      "red_noise_gamma": 3})
    nd = p.noisedict
    assert nd["J0000+0000_B_efac"] == 1.2 and "J0000+0000_B_log10_t2equad" not in nd
    assert nd["J0000+0000_A_log10_ecorr"] == -8 and nd["J0000+0000_red_noise_gamma"] == 3
    p.init_noisedict({"efac": 1.5, "log10_tnequad": -6.5})
    assert p.noisedict == {"J0000+0000_A_efac": 1.5, "J0000+0000_A_log10_tnequad": -6.5,
                           "J0000+0000_B_efac": 1.5, "J0000+0000_B_log10_tnequad": -6.5}


def test_reference_pickles_load_into_the_dropin():
    """Pulsar objects pickled by the reference itself (class path fakepta.fake_pta.Pulsar, as
    examples/make_fake_array.py:65 saves an array; fixture g7 written by tools/gen_golden.py) unpickle
    into this package's Pulsar with the reference's state, and this package's pickles record the same
    class path. The pickle is our own fixture file (written by the generator), not a reference artefact."""
    import os
    import pickle
    from tests.conftest import GOLDEN
    g = np.load(os.path.join(GOLDEN, "g7_ref_pulsars.npz"))
    with open(os.path.join(GOLDEN, "g7_ref_pulsars.pkl"), "rb") as fh:
        psrs = pickle.load(fh)
    assert len(psrs) == 4 and all(type(p) is fp.Pulsar for p in psrs)
    for i, p in enumerate(psrs):
        np.testing.assert_array_equal(p.residuals, g[f"residuals_{i}"])
        assert set(p.signal_model) == {"red_noise", "dm_gp", "gw_common"}
        assert p.signal_model["gw_common"]["orf"] == "hd"
    assert pickle.loads(pickle.dumps(psrs[0])).name == psrs[0].name
    assert b"fakepta.fake_pta" in pickle.dumps(psrs[0]) and b"fakepta_amd" not in pickle.dumps(psrs[0])


def test_reference_import_paths():
    """The reference's own import lines resolve (examples/make_fake_array.py:1,6, README.md:15)."""
    import importlib
    for mod, names in (("fakepta.fake_pta", ("Pulsar", "make_fake_array", "copy_array", "spec", "spec_params")),
                       ("fakepta.correlated_noises", ("add_common_correlated_noise", "hd", "monopole", "dipole",
                                                      "curn", "anisotropic", "get_correlations", "bin_curve")),
                       ("fakepta.spectrum", ("powerlaw", "turnover", "t_process", "t_process_adapt",
                                             "turnover_knee", "broken_powerlaw")),
                       ("fakepta.constants", ("fyr", "yr"))):
        m = importlib.import_module(mod)
        for n in names:
            assert hasattr(m, n), (mod, n)


def test_copy_array_noisedict_lookup_g8(golden):
    """copy_array with the reference's shipped EPTA noisedict / custom_models (fixture G8): the name-keyed
    init_noisedict branch, per-pulsar custom models, copied TOA attributes (fake_pta.py:76-147, 687-712)."""
    from fakepta import fake_pta as fp
    from tests.helpers import g8_inputs
    psrs_0, nd, cm, g = g8_inputs(golden)
    want = golden("g8_example_workflow.json")
    np.random.seed(int(g["seed"]))
    psrs = fp.copy_array(psrs_0, nd, cm)
    assert [p.name for p in psrs] == list(g["names"])
    np.testing.assert_array_equal(np.concatenate([p.freqs for p in psrs]), g["copied_freqs"])
    for p in psrs:
        # the final noisedict adds the GWB's keys (update_noisedict, correlated_noises.py:128-129)
        assert p.noisedict == {k: v for k, v in want["noisedicts"][p.name].items() if not k.startswith("gw_common")}
        assert p.Tspan == want["Tspan"][p.name]
        assert p.custom_model == cm[p.name]
        assert list(p.backends) == sorted(set(p.backend_flags))


def test_rccl_unique_id_rendezvous_threads():
    """RcclComm's rendezvous (fakepta_amd.batch._exchange_unique_id): rank 0 serves its 128-byte id to every other
    rank over one TCP socket; ranks that start before the server retry. Four ranks as threads, no GPU."""
    import socket
    import threading
    import time
    from fakepta_amd.batch import _exchange_unique_id
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    uid = bytes(range(128))
    got = {}

    def run(rank):
        if rank == 0:
            time.sleep(0.5)  # the clients start first and retry
        got[rank] = _exchange_unique_id(rank, 4, "127.0.0.1", port, lambda: uid, timeout=20.0)

    ts = [threading.Thread(target=run, args=(r,)) for r in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(30)
    assert got == {r: uid for r in range(4)}


def test_bench_refuses_world_size_mismatch():
    """bench.py --gpus N under a launcher that started a different number of ranks exits non-zero before any GPU
    call (the driver's scaling runs cannot silently measure a different N)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if not k.startswith("FPTA_")}
    env.update(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    res = subprocess.run([sys.executable, "bench.py", "--gpus", "2"], cwd=root, env=env, capture_output=True,
                         text=True, timeout=60)
    assert res.returncode != 0 and "WORLD_SIZE" in res.stderr
