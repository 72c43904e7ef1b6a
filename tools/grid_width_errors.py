"""Measured error of the gridded path against the oracle as a function of the kernel width (GPU box).

    python tools/grid_width_errors.py [--widths 12 13 14 15 16] [--sigma 150]

The worst case of tests/test_gpu_grid.py::test_flat_spectrum_real_epochs (flat spectrum, real-MJD-like epochs
t ~ 5e9 s, chromatic index 2, 4 ragged pulsars, 64 realizations) for 1, 30, 100 and 257 modes, at each width: one
JSON line per (width, modes) with the relative L2 error, the max-abs error over max|oracle| and the a-priori bound
exp(-pi w sqrt(1 - 1/sigma)). The oracle is the checker (tests/ infrastructure), as in the test.
"""
import argparse
import json
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--widths", type=int, nargs="+", default=[12, 13, 14, 15, 16])
    ap.add_argument("--sigma", type=int, default=150, help="oversampling x 100")
    args = ap.parse_args()
    from fakepta_amd import _capi
    from oracle import fakepta_oracle as O
    from tests.conftest import rel_err
    from tests.helpers import per_psr_signal, random_layout
    ctx = _capi.Context(0)
    ctx.set_option(_capi.OPT_SYNTH_PATH, 4)
    ctx.set_option(_capi.OPT_GRID_SIGMA, args.sigma)
    for n_modes in (1, 30, 100, 257):
        rng = np.random.default_rng(n_modes)  # the test's layout for this mode count
        offs, toas, nu = random_layout(rng, 4, (100, 300), t_max=1.6e8)
        toas = toas + 4.5e9
        ctx.batch_clear()
        ctx.batch_set_toas(offs, toas, nu)
        f, _ = per_psr_signal(rng, offs, toas, n_modes)
        a = np.full_like(f, 1e-7)
        ctx.batch_add_signal(0, f, a, idx=2.0)
        want = O.batch_synth(offs, toas, nu, [O.Segment(0, 2 * np.pi * f, a, 2.0)], 5, 0, 64)
        for w in args.widths:
            ctx.set_option(_capi.OPT_GRID_WIDTH, w)
            got = ctx.batch_synth(5, 0, 64)
            print(json.dumps({"width": w, "sigma": args.sigma / 100, "modes": n_modes,
                              "rel_l2": rel_err(got, want),
                              "max_abs_over_max": float(np.abs(got - want).max() / np.abs(want).max()),
                              "a_priori_bound": math.exp(-math.pi * w * math.sqrt(1 - 100 / args.sigma)),
                              "grid_info": {k: ctx.batch_grid_info()[k] for k in ("width", "err_bound")}}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
