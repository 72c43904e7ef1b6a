"""Host profile of the C1 drop-in path (GPU box): make_fake_array(25 psr, RN30) as tools/bench_configs.py c1 runs
it, warmed once, then five runs under cProfile; prints the top functions by own and by cumulative time.

    python tools/profile_c1.py > gpurun_out/c1_profile.txt
"""
import cProfile
import os
import pstats
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from fakepta import fake_pta as fp
    kw = dict(npsrs=25, Tobs=10, ntoas=1000, isotropic=True, gaps=True, toaerr=1e-7, backends="NUPPI.1400",
              custom_model={"RN": 30, "DM": None, "Sv": None})
    np.random.seed(0)
    fp.make_fake_array(**kw)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(5):
        np.random.seed(0)
        fp.make_fake_array(**kw)
    pr.disable()
    st = pstats.Stats(pr, stream=sys.stdout)
    st.sort_stats("tottime").print_stats(25)
    st.sort_stats("cumulative").print_stats(25)


if __name__ == "__main__":
    main()
