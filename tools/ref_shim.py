"""Container-only loader for the read-only reference at /root/reference.

Test infrastructure, never shipped: used by tools/gen_golden.py to produce the
committed fixtures under tests/golden/. It must never run on the GPU box (the
reference does not exist there). Only the modules the hot path does not use are
stubbed:
  * enterprise.constants  -> the reference's own copy, fakepta/constants.py
  * enterprise_extensions.deterministic.cw_delay -> raises (add_cgw is out of scope)
  * healpy.pix2ang / npix2nside -> raise (anisotropic ORF is out of scope)
"""
import importlib.util
import os
import sys
import types

REF = "/root/reference"


def load_reference():
    if not os.path.isdir(REF):
        raise RuntimeError("reference not present (container-only tool)")
    sys.dont_write_bytecode = True
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    spec = importlib.util.spec_from_file_location(
        "enterprise.constants", os.path.join(REF, "fakepta", "constants.py"))
    const = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(const)
    ent = types.ModuleType("enterprise")
    ent.constants = const
    sys.modules["enterprise"] = ent
    sys.modules["enterprise.constants"] = const

    def _absent(*a, **k):
        raise NotImplementedError("stubbed: not on the hot path")

    ee = types.ModuleType("enterprise_extensions")
    det = types.ModuleType("enterprise_extensions.deterministic")
    det.cw_delay = _absent
    ee.deterministic = det
    sys.modules["enterprise_extensions"] = ee
    sys.modules["enterprise_extensions.deterministic"] = det
    hp = types.ModuleType("healpy")
    hp.pix2ang = _absent
    hp.npix2nside = _absent
    sys.modules["healpy"] = hp
    if REF not in sys.path:
        sys.path.insert(0, REF)
    from fakepta import fake_pta, correlated_noises, spectrum  # noqa: E402
    return fake_pta, correlated_noises, spectrum
