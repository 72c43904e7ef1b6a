"""fakepta — drop-in for mfalxa/fakepta with the Fourier-basis GP synthesis on MI355X.

Same module names and public surface as the reference (fakepta/__init__.py:1):
`fakepta.fake_pta` (Pulsar, make_fake_array, copy_array), `fakepta.correlated_noises`
(ORFs, add_common_correlated_noise), `fakepta.spectrum` (PSD models), `fakepta.constants`.
Scripts written for the reference (`from fakepta.fake_pta import make_fake_array`) and
Pulsar pickles recorded as `fakepta.fake_pta.Pulsar` load unchanged.

The sums over Fourier modes run in libfakepta_amd.so (HIP, gfx950) through
`fakepta_amd._capi`; there is no CPU fallback. Many realizations on device:
`fakepta_amd.batch` (BatchSimulator, simulate_batch, simulate_sharded).
"""
__version__ = "0.1.0"
