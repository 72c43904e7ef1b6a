"""fakepta_amd — MI355X-native Fourier-basis GP residual synthesis for pulsar-timing arrays.

Drop-in modules for mfalxa/fakepta: `fake_pta` (Pulsar, make_fake_array, copy_array),
`correlated_noises` (ORFs, add_common_correlated_noise), `spectrum` (PSD models), plus
`batch` (BatchSimulator / simulate_batch: many realizations on device).
The compute path is libfakepta_amd.so (HIP, gfx950) loaded by `_capi`; no CPU fallback.
"""
__version__ = "0.1.0"
