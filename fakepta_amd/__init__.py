"""fakepta_amd — the MI355X-native layer under the `fakepta` drop-in package.

`_capi`: ctypes binding of libfakepta_amd.so (HIP kernels for gfx950 + C-ABI,
include/fakepta_amd.h). `batch`: many realizations of an array's noise model on device
(BatchSimulator, simulate_batch) and the realization-sharded multi-GPU driver
(simulate_sharded). The reference-compatible modules live in the `fakepta` package.
"""
__version__ = "0.1.0"
