"""ctypes binding of libfakepta_amd.so (C-ABI declared in include/fakepta_amd.h).

The product path has no CPU fallback: if the library is missing this module raises at
import, and if no MI355X is visible the first compute call raises FptaError.
"""
import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_DEFAULT_LIB = os.path.join(_HERE, "lib", "libfakepta_amd.so")
LIB_PATH = os.environ.get("FAKEPTA_AMD_LIB", _DEFAULT_LIB)

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"fakepta_amd: HIP library not found at {LIB_PATH}. Build it with "
        "`python -c 'import __graft_entry__ as g; g.build()'` (or `make -C fakepta_amd/csrc`).")

_lib = ctypes.CDLL(LIB_PATH)

_c_int = ctypes.c_int
_i32, _i64, _u64 = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64
_dbl = ctypes.c_double
_vp = ctypes.c_void_p
_ctx_p = ctypes.c_void_p

# (name, restype, argtypes) — mirrors include/fakepta_amd.h
_SIGS = [
    ("fpta_version", _c_int, []),
    ("fpta_create", _c_int, [_c_int, ctypes.POINTER(_ctx_p)]),
    ("fpta_destroy", _c_int, [_ctx_p]),
    ("fpta_last_error", ctypes.c_char_p, [_ctx_p]),
    ("fpta_device_count", _c_int, [ctypes.POINTER(_c_int)]),
    ("fpta_gp_accumulate", _c_int, [_ctx_p, _i64, _vp, _vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _dbl, _vp]),
    ("fpta_gp_accumulate_array", _c_int, [_ctx_p, _i32, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                          _dbl, _vp]),
    ("fpta_common_accumulate", _c_int, [_ctx_p, _i32, _vp, _vp, _vp, _i32, _vp, _vp, _dbl, _dbl, _vp, _vp, _vp,
                                        _vp]),
    ("fpta_white_accumulate", _c_int, [_ctx_p, _i64, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp]),
    ("fpta_gp_covariance", _c_int, [_ctx_p, _i64, _vp, _vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("fpta_noise_wiener", _c_int, [_ctx_p, _i64, _vp, _vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("fpta_noise_draw", _c_int, [_ctx_p, _i64, _vp, _vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _u64, _i64, _i32,
                                 _vp]),
    ("fpta_batch_set_toas", _c_int, [_ctx_p, _i32, _vp, _vp, _vp]),
    ("fpta_batch_add_signal", _c_int, [_ctx_p, _i32, _i32, _vp, _vp, _dbl, _dbl, _vp, _vp]),
    ("fpta_batch_set_white", _c_int, [_ctx_p, _vp, _i64, _vp, _vp, _vp]),
    ("fpta_batch_clear_signals", _c_int, [_ctx_p]),
    ("fpta_batch_synth", _c_int, [_ctx_p, _u64, _i64, _i32, _vp, _vp]),
    ("fpta_batch_synth_from_z", _c_int, [_ctx_p, _i32, _i32, _vp, _vp]),
    ("fpta_batch_download", _c_int, [_ctx_p, _i32, _i32, _vp]),
    ("fpta_batch_device_out", _c_int, [_ctx_p, ctypes.POINTER(_vp), ctypes.POINTER(_i64), ctypes.POINTER(_i32)]),
    ("fpta_batch_checksums", _c_int, [_ctx_p, _vp]),
    ("fpta_batch_synth_checksums", _c_int, [_ctx_p, _u64, _i64, _i64, _i32, _vp]),
    ("fpta_batch_correlations", _c_int, [_ctx_p, _i32, _vp]),
    ("fpta_batch_info", _c_int, [_ctx_p, _vp]),
    ("fpta_batch_grid_info", _c_int, [_ctx_p, _vp]),
    ("fpta_batch_grid_info_n", _c_int, [_ctx_p, _vp, _i32]),
    ("fpta_set_option", _c_int, [_ctx_p, _i32, _i64]),
    ("fpta_kernel_stats", _c_int, [_ctx_p, _i32, ctypes.POINTER(_i64), ctypes.POINTER(_dbl)]),
    ("fpta_reset_stats", _c_int, [_ctx_p]),
    ("fpta_synchronize", _c_int, [_ctx_p]),
    ("fpta_debug_philox", _c_int, [_ctx_p, _i64, _vp, _vp, _vp]),
    ("fpta_debug_normals", _c_int, [_ctx_p, _i64, _vp, _vp]),
    ("fpta_debug_fill_out", _c_int, [_ctx_p, _dbl]),
    ("fpta_get_option", _c_int, [_ctx_p, _i32, ctypes.POINTER(_i64)]),
    ("fpta_build_flags", _c_int, []),
    ("fpta_batch_path_reason", ctypes.c_char_p, [_ctx_p]),
    ("fpta_multi_create", _c_int, [_i32, _vp, ctypes.POINTER(_vp)]),
    ("fpta_multi_destroy", _c_int, [_vp]),
    ("fpta_multi_last_error", ctypes.c_char_p, [_vp]),
    ("fpta_multi_size", _c_int, [_vp]),
    ("fpta_multi_context", _ctx_p, [_vp, _i32]),
    ("fpta_multi_set_toas", _c_int, [_vp, _i32, _vp, _vp, _vp]),
    ("fpta_multi_add_signal", _c_int, [_vp, _i32, _i32, _vp, _vp, _dbl, _dbl, _vp, _vp]),
    ("fpta_multi_set_white", _c_int, [_vp, _vp, _i64, _vp, _vp, _vp]),
    ("fpta_multi_set_option", _c_int, [_vp, _i32, _i64]),
    ("fpta_multi_synth", _c_int, [_vp, _u64, _i64, _i64, _i32, _vp]),
    ("fpta_multi_set_gather", _c_int, [_vp, _i32]),
    ("fpta_multi_last_gather", _c_int, [_vp]),
    ("fpta_comm_unique_id", _c_int, [_vp]),
    ("fpta_comm_init_rank", _c_int, [_ctx_p, _i32, _i32, _vp, ctypes.POINTER(_vp)]),
    ("fpta_comm_destroy", _c_int, [_vp]),
    ("fpta_comm_last_error", ctypes.c_char_p, [_vp]),
    ("fpta_comm_size", _c_int, [_vp, ctypes.POINTER(_i32), ctypes.POINTER(_i32)]),
    ("fpta_comm_max", _c_int, [_vp, ctypes.POINTER(_dbl)]),
    ("fpta_comm_gather", _c_int, [_vp, _vp, _i64, _vp]),
]
# entry points newer than an older library a same-box A/B may load through FAKEPTA_AMD_LIB (tools/gpu_ab_cfg.sh LIB=):
# bound when present (the product library exports every one: tests/test_capi_symbols.py)
_OPTIONAL = {"fpta_debug_normals"}
for _name, _res, _args in _SIGS:
    try:
        _fn = getattr(_lib, _name)
    except AttributeError:
        if _name in _OPTIONAL and LIB_PATH != _DEFAULT_LIB:
            continue
        raise
    _fn.restype = _res
    _fn.argtypes = _args

EXPORTED = [s[0] for s in _SIGS]

OPT_SYNTH_PATH, OPT_MFMA_MIN_REAL, OPT_PROFILE, OPT_ANCHOR, OPT_VALU_VARIANT, OPT_FUSE_WHITE = 1, 2, 3, 4, 5, 6
OPT_GRID_WIDTH, OPT_GRID_SIGMA, OPT_GRID_MFMA, OPT_FUSE_CHECKSUMS = 7, 8, 9, 10
OPT_MIX_MFMA, OPT_OVERLAP, OPT_INTERP_LDS, OPT_GRID_COALESCE, OPT_INTERP_WS, OPT_SIDE_SPLIT = 11, 12, 13, 14, 15, 16
OPT_DFT_GEN, OPT_GEN_MIX, OPT_ASYNC_SUMS, OPT_PART_GROUP, OPT_INTERP_PSR, OPT_INTERP_WR = 17, 18, 19, 20, 21, 22
OPT_INTERP_FUSED, OPT_FUSED_WHITE, OPT_FUSED_NEXT_MIX = 23, 24, 25
OPTIONS = (OPT_SYNTH_PATH, OPT_MFMA_MIN_REAL, OPT_PROFILE, OPT_ANCHOR, OPT_VALU_VARIANT, OPT_FUSE_WHITE,
           OPT_GRID_WIDTH, OPT_GRID_SIGMA, OPT_GRID_MFMA, OPT_FUSE_CHECKSUMS, OPT_MIX_MFMA, OPT_OVERLAP,
           OPT_INTERP_LDS, OPT_GRID_COALESCE, OPT_INTERP_WS, OPT_SIDE_SPLIT, OPT_DFT_GEN, OPT_GEN_MIX,
           OPT_ASYNC_SUMS, OPT_PART_GROUP, OPT_INTERP_PSR, OPT_INTERP_WR, OPT_INTERP_FUSED, OPT_FUSED_WHITE,
           OPT_FUSED_NEXT_MIX)
K_GEN, K_MIX, K_SYNTH, K_WHITE, K_DENSE, K_GRID = 0, 1, 2, 3, 4, 5


def interp_kernel_name(code):
    """The gridded interpolation kernel of the last block (fpta_batch_grid_info_n slot 15: 1 + 4 kind + 2 white +
    partial checksums), as rocprofv3 names it; None before any gridded block."""
    if code <= 0:
        return None
    kind, white, part = (code - 1) >> 2, "true" if (code - 1) & 2 else "false", "true" if (code - 1) & 1 else "false"
    if kind >= INTERP_KIND_FUSED0:  # launch_grid_fused's / launch_grid_fused_w's instance tables
        i = kind - INTERP_KIND_FUSED0
        return FUSED_KERNELS[i] if i < len(FUSED_KERNELS) else None
    return {0: f"k_grid_interp_mfma<{white}, {part}, 8>", 1: f"k_grid_interp_ws<{part}>",
            2: f"k_grid_interp_ws2<{part}>", 3: f"k_grid_interp_lds<{white}, {part}>",
            4: f"k_grid_interp_st<{white}, {part}>", 5: f"k_grid_interp_u<{part}>",
            6: f"k_grid_interp_psr<{part}, 4>", 7: f"k_grid_interp_psr<{part}, 8>",
            10: "k_grid_interp_wr"}.get(kind)


# k_grid_fused<NQ, ODD, GEN, HALF> instances in launch_grid_fused's order (capi_host.h kInterpKindFused0 + index)
INTERP_KIND_FUSED0 = 11
FUSED_KERNELS = tuple(f"k_grid_fused<{nq}, {odd}, {gen}, {half}>" for nq, half in ((8, "false"), (12, "false"), (8, "true"))
                      for odd, gen in (("false", "false"), ("false", "true"), ("true", "true"))) + \
    ("k_grid_fused_w<16, false>", "k_grid_fused_w<16, true>")
BUILD_DEBUG, BUILD_DIAG = 1, 2
GATHER_AUTO, GATHER_RCCL, GATHER_HOST = 0, 1, 2
COMM_ID_BYTES = 128


def build_flags():
    """FPTA_BUILD_DEBUG (1) when the loaded library is the debug build (make debug), FPTA_BUILD_DIAG (2) when it
    holds the diagnostic kernels (make variant DEFS=-DFPTA_DIAG_KERNELS)."""
    return int(_lib.fpta_build_flags())


class FptaError(RuntimeError):
    pass


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _ptr(a):
    return None if a is None else a.ctypes.data_as(_vp)


class Context:
    """One device context (one GPU, one HIP stream). Not thread-safe: one per thread/process."""

    def __init__(self, device=0):
        h = _ctx_p()
        rc = _lib.fpta_create(int(device), ctypes.byref(h))
        if rc != 0:
            raise FptaError(f"fpta_create(device={device}) failed ({rc}): "
                            f"{_lib.fpta_last_error(None).decode()}")
        self._h = h
        self.device = device

    def close(self):
        if getattr(self, "_h", None):
            _lib.fpta_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc < 0:
            raise FptaError(f"{what} failed ({rc}): {_lib.fpta_last_error(self._h).decode()}")
        return rc

    # --------------------------------------------------------------- drop-in
    def gp_accumulate(self, toas, nu, segments, residuals, sign=1.0, masks=None):
        """segments: list of (f, ccos, csin, idx, freqf). residuals: float64 array updated in place."""
        toas, nu = _f64(toas), _f64(nu)
        n = len(toas)
        assert residuals.dtype == np.float64 and residuals.flags.c_contiguous and len(residuals) == n
        nm = np.array([len(s[0]) for s in segments], dtype=np.int32)
        f = _f64(np.concatenate([np.asarray(s[0], float) for s in segments]))
        cc = _f64(np.concatenate([np.asarray(s[1], float) for s in segments]))
        cs = _f64(np.concatenate([np.asarray(s[2], float) for s in segments]))
        idx = _f64([s[3] for s in segments])
        ff = _f64([s[4] for s in segments])
        m = None
        if masks is not None and any(x is not None for x in masks):
            m = np.ones((len(segments), n), dtype=np.uint8)
            for i, x in enumerate(masks):
                if x is not None:
                    m[i] = np.asarray(x, dtype=bool)
        self._check(_lib.fpta_gp_accumulate(self._h, n, _ptr(toas), _ptr(nu), len(segments), _ptr(nm), _ptr(f),
                                            _ptr(cc), _ptr(cs), _ptr(idx), _ptr(ff), _ptr(m), float(sign),
                                            _ptr(residuals)), "fpta_gp_accumulate")

    # ------------------------------------------------------------------ dense covariance
    @staticmethod
    def _dense_args(toas, nu, segments, white_var):
        """segments: list of (f [N], w = psd * df [N], idx, freqf)."""
        toas, nu = _f64(toas), _f64(nu)
        n = len(toas)
        assert len(nu) == n and len(segments) > 0
        nm = np.array([len(s[0]) for s in segments], dtype=np.int32)
        for s in segments:
            assert len(s[1]) == len(s[0])
        f = _f64(np.concatenate([np.asarray(s[0], float) for s in segments]))
        w = _f64(np.concatenate([np.asarray(s[1], float) for s in segments]))
        idx = _f64([s[2] for s in segments])
        ff = _f64([s[3] for s in segments])
        wv = None if white_var is None else _f64(white_var)
        if wv is not None:
            assert len(wv) == n
        keep = (toas, nu, nm, f, w, idx, ff, wv)
        args = (n, _ptr(toas), _ptr(nu), len(segments), _ptr(nm), _ptr(f), _ptr(w), _ptr(idx), _ptr(ff), _ptr(wv))
        return n, keep, args

    def gp_covariance(self, toas, nu, segments, white_var=None):
        """sum_s B_s diag(psd df) B_s^T (+ diag(white_var)) as a [n, n] float64 array."""
        n, keep, args = self._dense_args(toas, nu, segments, white_var)
        cov = np.empty((n, n), dtype=np.float64)
        self._check(_lib.fpta_gp_covariance(self._h, *args, _ptr(cov)), "fpta_gp_covariance")
        del keep
        return cov

    def noise_wiener(self, toas, nu, segments, white_var, residuals):
        """red_cov C^-1 residuals with C = red_cov + diag(white_var) (device Cholesky)."""
        n, keep, args = self._dense_args(toas, nu, segments, white_var)
        r = _f64(residuals)
        assert len(r) == n
        out = np.empty(n, dtype=np.float64)
        self._check(_lib.fpta_noise_wiener(self._h, *args, _ptr(r), _ptr(out)), "fpta_noise_wiener")
        del keep
        return out

    def noise_draw(self, toas, nu, segments, white_var, seed, real0, n_real):
        """[n_real, n] draws of N(0, red_cov + diag(white_var)) (Philox stream, device Cholesky)."""
        n, keep, args = self._dense_args(toas, nu, segments, white_var)
        out = np.empty((n_real, n), dtype=np.float64)
        self._check(_lib.fpta_noise_draw(self._h, *args, int(seed) & 0xFFFFFFFFFFFFFFFF, int(real0), int(n_real),
                                         _ptr(out)), "fpta_noise_draw")
        del keep
        return out

    def gp_accumulate_array(self, offs, toas, nu, segments, residuals, sign=1.0, masks=None):
        """Array form: segments = list of (f [P, N], ccos [P, N], csin [P, N], idx, freqf);
        masks: None or list (per segment) of None / bool [n_toa_total]. residuals updated in place."""
        offs = np.ascontiguousarray(offs, dtype=np.int64)
        toas, nu = _f64(toas), _f64(nu)
        P, n = len(offs) - 1, int(offs[-1])
        assert residuals.dtype == np.float64 and residuals.flags.c_contiguous and len(residuals) == n
        for s in segments:
            assert np.shape(s[0]) == np.shape(s[1]) == np.shape(s[2]) and np.shape(s[0])[0] == P
        nm = np.array([np.shape(s[0])[1] for s in segments], dtype=np.int32)
        f = _f64(np.concatenate([np.asarray(s[0], float).ravel() for s in segments]))
        cc = _f64(np.concatenate([np.asarray(s[1], float).ravel() for s in segments]))
        cs = _f64(np.concatenate([np.asarray(s[2], float).ravel() for s in segments]))
        idx = _f64([s[3] for s in segments])
        ff = _f64([s[4] for s in segments])
        m = None
        if masks is not None and any(x is not None for x in masks):
            m = np.ones((len(segments), n), dtype=np.uint8)
            for i, x in enumerate(masks):
                if x is not None:
                    m[i] = np.asarray(x, dtype=bool)
        self._check(_lib.fpta_gp_accumulate_array(self._h, P, _ptr(offs), _ptr(toas), _ptr(nu), len(segments),
                                                  _ptr(nm), _ptr(f), _ptr(cc), _ptr(cs), _ptr(idx), _ptr(ff), _ptr(m),
                                                  float(sign), _ptr(residuals)), "fpta_gp_accumulate_array")

    def common_accumulate(self, offs, toas, nu, f, amp, idx, freqf, L, z, residuals, want_x=True):
        offs = np.ascontiguousarray(offs, dtype=np.int64)
        toas, nu, f, amp, L, z = map(_f64, (toas, nu, f, amp, L, z))
        P = len(offs) - 1
        N = len(f)
        assert z.shape == (N, 2, P) and L.shape == (P, P) and len(residuals) == offs[-1]
        x = np.empty((N, 2, P)) if want_x else None
        self._check(_lib.fpta_common_accumulate(self._h, P, _ptr(offs), _ptr(toas), _ptr(nu), N, _ptr(f), _ptr(amp),
                                                float(idx), float(freqf), _ptr(L), _ptr(z), _ptr(residuals),
                                                _ptr(x)), "fpta_common_accumulate")
        return x

    def white_accumulate(self, sigma, z, residuals, blocks=None, ecorr_sigma=None, zb=None):
        sigma, z = _f64(sigma), _f64(z)
        n = len(sigma)
        nb = 0
        bo = bi = es = zbb = None
        if blocks:
            nb = len(blocks)
            bo = np.concatenate([[0], np.cumsum([len(b) for b in blocks])]).astype(np.int64)
            bi = np.concatenate([np.asarray(b, dtype=np.int64) for b in blocks]).astype(np.int64)
            es, zbb = _f64(ecorr_sigma), _f64(zb)
        self._check(_lib.fpta_white_accumulate(self._h, n, _ptr(sigma), _ptr(z), nb, _ptr(bo), _ptr(bi), _ptr(es),
                                               _ptr(zbb), _ptr(residuals)), "fpta_white_accumulate")

    # --------------------------------------------------------------- batch
    def batch_set_toas(self, offs, toas, nu):
        offs = np.ascontiguousarray(offs, dtype=np.int64)
        toas, nu = _f64(toas), _f64(nu)
        self._check(_lib.fpta_batch_set_toas(self._h, len(offs) - 1, _ptr(offs), _ptr(toas), _ptr(nu)),
                    "fpta_batch_set_toas")

    def batch_add_signal(self, kind, f, amp, idx=0.0, freqf=1400.0, L=None, mask=None):
        f, amp = _f64(f), _f64(amp)
        nm = f.shape[-1]
        L = None if L is None else _f64(L)
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        return self._check(_lib.fpta_batch_add_signal(self._h, int(kind), nm, _ptr(f), _ptr(amp), float(idx),
                                                      float(freqf), _ptr(L), _ptr(m)), "fpta_batch_add_signal")

    def batch_set_white(self, sigma=None, blocks=None, ecorr_sigma=None):
        s = None if sigma is None else _f64(sigma)
        nb = 0
        bo = bi = es = None
        if blocks:
            nb = len(blocks)
            bo = np.concatenate([[0], np.cumsum([len(b) for b in blocks])]).astype(np.int64)
            bi = np.concatenate([np.asarray(b, dtype=np.int64) for b in blocks]).astype(np.int64)
            es = _f64(ecorr_sigma)
        self._check(_lib.fpta_batch_set_white(self._h, _ptr(s), nb, _ptr(bo), _ptr(bi), _ptr(es)),
                    "fpta_batch_set_white")

    def batch_clear(self):
        self._check(_lib.fpta_batch_clear_signals(self._h), "fpta_batch_clear_signals")

    def batch_info(self):
        info = np.zeros(5, dtype=np.int64)
        self._check(_lib.fpta_batch_info(self._h, _ptr(info)), "fpta_batch_info")
        return dict(n_psr=int(info[0]), n_toa=int(info[1]), n_seg=int(info[2]), K=int(info[3]), max_np=int(info[4]))

    def batch_grid_info(self):
        """Gridded-path plan figures, the path of the last batch and why it was not the gridded path
        (fpta_batch_grid_info_n, fpta_batch_path_reason)."""
        g = np.zeros(19, dtype=np.float64)
        self._check(_lib.fpta_batch_grid_info_n(self._h, _ptr(g), len(g)), "fpta_batch_grid_info_n")
        keys = ("last_path", "ok", "n_chunks", "fma_dft", "fma_interp", "fma_direct", "grid_vals", "weight_bytes",
                "grid_mfma", "err_bound", "width", "sigma", "grid_signals", "signals", "band_rows_per_chunk")
        # slot 16: the interpolation FMAs per realization as the last block's kernel ran them (half-chunk bands)
        fma_run = float(g[16])
        d = dict(zip(keys, g.tolist()))
        d["last_path"] = int(d["last_path"])
        d["ok"] = bool(d["ok"])
        d["grid_mfma"] = int(d["grid_mfma"])
        d["width"] = int(d["width"])
        d["grid_signals"] = int(d["grid_signals"])
        d["signals"] = int(d["signals"])
        d["path_reason"] = _lib.fpta_batch_path_reason(self._h).decode()
        d["interp_kernel"] = interp_kernel_name(int(g[15]))
        d["fma_interp_run"] = fma_run if fma_run > 0 else d["fma_interp"]
        # slots 17, 18: the last block's kernel made the next block's common-signal mix / the last block took its mix
        # from the previous block's kernel (FPTA_OPT_FUSED_NEXT_MIX)
        d["next_mix_made"] = bool(g[17])
        d["next_mix_used"] = bool(g[18])
        return d

    def batch_synth(self, seed, real0, n_real, to_host=True, coeffs=False):
        info = self.batch_info()
        out = np.empty((n_real, info["n_toa"])) if to_host else None
        co = np.empty((info["n_psr"], info["K"], n_real)) if coeffs else None
        self._check(_lib.fpta_batch_synth(self._h, int(seed) & 0xFFFFFFFFFFFFFFFF, int(real0), int(n_real), _ptr(out),
                                          _ptr(co)), "fpta_batch_synth")
        return (out, co) if coeffs else out

    def batch_synth_from_z(self, z):
        z = _f64(z)
        info = self.batch_info()
        n_real = z.shape[0]
        assert z.ndim == 5 and z.shape[1:3] == (info["n_seg"], info["n_psr"]) and z.shape[4] == 2
        out = np.empty((n_real, info["n_toa"]))
        self._check(_lib.fpta_batch_synth_from_z(self._h, n_real, z.shape[3], _ptr(z), _ptr(out)),
                    "fpta_batch_synth_from_z")
        return out

    def batch_download(self, r_begin, r_count):
        """Realizations [r_begin, r_begin + r_count) of the last block -> host [r_count, n_toa]."""
        _, ld, _ = self.batch_device_out()
        out = np.empty((r_count, ld))
        self._check(_lib.fpta_batch_download(self._h, int(r_begin), int(r_count), _ptr(out)), "fpta_batch_download")
        return out

    def batch_device_out(self):
        p, ld, nr = _vp(), _i64(), _i32()
        self._check(_lib.fpta_batch_device_out(self._h, ctypes.byref(p), ctypes.byref(ld), ctypes.byref(nr)),
                    "fpta_batch_device_out")
        return p.value, ld.value, nr.value

    def batch_correlations(self, mode=2):
        """0: [R, P, P] per realization; 1: [P, P] sum; 2: [P, P] sum of normalized; 3: [R, P] autos."""
        info = self.batch_info()
        _, _, R = self.batch_device_out()
        P = info["n_psr"]
        shape = {0: (R, P, P), 1: (P, P), 2: (P, P), 3: (R, P)}[mode]
        out = np.empty(shape)
        self._check(_lib.fpta_batch_correlations(self._h, int(mode), _ptr(out)), "fpta_batch_correlations")
        return out

    def batch_checksums(self):
        _, _, nr = self.batch_device_out()
        s = np.empty((nr, 2))
        self._check(_lib.fpta_batch_checksums(self._h, _ptr(s)), "fpta_batch_checksums")
        return s

    def batch_synth_checksums(self, seed, real0, n_real, batch=4096):
        """Realizations real0 .. real0 + n_real - 1 streamed in batches of <= batch with no host round trip in
        between; returns their checksums [n_real, 2] (fpta_batch_synth_checksums)."""
        out = np.empty((int(n_real), 2))
        self._check(_lib.fpta_batch_synth_checksums(self._h, int(seed) & 0xFFFFFFFFFFFFFFFF, int(real0), int(n_real),
                                                    int(batch), _ptr(out)), "fpta_batch_synth_checksums")
        return out

    # --------------------------------------------------------------- tuning / profiling
    def set_option(self, key, value):
        self._check(_lib.fpta_set_option(self._h, int(key), int(value)), "fpta_set_option")

    def get_option(self, key):
        v = _i64()
        self._check(_lib.fpta_get_option(self._h, int(key), ctypes.byref(v)), "fpta_get_option")
        return int(v.value)

    def options(self):
        """Snapshot of every option (restore with set_options)."""
        return {k: self.get_option(k) for k in OPTIONS}

    def set_options(self, opts):
        for k, v in opts.items():
            self.set_option(k, v)

    def kernel_stats(self, which):
        n, ms = _i64(), _dbl()
        self._check(_lib.fpta_kernel_stats(self._h, int(which), ctypes.byref(n), ctypes.byref(ms)),
                    "fpta_kernel_stats")
        return n.value, ms.value

    def reset_stats(self):
        self._check(_lib.fpta_reset_stats(self._h), "fpta_reset_stats")

    def synchronize(self):
        self._check(_lib.fpta_synchronize(self._h), "fpta_synchronize")

    def debug_fill_out(self, value):
        """Fill the last device block with `value` (tests: the next batch must overwrite every sample)."""
        self._check(_lib.fpta_debug_fill_out(self._h, float(value)), "fpta_debug_fill_out")

    def debug_philox(self, ctr, key):
        ctr = np.ascontiguousarray(ctr, dtype=np.uint32).reshape(-1, 4)
        key = np.ascontiguousarray(key, dtype=np.uint32)
        out = np.empty_like(ctr)
        self._check(_lib.fpta_debug_philox(self._h, len(ctr), _ptr(ctr), _ptr(key), _ptr(out)), "fpta_debug_philox")
        return out

    def debug_normals(self, words):
        """philox.h normals4 on the device for uint32 words [n, 4] -> float64 [n, 4] (oracle normals4)."""
        words = np.ascontiguousarray(words, dtype=np.uint32).reshape(-1, 4)
        out = np.empty(words.shape, dtype=np.float64)
        self._check(_lib.fpta_debug_normals(self._h, len(words), _ptr(words), _ptr(out)), "fpta_debug_normals")
        return out


class _Borrowed(Context):
    """A device context owned by a MultiContext (not destroyed by this wrapper). It keeps its parent alive and is
    invalidated when the parent closes, so a call on it never reaches a context fpta_multi_destroy has freed."""

    def __init__(self, handle, device, parent):
        self._h = handle
        self.device = device
        self._parent = parent

    def close(self):
        self._h = None

    def __getattribute__(self, name):
        if name not in ("_h", "_parent", "device", "close", "__class__", "__dict__") and not name.startswith("__"):
            parent = object.__getattribute__(self, "_parent")
            if object.__getattribute__(self, "_h") is None or getattr(parent, "_h", None) is None:
                raise FptaError("context of a closed MultiContext")
        return object.__getattribute__(self, name)


class MultiContext:
    """Several devices driven from one process (fpta_multi_*): the layout is replicated on each device,
    realizations are sharded contiguously over them and only per-realization checksums come back."""

    def __init__(self, devices):
        devs = np.ascontiguousarray(devices, dtype=np.int32)
        h = _vp()
        rc = _lib.fpta_multi_create(len(devs), _ptr(devs), ctypes.byref(h))
        if rc != 0:
            raise FptaError(f"fpta_multi_create({list(devs)}) failed ({rc}): {_lib.fpta_last_error(None).decode()}")
        self._h = h
        self.devices = [int(d) for d in devs]

    def _check(self, rc, what):
        if rc < 0:
            raise FptaError(f"{what} failed ({rc}): {_lib.fpta_multi_last_error(self._h).decode()}")
        return rc

    def close(self):
        if getattr(self, "_h", None):
            for b in getattr(self, "_borrowed", ()):
                b.close()
            _lib.fpta_multi_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self):
        return int(_lib.fpta_multi_size(self._h))

    def context(self, i):
        if not getattr(self, "_h", None):
            raise FptaError("MultiContext is closed")
        b = _Borrowed(_lib.fpta_multi_context(self._h, int(i)), self.devices[i], self)
        self.__dict__.setdefault("_borrowed", []).append(b)
        return b

    def set_toas(self, offs, toas, nu):
        offs = np.ascontiguousarray(offs, dtype=np.int64)
        toas, nu = _f64(toas), _f64(nu)
        self._check(_lib.fpta_multi_set_toas(self._h, len(offs) - 1, _ptr(offs), _ptr(toas), _ptr(nu)),
                    "fpta_multi_set_toas")

    def add_signal(self, kind, f, amp, idx=0.0, freqf=1400.0, L=None, mask=None):
        f, amp = _f64(f), _f64(amp)
        L = None if L is None else _f64(L)
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        return self._check(_lib.fpta_multi_add_signal(self._h, int(kind), f.shape[-1], _ptr(f), _ptr(amp),
                                                      float(idx), float(freqf), _ptr(L), _ptr(m)),
                           "fpta_multi_add_signal")

    def set_white(self, sigma=None, blocks=None, ecorr_sigma=None):
        s = None if sigma is None else _f64(sigma)
        nb, bo, bi, es = 0, None, None, None
        if blocks:
            nb = len(blocks)
            bo = np.concatenate([[0], np.cumsum([len(b) for b in blocks])]).astype(np.int64)
            bi = np.concatenate([np.asarray(b, dtype=np.int64) for b in blocks]).astype(np.int64)
            es = _f64(ecorr_sigma)
        self._check(_lib.fpta_multi_set_white(self._h, _ptr(s), nb, _ptr(bo), _ptr(bi), _ptr(es)),
                    "fpta_multi_set_white")

    def set_option(self, key, value):
        self._check(_lib.fpta_multi_set_option(self._h, int(key), int(value)), "fpta_multi_set_option")

    def set_gather(self, mode):
        """GATHER_AUTO (RCCL when the devices are distinct), GATHER_RCCL or GATHER_HOST (fpta_multi_set_gather)."""
        self._check(_lib.fpta_multi_set_gather(self._h, int(mode)), "fpta_multi_set_gather")

    def last_gather(self):
        """The route the last synth_checksums took: GATHER_RCCL or GATHER_HOST (0 before any)."""
        return int(_lib.fpta_multi_last_gather(self._h))

    def synth_checksums(self, seed, real0, n_real, batch=4096):
        """Per-realization (sum, sum of squares) of realizations real0 .. real0 + n_real - 1: [n_real, 2]."""
        out = np.empty((int(n_real), 2))
        self._check(_lib.fpta_multi_synth(self._h, int(seed) & 0xFFFFFFFFFFFFFFFF, int(real0), int(n_real),
                                          int(batch), _ptr(out)), "fpta_multi_synth")
        return out


class Comm:
    """RCCL communicator of one rank on one context (fpta_comm_*): the library's own RCCL on the kernels' HIP
    runtime. Rank 0 makes the unique id (Comm.unique_id()); every rank passes it to Comm(ctx, nranks, rank, uid)."""

    @staticmethod
    def unique_id():
        buf = ctypes.create_string_buffer(COMM_ID_BYTES)
        rc = _lib.fpta_comm_unique_id(ctypes.cast(buf, _vp))
        if rc != 0:
            raise FptaError(f"fpta_comm_unique_id failed ({rc}): {_lib.fpta_last_error(None).decode()}")
        return buf.raw

    def __init__(self, ctx, nranks, rank, uid):
        if len(uid) != COMM_ID_BYTES:
            raise ValueError(f"RCCL unique id must be {COMM_ID_BYTES} bytes")
        buf = ctypes.create_string_buffer(bytes(uid), COMM_ID_BYTES)
        h = _vp()
        rc = _lib.fpta_comm_init_rank(ctx._h, int(nranks), int(rank), ctypes.cast(buf, _vp), ctypes.byref(h))
        if rc != 0:
            raise FptaError(f"fpta_comm_init_rank(nranks={nranks}, rank={rank}) failed ({rc}): "
                            f"{_lib.fpta_last_error(ctx._h).decode()}")
        self._h = h
        self.ctx = ctx  # the communicator runs on ctx's device and stream: keep it alive
        self.nranks, self.rank = int(nranks), int(rank)

    def _check(self, rc, what):
        if rc != 0:
            raise FptaError(f"{what} failed ({rc}): {_lib.fpta_comm_last_error(self._h).decode()}")

    def max(self, x):
        v = _dbl(float(x))
        self._check(_lib.fpta_comm_max(self._h, ctypes.byref(v)), "fpta_comm_max")
        return float(v.value)

    def gather(self, arr):
        """Rank 0: every rank's float64 `arr` (same shape on every rank) stacked in rank order; others: None."""
        a = _f64(arr)
        out = np.empty((self.nranks,) + a.shape) if self.rank == 0 else None
        self._check(_lib.fpta_comm_gather(self._h, _ptr(a), a.size, _ptr(out)), "fpta_comm_gather")
        return out

    def close(self):
        if getattr(self, "_h", None):
            _lib.fpta_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_default = {}
_lock = threading.Lock()


def default_device():
    return int(os.environ.get("FAKEPTA_AMD_DEVICE", os.environ.get("LOCAL_RANK", "0")))


def get_context(device=None):
    """Process-wide context for the drop-in Pulsar methods (created on first use)."""
    dev = default_device() if device is None else int(device)
    with _lock:
        ctx = _default.get(dev)
        if ctx is None:
            ctx = Context(dev)
            _default[dev] = ctx
        return ctx


def device_count():
    n = _c_int()
    rc = _lib.fpta_device_count(ctypes.byref(n))
    return n.value if rc == 0 else 0
