"""vbfm -- Python host side of libvbfm.so (the MI355X VB factorization machine).

Mirrors the reference's learner interface for `-method vb` (FMLearnVB),
`-method vb_online` (FMLearnVBOnline) and `-method mcmc | als` (FMLearnMCMC) so that driver
code reads like
the reference's main() (src/libfm/libfm.cpp:137-511):

    train = DataSubset.load("train.libfm")            # Data::load          (Data.h:106-283)
    test = DataSubset.load("test.libfm")
    D = num_all_attribute(train, test)                 # libfm.cpp:215
    fml = FMLearnVB(k0=1, k1=1, num_factor=8, num_attribute=D,
                    min_target=train.min_target, max_target=train.max_target)
    fml.init(seed=42, init_stdev=0.1)                  # fm.init + fm_learn_vb::init draws
    for it, st in enumerate(fml.learn(train, test, num_iter=20)):   # _learn
        print(it, st.rmse, st.free_energy)

Every numeric step runs in libvbfm.so on the GPU. There is no CPU fallback: without the
built library (make -C scalable-variational-bayesian-factorization-machine_amd) or without
a HIP device every call raises.
"""
import ctypes as C
import os

import numpy as np

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("VBFM_LIB", os.path.join(_PKG, "lib", "libvbfm.so"))

P_u32, P_u64, P_f32, P_f64, P_u8 = (C.POINTER(C.c_uint32), C.POINTER(C.c_uint64), C.POINTER(C.c_float),
                                    C.POINTER(C.c_double), C.POINTER(C.c_uint8))


ABI_VERSION = 4        # VBFM_ABI_VERSION of include/vbfm.h this binding is written for
LAYOUTS = {"auto": 0, "column": 1, "level": 2, "entry": 3}   # VBFM_LAYOUT_* (include/vbfm.h)
SYNTH_MODEL_SEED = 7   # tests/synth.py MODEL_SEED: the planted model shared by train, test and all shards


class VbfmError(RuntimeError):
    pass


class Entry(C.Structure):
    _fields_ = [("id", C.c_uint32), ("value", C.c_float)]


ENTRY_DTYPE = np.dtype([("id", "<u4"), ("value", "<f4")])


class Csc(C.Structure):
    _fields_ = [("num_rows", C.c_uint32), ("num_feature", C.c_uint32), ("nnz", C.c_uint64),
                ("col_ptr", P_u64), ("col_ent", C.c_void_p), ("target", P_f32)]


class Config(C.Structure):
    _fields_ = [("k0", C.c_int32), ("k1", C.c_int32), ("num_factor", C.c_int32),
                ("num_attribute", C.c_uint32), ("num_attr_groups", C.c_uint32), ("attr_group", P_u32),
                ("min_target", C.c_float), ("max_target", C.c_float), ("device", C.c_int32),
                ("task", C.c_int32), ("place_candidates", C.c_int32), ("place_budget_bytes", C.c_uint64)]


class SetupStats(C.Structure):
    _fields_ = [("s_set_train", C.c_double), ("s_schedule", C.c_double), ("s_store", C.c_double),
                ("s_placement", C.c_double), ("place_bytes", C.c_uint64), ("place_candidates", C.c_int32),
                ("place_kept", C.c_int32 * 2)]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_}
        d["place_kept"] = list(self.place_kept)
        return d


class Params(C.Structure):
    _fields_ = [("mu_w", P_f64), ("sigma_w", P_f64), ("mu_v", P_f64), ("sigma_v", P_f64),
                ("hyp_sigma_w", P_f64), ("hyp_sigma_v", P_f64), ("alpha", C.c_double),
                ("sigma_0", C.c_double), ("mu_0_dash", C.c_double), ("sigma_0_dash", C.c_double)]


class ExchangeStats(C.Structure):
    """vbfm_exchange_stats: the last iteration's all-reduces (include/vbfm.h)."""
    _fields_ = [("transport", C.c_int32), ("n_timed", C.c_int32), ("n_calls", C.c_uint64), ("bytes", C.c_uint64),
                ("ms_timed", C.c_double), ("ms_estimated", C.c_double), ("timeout_s", C.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class IterStats(C.Structure):
    _fields_ = [("rmse", C.c_double), ("mae", C.c_double), ("train_quirk", C.c_double),
                ("free_energy", C.c_double), ("free_energy_valid", C.c_int32), ("num_levels", C.c_int32),
                ("alpha", C.c_double), ("sigma_0", C.c_double), ("mu_0_dash", C.c_double),
                ("sigma_0_dash", C.c_double),
                ("nan_mu_w", C.c_uint32), ("nan_sigma_w", C.c_uint32), ("inf_mu_w", C.c_uint32),
                ("nan_mu_v", C.c_uint32), ("nan_sigma_v", C.c_uint32), ("inf_mu_v", C.c_uint32),
                ("nan_alpha", C.c_uint32), ("inf_alpha", C.c_uint32),
                ("ms_w0", C.c_double), ("ms_w", C.c_double), ("ms_qcache", C.c_double), ("ms_v", C.c_double),
                ("ms_hyper", C.c_double), ("ms_test", C.c_double), ("ms_total", C.c_double),
                ("ms_vlevel_kernels", C.c_double), ("ms_wlevel_kernels", C.c_double),
                ("ms_qcache_kernels", C.c_double), ("n_vlevel_launches", C.c_int32),
                ("n_wlevel_launches", C.c_int32), ("n_qcache_launches", C.c_int32), ("nnz_train", C.c_uint64),
                ("ms_test_predict", C.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


RNG_REFERENCE, RNG_DEVICE = 0, 1


class McmcConfig(C.Structure):
    _fields_ = [("do_sample", C.c_int32), ("do_multilevel", C.c_int32), ("rng", C.c_int32), ("seed", C.c_uint32),
                ("init_stdev", C.c_double), ("regular", P_f64), ("num_regular", C.c_int32)]


class McmcParams(C.Structure):
    _fields_ = [("w", P_f64), ("v", P_f64), ("w_mu", P_f64), ("w_lambda", P_f64), ("v_mu", P_f64),
                ("v_lambda", P_f64), ("w0", C.c_double), ("alpha", C.c_double), ("reg0", C.c_double)]


class McmcStats(C.Structure):
    _fields_ = ([("rmse_all", C.c_double), ("mae_all", C.c_double), ("rmse_this", C.c_double),
                 ("mae_this", C.c_double), ("train_rmse", C.c_double), ("alpha", C.c_double), ("w0", C.c_double)]
                + [(n, C.c_uint32) for n in ("nan_alpha", "inf_alpha", "nan_w0", "inf_w0", "nan_w", "inf_w",
                                             "nan_v", "inf_v", "nan_w_mu", "inf_w_mu", "nan_w_lambda",
                                             "inf_w_lambda", "nan_v_mu", "inf_v_mu", "nan_v_lambda",
                                             "inf_v_lambda", "rng_skipped")]
                + [("num_levels", C.c_int32), ("ms_hyper", C.c_double), ("ms_w", C.c_double), ("ms_v", C.c_double),
                   ("ms_predict", C.c_double), ("ms_total", C.c_double), ("ms_vlevel_kernels", C.c_double),
                   ("n_vlevel_launches", C.c_int32), ("nnz_train", C.c_uint64)])

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


ONLINE_INIT_HOST, ONLINE_INIT_REPLAY = 0, 1


class OnlineConfig(C.Structure):
    _fields_ = [("num_batch", C.c_uint32), ("seed", C.c_uint32), ("init_stdev", C.c_double),
                ("init_mode", C.c_int32), ("fm_v", P_f64)]


class OnlineStats(C.Structure):
    _fields_ = ([("rmse", C.c_double), ("mae", C.c_double), ("free_energy_first", C.c_double),
                 ("free_energy_last", C.c_double), ("alpha", C.c_double), ("sigma_0", C.c_double),
                 ("mu_0_dash", C.c_double), ("sigma_0_dash", C.c_double)]
                + [(n, C.c_uint32) for n in ("nan_mu_w", "nan_sigma_w", "inf_mu_w", "nan_mu_v", "nan_sigma_v",
                                             "inf_mu_v", "nan_alpha", "inf_alpha", "num_batch")]
                + [("num_levels", C.c_int32), ("ms_regroup", C.c_double), ("ms_batches", C.c_double),
                   ("ms_test", C.c_double), ("ms_total", C.c_double), ("ms_predict", C.c_double),
                   ("ms_w0", C.c_double), ("ms_w", C.c_double), ("ms_v", C.c_double), ("ms_hyper", C.c_double),
                   ("n_vlevel_launches", C.c_uint32), ("nnz_train", C.c_uint64), ("n_lord_batches", C.c_uint32),
                   ("n_pad_batches", C.c_uint32)])

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class HostData(C.Structure):
    _fields_ = [("num_rows", C.c_uint32), ("num_feature", C.c_uint32), ("nnz", C.c_uint64),
                ("min_target", C.c_float), ("max_target", C.c_float), ("target", P_f32),
                ("row_ptr", P_u64), ("row_ent", C.c_void_p), ("col_ptr", P_u64), ("col_ent", C.c_void_p)]


# every symbol include/vbfm.h declares (checked by tests/test_capi_cpu.py)
EXPORTS = ["vbfm_abi_version", "vbfm_last_error", "vbfm_create", "vbfm_destroy", "vbfm_set_train",
           "vbfm_set_test", "vbfm_synth_generate", "vbfm_synth_multihot", "vbfm_get_csc", "vbfm_get_shape", "vbfm_get_levels",
           "vbfm_set_params", "vbfm_get_params", "vbfm_init_params_device", "vbfm_init_params_replay", "vbfm_init_caches", "vbfm_iterate", "vbfm_get_test_pred",
           "vbfm_step_w0", "vbfm_step_w", "vbfm_step_qcache", "vbfm_step_v", "vbfm_step_w_level",
           "vbfm_step_v_level", "vbfm_step_hyper", "vbfm_device_count",
           "vbfm_free_energy", "vbfm_get_rows", "vbfm_get_test_e", "vbfm_factor_sweep", "vbfm_set_profiling",
           "vbfm_set_layout", "vbfm_get_layout", "vbfm_set_shard_mode",
           "vbfm_comm_unique_id", "vbfm_comm_init", "vbfm_comm_init_host", "vbfm_comm_info", "vbfm_exchange_info", "vbfm_placement_info", "vbfm_setup_info", "vbfm_load_data", "vbfm_free_host_data", "vbfm_save_data",
           "vbfm_init_params_host", "vbfm_mcmc_init", "vbfm_mcmc_set_params", "vbfm_mcmc_get_params",
           "vbfm_mcmc_init_caches", "vbfm_mcmc_iterate", "vbfm_mcmc_get_test_pred", "vbfm_mcmc_factor_sweep",
           "vbfm_online_init", "vbfm_online_epoch", "vbfm_online_get_state", "vbfm_save_state", "vbfm_load_state"]

# vbfm_exchange_fn: int fn(void *user, void *buf, uint64_t count, int32_t dtype, int32_t op)
EXCHANGE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_int32, C.c_int32)
_X_DTYPES = {0: np.float64, 1: np.uint32, 2: np.uint8}

_lib = None


def lib():
    """Load libvbfm.so (raises if it is not built: there is no fallback path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise VbfmError("libvbfm.so not built (expected %s); run `make -C %s`" % (LIB_PATH, _PKG))
        L = C.CDLL(LIB_PATH)
        if L.vbfm_abi_version() != ABI_VERSION:   # struct layouts / argument lists differ otherwise
            raise VbfmError("libvbfm.so has ABI %d, this binding expects %d (rebuild: make -C %s)" % (
                L.vbfm_abi_version(), ABI_VERSION, _PKG))
        V = C.c_void_p
        L.vbfm_last_error.argtypes = [V]
        L.vbfm_last_error.restype = C.c_char_p
        L.vbfm_create.argtypes = [C.POINTER(V), C.POINTER(Config)]
        L.vbfm_destroy.argtypes = [V]
        L.vbfm_destroy.restype = None
        L.vbfm_set_train.argtypes = [V, C.POINTER(Csc)]
        L.vbfm_set_test.argtypes = [V, C.POINTER(Csc)]
        L.vbfm_synth_generate.argtypes = [V, C.c_int32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64, C.c_int32,
                                          C.c_uint64, C.c_uint64]
        L.vbfm_synth_multihot.argtypes = [V, C.c_int32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64,
                                          C.c_int32, C.c_uint64, C.c_uint64]
        L.vbfm_get_csc.argtypes = [V, C.c_int32, P_u64, V, P_f32]
        L.vbfm_get_shape.argtypes = [V, C.c_int32, P_u32, P_u32, P_u64]
        L.vbfm_get_levels.argtypes = [V, P_u32, P_u32]
        L.vbfm_set_params.argtypes = [V, C.POINTER(Params)]
        L.vbfm_get_params.argtypes = [V, C.POINTER(Params)]
        L.vbfm_init_caches.argtypes = [V]
        L.vbfm_init_params_device.argtypes = [V, C.c_uint64]
        L.vbfm_init_params_replay.argtypes = [V, C.c_uint32, C.c_double, P_f64, P_f64]
        L.vbfm_iterate.argtypes = [V, C.POINTER(IterStats)]
        L.vbfm_get_test_pred.argtypes = [V, P_f64]
        for fn in ("vbfm_step_w0", "vbfm_step_w"):
            getattr(L, fn).argtypes = [V]
        L.vbfm_step_qcache.argtypes = [V, C.c_int32]
        L.vbfm_step_v.argtypes = [V, C.c_int32]
        L.vbfm_step_w_level.argtypes = [V, C.c_int32]
        L.vbfm_step_v_level.argtypes = [V, C.c_int32, C.c_int32]
        L.vbfm_device_count.argtypes = [C.POINTER(C.c_int32)]
        L.vbfm_step_hyper.argtypes = [V, C.POINTER(C.c_int32)]
        L.vbfm_free_energy.argtypes = [V, P_f64]
        L.vbfm_get_rows.argtypes = [V, P_f64, P_f64, P_f64, P_f64, P_f64]
        L.vbfm_get_test_e.argtypes = [V, P_f64]
        L.vbfm_factor_sweep.argtypes = [V, P_f64]
        L.vbfm_set_profiling.argtypes = [V, C.c_int32]
        L.vbfm_set_layout.argtypes = [V, C.c_int32]
        L.vbfm_set_shard_mode.argtypes = [V, C.c_int32, C.c_int32]
        L.vbfm_get_layout.argtypes = [V, C.POINTER(C.c_int32)]
        L.vbfm_comm_unique_id.argtypes = [C.POINTER(C.c_uint8)]
        L.vbfm_comm_init.argtypes = [V, C.c_int32, C.c_int32, C.POINTER(C.c_uint8)]
        L.vbfm_comm_init_host.argtypes = [V, C.c_int32, C.c_int32, EXCHANGE_FN, V]
        L.vbfm_comm_info.argtypes = [V, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        L.vbfm_exchange_info.argtypes = [V, C.POINTER(ExchangeStats)]
        L.vbfm_placement_info.argtypes = [V, C.POINTER(C.c_float), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        L.vbfm_setup_info.argtypes = [V, C.POINTER(SetupStats)]
        L.vbfm_load_data.argtypes = [C.c_char_p, C.POINTER(HostData)]
        L.vbfm_free_host_data.argtypes = [C.POINTER(HostData)]
        L.vbfm_save_data.argtypes = [C.c_char_p, C.POINTER(HostData)]
        L.vbfm_free_host_data.restype = None
        L.vbfm_init_params_host.argtypes = [C.c_uint32, C.c_double, C.c_int32, C.c_uint32, C.c_uint32,
                                            C.POINTER(Params), P_f64, P_f64]
        L.vbfm_mcmc_init.argtypes = [V, C.POINTER(McmcConfig)]
        L.vbfm_mcmc_set_params.argtypes = [V, C.POINTER(McmcParams)]
        L.vbfm_mcmc_get_params.argtypes = [V, C.POINTER(McmcParams)]
        L.vbfm_mcmc_init_caches.argtypes = [V]
        L.vbfm_mcmc_iterate.argtypes = [V, C.POINTER(McmcStats)]
        L.vbfm_mcmc_get_test_pred.argtypes = [V, C.c_int32, P_f64]
        L.vbfm_mcmc_factor_sweep.argtypes = [V, P_f64]
        L.vbfm_online_init.argtypes = [V, C.POINTER(OnlineConfig)]
        L.vbfm_online_epoch.argtypes = [V, C.POINTER(OnlineStats)]
        L.vbfm_online_get_state.argtypes = [V, P_f64, P_f64, P_f64, P_f64, P_f64, P_f64, P_f64]
        L.vbfm_save_state.argtypes = [V, C.c_char_p, C.c_uint32]
        L.vbfm_load_state.argtypes = [V, C.c_char_p, C.POINTER(C.c_uint32)]
        _lib = L
    return _lib


def _check(rc, ctx=None):
    if rc != 0:
        msg = lib().vbfm_last_error(ctx)
        raise VbfmError(msg.decode() if msg else "libvbfm error %d" % rc)


def _ptr(a, typ):
    return a.ctypes.data_as(typ) if a is not None else None


def _copy(ptr, n, dtype):
    dtype = np.dtype(dtype)
    if n == 0:
        return np.zeros(0, dtype=dtype)
    addr = ptr if isinstance(ptr, int) else C.cast(ptr, C.c_void_p).value
    buf = (C.c_char * (n * dtype.itemsize)).from_address(addr)
    return np.frombuffer(buf, dtype=dtype).copy()


class DataSubset:
    """A data set as the learner sees it: transposed copy (CSC) + targets (Data.h:73-104)."""

    def __init__(self, col_ptr, col_ent, target, num_feature=None, row_ptr=None, row_ent=None):
        self.col_ptr = np.ascontiguousarray(col_ptr, dtype=np.uint64)
        self.col_ent = np.ascontiguousarray(col_ent, dtype=ENTRY_DTYPE)
        self.target = np.ascontiguousarray(target, dtype=np.float32)
        self.num_feature = int(len(self.col_ptr) - 1 if num_feature is None else num_feature)
        self.num_cases = int(len(self.target))
        self.row_ptr, self.row_ent = row_ptr, row_ent
        # Data.h:161-166 (std::min / std::max over fp32 targets)
        self.min_target = float(np.min(self.target)) if self.num_cases else 3.4028234663852886e38
        self.max_target = float(np.max(self.target)) if self.num_cases else -3.4028234663852886e38

    @classmethod
    def load(cls, filename):
        """Data::load via the library's host loader (libfm text, or .x/.xt/.y binary)."""
        h = HostData()
        _check(lib().vbfm_load_data(filename.encode(), C.byref(h)))
        try:
            n, nf, z = h.num_rows, h.num_feature, h.nnz
            ds = cls(_copy(h.col_ptr, nf + 1, np.uint64), _copy(h.col_ent, z, ENTRY_DTYPE),
                     _copy(h.target, n, np.float32), num_feature=nf,
                     row_ptr=_copy(h.row_ptr, n + 1, np.uint64), row_ent=_copy(h.row_ent, z, ENTRY_DTYPE))
            ds.min_target, ds.max_target = float(h.min_target), float(h.max_target)
        finally:
            lib().vbfm_free_host_data(C.byref(h))
        return ds

    @classmethod
    def from_csr(cls, row_ptr, feat, val, target, num_feature=None):
        """Build the transposed copy like Data::create_data_t (stable by feature)."""
        row_ptr = np.asarray(row_ptr, dtype=np.uint64)
        feat = np.asarray(feat, dtype=np.uint32)
        n = len(target)
        nf = int(feat.max()) + 1 if num_feature is None and len(feat) else int(num_feature or 0)
        rows = np.repeat(np.arange(n, dtype=np.uint32), np.diff(row_ptr.astype(np.int64)))
        order = np.argsort(feat, kind="stable")
        col_ptr = np.zeros(nf + 1, dtype=np.uint64)
        np.cumsum(np.bincount(feat, minlength=nf)[:nf], out=col_ptr[1:])
        ent = np.empty(len(feat), dtype=ENTRY_DTYPE)
        ent["id"] = rows[order]
        ent["value"] = np.asarray(val, dtype=np.float32)[order]
        return cls(col_ptr, ent, target, num_feature=nf)

    def save_binary(self, basename):
        """Write <basename>.x/.xt/.y in the reference's binary format (tools/convert +
        tools/transpose); DataSubset.load(basename) reads it back."""
        if self.row_ptr is None:
            raise VbfmError("save_binary needs the row copy (a data set from DataSubset.load)")
        rp = np.ascontiguousarray(self.row_ptr, dtype=np.uint64)
        re = np.ascontiguousarray(self.row_ent, dtype=ENTRY_DTYPE)
        h = HostData(self.num_cases, self.num_feature, len(self.col_ent), self.min_target, self.max_target,
                     _ptr(self.target, P_f32), _ptr(rp, P_u64), re.ctypes.data if len(re) else None,
                     _ptr(self.col_ptr, P_u64), self.col_ent.ctypes.data if len(self.col_ent) else None)
        _check(lib().vbfm_save_data(basename.encode(), C.byref(h)))

    def _csc(self):
        c = Csc(self.num_cases, self.num_feature, len(self.col_ent), _ptr(self.col_ptr, P_u64),
                self.col_ent.ctypes.data if len(self.col_ent) else None, _ptr(self.target, P_f32))
        return c


def num_all_attribute(train, test):
    """libfm.cpp:215"""
    return max(train.num_feature, test.num_feature) + 1


def num_all_attribute_online(train, test):
    """-method vb_online: find_max_feature leaves the largest feature ids in num_feature
    (libfm.cpp:167-170, 528-600), so num_attribute = largest id of train and test + 1."""
    return max(train.num_feature, test.num_feature)


def load_meta(filename, num_attribute):
    """DataMetaInfo::loadGroupsFromFile (Data.h:49-61): one group id per attribute."""
    g = np.loadtxt(filename, dtype=np.int64, ndmin=1)
    out = np.zeros(num_attribute, dtype=np.uint32)
    m = min(len(g), num_attribute)
    out[:m] = g[:m]
    return out


class FMLearnVB:
    """fm_learn_vb_simultaneous on one MI355X (src/libfm/src/fm_learn_vb_simultaneous.h)."""

    def __init__(self, k0=1, k1=1, num_factor=8, num_attribute=0, attr_group=None,
                 min_target=1.0, max_target=5.0, device=0, layout="auto", place_candidates=0,
                 place_budget_bytes=0):
        self.k0, self.k1, self.k, self.D = int(bool(k0)), int(bool(k1)), int(num_factor), int(num_attribute)
        self.attr_group = None if attr_group is None else np.ascontiguousarray(attr_group, dtype=np.uint32)
        self.G = 1 if self.attr_group is None else int(self.attr_group.max()) + 1 if self.D else 1
        # place_candidates / place_budget_bytes: the store's record-buffer placement search
        # (include/vbfm.h vbfm_config; 0 = the library's defaults, place_candidates=1: no search)
        cfg = Config(self.k0, self.k1, self.k, self.D, self.G, _ptr(self.attr_group, P_u32),
                     min_target, max_target, device, 0, int(place_candidates), int(place_budget_bytes))
        self._ctx = C.c_void_p()
        _check(lib().vbfm_create(C.byref(self._ctx), C.byref(cfg)))
        _check(lib().vbfm_set_layout(self._ctx, LAYOUTS[layout]), self._ctx)
        self.num_iter_done = 0
        self.fm_v = self.fm_w = None

    def set_shard_mode(self, mode, num_shards=0):
        """"rows" (exact row shards, default) or "features" (the north star's column
        partition, Jacobi across shards; num_shards > 1 without a communicator runs the
        shards one after another in this process). Before set_data / synth."""
        _check(lib().vbfm_set_shard_mode(self._ctx, {"rows": 0, "features": 1}[mode], int(num_shards)), self._ctx)

    def layout(self):
        """Row layout in use for the sweeps: "column" (row order, gather), "level" (records
        kept in the current level's column order, streamed) or "entry" (one slot per train
        entry, for levels that miss rows)."""
        v = C.c_int32()
        _check(lib().vbfm_get_layout(self._ctx, C.byref(v)), self._ctx)
        return {1: "column", 2: "level", 3: "entry"}[v.value]

    # -- parameters ---------------------------------------------------------------------
    def _params_struct(self, arrs):
        return Params(*[_ptr(arrs[k], P_f64) for k in ("mu_w", "sigma_w", "mu_v", "sigma_v",
                                                      "hyp_sigma_w", "hyp_sigma_v")],
                      arrs.get("alpha", 1.0), arrs.get("sigma_0", 1.0), arrs.get("mu_0_dash", 0.0),
                      arrs.get("sigma_0_dash", 0.02))

    def _empty_params(self):
        kd = self.k * self.D
        return {"mu_w": np.zeros(self.D), "sigma_w": np.zeros(self.D), "mu_v": np.zeros(kd),
                "sigma_v": np.zeros(kd), "hyp_sigma_w": np.zeros(self.G), "hyp_sigma_v": np.zeros(self.G * self.k)}

    def init(self, seed, init_stdev=0.1, keep_model_draws=False):
        """srand(seed); fm.init(); fm.w.init_normal(); fml->init() (libfm.cpp:123-366)."""
        p = self._empty_params()
        fm_v = np.zeros(self.k * self.D) if keep_model_draws else None
        fm_w = np.zeros(self.D) if keep_model_draws else None
        ps = self._params_struct(p)
        _check(lib().vbfm_init_params_host(seed, init_stdev, self.k, self.D, self.G, C.byref(ps),
                                           _ptr(fm_v, P_f64), _ptr(fm_w, P_f64)))
        for k in ("alpha", "sigma_0", "mu_0_dash", "sigma_0_dash"):
            p[k] = getattr(ps, k)
        self.fm_v, self.fm_w = fm_v, fm_w
        self.set_params(p)
        return p

    def init_replay(self, seed, init_stdev=0.1, keep_model_draws=False):
        """init() with the reference's stream generated on the device (vbfm_init_params_replay):
        the same parameters bit for bit, without the host's sequential draws."""
        fm_v = np.zeros(self.k * self.D) if keep_model_draws else None
        fm_w = np.zeros(self.D) if keep_model_draws else None
        _check(lib().vbfm_init_params_replay(self._ctx, seed, init_stdev, _ptr(fm_v, P_f64), _ptr(fm_w, P_f64)),
               self._ctx)
        self.fm_v, self.fm_w = fm_v, fm_w

    def init_device(self, seed):
        """Random init on the device (bench scale; not the reference's RNG stream)."""
        _check(lib().vbfm_init_params_device(self._ctx, seed), self._ctx)

    def set_params(self, p):
        full = self._empty_params()
        full.update({k: np.ascontiguousarray(v, dtype=np.float64) if isinstance(v, np.ndarray) else v
                     for k, v in p.items()})
        _check(lib().vbfm_set_params(self._ctx, C.byref(self._params_struct(full))), self._ctx)

    def get_params(self):
        p = self._empty_params()
        ps = self._params_struct(p)
        _check(lib().vbfm_get_params(self._ctx, C.byref(ps)), self._ctx)
        for k in ("alpha", "sigma_0", "mu_0_dash", "sigma_0_dash"):
            p[k] = getattr(ps, k)
        return p

    # -- data ---------------------------------------------------------------------------
    def set_train(self, train):
        """vbfm_set_train alone: the train set from host memory (DataSubset)."""
        self._train_csc = train._csc()
        _check(lib().vbfm_set_train(self._ctx, C.byref(self._train_csc)), self._ctx)
        self.n_train = train.num_cases

    def set_data(self, train, test):
        self._train_csc, self._test_csc = train._csc(), test._csc()
        _check(lib().vbfm_set_train(self._ctx, C.byref(self._train_csc)), self._ctx)
        _check(lib().vbfm_set_test(self._ctx, C.byref(self._test_csc)), self._ctx)
        self.n_train, self.n_test = train.num_cases, test.num_cases

    def synth(self, which, num_rows, n_fields, ids_per_field, seed, xmode=0, model_seed=SYNTH_MODEL_SEED,
              row_offset=0):
        """tests/synth.py's generator on the device: seed draws the rows, model_seed the
        planted model; rows [row_offset, row_offset + num_rows) of the one-rank data set."""
        _check(lib().vbfm_synth_generate(self._ctx, which, num_rows, n_fields, ids_per_field, seed, xmode,
                                         model_seed, row_offset), self._ctx)
        if which == 0:
            self.n_train = num_rows
        else:
            self.n_test = num_rows

    def synth_multihot(self, which, num_rows, num_features, lo, hi, seed, xmode=0, model_seed=SYNTH_MODEL_SEED,
                       row_offset=0):
        """tests/synth.py generate_multihot on the device (rows of lo..hi distinct ids, no fields)."""
        _check(lib().vbfm_synth_multihot(self._ctx, which, num_rows, num_features, lo, hi, seed, xmode, model_seed,
                                         row_offset), self._ctx)
        if which == 0:
            self.n_train = num_rows
        else:
            self.n_test = num_rows

    def shape(self, which):
        n, nf, z = C.c_uint32(), C.c_uint32(), C.c_uint64()
        _check(lib().vbfm_get_shape(self._ctx, which, C.byref(n), C.byref(nf), C.byref(z)), self._ctx)
        return n.value, nf.value, z.value

    def get_csc(self, which):
        n, nf, z = self.shape(which)
        cp = np.zeros(nf + 1, dtype=np.uint64)
        ent = np.zeros(z, dtype=ENTRY_DTYPE)
        tg = np.zeros(n, dtype=np.float32)
        _check(lib().vbfm_get_csc(self._ctx, which, _ptr(cp, P_u64), ent.ctypes.data if z else None,
                                  _ptr(tg, P_f32)), self._ctx)
        return cp, ent, tg

    def levels(self):
        nf = self.shape(0)[1]
        lv = np.zeros(nf, dtype=np.uint32)
        L = C.c_uint32()
        _check(lib().vbfm_get_levels(self._ctx, _ptr(lv, P_u32), C.byref(L)), self._ctx)
        return lv, L.value

    # -- learning -----------------------------------------------------------------------
    def init_caches(self):
        _check(lib().vbfm_init_caches(self._ctx), self._ctx)

    def iterate(self):
        st = IterStats()
        _check(lib().vbfm_iterate(self._ctx, C.byref(st)), self._ctx)
        self.num_iter_done += 1
        return st

    def learn(self, train, test, num_iter):
        """fm_learn_vb::learn -> _learn: yields the IterStats of every iteration."""
        self.set_data(train, test)
        self.init_caches()
        for _ in range(num_iter):
            yield self.iterate()

    def save_state(self, path, num_iter=None):
        """Checkpoint the learner between iterations (include/vbfm.h vbfm_save_state)."""
        it = self.num_iter_done if num_iter is None else num_iter
        _check(lib().vbfm_save_state(self._ctx, os.fsencode(path), int(it)), self._ctx)

    def load_state(self, path):
        """Resume from vbfm_save_state's file instead of init_caches; returns its iteration count."""
        it = C.c_uint32()
        _check(lib().vbfm_load_state(self._ctx, os.fsencode(path), C.byref(it)), self._ctx)
        self.num_iter_done = it.value
        return it.value

    def predict(self):
        """pred_this: clipped test predictions of the last iteration."""
        out = np.zeros(self.n_test)
        _check(lib().vbfm_get_test_pred(self._ctx, _ptr(out, P_f64)), self._ctx)
        return out

    def evaluate(self, data=None):
        """fm_learn_vb::evaluate returns NaN (fm_learn_vb.h:27)."""
        return float("nan")

    # -- update_all step by step --------------------------------------------------------
    def step_w0(self):
        _check(lib().vbfm_step_w0(self._ctx), self._ctx)

    def step_w(self):
        _check(lib().vbfm_step_w(self._ctx), self._ctx)

    def step_qcache(self, f):
        _check(lib().vbfm_step_qcache(self._ctx, f), self._ctx)

    def step_v(self, f):
        _check(lib().vbfm_step_v(self._ctx, f), self._ctx)

    def step_w_level(self, level):
        """Level `level` (0-based, in order) of the w sweep (vbfm_step_w_level)."""
        _check(lib().vbfm_step_w_level(self._ctx, level), self._ctx)

    def step_v_level(self, f, level):
        """Level `level` (0-based, in order) of factor f's v sweep (vbfm_step_v_level)."""
        _check(lib().vbfm_step_v_level(self._ctx, f, level), self._ctx)

    def step_hyper(self):
        e = C.c_int32()
        _check(lib().vbfm_step_hyper(self._ctx, C.byref(e)), self._ctx)
        return bool(e.value)

    def free_energy(self):
        F = C.c_double()
        _check(lib().vbfm_free_energy(self._ctx, C.byref(F)), self._ctx)
        return F.value

    def set_profiling(self, on=True, stride=1):
        """Event pairs around the sweep launches; stride > 1 times every stride-th launch of a kind."""
        _check(lib().vbfm_set_profiling(self._ctx, max(1, int(stride)) if on else 0), self._ctx)

    def factor_sweep(self):
        ms = C.c_double()
        _check(lib().vbfm_factor_sweep(self._ctx, C.byref(ms)), self._ctx)
        return ms.value

    def rows(self):
        n = self.n_train
        out = {k: np.zeros(n) for k in ("e", "t", "q", "tq", "tz")}
        _check(lib().vbfm_get_rows(self._ctx, *[_ptr(out[k], P_f64) for k in ("e", "t", "q", "tq", "tz")]),
               self._ctx)
        return out

    def test_e(self):
        out = np.zeros(self.n_test)
        _check(lib().vbfm_get_test_e(self._ctx, _ptr(out, P_f64)), self._ctx)
        return out

    # -- multi-GPU ----------------------------------------------------------------------
    @staticmethod
    def comm_unique_id():
        buf = (C.c_uint8 * 128)()
        _check(lib().vbfm_comm_unique_id(buf))
        return bytes(buf)

    def comm_init(self, nranks, rank, uid):
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        _check(lib().vbfm_comm_init(self._ctx, nranks, rank, buf), self._ctx)

    def comm_init_host(self, nranks, rank, allreduce):
        """Ranks exchange through the caller instead of RCCL (vbfm_comm_init_host): every
        all-reduce of the path calls allreduce(array, op) with a numpy view of the staged host
        buffer (float64 / uint32 / uint8), op "sum" or "max", to be reduced in place across the
        ranks -- e.g. a torch.distributed gloo all_reduce, so that several ranks can share one
        GPU in tests."""
        def _fn(user, buf, count, dtype, op):
            try:
                dt = _X_DTYPES[dtype]
                n = int(count)
                arr = np.ctypeslib.as_array(C.cast(buf, C.POINTER(np.ctypeslib.as_ctypes_type(dt))), shape=(n,)) \
                    if n else np.zeros(0, dt)
                allreduce(arr, "max" if op == 1 else "sum")
                return 0
            except Exception:  # reported to the library as a failed exchange
                import traceback
                traceback.print_exc()
                return 1
        self._xfn = EXCHANGE_FN(_fn)          # kept alive as long as the context
        _check(lib().vbfm_comm_init_host(self._ctx, nranks, rank, self._xfn, None), self._ctx)

    def comm_info(self):
        """(nranks, rank, transport) as the communicator reports them (vbfm_comm_info)."""
        n, r, t = C.c_int32(), C.c_int32(), C.c_int32()
        _check(lib().vbfm_comm_info(self._ctx, C.byref(n), C.byref(r), C.byref(t)), self._ctx)
        return n.value, r.value, {0: "none", 1: "rccl", 2: "host"}[t.value]

    def exchange_info(self):
        """The last iteration's all-reduces (vbfm_exchange_info): calls, payload bytes per rank,
        the timed ones' summed ms, their estimate over all calls, and the deadline in force."""
        st = ExchangeStats()
        _check(lib().vbfm_exchange_info(self._ctx, C.byref(st)), self._ctx)
        return st.as_dict()

    def placement(self):
        """(score in ms of each candidate record buffer, [indices of the two kept]) of the level
        store's placement tuning (vbfm_placement_info); ([], [-1, -1]) when none ran."""
        cap = 256
        buf = (C.c_float * cap)()
        n, k = C.c_int32(cap), (C.c_int32 * 2)()
        _check(lib().vbfm_placement_info(self._ctx, buf, C.byref(n), k), self._ctx)
        return [float(buf[i]) for i in range(min(n.value, cap))], [k[0], k[1]]

    def setup_info(self):
        """What setting up the train set cost (vbfm_setup_info): host seconds of the train set's
        hand-over, of the dependency levels and of the row store (the placement search included),
        and the search's peak device memory, candidates and kept pair."""
        st = SetupStats()
        _check(lib().vbfm_setup_info(self._ctx, C.byref(st)), self._ctx)
        return st.as_dict()

    def close(self):
        if self._ctx:
            lib().vbfm_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class FMLearnMCMC(FMLearnVB):
    """fm_learn_mcmc_simultaneous on one MI355X (src/libfm/src/fm_learn_mcmc_simultaneous.h).

    method "mcmc" samples with hyper-prior inference, "als" is the same learner with neither
    (libfm.cpp:131-135). rng=RNG_REFERENCE replays the reference's rand() stream (draws
    identical to the reference's on the same inputs), RNG_DEVICE draws the per-attribute
    normals from a counter-based generator on the device (bench scale)."""

    def __init__(self, k0=1, k1=1, num_factor=8, num_attribute=0, attr_group=None,
                 min_target=1.0, max_target=5.0, device=0, method="mcmc", layout="auto"):
        if method not in ("mcmc", "als"):
            raise VbfmError("method must be mcmc or als")
        super().__init__(k0, k1, num_factor, num_attribute, attr_group, min_target, max_target, device, layout)
        self.method = method

    def init(self, seed, init_stdev=0.1, regular=(), rng=RNG_REFERENCE):
        """srand(seed); fm.init(); fm.w.init_normal(); fml->init(); -regular (libfm.cpp:123-411)."""
        sample = 1 if self.method == "mcmc" else 0
        self._reg = np.ascontiguousarray(list(regular), dtype=np.float64)
        cfg = McmcConfig(sample, sample, rng, seed, init_stdev, _ptr(self._reg, P_f64) if len(self._reg) else None,
                         len(self._reg))
        _check(lib().vbfm_mcmc_init(self._ctx, C.byref(cfg)), self._ctx)

    def init_device(self, seed, init_stdev=0.1):
        self.init(seed, init_stdev, rng=RNG_DEVICE)

    def _mc_struct(self, arrs):
        return McmcParams(*[_ptr(arrs.get(k), P_f64) for k in ("w", "v", "w_mu", "w_lambda", "v_mu", "v_lambda")],
                          arrs.get("w0", 0.0), arrs.get("alpha", 1.0), arrs.get("reg0", 0.0))

    def get_params(self):
        p = {"w": np.zeros(self.D), "v": np.zeros(self.k * self.D), "w_mu": np.zeros(self.G),
             "w_lambda": np.zeros(self.G), "v_mu": np.zeros(self.G * self.k), "v_lambda": np.zeros(self.G * self.k)}
        ps = self._mc_struct(p)
        _check(lib().vbfm_mcmc_get_params(self._ctx, C.byref(ps)), self._ctx)
        p.update(w0=ps.w0, alpha=ps.alpha, reg0=ps.reg0)
        return p

    def set_params(self, p):
        cur = self.get_params()
        cur.update({k: np.ascontiguousarray(v, dtype=np.float64) if isinstance(v, np.ndarray) else v
                    for k, v in p.items()})
        _check(lib().vbfm_mcmc_set_params(self._ctx, C.byref(self._mc_struct(cur))), self._ctx)

    def init_caches(self):
        _check(lib().vbfm_mcmc_init_caches(self._ctx), self._ctx)

    def iterate(self):
        st = McmcStats()
        _check(lib().vbfm_mcmc_iterate(self._ctx, C.byref(st)), self._ctx)
        self.num_iter_done += 1
        return st

    def predict(self, num_iter=None):
        """fm_learn_mcmc::predict (fm_learn_mcmc.h:355-381)."""
        out = np.zeros(self.n_test)
        n = self.num_iter_done if num_iter is None else num_iter
        _check(lib().vbfm_mcmc_get_test_pred(self._ctx, n, _ptr(out, P_f64)), self._ctx)
        return out

    def factor_sweep(self):
        ms = C.c_double()
        _check(lib().vbfm_mcmc_factor_sweep(self._ctx, C.byref(ms)), self._ctx)
        return ms.value


class FMLearnVBOnline(FMLearnVB):
    """fm_learn_vb_online_simultaneous on one MI355X (src/libfm/src/fm_learn_vb_online.h,
    fm_learn_vb_online_simultaneous.h): OVBFM, mini-batch natural-gradient VB.

        fml = FMLearnVBOnline(1, 1, 8, num_all_attribute_online(train, test), ...)
        fml.set_data(train, test)
        fml.init(seed=42, init_stdev=0.1, num_batch=50)   # fm.init ... fml->init()
        for st in fml.epochs(20): print(st.rmse)           # _learn's loop
    """

    def __init__(self, k0=1, k1=1, num_factor=8, num_attribute=0, attr_group=None,
                 min_target=1.0, max_target=5.0, device=0):
        super().__init__(k0, k1, num_factor, num_attribute, attr_group, min_target, max_target, device,
                         layout="auto")

    def init(self, seed, init_stdev=0.1, num_batch=50, replay=False):
        """srand(seed); the VB learner's initial draws; fm_learn_vb_online::init (needs set_data first)."""
        cfg = OnlineConfig(num_batch, seed, init_stdev, ONLINE_INIT_REPLAY if replay else ONLINE_INIT_HOST, None)
        _check(lib().vbfm_online_init(self._ctx, C.byref(cfg)), self._ctx)
        self.num_batch = num_batch

    def epoch(self):
        st = OnlineStats()
        _check(lib().vbfm_online_epoch(self._ctx, C.byref(st)), self._ctx)
        self.num_iter_done += 1
        return st

    def epochs(self, num_iter):
        for _ in range(num_iter):
            yield self.epoch()

    def learn(self, train, test, num_iter, seed=1, init_stdev=0.1, num_batch=50):
        """fm_learn_vb_online::learn -> _learn: yields the OnlineStats of every epoch."""
        self.set_data(train, test)
        self.init(seed, init_stdev, num_batch)
        return self.epochs(num_iter)

    def iterate(self):
        return self.epoch()

    def init_caches(self):
        raise VbfmError("the online learner builds its caches per mini-batch (use epoch())")

    def online_state(self):
        D, kd = self.D, self.k * self.D
        out = {"nat_mu_w": np.zeros(D), "nat_sigma_w": np.zeros(D), "nat_mu_v": np.zeros(kd),
               "nat_sigma_v": np.zeros(kd), "new_wj": np.zeros(D), "new_vj": np.zeros(D), "scalars": np.zeros(8)}
        _check(lib().vbfm_online_get_state(self._ctx, *[_ptr(out[k], P_f64) for k in
                                                        ("nat_mu_w", "nat_sigma_w", "nat_mu_v", "nat_sigma_v",
                                                         "new_wj", "new_vj", "scalars")]), self._ctx)
        return out
