"""ctypes view of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY (the checker).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
"""
import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "liboracle.so")

P_u32, P_u64, P_f32, P_f64 = (C.POINTER(C.c_uint32), C.POINTER(C.c_uint64),
                              C.POINTER(C.c_float), C.POINTER(C.c_double))


class OrData(C.Structure):
    _fields_ = [("num_rows", C.c_uint32), ("num_feature", C.c_uint32), ("nnz", C.c_uint64),
                ("min_target", C.c_float), ("max_target", C.c_float), ("target", P_f32),
                ("row_ptr", P_u64), ("row_feat", P_u32), ("row_val", P_f32),
                ("col_ptr", P_u64), ("col_row", P_u32), ("col_val", P_f32)]


class OrVB(C.Structure):
    _fields_ = [("k0", C.c_int), ("k1", C.c_int), ("k", C.c_int), ("D", C.c_uint32), ("G", C.c_uint32),
                ("attr_group", P_u32), ("num_attr_per_group", P_u32),
                ("alpha", C.c_double), ("sigma_0", C.c_double), ("mu_0_dash", C.c_double),
                ("sigma_0_dash", C.c_double), ("sigma_w", P_f64), ("sigma_v", P_f64),
                ("mu_w", P_f64), ("sig_w", P_f64), ("mu_v", P_f64), ("sig_v", P_f64),
                ("fm_v", P_f64), ("fm_w", P_f64), ("n_train", C.c_uint32), ("n_test", C.c_uint32),
                ("e", P_f64), ("q", P_f64), ("t", P_f64), ("tq", P_f64), ("tz", P_f64),
                ("e_test", P_f64), ("q_test", P_f64), ("pred_test", P_f64),
                ("min_target", C.c_float), ("max_target", C.c_float),
                ("nan_mu_w", C.c_uint32), ("nan_sigma_w", C.c_uint32), ("inf_mu_w", C.c_uint32),
                ("nan_mu_v", C.c_uint32), ("nan_sigma_v", C.c_uint32), ("inf_mu_v", C.c_uint32),
                ("nan_alpha", C.c_uint32), ("inf_alpha", C.c_uint32),
                ("last_free_energy", C.c_double), ("hyper_skipped", C.c_int)]


class OrALS(C.Structure):
    _fields_ = [("k0", C.c_int), ("k1", C.c_int), ("k", C.c_int), ("D", C.c_uint32), ("G", C.c_uint32),
                ("attr_group", P_u32), ("num_attr_per_group", P_u32), ("w0", C.c_double),
                ("alpha", C.c_double), ("w", P_f64), ("v", P_f64), ("w_lambda", P_f64),
                ("v_lambda", P_f64), ("w_mu", P_f64), ("v_mu", P_f64),
                ("n_train", C.c_uint32), ("n_test", C.c_uint32), ("e", P_f64), ("q", P_f64),
                ("e_test", P_f64), ("q_test", P_f64), ("pred_sum_all", P_f64), ("pred_this", P_f64),
                ("min_target", C.c_float), ("max_target", C.c_float), ("iter_done", C.c_uint32),
                ("do_sample", C.c_int), ("do_multilevel", C.c_int), ("reg0", C.c_double),
                ("nan_w", C.c_uint32), ("inf_w", C.c_uint32), ("nan_v", C.c_uint32), ("inf_v", C.c_uint32),
                ("tmp_g", P_f64)]


class OrOVB(C.Structure):
    _fields_ = [("vb", OrVB), ("nat_mu_w", P_f64), ("nat_sig_w", P_f64), ("nat_mu_v", P_f64),
                ("nat_sig_v", P_f64), ("nat_mu0", C.c_double), ("nat_sig0", C.c_double),
                ("new_w0", C.c_double), ("lamda", C.c_double), ("new_wj", P_f64), ("new_vj", P_f64),
                ("t_wj", P_u32), ("t_vj", P_u32), ("t_w0", C.c_uint32), ("t0_w0", C.c_uint32),
                ("t0_wj", C.c_uint32), ("t0_vj", C.c_uint32), ("col_count", P_u32),
                ("num_batch", C.c_uint32), ("n_total", C.c_uint32), ("size_except_last", C.c_uint32),
                ("shuffle", P_u32), ("fe_first", C.c_double), ("fe_last", C.c_double),
                ("hyper_skipped_any", C.c_int)]


ALLREDUCE_FN = C.CFUNCTYPE(None, P_f64, C.c_int, C.c_void_p)

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("oracle not built: run `make -C oracle` (missing %s)" % LIB_PATH)
        L = C.CDLL(LIB_PATH)
        L.or_load_libfm.argtypes = [C.c_char_p, C.POINTER(OrData), C.c_char_p, C.c_int]
        L.or_data_from_csr.argtypes = [C.c_uint32, C.c_uint64, P_u64, P_u32, P_f32, P_f32, C.POINTER(OrData)]
        L.or_free_data.argtypes = [C.POINTER(OrData)]
        L.or_srand.argtypes = [C.c_uint32]
        L.or_rand.restype = C.c_int32
        L.or_ran_gaussian.restype = C.c_double
        L.or_vb_create.argtypes = [C.POINTER(OrVB), C.c_int, C.c_int, C.c_int, C.c_uint32, P_u32]
        L.or_vb_init_params.argtypes = [C.POINTER(OrVB), C.c_uint32, C.c_double]
        L.or_vb_attach.argtypes = [C.POINTER(OrVB), C.POINTER(OrData), C.POINTER(OrData)]
        L.or_vb_init_caches.argtypes = [C.POINTER(OrVB), C.POINTER(OrData), C.POINTER(OrData)]
        for fn in ("or_vb_update_w0", "or_vb_update_w_all", "or_vb_update_all"):
            getattr(L, fn).argtypes = [C.POINTER(OrVB), C.POINTER(OrData)]
        L.or_vb_hyper.argtypes = [C.POINTER(OrVB), C.POINTER(OrData)]
        L.or_vb_free_energy.argtypes = [C.POINTER(OrVB), C.POINTER(OrData)]
        L.or_vb_free_energy.restype = C.c_double
        L.or_vb_add_main_q.argtypes = [C.POINTER(OrVB), C.POINTER(OrData), C.c_int]
        L.or_vb_update_v_all.argtypes = [C.POINTER(OrVB), C.POINTER(OrData), C.c_int]
        L.or_vb_iterate.argtypes = [C.POINTER(OrVB), C.POINTER(OrData), C.POINTER(OrData),
                                    P_f64, P_f64, P_f64]
        L.or_vb_update_all_sharded.argtypes = [C.POINTER(OrVB), C.POINTER(OrData), C.c_uint32,
                                               C.c_uint32, ALLREDUCE_FN, C.c_void_p]
        L.or_vb_destroy.argtypes = [C.POINTER(OrVB)]
        L.or_vb_update_all_fsharded.argtypes = [C.POINTER(OrVB), C.POINTER(OrData), C.c_int,
                                                C.POINTER(C.c_int32)]
        L.or_als_create.argtypes = [C.POINTER(OrALS), C.c_int, C.c_int, C.c_int, C.c_uint32, P_u32]
        L.or_als_init_params.argtypes = [C.POINTER(OrALS), C.c_uint32, C.c_double]
        L.or_als_attach.argtypes = [C.POINTER(OrALS), C.POINTER(OrData), C.POINTER(OrData)]
        L.or_als_iterate.argtypes = [C.POINTER(OrALS), C.POINTER(OrData), C.POINTER(OrData),
                                     P_f64, P_f64, P_f64]
        L.or_als_destroy.argtypes = [C.POINTER(OrALS)]
        L.or_als_configure.argtypes = [C.POINTER(OrALS), C.c_int, C.c_int, C.c_double]
        L.or_ovb_create.argtypes = [C.POINTER(OrOVB), C.c_int, C.c_int, C.c_int, C.c_uint32, P_u32, C.c_uint32]
        L.or_ovb_destroy.argtypes = [C.POINTER(OrOVB)]
        L.or_ovb_init.argtypes = [C.POINTER(OrOVB), C.c_uint32, C.c_double, C.POINTER(OrData), C.POINTER(OrData)]
        L.or_ovb_epoch.argtypes = [C.POINTER(OrOVB), C.POINTER(OrData), C.POINTER(OrData), P_f64, P_f64]
        L.or_ran_gamma.argtypes = [C.c_double]
        L.or_ran_gamma.restype = C.c_double
        _lib = L
    return _lib


def arr(ptr, n, dtype=np.float64):
    """Copy n elements behind a ctypes pointer into a numpy array."""
    if n == 0:
        return np.zeros(0, dtype=dtype)
    return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dtype, copy=True)


class Data:
    """A libfm data set loaded by the oracle (Data::load restated)."""

    def __init__(self, path=None, csr=None):
        self.d = OrData()
        err = C.create_string_buffer(512)
        if path is not None:
            if lib().or_load_libfm(path.encode(), C.byref(self.d), err, 512) != 0:
                raise ValueError(err.value.decode())
        else:
            n_rows, row_ptr, feat, val, y = csr
            self._keep = [np.ascontiguousarray(row_ptr, np.uint64), np.ascontiguousarray(feat, np.uint32),
                          np.ascontiguousarray(val, np.float32), np.ascontiguousarray(y, np.float32)]
            rp, fe, va, ta = self._keep
            lib().or_data_from_csr(n_rows, len(fe), rp.ctypes.data_as(P_u64), fe.ctypes.data_as(P_u32),
                                   va.ctypes.data_as(P_f32), ta.ctypes.data_as(P_f32), C.byref(self.d))

    @property
    def num_rows(self):
        return self.d.num_rows

    @property
    def num_feature(self):
        return self.d.num_feature

    def csr(self):
        n, z = self.d.num_rows, self.d.nnz
        return (arr(self.d.row_ptr, n + 1, np.uint64), arr(self.d.row_feat, z, np.uint32),
                arr(self.d.row_val, z, np.float32), arr(self.d.target, n, np.float32))

    def csc(self):
        nf, z = self.d.num_feature, self.d.nnz
        return (arr(self.d.col_ptr, nf + 1, np.uint64), arr(self.d.col_row, z, np.uint32),
                arr(self.d.col_val, z, np.float32))

    def __del__(self):
        try:
            lib().or_free_data(C.byref(self.d))
        except Exception:
            pass


class VB:
    """Oracle VB learner (fm_learn_vb restated)."""

    def __init__(self, k0, k1, k, D, attr_group=None):
        self.s = OrVB()
        self._g = None if attr_group is None else np.ascontiguousarray(attr_group, np.uint32)
        lib().or_vb_create(C.byref(self.s), int(k0), int(k1), int(k), int(D),
                           None if self._g is None else self._g.ctypes.data_as(P_u32))

    def __getattr__(self, name):
        return getattr(self.s, name)

    def init_params(self, seed, init_stdev=0.1):
        lib().or_vb_init_params(C.byref(self.s), seed, init_stdev)

    def attach(self, train, test):
        self.train, self.test = train, test
        lib().or_vb_attach(C.byref(self.s), C.byref(train.d), C.byref(test.d))

    def init_caches(self):
        lib().or_vb_init_caches(C.byref(self.s), C.byref(self.train.d), C.byref(self.test.d))

    def step(self, name, *args):
        return getattr(lib(), "or_vb_" + name)(C.byref(self.s), C.byref(self.train.d), *args)

    def update_all_fsharded(self, shard):
        """libvbfm's feature-sharded update_all (shard[j] = owning shard of train feature j)."""
        sh = np.ascontiguousarray(shard, dtype=np.int32)
        lib().or_vb_update_all_fsharded(C.byref(self.s), C.byref(self.train.d), int(sh.max()) + 1 if sh.size else 1,
                                        sh.ctypes.data_as(C.POINTER(C.c_int32)))

    def iterate(self):
        r, m, t = C.c_double(), C.c_double(), C.c_double()
        lib().or_vb_iterate(C.byref(self.s), C.byref(self.train.d), C.byref(self.test.d),
                            C.byref(r), C.byref(m), C.byref(t))
        return r.value, m.value, t.value

    def rows(self):
        n = self.s.n_train
        return {k: arr(getattr(self.s, k), n) for k in ("e", "t", "q", "tq", "tz")}

    def params(self):
        s = self.s
        return {"mu_w": arr(s.mu_w, s.D), "sigma_w": arr(s.sig_w, s.D),
                "mu_v": arr(s.mu_v, s.k * s.D), "sigma_v": arr(s.sig_v, s.k * s.D),
                "hyp_sigma_w": arr(s.sigma_w, s.G), "hyp_sigma_v": arr(s.sigma_v, s.G * s.k),
                "scalars": np.array([s.alpha, s.sigma_0, s.mu_0_dash, s.sigma_0_dash])}

    def __del__(self):
        try:
            lib().or_vb_destroy(C.byref(self.s))
        except Exception:
            pass


class ALS:
    """fm_learn_mcmc: method "als" (no sampling, no hyper-prior inference) or "mcmc"."""

    def __init__(self, k0, k1, k, D, attr_group=None, method="als", reg0=0.0):
        self.s = OrALS()
        self._groups = None if attr_group is None else np.ascontiguousarray(attr_group, dtype=np.uint32)
        gp = None if self._groups is None else self._groups.ctypes.data_as(P_u32)
        lib().or_als_create(C.byref(self.s), int(k0), int(k1), int(k), int(D), gp)
        mc = method == "mcmc"
        lib().or_als_configure(C.byref(self.s), int(mc), int(mc), float(reg0))

    def set_lambda(self, w_lambda, v_lambda):
        """-regular (libfm.cpp:367-411): w_lambda[G], v_lambda[G*k] at [g*k + f]"""
        s = self.s
        for i, x in enumerate(np.asarray(w_lambda, dtype=np.float64).ravel()):
            s.w_lambda[i] = x
        for i, x in enumerate(np.asarray(v_lambda, dtype=np.float64).ravel()):
            s.v_lambda[i] = x

    def init_params(self, seed, init_stdev=0.1):
        lib().or_als_init_params(C.byref(self.s), seed, init_stdev)

    def attach(self, train, test):
        self.train, self.test = train, test
        lib().or_als_attach(C.byref(self.s), C.byref(train.d), C.byref(test.d))

    def iterate(self):
        a, t, tr = C.c_double(), C.c_double(), C.c_double()
        lib().or_als_iterate(C.byref(self.s), C.byref(self.train.d), C.byref(self.test.d),
                             C.byref(a), C.byref(t), C.byref(tr))
        return a.value, t.value, tr.value

    def params(self):
        s = self.s
        return {"w": arr(s.w, s.D), "v": arr(s.v, s.k * s.D), "w0": s.w0, "alpha": s.alpha,
                "w_mu": arr(s.w_mu, s.G), "w_lambda": arr(s.w_lambda, s.G),
                "v_mu": arr(s.v_mu, s.G * s.k), "v_lambda": arr(s.v_lambda, s.G * s.k)}

    def __del__(self):
        try:
            lib().or_als_destroy(C.byref(self.s))
        except Exception:
            pass


def num_all_attribute(train, test):
    """libfm.cpp:215"""
    return max(train.num_feature, test.num_feature) + 1


class OVB:
    """Oracle online VB learner (fm_learn_vb_online + _simultaneous::_learn restated)."""

    def __init__(self, k0, k1, k, D, num_batch, attr_group=None):
        self.s = OrOVB()
        self._g = None if attr_group is None else np.ascontiguousarray(attr_group, np.uint32)
        lib().or_ovb_create(C.byref(self.s), int(k0), int(k1), int(k), int(D),
                            None if self._g is None else self._g.ctypes.data_as(P_u32), int(num_batch))

    def init(self, seed, init_stdev, train, test):
        self.train, self.test = train, test
        lib().or_ovb_init(C.byref(self.s), seed, init_stdev, C.byref(train.d), C.byref(test.d))

    def epoch(self):
        r, m = C.c_double(), C.c_double()
        lib().or_ovb_epoch(C.byref(self.s), C.byref(self.train.d), C.byref(self.test.d), C.byref(r), C.byref(m))
        return r.value, m.value, self.s.fe_first, self.s.fe_last

    def params(self):
        v, s = self.s.vb, self.s
        kd = v.k * v.D
        return {"mu_w": arr(v.mu_w, v.D), "sigma_w": arr(v.sig_w, v.D), "mu_v": arr(v.mu_v, kd),
                "sigma_v": arr(v.sig_v, kd), "hyp_sigma_w": arr(v.sigma_w, v.G),
                "hyp_sigma_v": arr(v.sigma_v, v.G * v.k), "nat_mu_w": arr(s.nat_mu_w, v.D),
                "nat_sigma_w": arr(s.nat_sig_w, v.D), "nat_mu_v": arr(s.nat_mu_v, kd),
                "nat_sigma_v": arr(s.nat_sig_v, kd),
                "steps": np.concatenate([arr(s.new_wj, v.D), arr(s.new_vj, v.D)]),
                "scalars": np.array([v.alpha, v.sigma_0, v.mu_0_dash, v.sigma_0_dash, s.nat_mu0, s.nat_sig0,
                                     s.new_w0, float(s.t_w0)]),
                "pred": arr(v.pred_test, v.n_test)}

    def __del__(self):
        try:
            lib().or_ovb_destroy(C.byref(self.s))
        except Exception:
            pass
