"""Field-structured synthetic libfm data, numpy version.

The same generator is implemented on the device by the product library
(`vbfm_synth_generate`, csrc/vbfm_kernels.hip k_synth_*) so that bench-scale data (10^8 rows) can be
generated in HBM; the definition below is the specification both follow:

Two seeds: the ROW seed draws the rows (ids, x, noise); the MODEL seed (shared by the
train and test sets, and by every rank's shard) draws the planted model, so a model fitted
on train predicts test. R = row_offset + r is the global row id, so a rank generating rows
[R0, R0 + n) of a data set produces exactly that slice of the one-rank data set.

  h_s(stream, i) = splitmix64(s * K1 + stream * K2 + i)              (uint64, wrapping)
  u_s(stream, i) = (h_s(stream, i) >> 11) * 2^-53                    (fp64 in [0, 1))
  feature(R, f)  = f * S + h_row(1, R * F + f) % S                   (one id per field)
  x(R, f)        = 1.0f                                  if xmode == 0
                 = 0.5f + (h_row(2, R * F + f) >> 40) * 2^-24 (fp32) if xmode == 1
  b(j)           = (u_model(3, j) - 0.5) * c,  c = sqrt(12 / F)      (planted per-id bias,
                                                                      unit variance summed)
  p(j, d)        = u_model(5, 2 j + d) - 0.5, d = 0, 1               (planted rank-2 factors)
  s    = sum_f b(j_f);  s_d = sum_f p(j_f, d);  q_d = sum_f p(j_f, d)^2   (field order)
  t    = 0.5 * (s_0 * s_0 - q_0) + 0.5 * (s_1 * s_1 - q_1)           (= sum_{f<f'} <p_f, p_f'>)
  g    = sqrt(72 / (F (F - 1) / 2))  (F >= 2; 0 for F = 1: unit-variance interaction)
  y(R) = clamp(rint(((3 + s) + g * t) + 1.5 * (u_row(4, R) - 0.5)), 1, 5)

All fp64 operations in the order written, no fused multiply-add. Rows list their features
in field order, i.e. in ascending feature id.
"""
import numpy as np

K1 = np.uint64(0x9E3779B97F4A7C15)
K2 = np.uint64(0xD1B54A32D192ED03)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = z + K1
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def h(seed, stream, i):
    with np.errstate(over="ignore"):
        base = np.uint64(seed) * K1 + np.uint64(stream) * K2
        return splitmix64(base + np.asarray(i, dtype=np.uint64))


MODEL_SEED = 7      # the planted model every data set shares unless a test asks otherwise


def _u(seed, stream, i):
    return (h(seed, stream, i) >> np.uint64(11)).astype(np.float64) * 2.0 ** -53


def bias_gain(F):
    return float(np.sqrt(12.0 / F))


def interaction_gain(F):
    return float(np.sqrt(72.0 / (F * (F - 1) / 2.0))) if F >= 2 else 0.0


def generate(n_rows, n_fields, ids_per_field, seed, xmode=0, model_seed=MODEL_SEED, row_offset=0):
    """Return (row_ptr uint64[N+1], feat uint32[N*F], val float32[N*F], y float32[N])."""
    N, F, S = int(n_rows), int(n_fields), int(ids_per_field)
    idx = np.arange(N * F, dtype=np.uint64) + np.uint64(int(row_offset) * F)
    fld = (idx % np.uint64(F)).astype(np.uint64)
    feat = (fld * np.uint64(S) + h(seed, 1, idx) % np.uint64(S)).astype(np.uint32)
    if xmode:
        val = (np.float32(0.5) + (h(seed, 2, idx) >> np.uint64(40)).astype(np.float32)
               * np.float32(2.0 ** -24)).astype(np.float32)
    else:
        val = np.ones(N * F, dtype=np.float32)
    D = F * S
    jd = np.arange(D, dtype=np.uint64)
    b = (_u(model_seed, 3, jd) - 0.5) * bias_gain(F)
    p0 = _u(model_seed, 5, 2 * jd) - 0.5
    p1 = _u(model_seed, 5, 2 * jd + np.uint64(1)) - 0.5
    s = np.zeros(N, dtype=np.float64)
    s0, s1, q0, q1 = (np.zeros(N, dtype=np.float64) for _ in range(4))
    fe = feat.reshape(N, F)
    for f in range(F):            # summed in field order (the device generator does the same)
        j = fe[:, f]
        s = s + b[j]
        a0, a1 = p0[j], p1[j]
        s0 = s0 + a0
        s1 = s1 + a1
        q0 = q0 + a0 * a0
        q1 = q1 + a1 * a1
    t = 0.5 * (s0 * s0 - q0) + 0.5 * (s1 * s1 - q1)
    noise = _u(seed, 4, np.arange(N, dtype=np.uint64) + np.uint64(int(row_offset))) - 0.5
    y = np.clip(np.rint(((3.0 + s) + interaction_gain(F) * t) + 1.5 * noise), 1.0, 5.0).astype(np.float32)
    row_ptr = np.arange(N + 1, dtype=np.uint64) * np.uint64(F)
    return row_ptr, feat, val, y


def write_libfm(path, row_ptr, feat, val, y):
    """libfm text: '<y> <id>:<x> ...' with x printed to round-trip fp32 exactly."""
    with open(path, "w") as fh:
        for r in range(len(y)):
            b, e = int(row_ptr[r]), int(row_ptr[r + 1])
            parts = ["%.9g" % float(y[r])]
            parts += ["%d:%.9g" % (int(feat[j]), float(val[j])) for j in range(b, e)]
            fh.write(" ".join(parts) + "\n")


def csr_to_csc(n_rows, n_feature, row_ptr, feat, val):
    """Data::create_data_t order (ascending rows per column, file order within a row)."""
    nnz = len(feat)
    rows = np.repeat(np.arange(n_rows, dtype=np.uint32), np.diff(row_ptr.astype(np.int64)))
    order = np.argsort(feat, kind="stable")
    col_ptr = np.zeros(n_feature + 1, dtype=np.uint64)
    np.cumsum(np.bincount(feat, minlength=n_feature)[:n_feature], out=col_ptr[1:])
    assert int(col_ptr[-1]) == nnz
    return col_ptr, rows[order], val[order]


def write_binary(base, n_feature, row_ptr, feat, val, y):
    """Reference binary format (src/util/fmatrix.h:46-52,66-82; matrix.h:296-312):
    base.x (rows), base.xt (transposed), base.y (targets)."""
    N = len(y)
    nnz = len(feat)

    def write_sparse(path, nrows, ncols, ptr, ids, vals):
        with open(path, "wb") as fh:
            hdr = np.zeros(1, dtype=[("id", "<u4"), ("fs", "<u4"), ("nv", "<u8"),
                                     ("nr", "<u4"), ("nc", "<u4")])
            hdr["id"], hdr["fs"], hdr["nv"], hdr["nr"], hdr["nc"] = 2, 4, nnz, nrows, ncols
            fh.write(hdr.tobytes())
            ptr64 = ptr.astype(np.int64)
            sizes = np.diff(ptr64).astype(np.uint32)
            words = np.empty(nrows + 2 * len(ids), dtype="<u4")
            row_off = np.arange(nrows, dtype=np.int64) + 2 * ptr64[:-1]
            words[row_off] = sizes
            ent_row = np.repeat(np.arange(nrows, dtype=np.int64), sizes.astype(np.int64))
            ent_off = ent_row + 1 + 2 * np.arange(len(ids), dtype=np.int64)
            words[ent_off] = ids
            words[ent_off + 1] = np.asarray(vals, dtype="<f4").view("<u4")
            fh.write(words.tobytes())

    write_sparse(base + ".x", N, n_feature, row_ptr, feat, val)
    col_ptr, crow, cval = csr_to_csc(N, n_feature, row_ptr, feat, val)
    write_sparse(base + ".xt", n_feature, N, col_ptr, crow, cval)
    with open(base + ".y", "wb") as fh:
        fh.write(np.array([1, 4, N], dtype="<u4").tobytes())
        fh.write(y.astype("<f4").tobytes())


def field_csr_from_csc(n_rows, n_fields, ids_per_field, col_ptr, crow, cval):
    """The CSR (rows in field order) of one-hot field data from its CSC: row r holds exactly one
    id of every field, field f's at position r * F + f."""
    nf = len(col_ptr) - 1
    col = np.repeat(np.arange(nf, dtype=np.uint32), np.diff(col_ptr.astype(np.int64)))
    pos = crow.astype(np.int64) * n_fields + col // np.uint32(ids_per_field)
    feat = np.empty(n_rows * n_fields, dtype=np.uint32)
    val = np.empty(n_rows * n_fields, dtype=np.float32)
    feat[pos] = col
    val[pos] = cval
    del pos, col
    return np.arange(n_rows + 1, dtype=np.uint64) * np.uint64(n_fields), feat, val


def write_binary_csc(base, n_feature, row_ptr, feat, val, y, col_ptr, crow, cval):
    """write_binary with the transposed copy given (no sort: large samples)."""
    N, nnz = len(y), len(feat)

    def write_sparse(path, nrows, ncols, ptr, ids, vals):
        with open(path, "wb") as fh:
            hdr = np.zeros(1, dtype=[("id", "<u4"), ("fs", "<u4"), ("nv", "<u8"), ("nr", "<u4"), ("nc", "<u4")])
            hdr["id"], hdr["fs"], hdr["nv"], hdr["nr"], hdr["nc"] = 2, 4, nnz, nrows, ncols
            fh.write(hdr.tobytes())
            ptr64 = ptr.astype(np.int64)
            for r0 in range(0, nrows, 1 << 20):           # in row blocks: bounded temporaries
                r1 = min(nrows, r0 + (1 << 20))
                b, e = int(ptr64[r0]), int(ptr64[r1])
                sizes = np.diff(ptr64[r0:r1 + 1]).astype(np.uint32)
                words = np.empty((r1 - r0) + 2 * (e - b), dtype="<u4")
                row_off = np.arange(r1 - r0, dtype=np.int64) + 2 * (ptr64[r0:r1] - b)
                words[row_off] = sizes
                ent_row = np.repeat(np.arange(r1 - r0, dtype=np.int64), sizes.astype(np.int64))
                ent_off = ent_row + 1 + 2 * np.arange(e - b, dtype=np.int64)
                words[ent_off] = ids[b:e]
                words[ent_off + 1] = np.asarray(vals[b:e], dtype="<f4").view("<u4")
                fh.write(words.tobytes())

    write_sparse(base + ".x", N, n_feature, row_ptr, feat, val)
    write_sparse(base + ".xt", n_feature, N, col_ptr, crow, cval)
    with open(base + ".y", "wb") as fh:
        fh.write(np.array([1, 4, N], dtype="<u4").tobytes())
        fh.write(y.astype("<f4").tobytes())


def generate_multihot(n_rows, n_features, lo, hi, seed, xmode=0, model_seed=MODEL_SEED, row_offset=0):
    """Multi-hot rows without field structure (the device's vbfm_synth_multihot follows this):

      L(R)    = lo + h_row(6, R) % (hi - lo + 1)                        (lo <= L <= hi <= 64)
      id i    = a_i + h_row(7, 64 R + i) % (a_{i+1} - a_i),  a_i = floor(i D / L)
                (one id per stratum: distinct and ascending within the row)
      x       = 1.0f, or 0.5f + (h_row(2, 64 R + i) >> 40) * 2^-24 if xmode
      s, t    = as generate() over the row's ids, with the raw bias u_model(3, j) - 0.5
      y(R)    = clamp(rint(((3 + c_L s) + g_L t) + 1.5 (u_row(4, R) - 0.5)), 1, 5),
                c_L = sqrt(12 / L), g_L = interaction_gain(L)
    Return (row_ptr uint64[N+1], feat uint32[nnz], val float32[nnz], y float32[N])."""
    N, D = int(n_rows), int(n_features)
    R = np.arange(N, dtype=np.uint64) + np.uint64(int(row_offset))
    L = (np.uint64(lo) + h(seed, 6, R) % np.uint64(hi - lo + 1)).astype(np.int64)
    row_ptr = np.zeros(N + 1, dtype=np.uint64)
    np.cumsum(L, out=row_ptr[1:])
    nnz = int(row_ptr[-1])
    row = np.repeat(np.arange(N, dtype=np.int64), L)
    i = np.arange(nnz, dtype=np.int64) - row_ptr[:-1].astype(np.int64)[row]
    Lr = L[row]
    a = i * D // Lr
    e = (i + 1) * D // Lr
    key = R[row] * np.uint64(64) + i.astype(np.uint64)
    feat = (a.astype(np.uint64) + h(seed, 7, key) % (e - a).astype(np.uint64)).astype(np.uint32)
    if xmode:
        val = (np.float32(0.5) + (h(seed, 2, key) >> np.uint64(40)).astype(np.float32)
               * np.float32(2.0 ** -24)).astype(np.float32)
    else:
        val = np.ones(nnz, dtype=np.float32)
    j = feat.astype(np.uint64)
    b = _u(model_seed, 3, j) - 0.5
    p0 = _u(model_seed, 5, 2 * j) - 0.5
    p1 = _u(model_seed, 5, 2 * j + np.uint64(1)) - 0.5
    s = np.zeros(N)
    s0, s1, q0, q1 = (np.zeros(N) for _ in range(4))
    for k in range(int(L.max()) if N else 0):   # the k-th entry of every row, in row order (sequential sums)
        m = L > k
        idx = row_ptr[:-1].astype(np.int64)[m] + k
        s[m] = s[m] + b[idx]
        s0[m] = s0[m] + p0[idx]
        s1[m] = s1[m] + p1[idx]
        q0[m] = q0[m] + p0[idx] * p0[idx]
        q1[m] = q1[m] + p1[idx] * p1[idx]
    t = 0.5 * (s0 * s0 - q0) + 0.5 * (s1 * s1 - q1)
    cl = np.sqrt(12.0 / L)
    gl = np.array([interaction_gain(int(x)) for x in range(0, 65)])[L]
    noise = _u(seed, 4, R) - 0.5
    y = np.clip(np.rint(((3.0 + cl * s) + gl * t) + 1.5 * noise), 1.0, 5.0).astype(np.float32)
    return row_ptr, feat, val, y


ML_USERS, ML_ITEMS = 6040, 3952      # MovieLens-1M (BASELINE configs[1])


def generate_movielens(n_rows, seed, row_offset=0, model_seed=MODEL_SEED):
    """ML-1M-shaped rows (BASELINE configs[1]): a user uniform over 6,040 ids, an
    item over 3,952 ids with popularity ~ u^3 (a few items own tens of thousands of rows), x = 1,
    targets 1..5 from per-id biases of the planted model:

      user(R) = h_row(1, R) % 6040;  item(R) = 6040 + min(floor(u_row(2, R)^3 * 3952), 3951)
      y(R)    = clamp(rint(3 + 1.5 (b(user) + b(item)) + 1.5 (u_row(4, R) - 0.5)), 1, 5),
      b(j)    = u_model(3, j) - 0.5
    R = row_offset + r, as generate(): a rank's rows are a slice of the one-rank data set."""
    U, I = ML_USERS, ML_ITEMS
    idx = np.arange(row_offset, row_offset + n_rows, dtype=np.uint64)
    user = (h(seed, 1, idx) % np.uint64(U)).astype(np.uint32)
    u = _u(seed, 2, idx)
    item = (U + np.minimum((u ** 3 * I).astype(np.int64), I - 1)).astype(np.uint32)
    feat = np.stack([user, item], axis=1).reshape(-1)
    val = np.ones(2 * n_rows, dtype=np.float32)
    bu = _u(model_seed, 3, np.arange(U + I, dtype=np.uint64)) - 0.5
    y = np.clip(np.rint(3.0 + 1.5 * (bu[user] + bu[item]) + 1.5 * (_u(seed, 4, idx) - 0.5)), 1, 5)
    rp = np.arange(n_rows + 1, dtype=np.uint64) * np.uint64(2)
    return rp, feat, val, y.astype(np.float32)
