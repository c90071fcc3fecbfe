"""Numpy restatement of the reference GMAT hot path (TEST INFRASTRUCTURE ONLY).

Every function restates the arithmetic of the reference function it names (file:line
under /root/reference/gmat) so that tests can check the HIP product path against it on
the same inputs.  It is pinned against the golden fixtures in tests/golden/, which the
reference code itself produced (tests/golden/make_golden.py + oracle/ref_shim.py).

Never imported by the product package ``gmat_amd``.
"""
import numpy as np
from scipy.stats import chi2

# ----------------------------------------------------------------------------- PLINK


def decode_bed(bed_bytes, n_id, n_snp):
    """(c^2+c)/6 decode of every 2-bit code, SNP-major, low bits first
    (process_plink/_read_plink_bed.c:17-44): 00->0, 01->1/3 (missing), 10->1, 11->2.
    Skips the 3 header bytes without checking them (:31).  Returns (n_snp, n_id) float64."""
    raw = np.frombuffer(bed_bytes, dtype=np.uint8)[3:]
    nb = (n_id + 3) // 4
    raw = raw[: nb * n_snp].reshape(n_snp, nb)
    codes = np.stack([(raw >> (2 * k)) & 3 for k in range(4)], axis=-1).reshape(n_snp, nb * 4)[:, :n_id]
    c = codes.astype(np.float64)
    return (c * c + c) / 6.0


def read_plink(prefix):
    """read_plink (process_plink.py:7-9) as the survey shim defines it: n x m dosage
    matrix with NaN for missing (read_plink_bed.py:26)."""
    n = sum(1 for _ in open(prefix + ".fam"))
    m = sum(1 for _ in open(prefix + ".bim"))
    with open(prefix + ".bed", "rb") as f:
        mat = decode_bed(f.read(), n, m)
    mat[np.abs(mat - 1.0 / 3) < 0.0001] = np.nan
    return np.ascontiguousarray(mat.T)


def impute_geno(snp_mat):
    """impute_geno (process_plink.py:12-25): each NaN becomes a draw from the SNP's observed
    0/1/2 frequencies, columns visited in the order of set(np.where(isnan)[1]), one
    np.random.choice per column on the global RNG.  In place; returns snp_mat."""
    for i in set(np.where(np.isnan(snp_mat))[1]):
        col = snp_mat[:, i]
        c0 = np.sum(np.absolute(col - 0.0) < 1e-10)
        c1 = np.sum(np.absolute(col - 1.0) < 1e-10)
        c2 = np.sum(np.absolute(col - 2.0) < 1e-10)
        tot = c0 + c1 + c2
        na = np.where(np.isnan(col))
        col[na] = np.random.choice([0.0, 1.0, 2.0], len(na[0]), p=[c0 / tot, c1 / tot, c2 / tot])
        snp_mat[:, i] = col
    return snp_mat


# ----------------------------------------------------------------------------- GRM


def agmat(snp_mat, small_val=0.001):
    """gmatrix.py:52-66 (no missing data)."""
    n = snp_mat.shape[0]
    freq = np.sum(snp_mat, axis=0) / (2 * n)
    scale = np.sum(2 * freq * (1 - freq))
    x = snp_mat - 2 * freq
    kin = x @ x.T / scale
    d = np.diag(kin).copy()
    np.fill_diagonal(kin, d + d * small_val)
    return kin


def dgmat_as(snp_mat, small_val=0.001):
    """gmatrix.py:115-130: het indicator centred by 2p(1-p), scale sum(s(1-s))."""
    n = snp_mat.shape[0]
    freq = np.sum(snp_mat, axis=0) / (2 * n)
    s = 2 * freq * (1 - freq)
    scale = np.sum(s * (1 - s))
    h = snp_mat.copy()
    h[h > 1.5] = 0.0
    h = h - s
    kin = h @ h.T / scale
    d = np.diag(kin).copy()
    np.fill_diagonal(kin, d + d * small_val)
    return kin


def codings(snp_mat):
    """Centred additive / dominance codings used by the scans:
    A = g - 2p (remma_epiAA.py:57-61), D = [g!=2]g - 2p(1-p) (remma_epiDD.py:60-66,
    remma_epiAD.py:61-63).  Returns (A, D), both n x m."""
    n = snp_mat.shape[0]
    freq = np.sum(snp_mat, axis=0) / (2 * n)
    a = snp_mat - 2 * freq
    h = snp_mat.copy()
    h[h > 1.5] = 0.0
    d = h - 2 * freq * (1 - freq)
    return a, d


# ----------------------------------------------------------------------------- design


def design_matrix(pheno_file, bed_file):
    """design_matrix_wemai_multi_gmat (uvlmm/design_matrix.py:7-57).  Returns y (n,1),
    X (n,p), and the record->individual index (Z as an index vector) and n_id."""
    fam = []
    with open(bed_file + ".fam") as f:
        for line in f:
            a = line.split()
            fam.append(a[0] + " " + a[1])
    recs = {}
    with open(pheno_file) as f:
        for line in f:
            a = line.split()
            if a[-1] in ("NA", "NaN", "nan", "na"):
                continue
            recs.setdefault(a[0] + " " + a[1], []).append(a)
    missing = set(fam) - set(recs)
    if missing:
        raise ValueError("genotyped ids without phenotype: %s" % sorted(missing)[:5])
    y, x, iid = [], [], []
    for key in fam:
        for a in recs[key]:
            y.append(float(a[-1]))
            x.append([float(v) for v in a[2:-1]])
            iid.append(a[1])
    order = {}
    col = []
    for v in iid:
        if v not in order:
            order[v] = len(order)
        col.append(order[v])
    return (np.array(y).reshape(-1, 1), np.array(x, dtype=float).reshape(len(y), -1),
            np.array(col, dtype=np.int64), len(order))


def design_matrix_pred(pheno_file, bed_file):
    """design_matrix_wemai_multi_gmat_pred (uvlmm/design_matrix.py:60-113): genotyped ids
    without records keep an empty column of Z.  Same return convention as design_matrix."""
    fam = []
    with open(bed_file + ".fam") as f:
        for line in f:
            a = line.split()
            fam.append(a[0] + " " + a[1])
    recs = {}
    with open(pheno_file) as f:
        for line in f:
            a = line.split()
            if a[-1] in ("NA", "NaN", "nan", "na"):
                continue
            recs.setdefault(a[0] + " " + a[1], []).append(a)
    y, x, iid = [], [], []
    for key in fam:
        if key in recs:
            for a in recs[key]:
                y.append(float(a[-1]))
                x.append([float(v) for v in a[2:-1]])
                iid.append(a[1])
        else:
            iid.append("NA")
    order, col, ncol = {}, [], 0
    for v in iid:
        if v != "NA":
            if v not in order:
                order[v] = ncol
                ncol += 1
            col.append(order[v])
        else:
            ncol += 1
    return (np.array(y).reshape(-1, 1), np.array(x, dtype=float).reshape(len(y), -1),
            np.array(col, dtype=np.int64), ncol)


def predict_random(y, xmat, col, n_id, gmat_lst, var_com):
    """Random-effect prediction of wemai_multi_gmat_pred (uvlmm_varcom.py:147-165) exactly as
    written there (its 'P' is built from V, not V^-1)."""
    n = y.shape[0]
    v = np.diag([var_com[-1]] * n)
    for k, g in enumerate(gmat_lst):
        v += zgz(col, n_id, g) * var_com[k]
    vx = v @ xmat
    p = v - vx @ np.linalg.inv(xmat.T @ vx) @ vx.T
    zt = np.zeros((n_id, n))
    zt[col, np.arange(n)] = 1.0
    zpy = zt @ (p @ y)
    return np.concatenate([(g @ zpy) * var_com[k] for k, g in enumerate(gmat_lst)], axis=1)


def zgz(col, n_id, g):
    """Z G Z' for an incidence Z given as record->individual index (uvlmm_varcom.py:34)."""
    return g[np.ix_(col, col)]


# ----------------------------------------------------------------------------- REML


def wemai_multi_gmat(y, xmat, col, n_id, gmat_lst, init=None, maxiter=200, cc_par=1.0e-8,
                     cc_gra=1.0e-6, history=None):
    """Weighted EM-AI REML (uvlmm_varcom.py:8-104).  ``history`` (list) receives the
    variance vector after every iteration."""
    var = np.array([1.0] * (len(gmat_lst) + 1) if init is None else list(init), dtype=float)
    y = np.asarray(y, dtype=float).reshape(-1, 1)
    n = y.shape[0]
    xmat = np.asarray(xmat, dtype=float).reshape(n, -1)
    zg = [zgz(col, n_id, g) for g in gmat_lst]
    it = 0
    cc_gra_val = cc_par_val = 1000.0
    while it < maxiter:
        it += 1
        v = np.diag([var[-1]] * n)
        for k, g in enumerate(zg):
            v += g * var[k]
        vi = np.linalg.inv(v)
        vx = vi @ xmat
        xvx_i = np.linalg.inv(xmat.T @ vx)
        p = vi - vx @ xvx_i @ vx.T
        py = p @ y
        fd, wv = [], []
        for g in zg:
            fd.append(0.5 * float(np.sum(-np.trace(p @ g) + py.T @ g @ py)))
            wv.append(g @ py)
        fd.append(0.5 * float(np.sum(-np.trace(p) + py.T @ py)))
        fd = np.array(fd)
        wv.append(py)
        w = np.concatenate(wv, axis=1)
        ai = 0.5 * (w.T @ p @ w)
        em = np.diag(n / (var * var))
        for j in range(101):
            wt = j * 0.01
            delta = np.linalg.inv((1 - wt) * ai + wt * em) @ fd
            new = var + delta
            if min(new) > 0:
                break
        cc_par_val = np.sqrt(np.sum(delta * delta) / np.sum(new * new))
        var = new
        cc_gra_val = np.sqrt(np.sum(fd * fd))
        if history is not None:
            history.append(var.copy())
        if cc_gra_val < cc_gra and cc_par_val < cc_par:
            break
    return var


def projection(y, xmat, col, n_id, gmat_lst, var_com):
    """P-matrix setup of _remma_epiAA (remma_epiAA.py:33-49): returns (Z'PZ, Z'Py)."""
    y = np.asarray(y, dtype=float).reshape(-1, 1)
    n = y.shape[0]
    xmat = np.asarray(xmat, dtype=float).reshape(n, -1)
    v = np.diag([var_com[-1]] * n)
    for k, g in enumerate(gmat_lst):
        v += zgz(col, n_id, g) * var_com[k]
    vi = np.linalg.inv(v)
    vx = vi @ xmat
    p = vi - vx @ np.linalg.inv(xmat.T @ vx) @ vx.T
    zt = np.zeros((n_id, n))
    zt[col, np.arange(n)] = 1.0
    return zt @ p @ zt.T, zt @ (p @ y)


# ----------------------------------------------------------------------------- scans


def _stat(e, pvp, py):
    eff = e.T @ py
    var = np.sum(e * (pvp @ e), axis=0).reshape(-1, 1)
    with np.errstate(divide="ignore", invalid="ignore"):
        chi = eff * eff / var
    return eff[:, 0], var[:, 0], chi[:, 0], chi2.sf(chi[:, 0], 1)


def epi_scan(kind, snp_mat, pvp, py, snp_lst_0=None, p_cut=1e-5):
    """Exact epistasis scan.  AA: remma_epiAA.py:63-82 (j>i), DD: remma_epiDD.py:68-86
    (j>i, dominance coding), AD: remma_epiAD.py:66-87 (all j, i==j included).
    Returns rows (i, j, eff, chi, p) with p < p_cut in the reference's row order."""
    a, d = codings(snp_mat)
    m = snp_mat.shape[1]
    if kind == "AA":
        left, right, rows = a, a, range(m - 1) if snp_lst_0 is None else snp_lst_0
    elif kind == "DD":
        left, right, rows = d, d, range(m - 1) if snp_lst_0 is None else snp_lst_0
    elif kind == "AD":
        left, right, rows = a, d, range(m) if snp_lst_0 is None else snp_lst_0
    else:
        raise ValueError(kind)
    out = []
    for i in rows:
        j = np.arange(m) if kind == "AD" else np.arange(i + 1, m)
        e = left[:, i:i + 1] * right[:, j]
        eff, var, chi, p = _stat(e, pvp, py)
        keep = p < p_cut
        out.append(np.column_stack([np.full(keep.sum(), i), j[keep], eff[keep], chi[keep], p[keep]]))
    return np.concatenate(out) if out else np.zeros((0, 5))


def epi_pair(kind, snp_mat, pvp, py, pairs):
    """Pair-list test (remma_epiAA_pair.py:79-84 and the AD/DD siblings): returns
    (eff, var, chi, p) for every pair, in input order."""
    a, d = codings(snp_mat)
    left, right = {"AA": (a, a), "DD": (d, d), "AD": (a, d)}[kind]
    pairs = np.asarray(pairs, dtype=np.int64)
    e = left[:, pairs[:, 0]] * right[:, pairs[:, 1]]
    return _stat(e, pvp, py)


def parallel_rows(num_snp, parallel, kind="AA"):
    """Triangle-folded row split of _remma_epiAA_parallel (remma_epiAA.py:125-139); for AD
    the first part extends to num_snp (remma_epiAD.py:134-140)."""
    n_part, k = parallel
    s = int(num_snp / (2 * n_part))
    p0, p1 = (k - 1) * s, k * s
    p2, p3 = (2 * n_part - k) * s, (2 * n_part - k + 1) * s
    if k == 1:
        p3 = num_snp if kind == "AD" else num_snp - 1
    return list(range(p0, p1)) + list(range(p2, p3))


def format_rows(rows, n_float):
    """Rows as the reference writes them (pandas to_csv: ints, then repr floats)."""
    lines = []
    for r in rows:
        lines.append(" ".join([str(int(r[0])), str(int(r[1]))] + [repr(float(v)) for v in r[2:2 + n_float]]))
    return lines


def annotation_snp_pos(res_lines, bim_lines, p_cut=1, dis=0):
    """annotation.py:22-73 without the LD filter: header rewrite + row filter."""
    info = [" ".join(line.split()) for line in bim_lines]
    hdr = res_lines[0].split()
    out = [" ".join([hdr[0], "snp0_chr", "snp0_ID", "snp0_cm", "snp0_bp", "snp0_allele1", "snp0_allele2",
                     hdr[1], "snp1_chr", "snp1_ID", "snp1_cm", "snp1_bp", "snp1_allele1", "snp1_allele2"])
           + " " + " ".join(hdr[2:])]
    for line in res_lines[1:]:
        a = line.split()
        s0 = info[int(a[0])].split()
        s1 = info[int(a[1])].split()
        if float(a[-1]) <= p_cut and (s0[0] != s1[0] or abs(float(s0[3]) - float(s1[3])) > dis):
            out.append(" ".join([a[0], info[int(a[0])], a[1], info[int(a[1])]]) + " " + " ".join(a[2:]))
    return out


def ld_filter(anno_lines, ld_lines, r2=0.2):
    """LD filter of annotation_snp_pos (annotation.py:57-73): drop annotated rows whose SNP id
    pair (columns 2 and 9) is listed in the LD file (ids in columns 2 and 5, r2 last, header
    skipped) with r2 above the cut, in either order."""
    ld = set()
    for line in ld_lines[1:]:
        a = line.split()
        if float(a[-1]) > r2:
            ld.add((a[2], a[5]))
            ld.add((a[5], a[2]))
    out = [anno_lines[0]]
    for line in anno_lines[1:]:
        a = line.split()
        if (a[2], a[9]) not in ld:
            out.append(line)
    return out


def epi_eff_screen(kind, snp_mat_dec, py, rows, eff_cut, freq_i=None, freq_j=None):
    """Effect-only screen of the C kernel (_remma_epi_eff_cpu.c:61-137 AA, :226-314 AD,
    :415-491 DD) on a decoded (n_snp, n_id) matrix (missing = 1/3 kept, as the C code does).
    Returns a sorted list of (i, j, eff) with the reference's thresholds (AD: >= for (i,j),
    > for (j,i)).  With freq_i / freq_j (the _maf forms, :141-166, :318-348, :500-522) the
    threshold of (i, j) is eff_cut[freq_i[i]*10 + freq_j[j]] for both AD orientations."""
    m, n = snp_mat_dec.shape
    g = snp_mat_dec
    pf = np.zeros(m)
    for i in range(m):  # per-element division accumulation order of :103-109
        acc = 0.0
        for v in g[i]:
            acc += v / (2 * n)
        pf[i] = acc
    a = g - 2 * pf[:, None]
    h = np.where(np.abs(g - 2.0) < 0.0001, 0.0, g)
    d = h - (2 * pf * (1 - pf))[:, None]
    py = np.asarray(py, dtype=float).reshape(-1)
    table = np.asarray(eff_cut, dtype=float).reshape(-1)
    out = []
    for i in rows:
        js = np.arange(i + 1, m)
        eff_cut = table[np.asarray(freq_i)[i] * 10 + np.asarray(freq_j)[js]] if freq_i is not None else table[0]
        if kind == "AA":
            eff = (a[js] * a[i]) @ py
            keep = np.abs(eff) > eff_cut
            out += [(i, j, e) for j, e in zip(js[keep], eff[keep])]
        elif kind == "DD":
            eff = (d[js] * d[i]) @ py
            keep = np.abs(eff) > eff_cut
            out += [(i, j, e) for j, e in zip(js[keep], eff[keep])]
        else:
            e1 = (d[js] * a[i]) @ py
            e2 = (a[js] * d[i]) @ py
            k1 = np.abs(e1) >= eff_cut
            k2 = np.abs(e2) > eff_cut
            out += [(i, j, e) for j, e in zip(js[k1], e1[k1])]
            out += [(j, i, e) for j, e in zip(js[k2], e2[k2])]
    out.sort(key=lambda t: (t[0], t[1]))
    return out


def eff_screen_c(kind, bed_body, n, m, rows, py, cut, freq_i=None, freq_j=None, threads=None):
    """The C++/OpenMP restatement of the reference's effect screen (oracle/eff_cpu.cpp, same fp64
    operation order as _remma_epi_eff_cpu.c:61-574): records (i, j, eff) in the reference's
    single-thread order.  bed_body: the .bed bytes after the magic."""
    import ctypes
    import os
    lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "build", "libgmat_oracle_eff.so"))
    fn = lib.oracle_eff_screen
    P = ctypes.c_void_p
    fn.restype = ctypes.c_int64
    fn.argtypes = [ctypes.c_int, P, ctypes.c_int64, ctypes.c_int64, P, ctypes.c_int64, P, P, P, P, ctypes.c_int64, P,
                   P, P]
    if threads:
        os.environ["OMP_NUM_THREADS"] = str(threads)
    body = np.ascontiguousarray(np.frombuffer(bed_body, dtype=np.uint8))
    rows = np.ascontiguousarray(rows, dtype=np.int64)
    py = np.ascontiguousarray(py, dtype=np.float64).reshape(-1)
    cut = np.ascontiguousarray(np.atleast_1d(cut), dtype=np.float64)
    fi = None if freq_i is None else np.ascontiguousarray(freq_i, dtype=np.int64)
    fj = None if freq_j is None else np.ascontiguousarray(freq_j, dtype=np.int64)
    ptr = lambda a: None if a is None else a.ctypes.data  # noqa: E731
    kid = {"AA": 0, "AD": 1, "DD": 2}[kind]
    cap = 1 << 16
    while True:
        oi, oj, oe = np.zeros(cap, np.int64), np.zeros(cap, np.int64), np.zeros(cap)
        k = fn(kid, ptr(body), n, m, ptr(rows), rows.size, ptr(py), ptr(cut), ptr(fi), ptr(fj), cap, ptr(oi), ptr(oj),
               ptr(oe))
        if k <= cap:
            return oi[:k], oj[:k], oe[:k]
        cap = int(k)


def maf_classes(kind, snp_mat):
    """Frequency classes of the _maf_approx pipelines from the (n, m) dosage matrix:
    AA minor-allele frequency (remma_epiAA_maf_approx.py:38-41), DD heterozygosity
    (remma_epiDD_maf_approx.py:39-44), AD both (remma_epiAD_maf_approx.py:39-50).
    Returns (freq_i, freq_j) as int64 class arrays (value*20 truncated)."""
    n = snp_mat.shape[0]
    if kind == "AA":
        f = 1 - np.sum(snp_mat, axis=0) / (2 * n)
        f[f > 0.5] = 1 - f[f > 0.5]
        c = np.array(list(map(np.longlong, f * 20)), dtype=np.int64)
        return c, c
    h = np.sum(np.absolute(snp_mat - 1.0) < 0.001, axis=0) / n
    h[h > 0.5] = 1 - h[h > 0.5]
    hc = np.array(h * 20, dtype=np.int64)
    if kind == "DD":
        return hc, hc
    a = np.sum(snp_mat, axis=0) / (2 * n)
    a[a > 0.5] = 1 - a[a > 0.5]
    return np.array(a * 20, dtype=np.int64), hc


def class_denominators(kind, random_rows, freq_i, freq_j):
    """Per-class mean exact variance of random pairs (remma_epiAA_maf_approx.py:43-71; AD
    one orientation, remma_epiAD_maf_approx.py:51-75).  random_rows: (i, j, var) tuples in
    file order.  Returns the 111-entry denominator table."""
    sums, counts = {}, {}
    for i, j, v in random_rows:
        keys = [(freq_i[i], freq_j[j])] if kind == "AD" else [(freq_i[i], freq_i[j]), (freq_i[j], freq_i[i])]
        for k in keys:
            counts[k] = counts.get(k, 0) + 1
            sums[k] = sums.get(k, 0.0) + v
    tot, cnt = 0, 0
    for k in counts:
        tot += sums[k]
        cnt += counts[k]
        sums[k] = sums[k] / counts[k]
    mean = tot / cnt
    deno = np.ones(111)
    for k1 in set(freq_i.tolist()):
        for k2 in set(freq_j.tolist()):
            deno[k1 * 10 + k2] = sums.get((k1, k2), mean)
    return deno


def remma_single(kind, snp_mat, pvp, py, sigma):
    """Single-SNP tests: remma_add.py:49-60 (kind "add") and remma_dom.py:49-64 ("dom") on an
    (n, m) dosage matrix without missing values.  Returns (eff, chi, eff_to_fixed, p)."""
    n, m = snp_mat.shape
    freq = (np.sum(snp_mat, axis=0) / (2 * n)).reshape(1, m)
    if kind == "add":
        x = snp_mat - 2 * freq
        scale = np.sum(2 * freq * (1 - freq))
    else:
        s = 2 * freq * (1 - freq)
        scale = np.sum(s * (1 - s))
        x = snp_mat.copy()
        x[x > 1.5] = 0.0
        x = x - s
    py = np.asarray(py, dtype=float).reshape(-1, 1)
    with np.errstate(divide="ignore", invalid="ignore"):
        eff = np.dot(x.T, py)[:, -1] * sigma / scale
        var = np.sum(x * np.dot(pvp, x), axis=0) * sigma * sigma / (scale * scale)
        fixed = eff * sigma / (var * scale)
        chi = eff * eff / var
    return eff, chi, fixed, chi2.sf(chi, 1)
