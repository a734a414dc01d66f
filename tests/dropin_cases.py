"""Drop-in API checks against the reference's golden vectors, shared by the
GPU suite (tests/test_gpu_dropin.py: real kernels, every key size) and the
CPU suite (tests/test_dropin_host.py: the device calls replaced by the oracle
through tests/oracle_ops.py, so the host logic is covered without a GPU)."""
import pickle

import numpy as np

from tests.conftest import fl, hx, load_fixture


def ctxs(g):
    from xfl_amd.paillier import PaillierContext
    k = g["key"]
    h = hx(k["h_pow_n"]) if k["djn_on"] else None
    priv = PaillierContext().init(hx(k["p"]), hx(k["q"]), djn_h_pow_n=h)
    return priv, priv.to_public()


def cts(ctx, d):
    from xfl_amd.paillier import PaillierCiphertext
    return np.array([PaillierCiphertext(ctx, hx(r), e) for r, e in zip(d["raw"], d["exp"])], dtype=object)


def raw(arr):
    flat = list(np.asarray(arr, dtype=object).reshape(-1)) if not hasattr(arr, "words") else list(arr.reshape(-1))
    return [c.raw_ciphertext for c in flat], [c.exponent for c in flat]


def ops_bit_exact(fx, vectorized):
    """vectorized=False: numpy's per-element object loop over PaillierCiphertext
    operators; True: PaillierArray's batched kernels (segmented product,
    batch inversion, multi-exponentiation matmul); "resident": the same with
    the operands held in HBM (every result stays there; GPU only)."""
    from xfl_amd.paillier import PaillierArray
    g = load_fixture(fx)
    priv, pub = ctxs(g)
    ops = g["ops"]
    a = cts(pub, ops["a"])
    b = cts(pub, ops["b"])
    if vectorized:
        a, b = PaillierArray(a), PaillierArray(b)
        if vectorized == "resident":
            a.to_device(), b.to_device()
            assert a.is_resident and (a + b).is_resident and (a * 2.5).is_resident
    sc = [fl(s) if isinstance(s, str) else s for s in ops["mul_pub"]["scalar"]]
    want = lambda name: ([hx(r) for r in ops[name]["raw"]], ops[name]["exp"])  # noqa: E731
    assert raw(a + b) == want("add")
    assert raw(a - b) == want("sub")
    assert raw(np.array([a[i] * sc[i] for i in range(len(a))], dtype=object)) == want("mul_pub")
    a_priv = cts(priv, ops["a"])
    assert raw(np.array([a_priv[i] * sc[i] for i in range(len(a))], dtype=object)) == want("mul_priv")
    if vectorized:
        scv = np.array(sc, dtype=object)
        assert raw(a * scv) == want("mul_pub")
        assert raw(a + scv) == want("add_scalar")
        assert raw(scv - a) == want("rsub_scalar")
        # numeric (non-object) scalar arrays: the float positions as float64,
        # the int positions as int64, each against its golden entries
        for kind, dt in ((float, np.float64), (int, np.int64)):
            idx = [i for i in range(len(sc)) if isinstance(sc[i], kind)]
            v = np.array([sc[i] for i in idx], dtype=dt)
            sub = lambda name: ([want(name)[0][i] for i in idx], [want(name)[1][i] for i in idx])  # noqa: E731
            assert raw(a[idx] * v) == sub("mul_pub") and raw(v * a[idx]) == sub("mul_pub")
            assert raw(a[idx] + v) == sub("add_scalar") and raw(v - a[idx]) == sub("rsub_scalar")
        assert raw(np.multiply(a, scv)) == want("mul_pub")
        assert raw(np.add(a, b)) == want("add")
    assert raw(np.array([a[i] + sc[i] for i in range(len(a))], dtype=object)) == want("add_scalar")
    assert raw(np.array([sc[i] - a[i] for i in range(len(a))], dtype=object)) == want("rsub_scalar")
    assert raw(a / 4.0) == want("truediv")
    assert raw(np.array([np.sum(a)], dtype=object)) == want("sum_a")
    assert raw(np.array([sum(a)], dtype=object)) == want("sum_pyfold")
    X = np.array([[fl(v) for v in row] for row in ops["matmul"]["X"]], dtype=np.float32)
    assert raw(np.matmul(a, X)) == want("matmul")
    if vectorized:
        assert raw(a @ X) == want("matmul")
        assert raw(X.T @ a) == want("matmul")
        assert raw(np.dot(a, X)) == want("matmul")


def histogram_groupby(fx):
    """pandas groupby(bin).sum over an object column built from a
    PaillierArray (the DataFrame materializes the reference's objects)."""
    import pandas as pd

    from xfl_amd.paillier import PaillierArray
    g = load_fixture(fx)
    priv, pub = ctxs(g)
    h = g["ops"]["hist"]
    want = ([hx(r) for r in h["sum"]["raw"]], h["sum"]["exp"])
    for c in (cts(pub, h["ct"]), PaillierArray(cts(pub, h["ct"]))):
        df = pd.DataFrame({"bin": h["bins"], "xfl_grad_hess": c})
        agg = df.groupby(["bin"])["xfl_grad_hess"].agg(["count", "sum"])
        assert list(agg["count"]) == h["count"]
        assert raw(np.array(list(agg["sum"]), dtype=object)) == want
    # Feature.create's form (core/tree/big_feature.py:43-46)
    df = pd.DataFrame(PaillierArray(cts(pub, h["ct"])), columns=["xfl_grad_hess"])
    df["bin"] = h["bins"]
    agg = df.groupby(["bin"])["xfl_grad_hess"].agg(["count", "sum"])
    assert raw(np.array(list(agg["sum"]), dtype=object)) == want


def _bin_sums(pub, raws, exps, bins, nbins):
    """per-bin oracle sums (A.9) -> ([raw], [exp], [count])"""
    from oracle import paillier_oracle as O
    k = O.derive_public(pub.n)
    out_r, out_e, cnt = [], [], []
    for b in range(nbins):
        sel = [i for i in range(len(bins)) if bins[i] == b]
        cnt.append(len(sel))
        r, e = O.sum_ct(k, [raws[i] for i in sel], [exps[i] for i in sel]) if sel else (1, 0)
        out_r.append(r)
        out_e.append(e)
    return out_r, out_e, cnt


def _col(df_col):
    """raw/exponent lists of a pandas column of ciphertexts"""
    return raw(np.array(list(df_col), dtype=object))


def xgb_histogram_pandas(fx, resident=False):
    """XFL's XGBoost histogram calls, verbatim, on a ciphertext column built
    from a PaillierArray: the column keeps the flat words (PaillierDtype, no
    object column) and each groupby sum is one segmented product, bit-exact
    against the oracle's per-bin sums and the reference's object column.
      - core/tree/big_feature.py:43-46 (Feature.create) and
        xgboost/decision_tree_trainer.py:146-183 (row batches, per-feature
        groupby agg({'count', 'sum'}), outer merge + fillna(0) + add);
      - core/tree_ray/big_feature.py:72-75 and xgb_actor.py:340-345, 447-455
        (groupby(observed=True)[[...]].agg, concat + groupby(index).sum)."""
    import pandas as pd

    from xfl_amd.paillier import PaillierArray
    from xfl_amd.paillier.array import PaillierDtype
    g = load_fixture(fx)
    priv, pub = ctxs(g)
    h = g["ops"]["hist"]
    R, E = [hx(r) for r in h["ct"]["raw"]], h["ct"]["exp"]
    n = len(R)
    # a second, mixed-exponent column (the alignment inside the folds) and 3 features
    a = g["ops"]["a"]
    R2 = R[:n - 16] + [hx(r) for r in a["raw"]]
    E2 = E[:n - 16] + list(a["exp"])
    bins0 = list(h["bins"])
    feats = {"f0": bins0, "f1": [(3 * b + i) % 5 for i, b in enumerate(bins0)], "f2": [(i * 7) % 3 for i in range(n)]}
    values = pd.DataFrame({k: np.asarray(v, dtype=np.uint8) for k, v in feats.items()})
    for RR, EE in ((R, E), (R2, E2)):
        grad_hess = PaillierArray(np.array([_ct(pub, r, e) for r, e in zip(RR, EE)], dtype=object))
        if resident:
            grad_hess.to_device()
        want = {f: _bin_sums(pub, RR, EE, b, max(b) + 1) for f, b in feats.items()}
        # Feature.create (core/tree/big_feature.py:43-46)
        data = pd.concat([pd.DataFrame(range(n), columns=['xfl_id']),
                          pd.DataFrame(grad_hess, columns=['xfl_grad_hess']), values], axis=1)
        assert isinstance(data['xfl_grad_hess'].dtype, PaillierDtype), "the ciphertext column became an object column"
        for f in feats:
            res = data.groupby([f])['xfl_grad_hess'].agg({'count', 'sum'})
            wr, we, wc = want[f]
            assert list(res['count']) == wc
            assert _col(res['sum']) == (wr, we), f
            assert isinstance(res['sum'].dtype, PaillierDtype)
            # res_hist['sum'].to_numpy(): the reference's object array (decision_tree_trainer.py:180)
            obj = res['sum'].to_numpy()
            assert obj.dtype == object and raw(obj) == (wr, we)
        # row batches merged as decision_tree_trainer.py:146-176 does
        rb = 13
        for f in feats:
            res = None
            for j in range((n + rb - 1) // rb):
                b = data.iloc[rb * j: rb * (j + 1), :].groupby([f])['xfl_grad_hess'].agg({'count', 'sum'})
                if res is None:
                    res = b
                    continue
                r = pd.merge(res, b, how='outer', left_index=True, right_index=True).fillna(0)
                r = pd.Series(b.columns).apply(lambda x: r[x + '_x'] + r[x + '_y']).T
                r.columns = list(b.columns)
                res = r
            wr, we, wc = want[f]
            assert [int(c) for c in res['count']] == wc
            assert raw(res['sum'].to_numpy()) == (wr, we), f
        # the reference's object column gives the same bits (pandas' object group_sum)
        obj_data = data.copy()
        obj_data['xfl_grad_hess'] = np.asarray(grad_hess)
        assert obj_data['xfl_grad_hess'].dtype == object
        ref = obj_data.groupby(['f1'])['xfl_grad_hess'].agg(['count', 'sum'])
        got = data.groupby(['f1'])['xfl_grad_hess'].agg(['count', 'sum'])
        assert _col(ref['sum']) == _col(got['sum'])
        # core/tree_ray: Feature.create (big_feature.py:72-75), node concat + groupby (xgb_actor.py:340-345)
        blocks = []
        for lo, hi in ((0, 17), (17, n)):
            idx = np.arange(lo, hi)
            d = pd.DataFrame(columns=['xfl_grad_hess'] + values.columns.to_list(), index=idx)
            d['xfl_grad_hess'] = grad_hess[lo:hi]
            d[values.columns] = values.loc[idx, :]
            assert isinstance(d['xfl_grad_hess'].dtype, PaillierDtype)
            blocks.append(d)
        agg_feature = pd.concat(blocks)
        hist = {f: agg_feature.groupby([f], observed=True)[['xfl_grad_hess']].agg({'sum', 'count'}) for f in feats}
        for f in feats:
            wr, we, wc = want[f]
            nz = [i for i in range(len(wc)) if wc[i]]
            assert _col(hist[f][('xfl_grad_hess', 'sum')]) == ([wr[i] for i in nz], [we[i] for i in nz])
            assert list(hist[f][('xfl_grad_hess', 'count')]) == [wc[i] for i in nz]
        # merge_hist over per-block partial histograms (xgb_actor.py:447-455)
        parts = [blk.groupby(['f0'], observed=True)[['xfl_grad_hess']].agg({'sum', 'count'}) for blk in blocks]
        hist_df = pd.concat(parts)
        merged = hist_df.groupby(hist_df.index).sum(numeric_only=False)
        wr, we, wc = want['f0']
        assert _col(merged[('xfl_grad_hess', 'sum')]) == (wr, we)
        assert list(merged[('xfl_grad_hess', 'count')]) == wc
        # Series.sum over the column = np.sum
        from oracle import paillier_oracle as O
        s = data['xfl_grad_hess'].sum()
        assert (s.raw_ciphertext, s.exponent) == O.sum_ct(O.derive_public(pub.n), RR, EE)
    # missing entries: NaN on read, skipped by the groupby sum, refused by arithmetic
    col = pd.Series(PaillierArray(np.array([_ct(pub, r, e) for r, e in zip(R[:6], E[:6])], dtype=object)))
    shifted = col.reindex(range(-2, 6))
    assert shifted.isna().tolist() == [True, True] + [False] * 6
    assert np.isnan(shifted.iloc[0])
    grp = pd.DataFrame({"k": [0, 0, 1, 1, 1, 1, 1, 1], "c": shifted.values})
    s = grp.groupby("k")["c"].sum()
    k = O.derive_public(pub.n)
    assert _col(s) == ([1, O.sum_ct(k, R[:6], E[:6])[0]], [0, O.sum_ct(k, R[:6], E[:6])[1]])
    filled = shifted.fillna(0)
    assert not filled.isna().any()
    assert (filled.iloc[0].raw_ciphertext, filled.iloc[0].exponent) == (1, 0)
    try:
        shifted.values + shifted.values
        raise AssertionError("arithmetic on missing ciphertexts must raise")
    except ValueError:
        pass


def _ct(ctx, r, e):
    from xfl_amd.paillier import PaillierCiphertext
    return PaillierCiphertext(ctx, r, e)


def decrypt_matches_reference(fx):
    """Paillier.decrypt of the reference's ciphertexts, as an object array and
    as a PaillierArray: float32 output hex-equal, out_origin values exact
    (floats RNE-53, integers exact), dtype='int' for the int32 case."""
    from xfl_amd.paillier import Paillier, PaillierArray
    from xfl_amd.paillier.encoder import int_to_float_gmpy
    g = load_fixture(fx)
    priv, pub = ctxs(g)
    for case in ("priv_f32_p7", "pub_f64_none_max-60", "priv_packed_p0", "pub_i32_none", "priv_edge_p7_noobf"):
        enc = g["encrypt"][case]
        dec = g["decrypt"][case]
        for c in (cts(priv, enc), PaillierArray(cts(priv, enc))):
            f32 = Paillier.decrypt(priv, c, dtype="float", num_cores=1)
            assert [float(v).hex() for v in np.asarray(f32).astype(np.float64)] == dec["float32"]
            org = Paillier.decrypt(priv, c, num_cores=1, out_origin=True)
            want_m = [hx(m) for m in dec["m"][len(dec["m"]) - len(enc["raw"]):]]
            n = priv.n
            for v, want, m, e in zip(org, dec["origin_f64"], want_m, enc["exp"]):
                if e >= 0:  # integer decode: the exact signed integer (an mpz in the reference)
                    assert isinstance(v, int) and v == (m - n if m >= priv.min_value_for_negative else m) << e
                    assert int_to_float_gmpy(v).hex() == want  # the reference's float(mpz), truncating
                else:
                    assert isinstance(v, float) and v.hex() == want
            if "int32" in dec:
                assert Paillier.decrypt(priv, c, dtype="int").tolist() == dec["int32"]


def wire_roundtrip(fx):
    from xfl_amd.paillier import Paillier, PaillierArray, PaillierContext
    g = load_fixture(fx)
    priv, pub = ctxs(g)
    ctx = PaillierContext.deserialize_from(bytes.fromhex(g["ops"]["wire_ctx_pub"]))
    assert ctx.n == pub.n
    arr = Paillier.ciphertext_from(None, bytes.fromhex(g["ops"]["wire_a4"]), compression=False)
    assert isinstance(arr, PaillierArray)
    assert [c.raw_ciphertext for c in arr] == [hx(r) for r in g["ops"]["a"]["raw"][:4]]
    for comp in (True, False):
        back = Paillier.ciphertext_from(priv, Paillier.serialize(arr, compression=comp), compression=comp)
        assert [c.raw_ciphertext for c in back] == [c.raw_ciphertext for c in arr]
        # a context-free decode (label_trainer.py:258) decrypts with the key passed to decrypt
        none = Paillier.ciphertext_from(None, Paillier.serialize(arr, compression=comp), compression=comp)
        assert raw(none) == raw(arr)
    # the bytes load with plain pickle into the reference's object graph
    from xfl_amd import compat
    obj = compat.loads(Paillier.serialize(arr, compression=False))
    assert isinstance(obj, np.ndarray) and obj.dtype == object
    assert [o.value for o in obj] == [hx(r) for r in g["ops"]["a"]["raw"][:4]]


def array_protocol(fx, resident=False):
    """The ndarray surface the operators use on encrypted arrays (resident:
    the array's words held in HBM first, so views, takes, copies and
    assignments go through the device copy)."""
    import pandas as pd

    from xfl_amd.paillier import Paillier, PaillierArray, PaillierCiphertext
    g = load_fixture(fx)
    priv, pub = ctxs(g)
    a_obj = cts(pub, g["ops"]["a"])  # 16 ciphertexts, mixed exponents
    a = PaillierArray(a_obj)
    if resident:
        a.to_device()
        a._st.h = None  # device copy only: every host read below downloads
    R, E = raw(a_obj)
    assert a.shape == (16,) and a.ndim == 1 and a.size == 16 and len(a) == 16 and a.dtype.kind == "O"
    assert isinstance(a[3], PaillierCiphertext) and (a[3].raw_ciphertext, a[3].exponent) == (R[3], E[3])
    assert (a[-1].raw_ciphertext, a[-1].exponent) == (R[-1], E[-1])
    assert raw(a[2:7]) == (R[2:7], E[2:7])
    assert raw(a[::3]) == (R[::3], E[::3])
    assert raw(a[[5, 1, 1]]) == ([R[5], R[1], R[1]], [E[5], E[1], E[1]])
    assert raw(a[np.arange(16) % 2 == 0]) == (R[::2], E[::2])
    m = a.reshape(4, 4)
    assert m.shape == (4, 4) and raw(m[1]) == (R[4:8], E[4:8])
    assert (m[2, 3].raw_ciphertext, m[2, 3].exponent) == (R[11], E[11])
    assert raw(m.T[0]) == ([R[0], R[4], R[8], R[12]], [E[0], E[4], E[8], E[12]])
    assert raw(m.flatten()) == (R, E) and raw(m.ravel()) == (R, E) and raw(np.reshape(m, -1)) == (R, E)
    assert raw(np.concatenate([a[:3], a[3:]])) == (R, E)
    assert raw(np.concatenate([a_obj[:3], a[3:]])) == (R, E)
    assert raw(np.stack([a[:8], a[8:]])[1]) == (R[8:], E[8:])
    assert raw(list(a)) == (R, E) and raw(a.tolist()) == (R, E)
    assert raw(np.asarray(a)) == (R, E) and np.asarray(a).dtype == object
    # np.sum over axes = the reference's object-array sums (order-free folds)
    want_rows = [np.sum(a_obj.reshape(4, 4)[i]) for i in range(4)]
    assert raw(np.sum(m, axis=1)) == raw(np.array(want_rows, dtype=object))
    assert raw(m.sum(axis=0)) == raw(np.array([np.sum(a_obj.reshape(4, 4)[:, j]) for j in range(4)], dtype=object))
    s = np.sum(a)
    assert isinstance(s, PaillierCiphertext) and raw([s]) == raw([np.sum(a_obj)])
    # broadcasting a ciphertext row against a column of scalars
    col = np.array([[1.5], [-2.0]])
    got = m[0] * col
    assert got.shape == (2, 4)
    assert raw(got[1]) == raw(np.array([c * -2.0 for c in a_obj[:4]], dtype=object))
    # assignment, copy, pickling
    b = a.copy()
    b[0] = a[5]
    assert raw(b[:2]) == ([R[5], R[1]], [E[5], E[1]]) and raw(a[:1]) == ([R[0]], [E[0]])
    assert raw(pickle.loads(pickle.dumps(a))) == (R, E)
    # serialize keeps the shape
    back = Paillier.ciphertext_from(pub, Paillier.serialize(m, compression=False), compression=False)
    assert back.shape == (4, 4) and raw(back) == (R, E)
    # a DataFrame column and Series.apply (binning_woe_iv/label_trainer.py:105)
    df = pd.DataFrame({"c": a})
    assert raw(np.array(list(df["c"]), dtype=object)) == (R, E)
    # different keys refuse to mix
    other = PaillierArray(cts(ctxs(load_fixture("paillier_2048_nodjn.json" if "nodjn" not in fx
                                                else "paillier_2048_djn.json"))[1], g["ops"]["a"]))
    try:
        a + other
        raise AssertionError("adding under different keys must raise")
    except ValueError:
        pass
    try:
        a * a
        raise AssertionError("ciphertext * ciphertext must raise")
    except TypeError:
        pass
    try:
        a + "342"
        raise AssertionError("adding a str must raise")
    except TypeError:
        pass


def encrypt_decrypt_shapes(fx):
    """Paillier.encrypt of arrays of every plaintext kind keeps the shape and
    decrypts back (float32/float64 within the reference's tolerance, ints
    exactly), public and private context, obfuscate in place."""
    from xfl_amd.paillier import Paillier, PaillierArray
    g = load_fixture(fx)
    priv, pub = ctxs(g)
    rng = np.random.default_rng(1)
    x = (rng.random((3, 5)) * 100 - 50).astype(np.float32)
    for ctx in (priv, pub):
        c = Paillier.encrypt(ctx, x, precision=7)
        assert isinstance(c, PaillierArray) and c.shape == (3, 5)
        assert np.all(np.abs(Paillier.decrypt(priv, c) - x) < 1e-4)
        before = raw(c)[0]
        same = Paillier.obfuscate(c)
        assert same is c and raw(c)[0] != before
        assert np.all(np.abs(Paillier.decrypt(priv, c) - x) < 1e-4)
    ints = np.array([[3, -7], [0, 123456]], dtype=np.int32)
    c = Paillier.encrypt(pub, ints)
    assert Paillier.decrypt(priv, c, dtype="int").tolist() == ints.tolist()
    mixed = np.array([1, 2.5, -3], dtype=object)
    assert Paillier.decrypt(priv, Paillier.encrypt(priv, mixed, precision=7)).tolist() == [1.0, 2.5, -3.0]
    empty = Paillier.encrypt(priv, np.zeros((0, 4)))
    assert empty.shape == (0, 4) and Paillier.decrypt(priv, empty).shape == (0, 4)
    # the object arrays the reference hands out keep working as inputs
    obj = np.asarray(Paillier.encrypt(pub, x[0], precision=7))
    assert obj.dtype == object and np.all(np.abs(Paillier.decrypt(priv, obj) - x[0]) < 1e-4)
    assert np.all(np.abs(Paillier.decrypt(priv, Paillier.obfuscate(obj)) - x[0]) < 1e-4)


def gap_alignment(fx, vectorized):
    """Adds across alignment gaps that take _raw_mul's negative branch
    (1 << d >= min_value_for_negative: c^(2^d - n), paillier.py:79-86,
    173-187), bit-exact vs the reference: the operands (a product with two
    2^-960 scalars), element-wise adds with the public and the private
    context, np.sum (numpy's left fold) and Python's sum() in four orders."""
    from xfl_amd.paillier import PaillierArray
    g = load_fixture(fx)
    priv, pub = ctxs(g)
    ops = g["ops"]
    want = lambda name: ([hx(r) for r in ops[name]["raw"]], ops[name]["exp"])  # noqa: E731
    cg = cts(pub, ops["gap"])
    scale = fl(ops["gap"]["scale"])
    if vectorized:
        A = PaillierArray(cg)
        if vectorized == "resident":
            A.to_device()
        first = A[:1] * scale * scale
        assert raw(first) == ([want("gap_operands")[0][0]], [want("gap_operands")[1][0]])
    else:
        gc = np.array([cg[0] * scale * scale] + list(cg[1:]), dtype=object)
        assert raw(gc) == want("gap_operands")
    pairs = ops["gap"]["pairs"]
    li, ri = [i for i, _ in pairs], [j for _, j in pairs]
    for name, ctx in (("pub", pub), ("priv", priv)):
        gc = cts(ctx, ops["gap_operands"])
        if vectorized:
            A = PaillierArray(gc)
            if vectorized == "resident":
                A.to_device()
            got = A[li] + A[ri]
        else:
            got = np.array([gc[i] + gc[j] for i, j in pairs], dtype=object)
        assert raw(got) == want(f"gap_add_{name}"), name
    gc = cts(pub, ops["gap_operands"])
    orders = ops["gap_sum"]["orders"]
    if vectorized:
        A = PaillierArray(gc)
        if vectorized == "resident":
            A.to_device()
        sums = [np.sum(A[o]) for o in orders]
    else:
        sums = [np.sum(gc[o]) for o in orders]
    assert raw(np.array(sums, dtype=object)) == want("gap_sum")
    assert raw(np.array([sum(gc[o]) for o in orders], dtype=object)) == want("gap_pyfold")
