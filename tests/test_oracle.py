"""Oracle (CPU restatement) pinned against SciPy/pandas: live in this
container and through the committed golden vectors (tests/golden)."""
import json
import os

import numpy as np
import pytest

import oracle
import synth

G = os.path.join(os.path.dirname(__file__), "golden")


def _g(name):
    return np.load(os.path.join(G, name), allow_pickle=False)


def test_c_oracle_built():
    assert oracle.have_c_oracle()


def test_design_matches_golden():
    g = _g("design.npz")
    for i, (N, Wn, bt) in enumerate(json.loads(str(g["cases"]))):
        sos = oracle.butter_sos(N, Wn, bt)
        ns = sos.shape[0]
        np.testing.assert_array_equal(sos, g["sos"][i][:ns])
        np.testing.assert_allclose(oracle.sosfilt_zi(sos), g["zi"][i][:ns], rtol=1e-13, atol=1e-15)


def test_sosfilt_bit_exact_golden():
    g = _g("sosfilt_small.npz")
    y, zf = oracle.sosfilt(g["sos"], g["x"], g["zi"])
    np.testing.assert_array_equal(y, g["y"])
    np.testing.assert_array_equal(zf, g["zf"])


def test_sosfiltfilt_bit_exact_golden():
    g = _g("sosfiltfilt_small.npz")
    np.testing.assert_array_equal(oracle.sosfiltfilt(g["sos"], g["x"]), g["y"])
    np.testing.assert_array_equal(oracle.sosfiltfilt_rows_c(g["sos"], g["x"]), g["y"])


def test_sosfiltfilt_errors():
    sos = oracle.butter_sos(4, 0.1)
    with pytest.raises(ValueError, match="greater than padlen, which is 15"):
        oracle.sosfiltfilt(sos, np.zeros(15))


@pytest.mark.parametrize("name", ["lfproc_cfg1.npz", "lfproc_cfg3_slice.npz", "lfproc_cfg5_slice.npz"])
def test_lfproc_restatement_matches_golden(name):
    g = _g(name)
    recipe = json.loads(str(g["recipe"]))["data"]
    if name == "lfproc_cfg1.npz":
        x = synth.random_das_spool_data().astype(np.float32)
    elif "cfg3" in name:
        x = synth.noise_sine(4, 750_000, 500.0, seed=3)
    else:
        x = synth.noise_sine(4, 600_000, 200.0, seed=5, dc=1000.0)
    assert synth.digest(x) == str(g["x_sha256"]), recipe
    fs, dt_out, P, B = float(g["fs"]), float(g["dt_out"]), int(g["P"]), int(g["B"])
    dt_ns = int(round(1e9 / fs))
    tg = g["tg"]
    out = oracle.lfproc_process(x, synth.T0_NS, dt_ns, tg[0], tg[-1] + 1, dt_out, P, B)
    sched = [tuple(r) for r in g["sched"]]
    assert [(oa, ob) for _, _, oa, ob in oracle.lfproc_schedule(len(tg), P, B)] == sched
    for (tt, yv), (oa, ob) in zip(out, sched):
        np.testing.assert_array_equal(tt, tg[oa:ob])
        np.testing.assert_allclose(yv, g["y"][:, oa:ob], rtol=0, atol=1e-12 * np.abs(g["y"][:, oa:ob]).max())


def test_schedule_golden_and_survey_table():
    tab = json.load(open(os.path.join(G, "schedule.json")))
    # SURVEY §3.1 worked table (cfg1: L=120, P=40, B=6)
    assert oracle.lfproc_schedule(120, 40, 6) == [(0, 40, 6, 34), (28, 68, 34, 62), (56, 96, 62, 90),
                                                  (84, 119, 90, 113)]
    for k, (L, P, B) in {"cfg1": (120, 40, 6), "cfg3": (3600, 600, 7), "short": (30, 40, 6),
                         "exact": (96, 40, 6)}.items():
        assert [list(t) for t in oracle.lfproc_schedule(L, P, B)] == tab[k]


def test_rolling_matches_pandas_golden():
    g = _g("rolling.npz")
    for key in g.files:
        if not key.startswith("x_"):
            continue
        _, n, W, S = key.split("_")
        ref = g["y_" + "_".join([n, W, S])]
        out = oracle.rolling_mean(g[key], int(W), int(S)).astype(np.float64)
        assert out.shape == ref.shape
        assert np.array_equal(np.isnan(out), np.isnan(ref))
        m = ~np.isnan(ref)
        np.testing.assert_allclose(out[m], ref[m], rtol=2e-7, atol=1e-7)


def test_interp_matches_scipy_live():
    from scipy.interpolate import interp1d
    rng = np.random.default_rng(1)
    t = np.arange(500) * 0.004
    y = rng.standard_normal((3, 500))
    tq = np.sort(rng.uniform(0, t[-1], 77))
    np.testing.assert_array_equal(oracle.interp1d_linear(t, y, tq), interp1d(t, y, kind="linear")(tq))


def test_patch_time_and_edge_helpers():
    assert oracle.get_patch_time(10000, 500, 10000) == pytest.approx(41.6666666667)
    e = oracle.get_edge_effect_time(1 / 250.0, 120.0, tol=1e-3, freq=5)
    assert 0.5 < e < 3.0
    with pytest.raises(ValueError):
        oracle.get_edge_effect_time(1 / 200.0, 20.8, tol=1e-3, freq=0.1)
