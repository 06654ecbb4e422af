"""Pin the CPU oracle (oracle/dad_oracle.py) against the reference's golden vectors.

The fixtures were produced by running the reference step itself with injected
randomness (tests/golden/gen_golden.py).  Tolerance: 1e-4 (the north_star's loss /
logit parity bound), relative to the tensor's max magnitude.
"""
import numpy as np
import pytest

from oracle import dad_oracle
import goldens

TOL = 1e-4


@pytest.mark.parametrize("name", goldens.variants())
def test_oracle_matches_reference(name):
    d, spec, cfg = goldens.load(name)
    W1, b1, W2, b2 = goldens.problem(spec)
    orc = dad_oracle.DADOracle(W1, b1, W2, b2, cfg, anchors=d["anchors"])
    idx = d["w1_index"]
    for s, epoch in goldens.schedule(d):
        p = "s%d_" % s
        orc.load_state(goldens.state(spec, s))
        o = orc.step(goldens.step_inputs(spec, s), epoch, lr=float(d[p + "lr"]))
        for k in ("total_loss", "supervised_ce_loss", "consistency_loss", "ecda_loss"):
            ref = float(d[p + k])
            assert abs(o[k] - ref) <= TOL * max(1.0, abs(ref)), (name, s, k, o[k], ref)
        assert goldens.rel_err(o["z_clean"], d[p + "z_clean"]) < TOL
        assert goldens.rel_err(o["e_clean"], d[p + "e_clean"]) < TOL
        if p + "z_strong" in d:
            assert goldens.rel_err(o["z_strong"], d[p + "z_strong"]) < TOL
            assert goldens.rel_err(o["z_teacher"], d[p + "z_teacher"]) < TOL
            assert goldens.rel_err(o["e_strong"], d[p + "e_strong"]) < TOL
        if p + "mask" in d:
            np.testing.assert_array_equal(o["mask"], d[p + "mask"])
            assert goldens.rel_err(o["score"], d[p + "score"]) < TOL
            np.testing.assert_allclose(o["tau_after"], d[p + "tau_after"], atol=1e-6)
            np.testing.assert_allclose(o["w"], d[p + "w"], atol=1e-6)
        assert abs(o["clip_norm"] - float(d[p + "clip_norm"])) <= TOL * max(1.0, float(d[p + "clip_norm"]))
        g = o["grads_clipped"]
        assert goldens.rel_err(g[0].reshape(-1)[idx], d[p + "gW1c_s"]) < TOL
        assert goldens.rel_err(g[1], d[p + "gb1c"]) < TOL
        assert goldens.rel_err(g[2], d[p + "gW2c"]) < TOL
        assert goldens.rel_err(g[3], d[p + "gb2c"]) < TOL
        for who, params in (("s", o["student"]), ("t", o["teacher"])):
            assert goldens.rel_err(params[0].reshape(-1)[idx], d[p + who + "W1_s"]) < TOL
            assert goldens.rel_err(params[1], d[p + who + "b1"]) < TOL
            assert goldens.rel_err(params[2], d[p + who + "W2"]) < TOL
            assert goldens.rel_err(params[3], d[p + who + "b2"]) < TOL
            s64 = float(np.sum(params[0].astype(np.float64)))
            assert abs(s64 - float(d[p + who + "W1_sum"])) < 1e-3 * max(1.0, abs(float(d[p + who + "W1_sum"])))
        assert goldens.rel_err(orc.m[1], d[p + "exp_avg_b1"]) < TOL
        assert goldens.rel_err(orc.v[2], d[p + "exp_avg_sq_W2"]) < TOL
    # epoch-end DACP quality update over the scores collected by the post-warm-up steps
    n = int(d["epoch_end_after_step"])
    orc.dacp.Q = goldens.state(spec, n)["Q"]
    np.testing.assert_array_equal(orc.dacp.score_cnt, d["epoch_end_counts"])
    orc.dacp.epoch_end(cfg["DACP_QUALITY_SMOOTHING_BETA"])
    np.testing.assert_allclose(orc.dacp.Q, d["epoch_end_Q"], rtol=0, atol=1e-6)


def test_quantile_matches_torch():
    torch = pytest.importorskip("torch")
    rs = np.random.RandomState(0)
    for n in (1, 2, 3, 7, 16, 64):
        for q in (0.4, 0.4 + 0.4 * 35 / 500, 0.4 + 0.4 * 60 / 500, 0.8, 0.5):
            v = rs.uniform(size=n).astype(np.float32)
            ref = torch.quantile(torch.from_numpy(v), q).item()
            assert np.float32(ref) == dad_oracle.quantile_linear(v, q), (n, q)
