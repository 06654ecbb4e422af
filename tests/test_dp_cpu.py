"""Data-parallel contract on CPU: world_size-2 gloo ranks running the oracle step with the
build's DP exchange: one SUM all-reduce of
[grads | tau' | score sums | counts | losses], rank-mean gradient and thresholds, summed
epoch statistics, replicated clip/Adam/EMA.  The GPU path (tests/test_gpu_dp.py) is held
to the same oracle.
"""
import multiprocessing as mp
import os
import socket

import numpy as np

from oracle import dad_oracle, synth

B, T, SEED = 8, 24, 11
SCHEDULE = [35, 60]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _shard(rank, k):
    return synth.make_step_inputs(SEED + 100 * rank, k, B, T)


def _snapshot(orc):
    return {"student": [p.copy() for p in orc.s], "teacher": [p.copy() for p in orc.t],
            "tau": orc.dacp.tau.copy(), "Q": orc.dacp.Q.copy(), "cnt": orc.dacp.score_cnt.copy()}


def _rank_main(rank, world, port, dup, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = dad_oracle.make_cfg("iemocap")
        orc = dad_oracle.DADOracle(*synth.init_weights(SEED)[:4], cfg)
        orc.load_state(synth.make_state(SEED, 1))

        def allreduce(v):
            t = torch.from_numpy(np.ascontiguousarray(v, np.float64))
            dist.all_reduce(t)
            return t.numpy()

        steps = []
        for k, epoch in enumerate(SCHEDULE):
            r = orc.step(_shard(0 if dup else rank, k), epoch, allreduce=allreduce, world=world)
            steps.append({"grads_mean": r["grads_mean"], "losses_mean": r["losses_mean"],
                          "total_loss": r["total_loss"], **_snapshot(orc)})
        orc.dacp.epoch_end(cfg["DACP_QUALITY_SMOOTHING_BETA"])
        q.put((rank, steps, orc.dacp.Q.copy()))
    finally:
        dist.destroy_process_group()


def _run(dup):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, dup, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = {}
    for _ in procs:
        rank, steps, Q = q.get(timeout=300)
        out[rank] = (steps, Q)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def test_dp_two_ranks_replicated_and_rank_mean():
    out = _run(dup=False)
    (s0, Q0), (s1, Q1) = out[0], out[1]
    # every rank holds identical parameters, thresholds and quality scores
    for a, b in zip(s0, s1):
        for k in range(4):
            np.testing.assert_array_equal(a["student"][k], b["student"][k])
            np.testing.assert_array_equal(a["teacher"][k], b["teacher"][k])
        np.testing.assert_array_equal(a["tau"], b["tau"])
        np.testing.assert_array_equal(a["cnt"], b["cnt"])
    np.testing.assert_array_equal(Q0, Q1)
    # the first step's gradient is the mean of the two shards' single-process gradients
    cfg = dad_oracle.make_cfg("iemocap")
    g = []
    for rank in range(2):
        orc = dad_oracle.DADOracle(*synth.init_weights(SEED)[:4], cfg)
        orc.load_state(synth.make_state(SEED, 1))
        g.append(orc.step(_shard(rank, 0), SCHEDULE[0])["grads"])
    for k in range(4):
        want = (g[0][k].astype(np.float64) + g[1][k]) / 2
        np.testing.assert_allclose(s0[0]["grads_mean"][k], want, rtol=0, atol=1e-6 * np.abs(want).max())
    # reported losses are the rank mean; each rank's own loss differs (its own shard)
    assert abs(s0[0]["losses_mean"][0] - (s0[0]["total_loss"] + s1[0]["total_loss"]) / 2) < 1e-9
    assert s0[0]["total_loss"] != s1[0]["total_loss"]
    assert s0[-1]["cnt"].sum() == 2 * 2 * B        # two post-warm-up steps, two ranks


def test_dp_duplicated_shards_equal_single_process():
    """Two ranks on the same shard == one process: mean grads and tau' unchanged, summed
    statistics only rescale the epoch mean."""
    out = _run(dup=True)
    steps, Q = out[0]
    cfg = dad_oracle.make_cfg("iemocap")
    orc = dad_oracle.DADOracle(*synth.init_weights(SEED)[:4], cfg)
    orc.load_state(synth.make_state(SEED, 1))
    for k, epoch in enumerate(SCHEDULE):
        orc.step(_shard(0, k), epoch)
        for i in range(4):
            np.testing.assert_allclose(steps[k]["student"][i], orc.s[i], rtol=0, atol=1e-7)
            np.testing.assert_allclose(steps[k]["teacher"][i], orc.t[i], rtol=0, atol=1e-7)
        np.testing.assert_allclose(steps[k]["tau"], orc.dacp.tau, rtol=0, atol=1e-7)
    orc.dacp.epoch_end(cfg["DACP_QUALITY_SMOOTHING_BETA"])
    np.testing.assert_allclose(Q, orc.dacp.Q, rtol=0, atol=1e-6)
