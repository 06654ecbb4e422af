"""Data-parallel HIP step, world_size 2 on the one-GPU box: two ranks share cuda:0 and
exchange the step's [grads | tau' | sums | counts | losses] buffer with ProcessGroupComm over
gloo.  That runs the kernels' DP path (dad_norm rank-mean, replicated clip/Adam/EMA, DACP
commit of the mean tau').  Each rank checks itself against the oracle's DP step on its own
shard.  RCCL cannot put two ranks on one GPU, so the RCCL transport (DPComm) with more than
one rank runs only where the node has a GPU per rank (the driver's multi-GPU bench, which
reports the ranks RCCL connected); here it is covered with one rank (test_gpu_rccl.py).
The last test drives `bench.py --gpus 2 --comm gloo` end to end: the launcher spawns both
ranks itself and the line must report two ranks.
"""
import json
import multiprocessing as mp
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

B, T, SEED = 12, 40, 21
SCHEDULE = [35, 60]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_main(rank, world, port, q):
    try:
        import torch
        import torch.distributed as dist
        import dadpkg
        import gpu_harness as gh
        from oracle import dad_oracle, synth
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        import datetime
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=120))
        p = dadpkg.pkg()
        cfg = dad_oracle.make_cfg("iemocap")
        model = p.SSRLModel().cuda()
        step = p.DADStep(model, p.ConfigView(cfg, flavor="iemocap"), precision="fp32", rng="explicit",
                         comm=p.ProcessGroupComm())
        st = synth.make_state(SEED, 1)
        gh.load_state(step, st)
        orc = dad_oracle.DADOracle(*synth.init_weights(SEED)[:4], cfg)
        orc.load_state(st)

        def allreduce(v):
            t = torch.from_numpy(np.ascontiguousarray(v, np.float64))
            dist.all_reduce(t)
            return t.numpy()

        msgs = []
        for k, epoch in enumerate(SCHEDULE):
            inp = synth.make_step_inputs(SEED + 100 * rank, k, B, T)
            o = gh.run_step(step, inp, epoch)
            r = orc.step(inp, epoch, allreduce=allreduce, world=world)
            gh.close(o["total_loss"], r["losses_mean"][0], 1e-4, "rank mean total loss")
            np.testing.assert_array_equal(o["mask"], r["mask"])
            for i in range(4):
                gh.close_grad(o["grads"][i], r["grads_mean"][i], "rank %d step %d mean grad %d" % (rank, k, i))
                gh.close_grad(o["student"][i], r["student"][i], "rank %d step %d student %d" % (rank, k, i))
                gh.close_grad(o["teacher"][i], r["teacher"][i], "rank %d step %d teacher %d" % (rank, k, i))
            np.testing.assert_allclose(o["dacp"][0:4], orc.dacp.tau, rtol=0, atol=1e-6)
            np.testing.assert_allclose(o["dacp"][12:16], orc.dacp.score_cnt, rtol=0, atol=0)
            msgs.append(o["student"][0].copy())
        # replicas agree bit-for-bit
        mine = torch.from_numpy(np.concatenate([m.reshape(-1) for m in msgs]).astype(np.float64))
        other = mine.clone()
        dist.broadcast(other, src=0)
        assert torch.equal(mine, other), "ranks diverged"
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except BaseException as e:  # report to the parent instead of hanging it
        import traceback
        q.put((rank, "FAIL: %r\n%s" % (e, traceback.format_exc())))


SCHEDULE16 = [35, 60, 60]


def _rank_main_fp16(rank, world, port, q):
    """The timed mode's DP path: fp16 operands, each step naming its next batch (its rows prepared inside
    this step's launches, the default; and its clean rows, or all of them, on a side stream under the
    exchange, DADStep.prep_under_exchange), gloo exchange.  Per rank: every step against the
    oracle's DP step on this rank's shard within the fp16 bounds of test_gpu_throughput_parity
    (losses 1e-4, mask bit-exact; logits within test_gpu_16bit's bound for short synthetic rows); the chain with next-batch preparation equals the
    chain without it bit for bit; the replicas stay bit-identical."""
    try:
        import torch
        import torch.distributed as dist
        import dadpkg
        import gpu_harness as gh
        from oracle import dad_oracle, synth
        from test_gpu_throughput_parity import TOL, _cos, _normrel
        from test_gpu_16bit import LOGIT_TOL
        tol = TOL["fp16"]
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        import datetime
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=120))
        p = dadpkg.pkg()
        cfg = dad_oracle.make_cfg("iemocap")
        st = synth.make_state(SEED, 1)
        dev = torch.device("cuda")
        inps = [synth.make_step_inputs(SEED + 100 * rank, k, B, T) for k in range(len(SCHEDULE16))]

        def dev_batch(inp):
            c, n, d = gh.batches(inp)
            mv = lambda b: {"net_input": {k: v.to(dev) for k, v in b["net_input"].items()}, "labels": b["labels"].to(dev)}
            # the dtypes DADStep uses, so the draws are not copied again (the prepared-ahead rows are
            # keyed on the next batch's device pointers)
            dt = {"nw": torch.float32, "ns": torch.float32, "u": torch.float32, "start": torch.int64,
                  "keep1": torch.bool, "keep2": torch.bool}
            return mv(c), mv(n), {k: torch.from_numpy(np.asarray(v)).to(dev, dt[k]) for k, v in d.items()}

        batches = [dev_batch(i) for i in inps]

        def allreduce(v):
            t = torch.from_numpy(np.ascontiguousarray(v, np.float64))
            dist.all_reduce(t)
            return t.numpy()

        def chain(ahead, check, split=0):
            model = p.SSRLModel().cuda()
            step = p.DADStep(model, p.ConfigView(cfg, flavor="iemocap"), precision="fp16", rng="explicit",
                             comm=p.ProcessGroupComm(), prep_under_exchange=split)
            gh.load_state(step, st)
            orc = None
            if check:
                orc = dad_oracle.DADOracle(*synth.init_weights(SEED)[:4], cfg)
                orc.load_state(st)
            prepped, losses = [], []
            for k, epoch in enumerate(SCHEDULE16):
                c, n, d = batches[k]
                nxt = batches[k + 1] if ahead and k + 1 < len(batches) and SCHEDULE16[k + 1] == epoch else None
                out = step.step(c, n, epoch, draws=d, next_batch=nxt)
                torch.cuda.synchronize()
                prepped.append(step.last_prepped)
                losses.append({key: float(v) for key, v in out.items()})
                if check:
                    o = {kk: (v.detach().cpu().numpy() if torch.is_tensor(v) else v) for kk, v in step.outputs(B, B).items()}
                    r = orc.step(inps[k], epoch, allreduce=allreduce, world=world)
                    err = abs(losses[-1]["total_loss"] - r["losses_mean"][0]) / max(1.0, abs(r["losses_mean"][0]))
                    assert err <= tol["loss"], (rank, k, "total loss", err)
                    assert np.array_equal(o["mask"], r["mask"]), (rank, k, "mask")
                    # synthetic 40-frame utterances: test_gpu_16bit's fp16 logit bound (the golden
                    # replays hold north_star's 1e-4; losses are held to it here too)
                    for key in ("z_clean",) + (("z_strong", "z_teacher") if epoch >= 30 else ()):
                        assert gh.rel(o[key], r[key]) <= LOGIT_TOL["fp16"], (rank, k, key, gh.rel(o[key], r[key]))
                    g = np.concatenate([x.reshape(-1) for x in gh.unflat(o["grad"])])
                    gr = np.concatenate([np.asarray(x).reshape(-1) for x in r["grads_mean"]])
                    assert _normrel(g, gr) <= tol["grad"] and _cos(g, gr) >= tol["cos"], (rank, k, _normrel(g, gr))
                    for name, flat in (("student", step.model.student_flat), ("teacher", step.model.teacher_flat)):
                        got = gh.unflat(flat.detach().cpu().numpy())
                        assert max(_normrel(a, b_) for a, b_ in zip(got, r[name])) <= tol["param"], (rank, k, name)
            state = torch.cat([step.model.student_flat.detach(), step.model.teacher_flat.detach(), step.exp_avg,
                               step.exp_avg_sq, step.dacp]).cpu()
            return state, losses, prepped

        plain, plain_losses, plain_prepped = chain(False, True)
        # the next batch's rows inside this step's launches (the default at every N)
        ahead, ahead_losses, ahead_prepped = chain(True, False)
        assert not any(plain_prepped) and ahead_prepped == [False, False, True], ahead_prepped
        assert torch.equal(plain, ahead) and plain_losses == ahead_losses, "next-batch preparation changed the DP chain"
        # the clean rows, and all of the next batch's rows, on a side stream under the exchange
        for split in (1, 3):
            tl, tl_losses, tl_prepped = chain(True, False, split=split)
            assert tl_prepped == [False, False, True] and torch.equal(plain, tl) and plain_losses == tl_losses, split
        other = plain.clone().double()
        dist.broadcast(other, src=0)
        assert torch.equal(plain.double(), other), "ranks diverged"
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except BaseException as e:  # report to the parent instead of hanging it
        import traceback
        q.put((rank, "FAIL: %r\n%s" % (e, traceback.format_exc())))


@pytest.mark.parametrize("fp16", [False, True], ids=["fp32", "fp16_ahead"])
def test_dp_step_two_ranks_match_oracle(fp16):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main_fp16 if fp16 else _rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in procs:
            rank, msg = q.get(timeout=300)
            res[rank] = msg
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.exitcode is None:
                p.kill()
    assert res == {0: "ok", 1: "ok"}, res


def test_bench_spawns_ranks_gloo():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--comm", "gloo",
                        "--steps", "5", "--warmup", "2", "--no-cpu-baseline", "--no-data-path", "--fp32-steps", "0"],
                       cwd=root, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2
    assert line["config"]["parallelism"] == "dp2"
    assert line["config"]["global_batch"] == 128
    assert line["comm"]["transport"] == "gloo" and line["comm"]["ranks_seen"] == 2
    assert line["value"] > 0 and line["ecda_on_last_step"] == 1.0
