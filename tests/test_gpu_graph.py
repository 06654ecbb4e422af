"""The fused step is enqueue-only and graph-capturable (include/dad.h conventions):
DADStep.step() captured into a torch.cuda.CUDAGraph with fixed device buffers replays bit for
bit like eager execution.

A captured step bakes its per-step host scalars (the Adam step count and the counter-RNG step
number) into the kernel arguments, so every replay repeats the step with the same scalars; the
eager side pins them the same way (adam_step / global_step reset before each call).  Every
replay reads and updates the device state (parameters, Adam moments, DACP thresholds and epoch
statistics), so K replays are K chained steps."""
import numpy as np
import pytest
import torch

import gpu_harness as gh
from oracle import dad_oracle, synth
from test_gpu_parity import _problem

pytestmark = pytest.mark.gpu
K = 10


def _device_batches(inp):
    clean, noisy, draws = gh.batches(inp)
    to = lambda d: {"net_input": {k: v.cuda() for k, v in d["net_input"].items()}, "labels": d["labels"].cuda()}
    dd = {k: torch.as_tensor(v).cuda() for k, v in draws.items()}
    for k in ("nw", "ns", "u"):
        dd[k] = dd[k].float()
    dd["keep1"] = dd["keep1"].bool()
    dd["keep2"] = dd["keep2"].bool()
    return to(clean), to(noisy), dd


def _state(step):
    return [t.detach().clone() for t in (step.model.student_flat, step.model.teacher_flat, step.exp_avg,
                                         step.exp_avg_sq, step.dacp, step.grad)]


@pytest.mark.parametrize("precision,rng", [("fp32", "explicit"), ("bf16", "counter"), ("fp16", "counter")])
def test_captured_step_replays_like_eager(precision, rng):
    cfg = dad_oracle.make_cfg("iemocap")
    inp = _problem(B=16, T=40, seed=21, Bn=12, Tn=50)
    st = synth.make_state(21, 1)
    clean, noisy, draws = _device_batches(inp)
    dr = draws if rng == "explicit" else None
    epoch = 60

    eager = gh.make_step(cfg, precision=precision, rng=rng, seed=3)
    gh.load_state(eager, st)
    n0, g0 = eager.adam_step, eager.global_step
    for _ in range(K):
        eager.adam_step, eager.global_step = n0, g0
        le = eager.step(clean, noisy, epoch, draws=dr)
    torch.cuda.synchronize()
    want = _state(eager)
    want_losses = {k: float(v) for k, v in le.items()}

    cap = gh.make_step(cfg, precision=precision, rng=rng, seed=3)
    gh.load_state(cap, st)
    # one eager step first (lazy buffers: workspace, per-shape outputs, the library's side
    # stream), then back to the start state
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        cap.step(clean, noisy, epoch, draws=dr)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    gh.load_state(cap, st)
    with torch.no_grad():
        cap.dacp[8:16].zero_()     # the warm-up step's epoch score sums / counts
    cap.adam_step, cap.global_step = n0, g0
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        lc = cap.step(clean, noisy, epoch, draws=dr)
    for _ in range(K):
        g.replay()
    torch.cuda.synchronize()
    got = _state(cap)
    for name, a, b in zip(("student", "teacher", "exp_avg", "exp_avg_sq", "dacp", "grad"), got, want):
        assert torch.equal(a, b), "%s differs after %d replays (max %.3g)" % (name, K, float((a - b).abs().max()))
    for k, v in lc.items():
        assert float(v) == want_losses[k], k
    # the replays really stepped: the parameters moved from the start state
    s0 = torch.from_numpy(gh.flat(st["student"])).cuda()
    assert not torch.equal(got[0], s0)


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
def test_cycled_graphs_with_rows_prepared_ahead(precision):
    """bench.py --launch graph with the next batch prepared in each tail launch: graphs of the
    steps g0, g0+1 on batches A, B, each preparing the next graph's rows (the last one for g0:
    next_counter), after one eager priming step that prepares A's.  Replays cycle the two graphs;
    the eager side runs the same chain with its counters pinned (global_step reset per step)."""
    import bench
    cfg = dad_oracle.make_cfg("iemocap")
    ins = [_problem(B=16, T=40, seed=s, Bn=12, Tn=50) for s in (31, 32)]
    st = synth.make_state(21, 1)
    data = []
    for inp in ins:
        c, n, _ = _device_batches(inp)
        data.append((c, n))
    epoch, R = 60, 6

    eager = gh.make_step(cfg, precision=precision, rng="counter", seed=3)
    gh.load_state(eager, st)
    g0 = eager.global_step + 1
    eager.step(*data[1], epoch, next_batch=data[0])            # the priming step (counter g0 - 1)
    a0 = eager.adam_step
    seen = []
    for k in range(R):
        i = k % 2
        eager.global_step, eager.adam_step = g0 + i, a0 + i
        eager.step(*data[i], epoch, next_batch=data[1 - i], next_counter=g0 if i == 1 else None)
        seen.append(eager.last_prepped)
    torch.cuda.synchronize()
    assert all(seen)
    want = _state(eager)

    cap = gh.make_step(cfg, precision=precision, rng="counter", seed=3)
    gh.load_state(cap, st)
    graphs = bench.capture_steps(cap, data, epoch, ahead=True)
    assert len(graphs) == 2 and cap.global_step == g0 + 2
    for k in range(R):
        graphs[k % 2][0].replay()
    torch.cuda.synchronize()
    got = _state(cap)
    for name, a, b in zip(("student", "teacher", "exp_avg", "exp_avg_sq", "dacp", "grad"), got, want):
        assert torch.equal(a, b), "%s differs after %d replays (max %.3g)" % (name, R, float((a - b).abs().max()))
