"""Launch-mode probe: the same fused fp16 step (B=64, T=300, bench.py's resident batches) timed
as eager launches, as one hipGraph per step, and as one hipGraph holding 8 consecutive steps.
Prints one line per mode (us per step, median of 3 rounds of 200 steps).

    python tools/graph_probe.py [--steps 200] [--rounds 3]
"""
import argparse
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

PKG = bench.PKG


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--precision", default="fp16")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    model = PKG.SSRLModel().to(dev)
    P = bench.init_model_weights(model, seed=0)
    step = PKG.DADStep(model, PKG.ConfigView(None, flavor="iemocap"), precision=args.precision, rng="counter", seed=1)
    data = bench.make_batches(P, 8, 64, 300, seed=17, device=dev)
    for i in range(30):
        step.step(*data[i % 8], 60)
    torch.cuda.synchronize()

    def timeit(fn, n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn(n)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e6

    def eager(n):
        for i in range(n):
            step.step(*data[i % 8], 60)

    per_step = []
    for c, nb in data:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step.step(c, nb, 60)
        per_step.append(g)

    def graph1(n):
        for i in range(n):
            per_step[i % 8].replay()

    g8 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g8):
        for c, nb in data:
            step.step(c, nb, 60)

    def graph8(n):
        for _ in range(n // 8):
            g8.replay()

    small = torch.zeros(64, device=dev)

    def eager_spacer(n):
        # a one-block fill between steps: does the optim -> encoder gap move in front of it?
        for i in range(n):
            step.step(*data[i % 8], 60)
            small.fill_(float(i))

    res = {"eager": [], "eager_spacer": [], "graph_per_step": [], "graph_8_steps": []}
    for _ in range(args.rounds):
        res["eager"].append(timeit(eager, args.steps))
        res["eager_spacer"].append(timeit(eager_spacer, args.steps))
        res["graph_per_step"].append(timeit(graph1, args.steps))
        res["graph_8_steps"].append(timeit(graph8, args.steps // 8 * 8))
    for k, v in res.items():
        print("%-16s %.1f us/step (rounds %s)" % (k, statistics.median(v), ", ".join("%.1f" % x for x in v)))
    if os.environ.get("PROBE_TRACE"):
        eager_spacer(8)
        for i in range(8):   # two spacers: is the optim -> next launch delay the first spacer's alone?
            step.step(*data[i % 8], 60)
            small.fill_(float(i))
            small.fill_(float(-i))
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
