"""Consecutive 20-step segments of the headline step right after a 5-step warm-up (the driver's
--steps 20 --warmup 5 region) on a GPU that has idled for IDLE_S seconds first: does the step time
settle, and how fast.   python tools/region_segments.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

PKG = bench.PKG


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B, T = 64, 300
    model = PKG.SSRLModel().to(dev)
    P = bench.init_model_weights(model, seed=0)
    view = PKG.ConfigView(None, flavor="iemocap")
    step = PKG.DADStep(model, view, precision="fp16", rng="counter", seed=1000)
    data = bench.make_batches(P, bench.N_BATCHES, B, T, seed=17, device=dev)
    pos = [0]

    def run(n):
        for _ in range(n):
            i = pos[0]
            pos[0] += 1
            c, nb = data[i % len(data)]
            step.step(c, nb, 60, next_batch=data[(i + 1) % len(data)])
    # the gap between the warm-up and the timed region (bench.py: synchronize, snapshot, the event
    # timer's creation): host time, and what an idle gap of that order costs the first segment
    run(20)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    snap = bench.snapshot(model, step)
    timer = PKG._lib.KernelTimer(bench.event_every(20), 20 // bench.event_every(20) + 1,
                                 kernels=bench.timed_kernels("fp16", True))
    torch.cuda.synchronize()
    print("snapshot + timer creation: %.2f ms of host time" % ((time.perf_counter() - t0) * 1e3), flush=True)
    timer.stop()
    del snap
    for gap in (0.0, 0.001, 0.003, 0.010, 0.030):
        run(40)
        torch.cuda.synchronize()
        time.sleep(gap)
        t0 = time.perf_counter()
        run(20)
        torch.cuda.synchronize()
        print("gap %.0f ms: first 20-step segment %.1f us/step" % (gap * 1e3, (time.perf_counter() - t0) / 20 * 1e6), flush=True)
    for idle in (float(os.environ.get("IDLE_S", "2")), 0.0):
        run(3)
        torch.cuda.synchronize()
        time.sleep(idle)
        run(5)
        torch.cuda.synchronize()
        segs = []
        for _ in range(12):
            t0 = time.perf_counter()
            run(20)
            torch.cuda.synchronize()
            segs.append((time.perf_counter() - t0) / 20 * 1e6)
        print("after %.1f s idle: us/step per 20-step segment: %s" % (idle, " ".join("%.1f" % s for s in segs)), flush=True)


if __name__ == "__main__":
    main()
