"""What a 20-step timed region pays before the GPU reaches its steady rate: 5 warm-up steps, then
(variant) a KernelTimer as bench.py creates it / a host pause of 1 or 10 ms / nothing, a
synchronize, and 20 timed steps; 200-step reference.   python tools/short_region.py"""
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
    PKG.lib()
    model = PKG.SSRLModel().to(dev)
    P = bench.init_model_weights(model, seed=0)
    view = PKG.ConfigView(None, flavor="iemocap")
    step = PKG.DADStep(model, view, precision="fp16", rng="counter", seed=1000)
    data = bench.make_batches(P, bench.N_BATCHES, 64, 300, seed=17, device=dev)
    pos = [0]

    def run(n):
        for _ in range(n):
            i = pos[0]
            pos[0] += 1
            c, nb = data[i % len(data)]
            step.step(c, nb, 60, next_batch=data[(i + 1) % len(data)])

    run(200)
    for rnd in range(2):
        for var in ("none", "timer", "pause1ms", "pause10ms", "long200"):
            run(5)
            torch.cuda.synchronize()
            timer = None
            if var == "timer":
                timer = PKG._lib.KernelTimer(bench.event_every(20), 21, kernels=["tail"])
            elif var.startswith("pause"):
                time.sleep(0.001 if var == "pause1ms" else 0.01)
            torch.cuda.synchronize()
            k = 200 if var == "long200" else 20
            t0 = time.perf_counter()
            run(k)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / k
            if timer is not None:
                timer.stop()
            print("r%d %-10s %7.1f us/step" % (rnd, var, dt * 1e6), flush=True)


if __name__ == "__main__":
    main()
